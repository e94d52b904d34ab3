/*
 * Native entry points of include/tekukzg.h (the KZG side of
 * libtekubls_hip.so), bound by integration/native/tekukzg_jni.c.  Each
 * method returns the TKZG_* status; HipKZG turns a non-zero status into the
 * exception CKZG4844 would throw.
 */
package tech.pegasys.teku.kzg;

final class TekuKzgHip {
  static final int OK = 0;
  static final int BADARGS = 1;
  static final int ERROR = 2;
  static final int MALLOC = 3;

  private TekuKzgHip() {}

  static native int loadTrustedSetup(byte[] g1Monomial, byte[] g1Lagrange, byte[] g2Monomial, long precompute);
  static native int freeTrustedSetup();
  static native int blobToKzgCommitment(byte[] blob, byte[] out48);
  static native int computeBlobKzgProof(byte[] blob, byte[] commitment48, byte[] out48);
  static native int verifyBlobKzgProof(byte[] blob, byte[] commitment48, byte[] proof48, int[] ok);
  static native int verifyBlobKzgProofBatch(byte[] blobs, byte[] commitments, byte[] proofs, long count, int[] ok);
  static native String lastError();
}
