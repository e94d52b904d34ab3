/*
 * KZG (infrastructure/kzg/.../KZG.java) on libtekubls_hip.so, with the
 * structure of CKZG4844 (CKZG4844.java:40-150): one trusted setup at a time,
 * loading the same file twice is a no-op, every failure is a KZGException.
 * Selected where KZG.getInstance() is wired (KZG.java), e.g. behind a system
 * property, falling back to CKZG4844.  Mirror and tests: teku_amd/kzg.py,
 * tests/test_gpu_kzg.py.
 */
package tech.pegasys.teku.kzg;

import java.util.List;
import java.util.Optional;
import org.apache.tuweni.bytes.Bytes;

public final class HipKZG implements KZG {
  private static final int PRECOMPUTE_DEFAULT = 0;
  private static HipKZG instance;

  private Optional<String> loadedTrustedSetupFile = Optional.empty();

  public static synchronized HipKZG getInstance() {
    if (instance == null) {
      instance = new HipKZG();
    }
    return instance;
  }

  private HipKZG() {
    try {
      System.loadLibrary("tekukzg_jni"); // links libtekubls_hip.so
    } catch (final UnsatisfiedLinkError ex) {
      throw new KZGException("Failed to load the GPU KZG library", ex);
    }
  }

  private static void check(final int rc, final String what) {
    if (rc == TekuKzgHip.OK) {
      return;
    }
    final String msg = what + ": " + TekuKzgHip.lastError();
    // as CKZG4844JNI: argument errors are CKZGException(C_KZG_BADARGS), a
    // missing setup a RuntimeException; both wrapped by the callers below
    throw rc == TekuKzgHip.BADARGS ? new IllegalArgumentException(msg) : new IllegalStateException(msg);
  }

  @Override
  public synchronized void loadTrustedSetup(final String trustedSetupFile) throws KZGException {
    if (loadedTrustedSetupFile.isPresent() && loadedTrustedSetupFile.get().equals(trustedSetupFile)) {
      return;
    }
    try {
      if (loadedTrustedSetupFile.isPresent()) {
        freeTrustedSetup();
      }
      final TrustedSetup ts = CKZG4844Utils.parseTrustedSetupFile(trustedSetupFile);
      check(TekuKzgHip.loadTrustedSetup(CKZG4844Utils.flattenG1Points(ts.g1Monomial()),
                                        CKZG4844Utils.flattenG1Points(ts.g1Lagrange()),
                                        CKZG4844Utils.flattenG2Points(ts.g2Monomial()), PRECOMPUTE_DEFAULT),
            "loadTrustedSetup");
      loadedTrustedSetupFile = Optional.of(trustedSetupFile);
    } catch (final Exception ex) {
      throw new KZGException("Failed to load trusted setup from " + trustedSetupFile, ex);
    }
  }

  @Override
  public synchronized void freeTrustedSetup() throws KZGException {
    try {
      check(TekuKzgHip.freeTrustedSetup(), "freeTrustedSetup");
      loadedTrustedSetupFile = Optional.empty();
    } catch (final Exception ex) {
      throw new KZGException("Failed to free trusted setup", ex);
    }
  }

  @Override
  public boolean verifyBlobKzgProof(final Bytes blob, final KZGCommitment kzgCommitment, final KZGProof kzgProof)
      throws KZGException {
    try {
      final int[] ok = new int[1];
      check(TekuKzgHip.verifyBlobKzgProof(blob.toArrayUnsafe(), kzgCommitment.toArrayUnsafe(), kzgProof.toArrayUnsafe(), ok),
            "verifyBlobKzgProof");
      return ok[0] == 1;
    } catch (final Exception ex) {
      throw new KZGException("Failed to verify blob and commitment against KZG proof " + kzgProof, ex);
    }
  }

  @Override
  public boolean verifyBlobKzgProofBatch(final List<Bytes> blobs, final List<KZGCommitment> kzgCommitments,
                                         final List<KZGProof> kzgProofs) throws KZGException {
    try {
      final int[] ok = new int[1];
      check(TekuKzgHip.verifyBlobKzgProofBatch(CKZG4844Utils.flattenBlobs(blobs),
                                               CKZG4844Utils.flattenCommitments(kzgCommitments),
                                               CKZG4844Utils.flattenProofs(kzgProofs), blobs.size(), ok),
            "verifyBlobKzgProofBatch");
      return ok[0] == 1;
    } catch (final Exception ex) {
      throw new KZGException("Failed to verify blobs and commitments against KZG proofs " + kzgProofs, ex);
    }
  }

  @Override
  public KZGCommitment blobToKzgCommitment(final Bytes blob) throws KZGException {
    try {
      final byte[] out = new byte[BYTES_PER_G1];
      check(TekuKzgHip.blobToKzgCommitment(blob.toArrayUnsafe(), out), "blobToKzgCommitment");
      return KZGCommitment.fromArray(out);
    } catch (final Exception ex) {
      throw new KZGException("Failed to produce KZG commitment from blob", ex);
    }
  }

  @Override
  public KZGProof computeBlobKzgProof(final Bytes blob, final KZGCommitment kzgCommitment) throws KZGException {
    try {
      final byte[] out = new byte[BYTES_PER_G1];
      check(TekuKzgHip.computeBlobKzgProof(blob.toArrayUnsafe(), kzgCommitment.toArrayUnsafe(), out),
            "computeBlobKzgProof");
      return KZGProof.fromArray(out);
    } catch (final Exception ex) {
      throw new KZGException("Failed to compute KZG proof for blob with commitment " + kzgCommitment, ex);
    }
  }
}
