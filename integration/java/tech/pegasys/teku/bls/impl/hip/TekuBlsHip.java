/*
 * Native entry points of libtekubls_hip.so (include/tekubls.h), bound by
 * integration/native/tekubls_jni.c.  Every method returns the library status
 * code (TBLS_*); outputs go to the caller's arrays.  No Java memory is
 * referenced after a call returns (the glue copies in and out).
 */
package tech.pegasys.teku.bls.impl.hip;

final class TekuBlsHip {
  static final int SUCCESS = 0;
  static final int BAD_ENCODING = 1;
  static final int POINT_NOT_ON_CURVE = 2;
  static final int POINT_NOT_IN_GROUP = 3;
  static final int AGGR_TYPE_MISMATCH = 4;
  static final int VERIFY_FAIL = 5;
  static final int PK_IS_INFINITY = 6;
  static final int BAD_SCALAR = 7;
  static final int DEVICE_ERROR = 8;
  static final int BAD_ARGUMENT = 9;

  private TekuBlsHip() {}

  static native int init(int nDevices, int flags); // tbls_init
  static native void shutdown(); // tbls_shutdown
  static native int deviceCount(); // tbls_device_count

  /* host decoding, no device call: BlstPublicKey / BlstSignature.fromBytes */
  static native int pkDecode(byte[] pk48); // tbls_pk_decode
  static native int sigDecode(byte[] sig96); // tbls_sig_decode
  static native int pkDecodeMany(byte[] pks, int n, byte[] codes); // tbls_pk_decode_many
  static native int sigDecodeMany(byte[] sigs, int n, byte[] codes); // tbls_sig_decode_many

  static native int pkValidate(byte[] pk48); // tbls_pk_validate
  static native int sigValidate(byte[] sig96, int[] isInf); // tbls_sig_validate
  static native int aggregatePks(byte[] pks, int k, byte[] out48); // tbls_aggregate_pks
  static native int aggregateSigs(byte[] sigs, int k, byte[] out96); // tbls_aggregate_sigs
  static native int sign(byte[] sk32, byte[] msg, byte[] dst, byte[] out96); // tbls_sign
  static native int skToPk(byte[] sk32, byte[] out48); // tbls_sk_to_pk
  static native int verify(byte[] pk48, byte[] msg, byte[] sig96, byte[] dst, int[] ok); // tbls_verify

  /* aggregateVerify: n (pk, msg) pairs, messages concatenated with msgOff[n + 1] */
  static native int aggregateVerify(byte[] pks, byte[] msgs, int[] msgOff, byte[] sig96, int[] ok); // tbls_aggregate_verify

  /* Sets flattened: pks (sum nPks * 48 bytes), nPks[n], messages concatenated
   * with msgOff[n + 1], sigs (n * 96), rand[n] (unsigned 64-bit). */
  static native int batchVerify(byte[] pks, int[] nPks, byte[] msgs, int[] msgOff, byte[] sigs, long[] rand,
                                int nGpus, int[] ok); // tbls_batch_verify

  /* batchVerify + every set's verdict when the batch fails, settled from the
   * batch's own Miller work (okPerSet[n]; all 1 when ok[0] == 1) */
  static native int batchVerifyEach(byte[] pks, int[] nPks, byte[] msgs, int[] msgOff, byte[] sigs, long[] rand,
                                    int nGpus, int[] ok, int[] okPerSet); // tbls_batch_verify_each

  /* device-resident validator key table */
  static native int pkTableLoad(byte[] pks, int k, byte[] codes); // tbls_pk_table_load
  static native int batchVerifyIdx(int[] keyIdx, int[] nPks, byte[] msgs, int[] msgOff, byte[] sigs, long[] rand,
                                   int nGpus, int[] ok); // tbls_batch_verify_idx

  /* per-set verdicts in one device pass */
  static native int verifyEach(byte[] pks, int[] nPks, byte[] msgs, int[] msgOff, byte[] sigs, int nGpus,
                               int[] okPerSet); // tbls_verify_each

  /* batched deserialization / aggregation */
  static native int pkValidateMany(byte[] pks, int n, byte[] codes); // tbls_pk_validate_many
  static native int sigValidateMany(byte[] sigs, int n, byte[] codes, byte[] isInf); // tbls_sig_validate_many
  static native int aggregateSigsMany(byte[] sigs, int[] off, int groups, byte[] out, int[] status); // tbls_aggregate_sigs_many
}
