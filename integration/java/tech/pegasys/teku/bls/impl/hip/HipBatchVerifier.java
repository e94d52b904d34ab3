/*
 * Public entry of the GPU batch path for callers outside the SPI: the
 * gossip service's batch with its failure path in one device call
 * (tbls_batch_verify_each, include/tekubls.h), used by
 * HipAggregatingSignatureVerificationService.  Mirror and tests:
 * teku_amd/service.py (_hip_batch_each), tests/test_gpu_configs.py
 * test_config4_16k_through_service.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.util.List;
import org.apache.tuweni.bytes.Bytes;
import tech.pegasys.teku.bls.BLSPublicKey;
import tech.pegasys.teku.bls.BLSSignature;
import tech.pegasys.teku.bls.impl.BlsException;

public final class HipBatchVerifier {
  private HipBatchVerifier() {}

  /* Library devices (tbls_device_count): the service runs one worker per device. */
  public static int deviceCount() {
    return HipLoader.INSTANCE.isPresent() ? Math.max(1, TekuBlsHip.deviceCount()) : 1;
  }

  /*
   * BLS.batchVerify(keys, messages, signatures) over all sets as one
   * randomized device batch (BLS.java:230-336); when it fails, okPerSet[i] =
   * BLS.fastAggregateVerify(set i) (BLS.java:185-207), settled on the devices
   * that ran the batch from its own Miller work.  Returns the batch verdict
   * (okPerSet all true when it passes).  A set with no keys is false and makes
   * the batch false.  nGpus: at most that many devices (0 = every idle one);
   * a caller with more batches waiting passes 1.
   */
  public static boolean batchVerifyEach(final List<List<BLSPublicKey>> keys, final List<Bytes> messages,
                                        final List<BLSSignature> signatures, final int nGpus, final boolean[] okPerSet) {
    final int n = keys.size();
    if (messages.size() != n || signatures.size() != n || okPerSet.length < n) {
      throw new IllegalArgumentException("Different collection sizes");
    }
    int k = 0;
    int m = 0;
    for (int i = 0; i < n; i++) {
      k += keys.get(i).size();
      m += messages.get(i).size();
    }
    final byte[] pks = new byte[48 * k];
    final int[] nPks = new int[n];
    final byte[] msgs = new byte[m];
    final int[] msgOff = new int[n + 1];
    final byte[] sigs = new byte[96 * n];
    final long[] rand = new long[n];
    int kk = 0;
    for (int i = 0; i < n; i++) {
      final List<BLSPublicKey> ks = keys.get(i);
      for (BLSPublicKey pk : ks) {
        System.arraycopy(pk.toBytesCompressed().toArrayUnsafe(), 0, pks, 48 * kk++, 48);
      }
      nPks[i] = ks.size();
      final byte[] msg = messages.get(i).toArrayUnsafe();
      System.arraycopy(msg, 0, msgs, msgOff[i], msg.length);
      msgOff[i + 1] = msgOff[i] + msg.length;
      System.arraycopy(signatures.get(i).toBytesCompressed().toArrayUnsafe(), 0, sigs, 96 * i, 96);
      rand[i] = HipBLS12381.nextBatchRandomMultiplier();
    }
    final int[] ok = new int[1];
    final int[] each = new int[n];
    final int rc = TekuBlsHip.batchVerifyEach(pks, nPks, msgs, msgOff, sigs, rand, nGpus, ok, each);
    if (rc != TekuBlsHip.SUCCESS) {
      throw new BlsException("GPU BLS backend: batchVerifyEach failed, code " + rc);
    }
    for (int i = 0; i < n; i++) {
      okPerSet[i] = each[i] == 1;
    }
    return ok[0] == 1;
  }
}
