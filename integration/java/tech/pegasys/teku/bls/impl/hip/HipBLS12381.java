/*
 * BLS12381 SPI (infrastructure/bls/.../impl/BLS12381.java:34-157) on
 * libtekubls_hip.so, installed beside BlstBLS12381 with
 * BLS.setBlsImplementation (BLS.java:51-53).  Mirror and tests:
 * teku_amd/bls.py HipBLS12381, tests/test_gpu_bls.py.
 *
 * prepareBatchVerify only captures the set; completeBatchVerify draws the
 * randomizers (8 random bytes + 1, BlstBLS12381.java:191-195) and runs every
 * set of the batch as one device batch.  eager = true moves the signature's
 * G2 check into prepare, the point where BlstBLS12381 throws for it
 * (BlstTest.java:93-103); the verdicts are identical either way.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.security.SecureRandom;
import java.util.List;
import java.util.Random;
import org.apache.tuweni.bytes.Bytes;
import org.apache.tuweni.bytes.Bytes32;
import org.apache.tuweni.bytes.Bytes48;
import tech.pegasys.teku.bls.BatchSemiAggregate;
import tech.pegasys.teku.bls.impl.BLS12381;
import tech.pegasys.teku.bls.impl.BlsException;
import tech.pegasys.teku.bls.impl.KeyPair;
import tech.pegasys.teku.bls.impl.PublicKey;
import tech.pegasys.teku.bls.impl.SecretKey;
import tech.pegasys.teku.bls.impl.Signature;

public class HipBLS12381 implements BLS12381 {
  private static final SecureRandom RANDOM = new SecureRandom();
  private final boolean eager;
  private final int nGpus;

  public HipBLS12381() {
    this(false, 0);
  }

  public HipBLS12381(final boolean eager, final int nGpus) {
    this.eager = eager;
    this.nGpus = nGpus;
  }

  @Override
  public KeyPair generateKeyPair(final Random random) {
    final HipSecretKey sk = HipSecretKey.generateNew(random);
    return new KeyPair(sk, sk.derivePublicKey());
  }

  @Override
  public PublicKey publicKeyFromCompressed(final Bytes48 compressedPublicKeyBytes) throws BlsException {
    return HipPublicKey.fromBytes(compressedPublicKeyBytes);
  }

  @Override
  public Signature signatureFromCompressed(final Bytes compressedSignatureBytes) {
    return HipSignature.fromBytes(compressedSignatureBytes);
  }

  @Override
  public SecretKey secretKeyFromBytes(final Bytes32 secretKeyBytes) {
    return HipSecretKey.fromBytes(secretKeyBytes);
  }

  @Override
  public PublicKey aggregatePublicKeys(final List<? extends PublicKey> publicKeys) {
    return HipPublicKey.aggregate(publicKeys.stream().map(HipPublicKey::fromPublicKey).toList());
  }

  @Override
  public Signature aggregateSignatures(final List<? extends Signature> signatures) throws IllegalArgumentException {
    final byte[] blob = new byte[96 * signatures.size()];
    for (int i = 0; i < signatures.size(); i++) {
      System.arraycopy(HipSignature.fromSignature(signatures.get(i)).raw(), 0, blob, 96 * i, 96);
    }
    final byte[] out = new byte[96];
    final int rc = TekuBlsHip.aggregateSigs(blob, signatures.size(), out);
    if (rc == TekuBlsHip.DEVICE_ERROR) {
      throw new BlsException("GPU BLS backend: device error");
    }
    if (rc != TekuBlsHip.SUCCESS) {
      throw new IllegalArgumentException("Failed to aggregate signatures"); // BlstSignature.java:64-67
    }
    return new HipSignature(out);
  }

  @Override
  public BatchSemiAggregate prepareBatchVerify(final int index, final List<? extends PublicKey> publicKeys,
                                               final Bytes message, final Signature signature) {
    if (publicKeys.isEmpty()) {
      throw new IllegalArgumentException("empty public key list"); // BlstPublicKey.aggregate, l.56
    }
    final HipSignature sig = HipSignature.fromSignature(signature);
    if (eager && !sig.isInfinity() && !sig.isInGroup()) {
      throw new BlsException("Error in Blst, error code: BLST_POINT_NOT_IN_GROUP");
    }
    final List<HipPublicKey> keys = publicKeys.stream().map(HipPublicKey::fromPublicKey).toList();
    return new HipSemiAggregate(new HipSemiAggregate.SigSet(keys, message.toArray(), sig), true);
  }

  @Override
  public BatchSemiAggregate prepareBatchVerify2(final int index, final List<? extends PublicKey> publicKeys1,
                                                final Bytes message1, final Signature signature1,
                                                final List<? extends PublicKey> publicKeys2, final Bytes message2,
                                                final Signature signature2) {
    return new HipSemiAggregate((HipSemiAggregate) prepareBatchVerify(index, publicKeys1, message1, signature1),
                                (HipSemiAggregate) prepareBatchVerify(index + 1, publicKeys2, message2, signature2));
  }

  /* BlstBLS12381.nextBatchRandomMultiplier (l.191-195): 8 random bytes + 1;
   * the value 2^64 (probability 2^-64) is redrawn to fit the u64 ABI. */
  static long nextBatchRandomMultiplier() {
    long r;
    do {
      r = RANDOM.nextLong() + 1; // unsigned: 0 would be 2^64
    } while (r == 0);
    return r;
  }

  @Override
  public boolean completeBatchVerify(final List<? extends BatchSemiAggregate> preparedList) {
    if (preparedList.isEmpty()) {
      return true; // BlstBLS12381.java:163-165
    }
    int n = 0;
    int k = 0;
    int m = 0;
    for (BatchSemiAggregate p : preparedList) {
      if (!(p instanceof HipSemiAggregate s) || !s.valid) {
        return false; // l.169-177, 185-188
      }
      for (HipSemiAggregate.SigSet set : s.sets) {
        n++;
        k += set.keys().size();
        m += set.message().length;
      }
    }
    final byte[] pks = new byte[48 * k];
    final int[] nPks = new int[n];
    final byte[] msgs = new byte[m];
    final int[] msgOff = new int[n + 1];
    final byte[] sigs = new byte[96 * n];
    final long[] rand = new long[n];
    int i = 0;
    int kk = 0;
    for (BatchSemiAggregate p : preparedList) {
      for (HipSemiAggregate.SigSet set : ((HipSemiAggregate) p).sets) {
        for (HipPublicKey pk : set.keys()) {
          System.arraycopy(pk.raw(), 0, pks, 48 * kk++, 48);
        }
        nPks[i] = set.keys().size();
        System.arraycopy(set.message(), 0, msgs, msgOff[i], set.message().length);
        msgOff[i + 1] = msgOff[i] + set.message().length;
        System.arraycopy(set.signature().raw(), 0, sigs, 96 * i, 96);
        rand[i] = nextBatchRandomMultiplier();
        i++;
      }
    }
    final int[] ok = new int[1];
    final int rc = TekuBlsHip.batchVerify(pks, nPks, msgs, msgOff, sigs, rand, nGpus, ok);
    if (rc == TekuBlsHip.DEVICE_ERROR) {
      throw new BlsException("GPU BLS backend: device error");
    }
    return rc == TekuBlsHip.SUCCESS && ok[0] == 1;
  }
}
