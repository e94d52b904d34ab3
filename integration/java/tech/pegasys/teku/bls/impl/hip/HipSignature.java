/*
 * Signature (impl/Signature.java) over the compressed bytes.  Mirror:
 * teku_amd/bls.py HipSignature.  fromBytes decodes on the calling thread
 * (tbls_sig_decode: blst_p2_uncompress's checks, no device call); the G2
 * subgroup check runs on the device when isInGroup is first asked, memoised,
 * or inside the batch.  Failures of the device are BlsExceptions, the failure
 * mode of a broken blst load.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.nio.charset.StandardCharsets;
import java.util.Arrays;
import java.util.List;
import java.util.Objects;
import org.apache.tuweni.bytes.Bytes;
import tech.pegasys.teku.bls.impl.BlsException;
import tech.pegasys.teku.bls.impl.PublicKey;
import tech.pegasys.teku.bls.impl.PublicKeyMessagePair;
import tech.pegasys.teku.bls.impl.Signature;

final class HipSignature implements Signature {
  static final byte[] INFINITY = HipPublicKey.infinity(96);
  static final byte[] ETH2_DST = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_".getBytes(StandardCharsets.US_ASCII);

  private final byte[] bytes;
  private volatile Boolean inGroup;

  HipSignature(final byte[] compressed) {
    this.bytes = compressed.clone();
  }

  /* BlstSignature.fromBytes (BlstSignature.java:35-47) */
  static HipSignature fromBytes(final Bytes compressed) {
    if (compressed.size() != 96) {
      throw new BlsException("Expected 96 bytes of input but got " + compressed.size());
    }
    final byte[] b = compressed.toArrayUnsafe();
    // BAD_ENCODING, POINT_NOT_ON_CURVE, or POINT_NOT_IN_GROUP for x = 0: P2_Affine throws
    if (TekuBlsHip.sigDecode(b) != TekuBlsHip.SUCCESS) {
      throw new BlsException("Deserialization of signature bytes failed: " + compressed);
    }
    return new HipSignature(b);
  }

  static HipSignature fromSignature(final Signature s) {
    if (s instanceof HipSignature h) {
      return h;
    }
    return fromBytes(s.toBytesCompressed());
  }

  byte[] raw() {
    return bytes;
  }

  @Override
  public Bytes toBytesCompressed() {
    return Bytes.wrap(bytes.clone());
  }

  @Override
  public boolean verify(final List<PublicKeyMessagePair> keysToMessages) {
    final int n = keysToMessages.size();
    final byte[] pks = new byte[48 * n];
    final int[] off = new int[n + 1];
    for (int i = 0; i < n; i++) {
      final HipPublicKey pk = HipPublicKey.fromPublicKey(keysToMessages.get(i).getPublicKey());
      if (pk.isInfinity()) {
        return false; // BlstSignature.java:106-111
      }
      System.arraycopy(pk.raw(), 0, pks, 48 * i, 48);
      off[i + 1] = off[i] + keysToMessages.get(i).getMessage().size();
    }
    final byte[] msgs = new byte[off[n]];
    for (int i = 0; i < n; i++) {
      keysToMessages.get(i).getMessage().copyTo(msgs, off[i]);
    }
    final int[] ok = new int[1];
    final int rc = TekuBlsHip.aggregateVerify(pks, msgs, off, bytes, ok);
    if (rc == TekuBlsHip.DEVICE_ERROR) {
      throw new BlsException("GPU BLS backend: device error");
    }
    return rc == TekuBlsHip.SUCCESS && ok[0] == 1;
  }

  @Override
  public boolean verify(final List<PublicKey> publicKeys, final Bytes message) {
    return verify(HipPublicKey.aggregate(publicKeys.stream().map(HipPublicKey::fromPublicKey).toList()), message);
  }

  @Override
  public boolean verify(final PublicKey publicKey, final Bytes message) {
    return coreVerify(HipPublicKey.fromPublicKey(publicKey), message, ETH2_DST);
  }

  @Override
  public boolean verify(final PublicKey publicKey, final Bytes message, final String dst) {
    return coreVerify(HipPublicKey.fromPublicKey(publicKey), message, dst.getBytes(StandardCharsets.US_ASCII));
  }

  private boolean coreVerify(final HipPublicKey pk, final Bytes message, final byte[] dst) {
    final int[] ok = new int[1];
    final int rc = TekuBlsHip.verify(pk.raw(), message.toArrayUnsafe(), bytes, dst, ok);
    if (rc == TekuBlsHip.DEVICE_ERROR) {
      throw new BlsException("GPU BLS backend: device error");
    }
    return rc == TekuBlsHip.SUCCESS && ok[0] == 1;
  }

  @Override
  public boolean isInfinity() {
    return Arrays.equals(bytes, INFINITY);
  }

  // BlstSignature.isInGroup (BlstSignature.java:147-149), memoised: one
  // device check per object at most; the infinity point is in the group
  @Override
  public boolean isInGroup() {
    Boolean g = inGroup;
    if (g == null) {
      if (isInfinity()) {
        g = Boolean.TRUE;
      } else {
        final int rc = TekuBlsHip.sigValidate(bytes, new int[1]);
        if (rc == TekuBlsHip.DEVICE_ERROR) {
          throw new BlsException("GPU BLS backend: device error");
        }
        g = rc == TekuBlsHip.SUCCESS;
      }
      inGroup = g;
    }
    return g;
  }

  // BlstSignature.java:152-165: the compressed bytes' hash, and equal to any
  // Signature (of any implementation) with the same compressed bytes
  @Override
  public int hashCode() {
    return toBytesCompressed().hashCode();
  }

  @Override
  public boolean equals(final Object obj) {
    if (this == obj) {
      return true;
    }
    if (!(obj instanceof Signature o)) {
      return false;
    }
    return Objects.equals(toBytesCompressed(), o.toBytesCompressed());
  }
}
