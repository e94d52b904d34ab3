/*
 * PublicKey (impl/PublicKey.java) over the compressed bytes.  fromBytes
 * decodes on the calling thread (tbls_pk_decode: blst_p1_uncompress's checks,
 * no device call); validity (!infinity && in G1) is computed on the device
 * when first asked and memoised, as BlstPublicKey.java:74-75.  Mirror:
 * teku_amd/bls.py HipPublicKey.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.util.Arrays;
import java.util.List;
import java.util.Objects;
import org.apache.tuweni.bytes.Bytes48;
import tech.pegasys.teku.bls.impl.BlsException;
import tech.pegasys.teku.bls.impl.PublicKey;

final class HipPublicKey implements PublicKey {
  static final byte[] INFINITY = infinity(48);

  private final byte[] bytes;
  private volatile Boolean valid;

  HipPublicKey(final byte[] compressed, final Integer checkedCode) {
    this.bytes = compressed.clone();
    this.valid = checkedCode == null ? null : checkedCode == TekuBlsHip.SUCCESS;
  }

  static byte[] infinity(final int n) {
    final byte[] b = new byte[n];
    b[0] = (byte) 0xc0;
    return b;
  }

  /* BlstPublicKey.fromBytes: decode failures throw (BlstPublicKey.java:38-45) */
  static HipPublicKey fromBytes(final Bytes48 compressed) {
    final byte[] b = compressed.toArrayUnsafe();
    // BAD_ENCODING, POINT_NOT_ON_CURVE, or POINT_NOT_IN_GROUP for x = 0 (blst:
    // "(0, +-2) is not in group"): P1_Affine throws
    if (TekuBlsHip.pkDecode(b) != TekuBlsHip.SUCCESS) {
      throw new BlsException("Deserialization of public key bytes failed: " + compressed);
    }
    return new HipPublicKey(b, null);
  }

  static HipPublicKey fromPublicKey(final PublicKey pk) {
    if (pk instanceof HipPublicKey h) {
      return h;
    }
    return fromBytes(pk.toBytesCompressed());
  }

  static HipPublicKey aggregate(final List<HipPublicKey> keys) {
    if (keys.isEmpty()) {
      throw new IllegalArgumentException("empty public key list"); // BlstPublicKey.java:56
    }
    final byte[] blob = new byte[48 * keys.size()];
    for (int i = 0; i < keys.size(); i++) {
      System.arraycopy(keys.get(i).bytes, 0, blob, 48 * i, 48);
    }
    final byte[] out = new byte[48];
    final int rc = TekuBlsHip.aggregatePks(blob, keys.size(), out);
    if (rc == TekuBlsHip.BAD_ENCODING || rc == TekuBlsHip.POINT_NOT_ON_CURVE) {
      throw new BlsException("Deserialization of public key bytes failed");
    }
    if (rc != TekuBlsHip.SUCCESS) {
      throw new BlsException("GPU BLS backend: aggregate failed, code " + rc);
    }
    return new HipPublicKey(out, null);
  }

  byte[] raw() {
    return bytes;
  }

  boolean isInfinity() {
    return Arrays.equals(bytes, INFINITY);
  }

  @Override
  public Bytes48 toBytesCompressed() {
    return Bytes48.wrap(bytes.clone());
  }

  @Override
  public void forceValidation() throws IllegalArgumentException {
    if (!isValid()) {
      throw new IllegalArgumentException("Invalid PublicKey: " + toBytesCompressed());
    }
  }

  @Override
  public boolean isInGroup() {
    return isInfinity() || isValid();
  }

  @Override
  public boolean isValid() {
    Boolean v = valid;
    if (v == null) {
      final int rc = TekuBlsHip.pkValidate(bytes);
      if (rc == TekuBlsHip.DEVICE_ERROR) {
        throw new BlsException("GPU BLS backend: device error");
      }
      v = rc == TekuBlsHip.SUCCESS;
      valid = v;
    }
    return v;
  }

  // BlstPublicKey.java:115-130: the compressed bytes' hash, and equal to any
  // PublicKey (of any implementation) with the same compressed bytes
  @Override
  public int hashCode() {
    return toBytesCompressed().hashCode();
  }

  @Override
  public boolean equals(final Object obj) {
    if (this == obj) {
      return true;
    }
    if (!(obj instanceof PublicKey o)) {
      return false;
    }
    return Objects.equals(toBytesCompressed(), o.toBytesCompressed());
  }
}
