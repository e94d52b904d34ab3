/*
 * SecretKey (impl/SecretKey.java).  KeyGen (draft-irtf-cfrg-bls-signature-04
 * section 2.3, as BlstSecretKey.generateNew) runs on the host; signing and
 * key derivation run on the device.  Mirror: teku_amd/bls.py HipSecretKey.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.math.BigInteger;
import java.nio.charset.StandardCharsets;
import java.security.GeneralSecurityException;
import java.security.MessageDigest;
import java.util.Arrays;
import java.util.Random;
import javax.crypto.Mac;
import javax.crypto.spec.SecretKeySpec;
import org.apache.tuweni.bytes.Bytes;
import org.apache.tuweni.bytes.Bytes32;
import tech.pegasys.teku.bls.impl.BlsException;
import tech.pegasys.teku.bls.impl.PublicKey;
import tech.pegasys.teku.bls.impl.SecretKey;
import tech.pegasys.teku.bls.impl.Signature;

final class HipSecretKey implements SecretKey {
  static final BigInteger CURVE_ORDER =
      new BigInteger("73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001", 16);

  private final byte[] k; // 32 bytes big-endian, reduced mod r

  HipSecretKey(final BigInteger v) {
    this.k = toBytes32(v.mod(CURVE_ORDER));
  }

  static HipSecretKey fromBytes(final Bytes32 b) {
    return new HipSecretKey(new BigInteger(1, b.toArrayUnsafe()));
  }

  static HipSecretKey generateNew(final Random random) {
    final byte[] ikm = new byte[128];
    random.nextBytes(ikm);
    return new HipSecretKey(keyGen(ikm));
  }

  private static byte[] toBytes32(final BigInteger v) {
    final byte[] b = v.toByteArray();
    final byte[] out = new byte[32];
    final int n = Math.min(b.length, 32);
    System.arraycopy(b, b.length - n, out, 32 - n, n);
    return out;
  }

  private static byte[] hmac(final byte[] key, final byte[] data) throws GeneralSecurityException {
    final Mac m = Mac.getInstance("HmacSHA256");
    m.init(new SecretKeySpec(key, "HmacSHA256"));
    return m.doFinal(data);
  }

  /* HKDF-based KeyGen: salt = SHA256 chain from "BLS-SIG-KEYGEN-SALT-", L = 48 */
  static BigInteger keyGen(final byte[] ikm) {
    try {
      byte[] salt = "BLS-SIG-KEYGEN-SALT-".getBytes(StandardCharsets.US_ASCII);
      BigInteger sk = BigInteger.ZERO;
      while (sk.signum() == 0) {
        salt = MessageDigest.getInstance("SHA-256").digest(salt);
        final byte[] prk = hmac(salt, Bytes.concatenate(Bytes.wrap(ikm), Bytes.of(0)).toArrayUnsafe());
        final byte[] okm = new byte[64];
        byte[] t = new byte[0];
        for (int i = 1, o = 0; o < 48; i++, o += 32) {
          t = hmac(prk, Bytes.concatenate(Bytes.wrap(t), Bytes.of(0, 48, i)).toArrayUnsafe());
          System.arraycopy(t, 0, okm, o, 32);
        }
        sk = new BigInteger(1, Arrays.copyOf(okm, 48)).mod(CURVE_ORDER);
      }
      return sk;
    } catch (GeneralSecurityException e) {
      throw new IllegalStateException(e);
    }
  }

  boolean isZero() {
    for (byte b : k) {
      if (b != 0) {
        return false;
      }
    }
    return true;
  }

  @Override
  public Bytes32 toBytes() {
    return Bytes32.wrap(k.clone());
  }

  @Override
  public PublicKey derivePublicKey() {
    final byte[] out = new byte[48];
    if (TekuBlsHip.skToPk(k, out) != TekuBlsHip.SUCCESS) {
      throw new BlsException("GPU BLS backend: sk_to_pk failed");
    }
    return new HipPublicKey(out, null);
  }

  @Override
  public Signature sign(final Bytes message) {
    return sign(message, HipSignature.ETH2_DST);
  }

  @Override
  public Signature sign(final Bytes message, final String dst) {
    return sign(message, dst.getBytes(StandardCharsets.US_ASCII));
  }

  private Signature sign(final Bytes message, final byte[] dst) {
    if (isZero()) {
      throw new IllegalArgumentException("Signing with zero private key is prohibited"); // BlstBLS12381.java:54-56
    }
    final byte[] out = new byte[96];
    if (TekuBlsHip.sign(k, message.toArrayUnsafe(), dst, out) != TekuBlsHip.SUCCESS) {
      throw new BlsException("GPU BLS backend: sign failed");
    }
    return new HipSignature(out);
  }

  @Override
  public void destroy() {
    Arrays.fill(k, (byte) 0);
  }

  @Override
  public int hashCode() {
    return Arrays.hashCode(k);
  }

  @Override
  public boolean equals(final Object obj) {
    return obj instanceof HipSecretKey o && Arrays.equals(o.k, k);
  }
}
