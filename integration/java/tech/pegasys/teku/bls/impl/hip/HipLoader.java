/*
 * Loader in the pattern of BlstLoader (infrastructure/bls/.../blst/BlstLoader.java:29-51):
 * an absent library, a failed device initialisation or a machine without a
 * GPU leaves INSTANCE empty and the node keeps blst.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.util.Optional;
import tech.pegasys.teku.bls.impl.BLS12381;

public final class HipLoader {
  public static final Optional<BLS12381> INSTANCE = load();

  private HipLoader() {}

  private static Optional<BLS12381> load() {
    try {
      System.loadLibrary("tekubls_jni"); // links libtekubls_hip.so
      if (TekuBlsHip.init(-1, 0) != TekuBlsHip.SUCCESS || TekuBlsHip.deviceCount() < 1) {
        return Optional.empty();
      }
      Runtime.getRuntime().addShutdownHook(new Thread(TekuBlsHip::shutdown));
      return Optional.of(new HipBLS12381());
    } catch (UnsatisfiedLinkError | SecurityException e) {
      return Optional.empty();
    }
  }
}
