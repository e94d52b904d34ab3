"""teku_amd: MI355X-native BLS12-381 verification backend for Teku.

``teku_amd.native``  -- ctypes binding of libtekubls_hip.so (the C ABI)
``teku_amd.bls``     -- host-side mirror of Teku's BLS12381 SPI and BLS facade
"""

__all__ = ["native", "bls"]
