"""Deterministic key/message generators used by the reference's tests and by
the benchmark's synthetic workloads (TEST INFRASTRUCTURE ONLY).

* ``JavaRandom``: a faithful port of ``java.util.Random`` (48-bit LCG), so that
  ``BLSTestUtil.randomKeyPair(seed)``
  (``infrastructure/bls/src/testFixtures/java/tech/pegasys/teku/bls/BLSTestUtil.java:63-67``)
  yields the same secret keys as in the reference tests.
* ``interop_sk(i)``: ``MockStartValidatorKeyPairFactory.createKeyPairForValidator``
  (``ethereum/spec/.../interop/MockStartValidatorKeyPairFactory.java:36-42``):
  ``sk = LE(sha256(LE32(i))) mod r``.
* ``bench_message(seed, j)``: ``sha256(b"teku-bench" || LE64(seed) || LE64(j))``
  (SURVEY.md §8(d)).
"""

from __future__ import annotations

import hashlib

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class JavaRandom:
    MULT = 0x5DEECE66D
    MASK = (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self.MULT) & self.MASK

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * self.MULT + 0xB) & self.MASK
        v = self.seed >> (48 - bits)
        if v & (1 << (bits - 1)):
            v -= 1 << bits  # Java int is signed
        return v

    def next_int(self) -> int:
        return self._next(32)

    def next_bytes(self, n: int) -> bytes:
        out = bytearray()
        while len(out) < n:
            rnd = self.next_int()
            for _ in range(min(n - len(out), 4)):
                out.append(rnd & 0xFF)
                rnd >>= 8
        return bytes(out)

    def next_long(self) -> int:
        v = (self._next(32) << 32) + self._next(32)
        v &= (1 << 64) - 1
        if v >> 63:
            v -= 1 << 64
        return v


def blstestutil_sk(seed: int) -> int:
    """BLSTestUtil.randomKeyPair(seed): Bytes32.random(new Random(seed)), then
    BLSSecretKey.fromBytesModR (BLSSecretKey.java:42-54)."""
    b = JavaRandom(seed).next_bytes(32)
    return int.from_bytes(b, "big") % R


def interop_sk(i: int) -> int:
    h = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(h, "little") % R


def sk_to_bytes(sk: int) -> bytes:
    return sk.to_bytes(32, "big")


def bench_message(seed: int, j: int) -> bytes:
    return hashlib.sha256(b"teku-bench" + seed.to_bytes(8, "little") + j.to_bytes(8, "little")).digest()
