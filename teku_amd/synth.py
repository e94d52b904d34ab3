"""Synthetic signature sets of the BASELINE.json configs.

Keys are Teku's interop keys, sk_i = LE(sha256(LE32(i))) mod r
(ethereum/spec/.../interop/MockStartValidatorKeyPairFactory.java:32-42);
messages are distinct 32-byte digests m_j = sha256("teku-bench" || LE64(seed)
|| LE64(j)); keys and signatures are produced on the GPU through the C ABI
(tbls_sk_to_pk_many / tbls_sign_many, pinned to the oracle by the sign and
sk->pk KATs).  A set signed by k keys on one message carries the aggregate
signature sum_j sk_j H(m) = (sum_j sk_j mod r) H(m), which is what
BlstSignature.aggregate of the k individual signatures gives.

Used by bench.py and the GPU parity tests; only the C ABI is called.
"""

from __future__ import annotations

import ctypes
import hashlib
from operator import itemgetter
from typing import List, Sequence, Tuple

import numpy as np

from . import native

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
ETH2_DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
NOT_IN_G2 = bytes.fromhex("80" + "00" * 94 + "04")  # BLSTest.notInG2 (BLSTest.java:248-256)
BAD_PK = bytes.fromhex("9378a6e3984e96d2cd50450c76ca14732f1300efa04aecdb805b22e6d6926a85ef409e8f3acf494a1481090bf32ce3bd")
INFINITY_G1 = bytes([0xC0]) + bytes(47)
INFINITY_G2 = bytes([0xC0]) + bytes(95)

CHUNK = 65536  # items per generator call (bounds the staging buffers)


def interop_sk(i: int) -> int:
    h = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(h, "little") % R_ORDER


def bench_message(seed: int, j: int) -> bytes:
    return hashlib.sha256(b"teku-bench" + seed.to_bytes(8, "little") + j.to_bytes(8, "little")).digest()


def pubkeys(sks: Sequence[int]) -> List[bytes]:
    """pk_i = sk_i g1 (compressed), on the GPU."""
    L = native.lib()
    out: List[bytes] = []
    for s in range(0, len(sks), CHUNK):
        part = sks[s : s + CHUNK]
        buf = ctypes.create_string_buffer(48 * len(part))
        native.check(L.tbls_sk_to_pk_many(b"".join(k.to_bytes(32, "big") for k in part), len(part), buf), "sk_to_pk_many")
        raw = buf.raw
        out += [raw[48 * i : 48 * i + 48] for i in range(len(part))]
    return out


def sign_blob(sks: Sequence[int], msgs: Sequence[bytes], dst: bytes = ETH2_DST) -> bytes:
    """sig_i = sk_i H(m_i) (compressed, concatenated), on the GPU."""
    L = native.lib()
    parts = []
    for s in range(0, len(sks), CHUNK):
        ks, ms = sks[s : s + CHUNK], msgs[s : s + CHUNK]
        n = len(ks)
        off = (ctypes.c_uint32 * (n + 1))()
        acc = 0
        for i, m in enumerate(ms):
            off[i] = acc
            acc += len(m)
        off[n] = acc
        buf = ctypes.create_string_buffer(96 * n)
        native.check(
            L.tbls_sign_many(b"".join(k.to_bytes(32, "big") for k in ks), b"".join(ms) or b"\0", off, n, dst, len(dst), buf), "sign_many"
        )
        parts.append(buf.raw)
    return b"".join(parts)


def single_signer(first: int, count: int, n_keys_uniq: int = 65536, seed: int = 0) -> Tuple[bytes, bytes, bytes]:
    """Sets [first, first + count) of the single-signer configs (1, 4, 5): set j
    is signed by interop key (first + j) mod n_keys_uniq on bench_message(seed,
    first + j).  Returns (pks 48*count, msgs 32*count, sigs 96*count)."""
    kidx = [(first + j) % n_keys_uniq for j in range(count)]
    uniq = sorted(set(kidx))
    sk_of = {k: interop_sk(k) for k in uniq}
    pk_list = pubkeys([sk_of[k] for k in uniq])
    pk_of = dict(zip(uniq, pk_list))
    msgs = [bench_message(seed, first + j) for j in range(count)]
    sigs = sign_blob([sk_of[k] for k in kidx], msgs)
    return b"".join(pk_of[k] for k in kidx), b"".join(msgs), sigs


def multi_key(n_sets: int, keys_per_set: int, first_key: int = 0, seed: int = 1) -> Tuple[List[List[bytes]], List[bytes], List[bytes]]:
    """Configs 2/3: set s is signed by the keys_per_set interop keys
    first_key + s*keys_per_set + [0, keys_per_set) on bench_message(seed, s), with
    the aggregate signature.  Returns (key lists, messages, signatures)."""
    n_keys = n_sets * keys_per_set
    sks = [interop_sk(first_key + i) for i in range(n_keys)]
    pks = pubkeys(sks)
    msgs = [bench_message(seed, s) for s in range(n_sets)]
    agg_sk = [sum(sks[s * keys_per_set : (s + 1) * keys_per_set]) % R_ORDER for s in range(n_sets)]
    sig = sign_blob(agg_sk, msgs)
    return (
        [pks[s * keys_per_set : (s + 1) * keys_per_set] for s in range(n_sets)],
        msgs,
        [sig[96 * s : 96 * s + 96] for s in range(n_sets)],
    )


def random_multipliers(n: int, rng=None) -> List[int]:
    """Randomizers in [1, 2^64) (BlstBLS12381.nextBatchRandomMultiplier, l.191-195;
    2^64 itself does not fit the C ABI's uint64)."""
    import secrets

    out = []
    for _ in range(n):
        r = 0
        while r == 0:
            r = rng.getrandbits(64) if rng is not None else secrets.randbits(64)
        out.append(r)
    return out


def fast_multipliers(n: int) -> np.ndarray:
    """n randomizers in [1, 2^64) as a uint64 array from the OS CSPRNG in one
    call (the per-set Python loop of random_multipliers costs ~1 us per set,
    which at 16,384 sets is host time the reference spends in Java)."""
    import os

    a = np.frombuffer(os.urandom(8 * max(1, n)), dtype=np.uint64).copy()[:n]
    a[a == 0] = 1
    return a


# ---- contiguous C-ABI set arrays (no per-set Python buffers) -------------------
def _addr(p: ctypes.c_char_p) -> int:
    return ctypes.cast(p, ctypes.c_void_p).value

_SET_DTYPE = np.dtype([("pks", "<u8"), ("n_pks", "<u4"), ("msg", "<u8"), ("msg_len", "<u4"), ("sig", "<u8")], align=True)
assert _SET_DTYPE.itemsize == ctypes.sizeof(native.TblsSet)


_G0, _G1, _G2, _G3 = (itemgetter(k) for k in range(4))


class SetArray:
    """tbls_set[n] over contiguous blobs: set i has keys pks[48 k_off[i] ..],
    message msgs[m_off[i] .. m_off[i+1]) and signature sigs[96 i ..]."""

    def __init__(self, pks: bytes, n_pks: Sequence[int], msgs: bytes, msg_lens: Sequence[int], sigs: bytes):
        n = len(n_pks)
        # the blobs in place (the library only reads them): a c_char_p keeps its
        # bytes object alive and points at its data, no copy
        self._pks, self._msgs, self._sigs = (ctypes.c_char_p(bytes(x) if x else b"\0") for x in (pks, msgs, sigs))
        k = np.asarray(n_pks, dtype=np.uint64)
        ml = np.asarray(msg_lens, dtype=np.uint64)
        k_off = np.concatenate([[0], np.cumsum(k)[:-1]]).astype(np.uint64) if n else k
        m_off = np.concatenate([[0], np.cumsum(ml)[:-1]]).astype(np.uint64) if n else ml
        a = np.zeros(n, dtype=_SET_DTYPE)
        a["pks"] = _addr(self._pks) + 48 * k_off
        a["n_pks"] = k
        a["msg"] = _addr(self._msgs) + m_off
        a["msg_len"] = ml
        a["sig"] = _addr(self._sigs) + 96 * np.arange(n, dtype=np.uint64)
        self._arr = a
        self.n = n
        self.ptr = ctypes.cast(a.ctypes.data, ctypes.POINTER(native.TblsSet))

    @classmethod
    def single(cls, pks: bytes, msgs: bytes, sigs: bytes, msg_len: int = 32) -> "SetArray":
        n = len(sigs) // 96
        return cls(pks, [1] * n, msgs, [msg_len] * n, sigs)

    @classmethod
    def from_lists(cls, key_lists: Sequence[Sequence[bytes]], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> "SetArray":
        return cls(
            b"".join(b"".join(ks) for ks in key_lists), [len(ks) for ks in key_lists], b"".join(msgs), [len(m) for m in msgs], b"".join(sigs)
        )

    @classmethod
    def from_tuples(cls, sets: Sequence[Tuple[bytes, int, bytes, bytes]]) -> "SetArray":
        """[(pk_blob, n_pks, msg, sig96)] (the tuples of bls.batch_verify_raw)."""
        msgs = list(map(_G2, sets))
        return cls(b"".join(map(_G0, sets)), list(map(_G1, sets)), b"".join(msgs), list(map(len, msgs)), b"".join(map(_G3, sets)))

    def batch_verify(self, rands: Sequence[int], n_gpus: int = 0, timing: "native.TblsTiming" = None) -> bool:
        if isinstance(rands, np.ndarray):  # uint64 array (fast_multipliers): passed in place
            assert rands.dtype == np.uint64 and rands.flags.c_contiguous and len(rands) >= self.n
            rr = rands.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        else:
            rr = (ctypes.c_uint64 * max(1, self.n))(*rands)
        ok = ctypes.c_int(0)
        rc = native.lib().tbls_batch_verify(self.ptr, self.n, rr, n_gpus, ctypes.byref(ok), ctypes.byref(timing) if timing is not None else None)
        if rc == native.BAD_ARGUMENT:
            raise ValueError("empty public key list in batch")
        native.check(rc, "tbls_batch_verify")
        return ok.value == 1

    def batch_verify_each(self, rands: Sequence[int], n_gpus: int = 0, timing: "native.TblsTiming" = None):
        """(batch verdict, per-set verdicts): tbls_batch_verify_each -- the
        randomized batch, and when it fails every set's verdict settled from
        the batch's own work (per-set values are all True when it passes)."""
        if isinstance(rands, np.ndarray):
            assert rands.dtype == np.uint64 and rands.flags.c_contiguous and len(rands) >= self.n
            rr = rands.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        else:
            rr = (ctypes.c_uint64 * max(1, self.n))(*rands)
        ok = ctypes.c_int(0)
        each = (ctypes.c_int * max(1, self.n))()
        rc = native.lib().tbls_batch_verify_each(self.ptr, self.n, rr, n_gpus, ctypes.byref(ok), each,
                                                  ctypes.byref(timing) if timing is not None else None)
        native.check(rc, "tbls_batch_verify_each")
        return ok.value == 1, [v == 1 for v in each[: self.n]]

    def fast_aggregate_verify_many(self) -> List[bool]:
        ok = (ctypes.c_int * max(1, self.n))()
        native.check(native.lib().tbls_fast_aggregate_verify_many(self.ptr, self.n, ok), "tbls_fast_aggregate_verify_many")
        return [v == 1 for v in ok[: self.n]]

    def verify_each(self, n_gpus: int = 0) -> List[bool]:
        ok = (ctypes.c_int * max(1, self.n))()
        native.check(native.lib().tbls_verify_each(self.ptr, self.n, n_gpus, ok), "tbls_verify_each")
        return [v == 1 for v in ok[: self.n]]
