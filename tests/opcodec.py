"""Record codec for the primitive test ops (tests/native/tb_testops.h).

Used by the CPU hostsim tests and by the -m gpu tests (same records, same
expected values from the oracle).
"""

import ctypes
import os

import numpy as np

from oracle import bls12_381 as O

TEST_IN = 1536
TEST_OUT = 640

OPS = dict(
    FP_MUL=1, FP_INV=2, FP2_MUL=3, FP2_SQRT=4, FP12_MUL=5, FP12_CYC_SQR=6, FP12_FROB=7, FINAL_EXP=8,
    MILLER=9, G1_DECOMP=10, G2_DECOMP=11, HASH_TO_G2=12, G1_IN_GROUP=13, G2_IN_GROUP=14, SSWU=15,
    ISO=16, CLEAR_COF=17, FP12_SQR=18, FP12_INV=19, HASH_TO_FIELD=20, FP_SQR=21, FP_ADD=22, FP_SUB=23, FINAL_EXP_WAVE=29, MILLER2=30, MILLER_WAVE=31,
)


def enc_fp(v):
    return (v % O.P).to_bytes(48, "big")


def dec_fp(b):
    return int.from_bytes(b[:48], "big")


def enc_fp2(a):
    return enc_fp(a[0]) + enc_fp(a[1])


def dec_fp2(b):
    return (dec_fp(b[:48]), dec_fp(b[48:96]))


def enc_fp12(f):
    (a0, a1, a2), (b0, b1, b2) = f
    return b"".join(enc_fp2(x) for x in (a0, a1, a2, b0, b1, b2))


def dec_fp12(b):
    xs = [dec_fp2(b[96 * i : 96 * i + 96]) for i in range(6)]
    return ((xs[0], xs[1], xs[2]), (xs[3], xs[4], xs[5]))


def enc_h2c(msg, dst=O.ETH2_DST):
    assert len(msg) <= 1024 and len(dst) <= 255
    b = len(msg).to_bytes(4, "little") + len(dst).to_bytes(4, "little") + msg.ljust(1024, b"\0") + dst
    return b


def pack(records):
    buf = bytearray(TEST_IN * len(records))
    for i, r in enumerate(records):
        assert len(r) <= TEST_IN
        buf[i * TEST_IN : i * TEST_IN + len(r)] = r
    return bytes(buf)


def unpack(out, n):
    return [bytes(out[i * TEST_OUT : (i + 1) * TEST_OUT]) for i in range(n)]


def u32(b, off=0):
    return int.from_bytes(b[off : off + 4], "little")


def run_ops(fn, op, records):
    """fn(op, in_ptr, out_ptr, n) -> int ; returns list of output records."""
    n = len(records)
    inb = np.frombuffer(pack(records), dtype=np.uint8).copy()
    outb = np.zeros(TEST_OUT * n, dtype=np.uint8)
    rc = fn(OPS[op], inb.ctypes.data_as(ctypes.c_void_p), outb.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n))
    assert rc == 0, rc
    return unpack(outb.tobytes(), n)


TEST_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "native", "_build", "libtekubls_test.so")


def load_test_lib():
    """libtekubls_test.so (tests/native/k_test.hip): the primitive-op kernels,
    kept out of the product library.  The product library is initialised first
    so both share one HIP runtime and device."""
    from teku_amd import native

    native.lib()
    if not os.path.exists(TEST_LIB_PATH):
        raise RuntimeError("test library not built: __graft_entry__.build()")
    L = ctypes.CDLL(TEST_LIB_PATH)
    L.tbls_test_ops.restype = ctypes.c_int
    L.tbls_test_ops.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    return L
