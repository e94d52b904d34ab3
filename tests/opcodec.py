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
    ISO=16, CLEAR_COF=17, FP12_SQR=18, FP12_INV=19, HASH_TO_FIELD=20, FP_SQR=21, FP_ADD=22, FP_SUB=23, FINAL_EXP_WAVE=29, MILLER2=30, MILLER_WAVE=31, MILLER_PROG=40, CLEAR_COF_PROG=41, WAVE_TIMING=42, COOP_MUL=43, COOP_TIMING=44, COOP_INV=47, FP_INV_ROW=38, FINAL_EXP_COOP=45, CFE_OPS=46,
    FP_MUL_RAW=32, FP_SQR_RAW=33, FP2_MUL_RAW=34, FP2_SQR_RAW=35, CLEAR_COF_NX=36, G2_IN_GROUP_NX=37, STAGE_PK=24, STAGE_SET_PK=25, STAGE_SET_SIG=26, STAGE_SET_HASH=27, G2_JADD=28,
)

R_MONT = 1 << 406  # tb_fp.h Montgomery radix
R_INV = pow(R_MONT, -1, O.P)


def raw_bound_cases(rng, n):
    """Operands across the weakly reduced contract of tb_fp.h: canonical values,
    [p, 2p) (every op's output range), [2p, 4p) (unreduced sums fp_add_nr feeds
    to products) and the top of 2^384 (the lazy Fp2 product's input bound)."""
    top = (1 << 384) - 1
    pool = [0, 1, O.P - 1, O.P, O.P + 1, 2 * O.P - 1, 2 * O.P, 3 * O.P + 7, 4 * O.P - 1, top, top - O.P]
    out = list(pool)
    for _ in range(n):
        k = rng.randrange(4)
        hi = [O.P, 2 * O.P, 4 * O.P, 1 << 384][k]
        out.append(rng.randrange(hi))
    return out


def check_raw_ops(run, rng):
    """FP_MUL/SQR_RAW on operands < 2^384 and FP2_MUL/SQR_RAW on coordinates
    < 2p: canonical value == a b / R mod p and the raw output < 2p (tb_fp.h /
    tb_tower.h contract)."""
    X = raw_bound_cases(rng, 60)
    Y = list(reversed(X))
    be = lambda v: v.to_bytes(48, "big")  # noqa: E731
    out = run("FP_MUL_RAW", [be(a) + be(b) for a, b in zip(X, Y)])
    for o, a, b in zip(out, X, Y):
        assert int.from_bytes(o[:48], "big") == a * b * R_INV % O.P
        assert int.from_bytes(o[48:96], "big") < 2 * O.P
    out = run("FP_SQR_RAW", [be(a) for a in X])
    for o, a in zip(out, X):
        assert int.from_bytes(o[:48], "big") == a * a * R_INV % O.P
        assert int.from_bytes(o[48:96], "big") < 2 * O.P
    # Fp2 coordinates are weakly reduced (< 2p): the Karatsuba sums a0 + a1 (< 4p)
    # are then products' operands; cover [p, 2p) and its top
    W = [v % (2 * O.P) for v in X] + [2 * O.P - 1, O.P, O.P - 1]
    A = list(zip(W, W[7:] + W[:7]))
    B = list(zip(reversed(W), W[3:] + W[:3]))
    out = run("FP2_MUL_RAW", [be(a[0]) + be(a[1]) + be(b[0]) + be(b[1]) for a, b in zip(A, B)])
    for o, a, b in zip(out, A, B):
        re = (a[0] * b[0] - a[1] * b[1]) * R_INV % O.P
        im = (a[0] * b[1] + a[1] * b[0]) * R_INV % O.P
        assert (int.from_bytes(o[:48], "big"), int.from_bytes(o[96:144], "big")) == (re, im)
        assert int.from_bytes(o[48:96], "big") < 2 * O.P and int.from_bytes(o[144:192], "big") < 2 * O.P
    # fp2_sqr's operands are formed from weakly reduced inputs (< 2p)
    S = A
    out = run("FP2_SQR_RAW", [be(a[0]) + be(a[1]) for a in S])
    for o, a in zip(out, S):
        re = (a[0] * a[0] - a[1] * a[1]) * R_INV % O.P
        im = 2 * a[0] * a[1] * R_INV % O.P
        assert (int.from_bytes(o[:48], "big"), int.from_bytes(o[96:144], "big")) == (re, im)
        assert int.from_bytes(o[48:96], "big") < 2 * O.P and int.from_bytes(o[144:192], "big") < 2 * O.P


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
