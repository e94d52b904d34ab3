"""Lane-cooperative Fp products (teku_amd/csrc/tb_coop.h) on the host emulation
of a 16-lane row, checked against Python integers.

The digit-class bounds of the file comment are exercised with worst-case
digits (every digit at its class bound, both signs), the conversions from and
to the 12 x 32-bit [0, 2p) form with edge values, and a chain of products fed
back as operands (what the serial exponentiations do).  Test infrastructure
only: the product path runs the same source on the GPU (tests/test_gpu_ops.py).
"""

import ctypes
import random

import numpy as np
import pytest

from oracle import bls12_381 as O

P = O.P
R = 1 << 406
RINV = pow(R, -1, P)


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as ge

    L = ctypes.CDLL(ge.build_hostsim())
    for name in ("tbls_hostsim_coop_mul_digits", "tbls_hostsim_coop_mul_fp"):
        getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.tbls_hostsim_coop_to_fp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    return L


def val(d):
    return sum(int(x) << (29 * j) for j, x in enumerate(d[:14]))


def mul_digits(L, A, B):
    a = np.ascontiguousarray(np.array(A, dtype=np.int32))
    b = np.ascontiguousarray(np.array(B, dtype=np.int32))
    out = np.zeros_like(a)
    L.tbls_hostsim_coop_mul_digits(a.ctypes.data, b.ctypes.data, out.ctypes.data, len(A))
    return out


def rnd_digits(rng, T, top=31, worst=False):
    """14 digits of class T (|d| <= T 2^28), lanes 14, 15 zero."""
    lim = T << 28
    if worst:
        d = [rng.choice((-lim, lim - 1)) for _ in range(13)]
    else:
        d = [rng.randint(-lim, lim - 1) for _ in range(13)]
    return d + [rng.randint(-top, top), 0, 0]


def check(L, A, B):
    out = mul_digits(L, A, B)
    for a, b, r in zip(A, B, out):
        assert r[14] == 0 and r[15] == 0
        assert all(abs(int(x)) <= (1 << 28) + 8 for x in r[:13]), "output digit class"
        assert abs(int(r[13])) < 32, "output top digit"
        v = val(r)
        assert abs(v) < P + P // 100
        assert (v - val(a) * val(b) * RINV) % P == 0
    return out


@pytest.mark.parametrize("ta,tb", [(1, 1), (1, 7), (7, 1), (2, 3), (3, 2), (1, 2), (2, 2)])
def test_coop_mul_classes(lib, ta, tb):
    rng = random.Random(1000 * ta + tb)
    for worst in (False, True):
        A = [rnd_digits(rng, ta, worst=worst) for _ in range(300)]
        B = [rnd_digits(rng, tb, worst=worst) for _ in range(300)]
        check(lib, A, B)


def test_coop_mul_chain(lib):
    """Outputs fed back as operands, and sums of up to 7 outputs times an output."""
    rng = random.Random(7)
    x = [rnd_digits(rng, 1) for _ in range(64)]
    y = [rnd_digits(rng, 1) for _ in range(64)]
    for _ in range(30):
        z = check(lib, x, y)
        x, y = y, [list(map(int, r)) for r in z]
    s = [[sum(int(r[j]) for r in (x[i], y[i], x[i], y[i], x[i], y[i], x[i])) for j in range(16)] for i in range(64)]
    check(lib, s, y)


def test_coop_fp_roundtrip(lib):
    """[0, 2p) 12-word operands through cfrom_words / cmul / cdigits_to_fp equal
    fp_mul's residue, with the result back in [0, 2p)."""
    rng = random.Random(3)
    vals = [0, 1, P - 1, P, P + 1, 2 * P - 1] + [rng.randrange(2 * P) for _ in range(200)]
    A = vals
    B = list(reversed(vals))
    w = lambda v: np.array([(v >> (32 * i)) & 0xFFFFFFFF for i in range(12)], dtype=np.uint32)  # noqa: E731
    a = np.ascontiguousarray(np.stack([w(v) for v in A]))
    b = np.ascontiguousarray(np.stack([w(v) for v in B]))
    out = np.zeros_like(a)
    lib.tbls_hostsim_coop_mul_fp(a.ctypes.data, b.ctypes.data, out.ctypes.data, len(A))
    for x, y, r in zip(A, B, out):
        v = sum(int(r[i]) << (32 * i) for i in range(12))
        assert v < 2 * P
        assert v % P == x * y * RINV % P


def test_coop_to_fp_signed(lib):
    """cdigits_to_fp on signed digit vectors of |value| < 64p."""
    rng = random.Random(4)
    D = []
    for _ in range(300):
        v = rng.choice([rng.randrange(-64 * P + 1, 64 * P), rng.randrange(-P, P), -64 * P + 1, 64 * P - 1])
        d = []
        for _ in range(13):
            lo = ((v + (1 << 28)) & ((1 << 29) - 1)) - (1 << 28)
            d.append(lo)
            v = (v - lo) >> 29
        D.append(d + [v, 0, 0])
    d = np.ascontiguousarray(np.array(D, dtype=np.int32))
    out = np.zeros((len(D), 12), dtype=np.uint32)
    lib.tbls_hostsim_coop_to_fp(d.ctypes.data, out.ctypes.data, len(D))
    for dd, r in zip(D, out):
        v = sum(int(r[i]) << (32 * i) for i in range(12))
        assert v < 2 * P and v % P == val(dd) % P


def test_coop_pow_win(lib):
    """cpow_win_n<2> with the (p+1)/4 schedule equals a^((p+1)/4) (Montgomery
    form in and out: the residue a R^-1 ... handled by comparing x^2 == a)."""
    lib.tbls_hostsim_coop_sqrt_cand.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    rng = random.Random(9)
    vals = [rng.randrange(P) for _ in range(6)] + [1, P - 1]
    w = lambda v: np.array([(v >> (32 * i)) & 0xFFFFFFFF for i in range(12)], dtype=np.uint32)  # noqa: E731
    a = np.ascontiguousarray(np.stack([w(v * R % P) for v in vals]))  # Montgomery form
    out = np.zeros_like(a)
    lib.tbls_hostsim_coop_sqrt_cand(a.ctypes.data, out.ctypes.data, len(vals))
    for v, r in zip(vals, out):
        m = sum(int(r[i]) << (32 * i) for i in range(12)) * RINV % P
        assert m == pow(v, (P + 1) // 4, P)


def test_coop_reduce(lib):
    """creduce64: sums of up to 64 product outputs (64-bit digit sums, |v| up to
    2^395) -> T = 1 digits with |v| < 1.6 p, same residue."""
    lib.tbls_hostsim_coop_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    rng = random.Random(11)
    X = []
    for _ in range(400):
        k = rng.choice([1, 2, 8, 36, 64, 4096])
        d = [sum(rng.randint(-(1 << 28), 1 << 28) for _ in range(min(k, 8))) * max(1, k // 8) for _ in range(13)]
        top = rng.randint(-(1 << 5), 1 << 5) * k
        X.append(d + [top, 0, 0])
    x = np.ascontiguousarray(np.array(X, dtype=np.int64))
    out = np.zeros((len(X), 16), dtype=np.int32)
    lib.tbls_hostsim_coop_reduce(x.ctypes.data, out.ctypes.data, len(X))
    for a, r in zip(X, out):
        assert r[14] == 0 and r[15] == 0
        assert all(abs(int(v)) <= (1 << 28) + (1 << 12) for v in r[:13])
        assert abs(val(r)) < 1.6 * P
        assert (val(r) - val(a)) % P == 0


# ---- point arithmetic (tb_cpoint.h) -----------------------------------------
def _words(v):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(12)]


def _mont(v):
    return v * R % P


def _unwords(ws):
    return sum(int(w) << (32 * i) for i, w in enumerate(ws)) * RINV % P


def _g1_points(rng, k):
    return [O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), rng.randrange(1, O.R))) for _ in range(k)]


def _g2_points(rng, k):
    return [O.jac_to_affine(O.FP2, O.jac_mul(O.FP2, O.jac_from_affine(O.FP2, O.G2_GEN), rng.randrange(1, O.R))) for _ in range(k)]


def _eq_jac(F, got, exp_aff):
    return O.jac_to_affine(F, got) == exp_aff


@pytest.mark.parametrize("op", [0, 1, 2, 3, 4, 5])
def test_cpoint_g1(lib, op):
    lib.tbls_hostsim_cpoint_g1.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    rng = random.Random(100 + op)
    n = 6
    A, B = _g1_points(rng, n), _g1_points(rng, n)
    k = O.X_ABS if op == 5 else rng.getrandbits(64) | (1 << 63)
    inp = np.array([w for a, b in zip(A, B) for v in (a[0], a[1], b[0], b[1]) for w in _words(_mont(v))], dtype=np.uint32)
    out = np.zeros(36 * n, dtype=np.uint32)
    lib.tbls_hostsim_cpoint_g1(op, inp.ctypes.data, out.ctypes.data, n, k)
    F = O.FP
    for i, (a, b) in enumerate(zip(A, B)):
        ja, jb = O.jac_from_affine(F, a), O.jac_from_affine(F, b)
        exp = {
            0: lambda: O.jac_double(F, ja),
            1: lambda: O.jac_add(F, O.jac_double(F, ja), jb),
            2: lambda: O.jac_add(F, O.jac_double(F, ja), O.jac_double(F, jb)),
            3: lambda: O.jac_mul(F, ja, k),
            4: lambda: O.jac_mul(F, O.jac_double(F, ja), k),
            5: lambda: O.jac_mul(F, ja, k * k),
        }[op]()
        got = tuple(_unwords(out[36 * i + 12 * j : 36 * i + 12 * j + 12]) for j in range(3))
        assert _eq_jac(F, got, O.jac_to_affine(F, exp)), (op, i)


@pytest.mark.parametrize("op", [0, 1, 3])
def test_cpoint_g2(lib, op):
    lib.tbls_hostsim_cpoint_g2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    rng = random.Random(200 + op)
    n = 3
    A, B = _g2_points(rng, n), _g2_points(rng, n)
    k = O.X_ABS if op == 3 else 0
    inp = np.array([w for a, b in zip(A, B) for v in (a[0], a[1], b[0], b[1]) for c in v for w in _words(_mont(c))], dtype=np.uint32)
    out = np.zeros(72 * n, dtype=np.uint32)
    lib.tbls_hostsim_cpoint_g2(op, inp.ctypes.data, out.ctypes.data, n, k)
    F = O.FP2
    for i, (a, b) in enumerate(zip(A, B)):
        ja, jb = O.jac_from_affine(F, a), O.jac_from_affine(F, b)
        exp = {0: lambda: O.jac_double(F, ja), 1: lambda: O.jac_add(F, O.jac_double(F, ja), jb), 3: lambda: O.jac_mul(F, ja, k)}[op]()
        c = [_unwords(out[72 * i + 12 * j : 72 * i + 12 * j + 12]) for j in range(6)]
        got = ((c[0], c[1]), (c[2], c[3]), (c[4], c[5]))
        assert _eq_jac(F, got, O.jac_to_affine(F, exp)), (op, i)
