"""CPU logic checks of the kernel code (host build of teku_amd/csrc/tb_*.h) vs the oracle.

The same op records as tests/test_gpu_ops.py; here they run through the
hostsim build in this GPU-less container.  (Test infrastructure only: the
product library has no CPU path.)
"""

import ctypes
import os
import random

import pytest

from oracle import bls12_381 as O
from oracle.keys import interop_sk
from tests.opcodec import *  # noqa: F401,F403

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def run():
    import __graft_entry__ as ge

    path = ge.build_hostsim()
    lib = ctypes.CDLL(path)
    fn = lib.tbls_hostsim_test_ops
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    return lambda op, recs: run_ops(fn, op, recs)


def test_fp(run):
    rng = random.Random(5)
    A = [rng.randrange(O.P) for _ in range(100)] + [0, 1, O.P - 1]
    B = [rng.randrange(O.P) for _ in range(100)] + [O.P - 1] * 3
    recs = [enc_fp(a) + enc_fp(b) for a, b in zip(A, B)]
    assert [dec_fp(x) for x in run("FP_MUL", recs)] == [a * b % O.P for a, b in zip(A, B)]
    assert [dec_fp(x) for x in run("FP_ADD", recs)] == [(a + b) % O.P for a, b in zip(A, B)]
    assert [dec_fp(x) for x in run("FP_SUB", recs)] == [(a - b) % O.P for a, b in zip(A, B)]


def test_fp_inv_row(run):
    """tb_cinv.h: the coop-row Bernstein-Yang inversion (host emulation of the
    16 lanes) against pow(a, -1, p), and against the lone-lane fp_inv; 0 -> 0."""
    rng = random.Random(11)
    A = [rng.randrange(O.P) for _ in range(300)] + [0, 1, 2, 3, O.P - 1, O.P - 2, (O.P - 1) // 2, 1 << 380, (1 << 381) % O.P]
    A += [rng.randrange(1 << rng.randrange(1, 381)) for _ in range(60)]  # short values: long runs of zero bits
    recs = [enc_fp(a) for a in A]
    got = [dec_fp(x) for x in run("FP_INV_ROW", recs)]
    assert got == [pow(a, -1, O.P) if a else 0 for a in A]
    assert got == [dec_fp(x) for x in run("FP_INV", recs)]


def test_tower(run):
    rng = random.Random(6)
    rf2 = lambda: (rng.randrange(O.P), rng.randrange(O.P))  # noqa: E731
    X, Y = [rf2() for _ in range(20)], [rf2() for _ in range(20)]
    assert [dec_fp2(x) for x in run("FP2_MUL", [enc_fp2(a) + enc_fp2(b) for a, b in zip(X, Y)])] == [O.f2_mul(a, b) for a, b in zip(X, Y)]
    rf12 = lambda: tuple(tuple(rf2() for _ in range(3)) for _ in range(2))  # noqa: E731
    F, G = [rf12() for _ in range(2)], [rf12() for _ in range(2)]
    assert [dec_fp12(x) for x in run("FP12_MUL", [enc_fp12(a) + enc_fp12(b) for a, b in zip(F, G)])] == [O.f12_mul(a, b) for a, b in zip(F, G)]
    assert [dec_fp12(x) for x in run("FP12_FROB", [enc_fp12(a) for a in F])] == [O.f12_pow(a, O.P) for a in F]


def test_codec_groups_hash(run):
    sks = [interop_sk(i) for i in range(3)]
    pks = [O.sk_to_pk(s) for s in sks] + [O.INFINITY_G1, bytes(48), bytes([0x80]) + bytes(47)]
    for x, b in zip(run("G1_DECOMP", pks), pks):
        assert u32(x) & 0xFF == O.g1_decompress(b)[0]
    msgs = [b"", b"abc", b"\x01" * 32]
    assert [x[:96] for x in run("HASH_TO_G2", [enc_h2c(m) for m in msgs])] == [O.g2_compress(O.hash_to_g2(m)) for m in msgs]


def test_pairing(run):
    f = dec_fp12(run("MILLER", [enc_fp(O.G1_GEN[0]) + enc_fp(O.G1_GEN[1]) + enc_fp2(O.G2_GEN[0]) + enc_fp2(O.G2_GEN[1])])[0])
    assert O.final_exponentiation(f) == O.pairing(O.G1_GEN, O.G2_GEN)


def test_miller2_shared_accumulator(run):
    """miller_loop2 (two pairs, one Fp12 accumulator) == product of pairings."""
    P0, Q0 = O.G1_GEN, O.G2_GEN
    P1 = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), 7))
    Q1 = O.hash_to_g2(b"second pair")
    rec = enc_fp(P0[0]) + enc_fp(P0[1]) + enc_fp2(Q0[0]) + enc_fp2(Q0[1]) + enc_fp(P1[0]) + enc_fp(P1[1]) + enc_fp2(Q1[0]) + enc_fp2(Q1[1])
    f = dec_fp12(run("MILLER2", [rec])[0])
    assert O.final_exponentiation(f) == O.f12_mul(O.pairing(P0, Q0), O.pairing(P1, Q1))


def test_fp_bounds_of_weak_reduction(run):
    """tb_fp.h / tb_tower.h contract at its bounds (host build of the kernel
    code): products of operands in [p, 2^384), incl. the lazy Fp2 product."""
    check_raw_ops(run, random.Random(11))


def _g2_aff_rec(b):
    """tio_put_g2j_aff record (u32 finite flag || x || y) -> affine or None."""
    if u32(b[:4]) == 0:
        return None
    return (dec_fp2(b[4:100]), dec_fp2(b[100:196]))


def test_clear_cofactor_branch_free(run):
    """g2_clear_cofactor_nx (the throughput hash's cofactor clearing, no
    exceptional branches) equals the exact g2_clear_cofactor and the oracle on
    random E2 points whenever it reports ok, and reports !ok (the caller then
    runs the exact formulas) on the torsion points where its chain meets P = +-Q
    or infinity."""
    import random as _r

    from tests.test_gpu_kcoop import N2, _rand_e2, _torsion

    rng = _r.Random(31)
    pts = [_rand_e2(rng) for _ in range(6)]
    tors = [_torsion(O.FP2, _rand_e2, m, N2, rng) for m in (13, 23, 299)]
    pts += tors + [O.jac_to_affine(O.FP2, O.jac_add(O.FP2, O.jac_from_affine(O.FP2, tors[0]), O.jac_from_affine(O.FP2, pts[0])))]
    recs = [enc_fp2(x) + enc_fp2(y) for x, y in pts]
    n_ok = 0
    for (x, y), out in zip(pts, run("CLEAR_COF_NX", recs)):
        ok = u32(out[:4])
        nx, exact = _g2_aff_rec(out[4:200]), _g2_aff_rec(out[204:400])
        want = O.jac_to_affine(O.FP2, O.clear_cofactor_g2(O.jac_from_affine(O.FP2, (x, y))))
        assert exact == want
        if ok:
            n_ok += 1
            assert nx == want
        else:
            assert nx is None  # Z = 0: the exceptional chain is flagged, never a wrong finite point
    assert n_ok >= 6  # every random point takes the branch-free path


def test_stage_set_hash_bytes(run):
    """The throughput hash stage (tb_stages.h stage_set_hash: branch-free
    cofactor clearing with the exact fall-back) bit-exact with the oracle."""
    from oracle import c_oracle as C

    msgs = [b"", b"abc", bytes(200), b"\x01" * 32, bytes(range(77))]
    nul = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
    for dst in (O.ETH2_DST, nul):
        outs = run("STAGE_SET_HASH", [enc_h2c(m, dst) for m in msgs])
        for m, out in zip(msgs, outs):
            assert u32(out[:4]) == 1
            assert out[4:100] == C.hash_to_g2(m, dst), m


def test_g2_in_group_branch_free(run):
    """g2_in_group_nx (the two-wave signature check's subgroup test) gives
    g2_in_group's verdict on G2 points, random E2 points and small-order
    points (whose [|x|] chain may meet P = +-Q)."""
    import random as _r

    from tests.test_gpu_kcoop import N2, _rand_e2, _torsion

    rng = _r.Random(41)
    g2 = [O.jac_to_affine(O.FP2, O.clear_cofactor_g2(O.jac_from_affine(O.FP2, _rand_e2(rng)))) for _ in range(4)]
    other = [_rand_e2(rng) for _ in range(4)] + [_torsion(O.FP2, _rand_e2, m, N2, rng) for m in (13, 23, 299)]
    recs = [enc_fp2(x) + enc_fp2(y) for x, y in g2 + other]
    a = [u32(x) for x in run("G2_IN_GROUP_NX", recs)]
    b = [u32(x) for x in run("G2_IN_GROUP", recs)]
    assert a == b == [1] * len(g2) + [0] * len(other)


def test_stage_set_pk_windowed(run):
    """tb_stages.h stage_set_pk for one key: P = [r] pk affine by the fixed
    2-bit-window form (tb_curve.h g1_mul_u64_aff_w2) -- random 64-bit r and
    the edge scalars (1, 2, 3, 4, a lone top bit, all ones, zero windows
    between set ones), against the oracle; r = 0 reports infinity."""
    rng = random.Random(17)
    g = O.jac_from_affine(O.FP, O.G1_GEN)
    pts = [O.jac_to_affine(O.FP, O.jac_mul(O.FP, g, rng.randrange(1, O.R))) for _ in range(6)]
    rs = [1, 2, 3, 4, 5, 7, 1 << 63, (1 << 64) - 1, 0x8000000000000001, 0x5555555555555555, 0xC000000000000003, 0x100000000]
    rs += [rng.getrandbits(64) | 1 for _ in range(30)]
    recs, want = [], []
    for i, r in enumerate(rs):
        pt = pts[i % len(pts)]
        recs.append(enc_fp(pt[0]) + enc_fp(pt[1]) + (r & 0xFFFFFFFF).to_bytes(4, "little") + (r >> 32).to_bytes(4, "little"))
        want.append(O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, pt), r)))
    out = run("STAGE_SET_PK", recs)
    for o, w in zip(out, want):
        assert u32(o) == 0
        assert (dec_fp(o[4:52]), dec_fp(o[52:100])) == w
    z = run("STAGE_SET_PK", [enc_fp(pts[0][0]) + enc_fp(pts[0][1]) + bytes(8)])
    assert u32(z[0]) != 0
