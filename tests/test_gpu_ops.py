"""GPU parity of the primitive kernels (tests/native/tb_testops.h via the test library libtekubls_test.so) against the oracle."""

import random

import pytest

from oracle import bls12_381 as O
from oracle.keys import interop_sk
from tests.opcodec import *  # noqa: F401,F403

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def run():
    L = load_test_lib()
    return lambda op, recs: run_ops(L.tbls_test_ops, op, recs)


def _rng():
    return random.Random(1234)


def test_fp_ops(run):
    rng = _rng()
    A = [rng.randrange(O.P) for _ in range(200)] + [0, 1, O.P - 1]
    B = [rng.randrange(O.P) for _ in range(200)] + [O.P - 1, O.P - 1, O.P - 1]
    recs = [enc_fp(a) + enc_fp(b) for a, b in zip(A, B)]
    assert [dec_fp(x) for x in run("FP_MUL", recs)] == [a * b % O.P for a, b in zip(A, B)]
    assert [dec_fp(x) for x in run("FP_ADD", recs)] == [(a + b) % O.P for a, b in zip(A, B)]
    assert [dec_fp(x) for x in run("FP_SUB", recs)] == [(a - b) % O.P for a, b in zip(A, B)]
    out = run("FP_INV", [enc_fp(a) for a in A[:16]])
    assert all(dec_fp(x) * a % O.P == 1 for x, a in zip(out, A[:16]) if a)


def test_fp2_fp12(run):
    rng = _rng()
    rf2 = lambda: (rng.randrange(O.P), rng.randrange(O.P))  # noqa: E731
    X = [rf2() for _ in range(64)]
    Y = [rf2() for _ in range(64)]
    out = run("FP2_MUL", [enc_fp2(a) + enc_fp2(b) for a, b in zip(X, Y)])
    assert [dec_fp2(x) for x in out] == [O.f2_mul(a, b) for a, b in zip(X, Y)]
    sq = [O.f2_sqr(x) for x in X[:8]] + X[8:16] + [(0, 0), (5, 0), (O.P - 5, 0), (0, 7)]
    out = run("FP2_SQRT", [enc_fp2(a) for a in sq])
    for x, a in zip(out, sq):
        exp = O.f2_sqrt(a) is not None
        assert u32(x) == exp
        if exp:
            assert O.f2_sqr(dec_fp2(x[4:])) == a
    rf12 = lambda: tuple(tuple(rf2() for _ in range(3)) for _ in range(2))  # noqa: E731
    F = [rf12() for _ in range(4)]
    G = [rf12() for _ in range(4)]
    assert [dec_fp12(x) for x in run("FP12_MUL", [enc_fp12(a) + enc_fp12(b) for a, b in zip(F, G)])] == [
        O.f12_mul(a, b) for a, b in zip(F, G)
    ]
    assert [dec_fp12(x) for x in run("FP12_SQR", [enc_fp12(a) for a in F])] == [O.f12_mul(a, a) for a in F]
    cyc = []
    for a in F:
        t = O.f12_mul(O.f12_conj(a), O.f12_inv(a))
        cyc.append(O.f12_mul(O.f12_pow(t, O.P * O.P), t))
    assert [dec_fp12(x) for x in run("FP12_CYC_SQR", [enc_fp12(a) for a in cyc])] == [O.f12_mul(a, a) for a in cyc]
    out = run("FP12_INV", [enc_fp12(a) for a in F[:2]])
    assert all(O.f12_mul(dec_fp12(x), a) == O.F12_ONE for x, a in zip(out, F[:2]))


def test_decompress_and_groups(run):
    sks = [interop_sk(i) for i in range(6)]
    pks = [O.sk_to_pk(s) for s in sks] + [
        O.INFINITY_G1,
        bytes(48),
        bytes.fromhex("9378a6e3984e96d2cd50450c76ca14732f1300efa04aecdb805b22e6d6926a85ef409e8f3acf494a1481090bf32ce3bd"),
        bytes([0x80]) + bytes(47),
        bytes([0xC0]) + bytes(46) + b"\x01",
        bytes([0x9F]) + b"\xff" * 47,
    ]
    for x, b in zip(run("G1_DECOMP", pks), pks):
        code, a = O.g1_decompress(b)
        c = u32(x)
        assert c & 0xFF == code
        assert bool(c & 0x100) == (code == O.SUCCESS and a is None)
        if code == O.SUCCESS and a is not None:
            assert (dec_fp(x[4:]), dec_fp(x[52:])) == a
    sigs = [O.sign(s, b"m%d" % i) for i, s in enumerate(sks[:3])] + [
        O.INFINITY_G2,
        bytes(96),
        bytes.fromhex("80" + "00" * 94 + "04"),
        bytes([0xA0]) + bytes(95),
    ]
    for x, b in zip(run("G2_DECOMP", sigs), sigs):
        code, a = O.g2_decompress(b)
        c = u32(x)
        assert c & 0xFF == code
        if code == O.SUCCESS and a is not None:
            assert (dec_fp2(x[4:100]), dec_fp2(x[100:196])) == a
    pts = [O.g1_decompress(b)[1] for b in pks[:4]] + [O.g1_decompress(pks[8])[1]]
    got = [u32(x) for x in run("G1_IN_GROUP", [enc_fp(a[0]) + enc_fp(a[1]) for a in pts])]
    assert got == [1, 1, 1, 1, 0]
    p2 = [O.g2_decompress(s)[1] for s in sigs[:3]] + [O.g2_decompress(sigs[5])[1]]
    got = [u32(x) for x in run("G2_IN_GROUP", [enc_fp2(a[0]) + enc_fp2(a[1]) for a in p2])]
    assert got == [1, 1, 1, 0]


def test_hash_to_g2(run):
    msgs = [b"", b"abc", b"\x99" * 32, bytes(range(256)) * 2, b"Hello, world!"]
    recs = [enc_h2c(m) for m in msgs] + [enc_h2c(b"abc", b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_")]
    exp = [O.g2_compress(O.hash_to_g2(m)) for m in msgs] + [
        O.g2_compress(O.hash_to_g2(b"abc", b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"))
    ]
    assert [x[:96] for x in run("HASH_TO_G2", recs)] == exp


def test_pairing_pieces(run):
    P1, Q1 = O.G1_GEN, O.G2_GEN
    out = run("MILLER", [enc_fp(P1[0]) + enc_fp(P1[1]) + enc_fp2(Q1[0]) + enc_fp2(Q1[1])])
    f = dec_fp12(out[0])
    assert O.final_exponentiation(f) == O.pairing(P1, Q1)
    g = dec_fp12(run("FINAL_EXP", [enc_fp12(f)])[0])
    e = O.pairing(P1, Q1)
    assert g == O.f12_mul(O.f12_mul(e, e), e)
    # wave-parallel final exponentiation == single-lane version, bit for bit
    rng = _rng()
    fs = [f] + [tuple(tuple((rng.randrange(O.P), rng.randrange(O.P)) for _ in range(3)) for _ in range(2)) for _ in range(2)]
    single = [dec_fp12(x) for x in run("FINAL_EXP", [enc_fp12(x) for x in fs])]
    wave = [dec_fp12(x) for x in run("FINAL_EXP_WAVE", [enc_fp12(x) for x in fs])]
    assert wave == single
    # lane-cooperative final exponentiation (tb_cfe.h) == the same, bit for bit
    out = run("FINAL_EXP_COOP", [enc_fp12(x) for x in fs])
    assert [dec_fp12(x) for x in out] == single
    print("\ncoop final exponentiation: %d cycles" % int.from_bytes(out[0][576:584], "little"))


def test_miller2_shared_accumulator(run):
    P0, Q0 = O.G1_GEN, O.G2_GEN
    P1 = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), 7))
    Q1 = O.hash_to_g2(b"second pair")
    rec = enc_fp(P0[0]) + enc_fp(P0[1]) + enc_fp2(Q0[0]) + enc_fp2(Q0[1]) + enc_fp(P1[0]) + enc_fp(P1[1]) + enc_fp2(Q1[0]) + enc_fp2(Q1[1])
    f = dec_fp12(run("MILLER2", [rec])[0])
    assert O.final_exponentiation(f) == O.f12_mul(O.pairing(P0, Q0), O.pairing(P1, Q1))


def test_miller_wave_matches_single_lane(run):
    """k_miller_wave's loop (tb_fp12_wave.h miller_loop_wave: lane-parallel
    f^2, doubling step and line products) == the one-thread miller_loop, as
    field elements, and pairs to e(P, Q) after the final exponentiation."""
    P1 = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), 12345))
    pairs = [(O.G1_GEN, O.G2_GEN), (P1, O.hash_to_g2(b"wave miller")), (O.G1_GEN, O.hash_to_g2(b"x" * 32))]
    recs = [enc_fp(P[0]) + enc_fp(P[1]) + enc_fp2(Q[0]) + enc_fp2(Q[1]) for P, Q in pairs]
    single = [dec_fp12(x) for x in run("MILLER", recs)]
    wave = [dec_fp12(x) for x in run("MILLER_WAVE", recs)]
    assert wave == single
    assert O.final_exponentiation(wave[1]) == O.pairing(*pairs[1])


def test_miller_prog_matches_single_lane(run):
    """k_miller_wave's pipelined level program (tb_mprog.h, tables from
    tools/gen_miller_prog.py) == the one-thread miller_loop up to a factor in
    Fp (its doubling step works on 4T), and pairs to e(P, Q) after the final
    exponentiation; the batch paths only ever use the final exponentiation."""
    P1 = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), 12345))
    pairs = [(O.G1_GEN, O.G2_GEN), (P1, O.hash_to_g2(b"wave miller")), (O.G1_GEN, O.hash_to_g2(b"x" * 32))]
    recs = [enc_fp(P[0]) + enc_fp(P[1]) + enc_fp2(Q[0]) + enc_fp2(Q[1]) for P, Q in pairs]
    single = [dec_fp12(x) for x in run("MILLER", recs)]
    prog = [dec_fp12(x) for x in run("MILLER_PROG", recs)]
    for s, w in zip(single, prog):
        ratio = O.f12_mul(w, O.f12_inv(s))
        flat = [c for f6 in ratio for f2_ in f6 for c in f2_]
        assert flat[0] != 0 and all(c == 0 for c in flat[1:]), "ratio not in Fp"
    for (P, Q), w in zip(pairs, prog):
        assert O.final_exponentiation(w) == O.pairing(P, Q)


def test_clear_cofactor_prog(run):
    """The wave cofactor-clearing program (tb_cofprog.h, tables from
    tools/gen_cofactor_prog.py, used by k_set_hash_wave) == the oracle's
    clear_cofactor_g2 on SSWU/isogeny points given with random Jacobian Z, on
    G2 points, and -- through the one-lane fallback the kernel takes when the
    program ends with Z = 0 -- on the point at infinity."""
    rng = _rng()
    pts = [O.iso_map_g2(O.map_to_curve_sswu_g2((rng.randrange(O.P), rng.randrange(O.P)))) for _ in range(3)] + [O.G2_GEN]
    recs, exps = [], []
    for q in pts:
        z = (rng.randrange(1, O.P), rng.randrange(O.P))
        zz = O.f2_sqr(z)
        recs.append(enc_fp2(O.f2_mul(q[0], zz)) + enc_fp2(O.f2_mul(q[1], O.f2_mul(zz, z))) + enc_fp2(z))
        exps.append(O.jac_to_affine(O.FP2, O.clear_cofactor_g2(O.jac_from_affine(O.FP2, q))))
    recs.append(enc_fp2((1, 0)) + enc_fp2((1, 0)) + enc_fp2((0, 0)))  # infinity
    out = run("CLEAR_COF_PROG", recs)
    for o, e in zip(out, exps):
        assert u32(o, 384) == 1
        assert (dec_fp2(o[:96]), dec_fp2(o[96:192])) == e
    assert u32(out[-1], 384) == 0


def test_fp_bounds_of_weak_reduction(run):
    """The same bound checks on the GPU build (tests/opcodec.check_raw_ops)."""
    check_raw_ops(run, random.Random(12))


def test_coop_mul_and_timing(run):
    """Lane-cooperative products (tb_coop.h) on the GPU: one product per 16-lane
    row equals the oracle's a*b; a 64-long chain of products equals a b^64; the
    clock64 cycles of the chains (one and two interleaved per row) against the
    lone-lane fp_mul chain are printed (tools/hash_parts.py reads them too)."""
    rng = _rng()
    A = [rng.randrange(O.P) for _ in range(61)] + [0, 1, O.P - 1]
    B = [rng.randrange(O.P) for _ in range(61)] + [O.P - 1, O.P - 1, 2]
    out = run("COOP_MUL", [enc_fp(a) + enc_fp(b) for a, b in zip(A, B)])
    assert [dec_fp(x) for x in out] == [a * b % O.P for a, b in zip(A, B)]
    a, b = 0x1234567 * 0x9ABCDEF0123, O.P - 12345
    o = run("COOP_TIMING", [enc_fp(a) + enc_fp(b)])[0]
    cyc = [int.from_bytes(o[8 * i : 8 * i + 8], "little") / 64 for i in range(3)]
    print("\ncoop cycles per product: chain %.0f, two interleaved chains %.0f per step; lone-lane fp_mul %.0f" % tuple(cyc))
    assert int.from_bytes(o[64:112], "big") == a * pow(b, 64, O.P) % O.P
    assert int.from_bytes(o[112:160], "big") == b * pow(a, 64, O.P) % O.P
    assert int.from_bytes(o[160:208], "big") == a * pow(b, 64, O.P) % O.P


def test_coop_row_inversion(run):
    """tb_cinv.h on the GPU: one Bernstein-Yang inversion per 16-lane row
    equals pow(a, -1, p) (0 -> 0), short inputs included; record 0's row also
    times one row inversion against the lone-lane fp_inv (printed) and checks
    that fp_inv agrees."""
    rng = _rng()
    A = [rng.randrange(O.P) for _ in range(100)] + [0, 1, 2, O.P - 1, O.P - 2, 1 << 380]
    A += [rng.randrange(1 << rng.randrange(1, 381)) for _ in range(30)]
    out = run("COOP_INV", [enc_fp(a) for a in A])
    assert [dec_fp(x[:48]) for x in out] == [pow(a, -1, O.P) if a else 0 for a in A]
    o = out[0]
    cyc = [int.from_bytes(o[48 + 8 * i : 56 + 8 * i], "little") for i in range(2)]
    print("\nFp inversion cycles: coop row %d, lone-lane fp_inv %d" % tuple(cyc))
    assert int.from_bytes(o[64:112], "big") == pow(A[0], -1, O.P)


def test_cfe_ops(run):
    """Single lane-cooperative Fp12 ops (tb_cfe.h) vs the oracle: product,
    cyclotomic squaring (on f^((p^6-1)(p^2+1))), Frobenius, conjugation."""
    rng = _rng()
    rf12 = lambda: tuple(tuple((rng.randrange(O.P), rng.randrange(O.P)) for _ in range(3)) for _ in range(2))  # noqa: E731
    f, g = rf12(), rf12()
    c = O.f12_pow(f, (O.P ** 6 - 1) * (O.P ** 2 + 1))
    op = lambda k: k.to_bytes(4, "little")  # noqa: E731
    recs = [enc_fp12(f) + enc_fp12(g) + op(0), enc_fp12(c) + enc_fp12(g) + op(1), enc_fp12(f) + enc_fp12(g) + op(2),
            enc_fp12(f) + enc_fp12(g) + op(3), enc_fp12(f) + enc_fp12(g) + op(4)]
    got = [dec_fp12(x) for x in run("CFE_OPS", recs)]
    exp = [O.f12_mul(f, g), O.f12_mul(c, c), O.f12_pow(f, O.P), O.f12_conj(f) if hasattr(O, "f12_conj") else None, f]
    names = ["mul", "cyc_sqr", "frob", "conj", "copy"]
    bad = [n for n, a, b in zip(names, got, exp) if b is not None and a != b]
    X = -0xD201000000010000
    t = O.f12_pow(f, (O.P ** 6 - 1) * (O.P ** 2 + 1))
    recs = [enc_fp12(f) + enc_fp12(g) + op(5), enc_fp12(c) + enc_fp12(g) + op(6), enc_fp12(f) + enc_fp12(g) + op(7)]
    got = [dec_fp12(x) for x in run("CFE_OPS", recs)]
    e = O.final_exponentiation(f)
    exp = [O.f12_inv(f), O.f12_conj(O.f12_pow(c, -X)), O.f12_mul(O.f12_mul(e, e), e)]  # the device chain computes the 3 x hard part
    bad += [n for n, a, b in zip(["inv", "exp_x", "final"], got, exp) if a != b]
    assert not bad, bad
    o = run("CFE_OPS", [enc_fp12(c) + enc_fp12(g) + op(8)])[0]
    cyc = [int.from_bytes(o[576 + 8 * i : 584 + 8 * i], "little") for i in range(3)]
    print("\ncoop levels: cyc_sqr %.0f, mul %.0f cycles; inversion %d cycles" % (cyc[0] / 64, cyc[1] / 64, cyc[2]))
