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
