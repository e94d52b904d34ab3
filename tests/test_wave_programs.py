"""CPU checks of the wave-program arithmetic (no GPU):

* reduce13 (tb_fp12_wave.h): the quotient estimate from the top 64 bits
  leaves v - q p in [0, 3p) for every v < 2^392, so one conditional
  subtraction of p lands in [0, 2p) -- mirrored here on edge and random values.
* tb_miller_prog.h / tb_cofactor_prog.h are exactly what
  tools/gen_miller_prog.py / gen_cofactor_prog.py generate, and the
  generators' own checks pass (the emitted level tables executed on field
  values give the oracle's e(P, Q) / clear_cofactor_g2).
"""
import os
import random
import sys

from oracle import bls12_381 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

P_TOP = O.P >> 352


def reduce13(v):
    """tb_fp12_wave.h reduce13 on a Python integer."""
    assert 0 <= v < 1 << 416
    C = (1 << 50) // (P_TOP + 1)
    t = (v >> 352) & ((1 << 64) - 1)
    q = ((t * C) >> 50) & 0xFFFFFFFF
    r = v - q * O.P
    assert 0 <= r < 3 * O.P
    return r - O.P if r >= O.P else r


def test_reduce13_bound():
    rng = random.Random(7)
    cases = [0, 1, O.P - 1, O.P, 2 * O.P - 1, 2 * O.P, (1 << 392) - 1, 4096 * O.P, 4096 * O.P - 1]
    for k in range(1, 300):
        cases += [k * O.P - 1, k * O.P, k * O.P + 1]
    cases += [rng.randrange(1 << 392) for _ in range(20000)]
    for v in cases:
        r = reduce13(v)
        assert 0 <= r < 2 * O.P and (r - v) % O.P == 0


def cs_sum(terms):
    """tb_fp12_wave.h cs_term / cs_norm on Python integers: terms (c, v) with
    v < 2^384 given as 12 limbs; returns the normalized 13-limb value."""
    G = (O.P - ((1 << 384) - 1) % O.P) % O.P
    cols, mneg = [0] * 12, 0
    for c, v in terms:
        m, neg = abs(c), c < 0
        for i in range(12):
            li = (v >> (32 * i)) & 0xFFFFFFFF
            cols[i] += (li ^ (0xFFFFFFFF if neg else 0)) * m
            assert cols[i] < 1 << 64
        mneg += m if neg else 0
    out, carry = 0, 0
    for i in range(12):
        s = ((G >> (32 * i)) & 0xFFFFFFFF) * mneg + cols[i] + carry
        assert s < 1 << 64
        out |= (s & 0xFFFFFFFF) << (32 * i)
        carry = s >> 32
    return out | (carry << 384)


def test_carry_save_sums():
    rng = random.Random(9)
    for _ in range(3000):
        n = rng.randrange(1, 9)
        terms = [(rng.choice([-1, 1]) * rng.randrange(1, 40), rng.choice([0, O.P - 1, 2 * O.P - 1, rng.randrange(2 * O.P)])) for _ in range(n)]
        v = cs_sum(terms)
        total = sum(abs(c) for c, _ in terms) + sum(-c for c, _ in terms if c < 0)
        assert v < total << 384 and v < 1 << 392
        assert (v - sum(c * x for c, x in terms)) % O.P == 0
        assert 0 <= reduce13(v) < 2 * O.P


def test_miller_program_is_generated_and_pairs_to_oracle():
    import gen_miller_prog as G

    text = G.generate(check_pairs=1, verbose=False)
    with open(os.path.join(ROOT, "teku_amd", "csrc", "tb_miller_prog.h")) as f:
        assert f.read() == text, "tb_miller_prog.h is stale: run tools/gen_miller_prog.py"


def test_cofactor_program_is_generated_and_matches_oracle():
    import gen_cofactor_prog as G

    text = G.generate(check_points=1, verbose=False)
    with open(os.path.join(ROOT, "teku_amd", "csrc", "tb_cofactor_prog.h")) as f:
        assert f.read() == text, "tb_cofactor_prog.h is stale: run tools/gen_cofactor_prog.py"
