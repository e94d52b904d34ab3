"""Small-batch lane-cooperative key and signature stages (k_kcoop.hip) vs the
oracle: the batches of <= 512 sets that take k_keys_coop / k_sig_check_coop.

Beyond the reference's tampered sets (tests/test_gpu_bls.py) these feed the
cases the branch-free scalar multiplications of tb_ccurve.h must reject:
on-curve keys and signatures outside the prime-order groups, among them
points of small order (3, 11, 33 on E1; 13, 23, 299 on E2: the 11- and
13-parts are not cyclic, so no points of order 121, 169) whose
multiples meet the exceptional addition cases inside the [|x|] chains, placed
in each row of a workgroup; batch sizes around the 4-sets-per-workgroup
packing; and, through the device-batch API, a batch with as many keys as sets
but one empty set beside a two-key set (the one-lane fallback).
"""

import ctypes
import random

import pytest

from oracle import bls12_381 as O
from oracle.keys import interop_sk

pytestmark = pytest.mark.gpu

N1 = O.P + 1 - (O.X + 1)  # #E1(Fp)
H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5
N2 = H2 * O.R  # #E2(Fp2)


@pytest.fixture(scope="module")
def hip():
    import torch  # noqa: F401

    from teku_amd import bls, native

    return bls, native, native.lib()


@pytest.fixture(scope="module")
def sets():
    n = 132
    sks = [interop_sk(i) for i in range(n)]
    msgs = [i.to_bytes(4, "big") * 8 for i in range(n)]
    pks = [O.sk_to_pk(s) for s in sks]
    sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
    return pks, msgs, sigs


def _rand_e1(rng):
    while True:
        x = rng.randrange(O.P)
        y = O.fp_sqrt(x**3 + 4)
        if y is not None:
            return (x, y)


def _rand_e2(rng):
    while True:
        x = (rng.randrange(O.P), rng.randrange(O.P))
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(x), x), O.B_G2))
        if y is not None:
            return (x, y)


def _torsion(F, rand_pt, order, cof, rng):
    """A point of exactly `order` (squarefree, dividing the curve order cof):
    cof stripped of those primes' whole powers (the 3-, 11-, 13-, 23-parts
    have exponent q), times a random point."""
    for q in (3, 11, 13, 23):
        if order % q == 0:
            while cof % q == 0:
                cof //= q
    while True:
        p = O.jac_mul(F, O.jac_from_affine(F, rand_pt(rng)), cof)
        a = O.jac_to_affine(F, p)
        if a is not None and all(O.jac_to_affine(F, O.jac_mul(F, p, order // q)) is not None for q in (3, 11, 13, 23) if order % q == 0):
            return a


def bad_keys():
    rng = random.Random(21)
    out = {"rand non-G1": O.g1_compress(_rand_e1(rng))}
    for m in (3, 11, 33):
        out[f"order {m}"] = O.g1_compress(_torsion(O.FP, _rand_e1, m, N1, rng))
    return out


def bad_sigs():
    rng = random.Random(22)
    out = {"rand non-G2": O.g2_compress(_rand_e2(rng))}
    for m in (13, 23, 299):
        out[f"order {m}"] = O.g2_compress(_torsion(O.FP2, _rand_e2, m, N2, rng))
    return out


def _raw(bls, pks, msgs, sigs):
    rands = [random.getrandbits(64) | 1 for _ in sigs]
    return bls.batch_verify_raw([(p, 1, m, s) for p, m, s in zip(pks, msgs, sigs)], rands)


def test_outside_points_are_on_curve_and_outside_group():
    rng = random.Random(5)
    for m in (3, 11, 33):
        a = _torsion(O.FP, _rand_e1, m, N1, rng)
        assert O.on_curve_g1(a) and not O.g1_in_group(O.jac_from_affine(O.FP, a))
    for m in (13, 23):
        a = _torsion(O.FP2, _rand_e2, m, N2, rng)
        assert O.on_curve_g2(a) and not O.g2_in_group(O.jac_from_affine(O.FP2, a))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 63, 128, 129, 131])
def test_small_batches_valid_and_swapped(hip, sets, n):
    bls = hip[0]
    pks, msgs, sigs = (x[:n] for x in sets)
    assert _raw(bls, pks, msgs, sigs) is True
    if n > 1:
        s2 = list(sigs)
        s2[n - 1], s2[0] = s2[0], s2[n - 1]
        assert _raw(bls, pks, msgs, s2) is False


def test_keys_outside_g1_each_row(hip, sets):
    bls = hip[0]
    pks, msgs, sigs = (x[:8] for x in sets)
    for name, bad in bad_keys().items():
        for pos in (0, 1, 2, 3, 5):  # every row of a workgroup, and the second workgroup
            p2 = list(pks)
            p2[pos] = bad
            got = _raw(bls, p2, msgs, sigs)
            assert got is False, (name, pos)
    assert O.batch_verify([[bad_keys()["order 11"]]], [msgs[0]], [sigs[0]]) is False


def test_sigs_outside_g2_each_row(hip, sets):
    bls = hip[0]
    pks, msgs, sigs = (x[:8] for x in sets)
    for name, bad in bad_sigs().items():
        for pos in (0, 1, 2, 3, 6):
            s2 = list(sigs)
            s2[pos] = bad
            assert _raw(bls, pks, msgs, s2) is False, (name, pos)
    assert O.batch_verify([[pks[0]]], [msgs[0]], [bad_sigs()["order 13"]]) is False


def test_verify_each_codes_for_outside_points(hip, sets):
    """Per-set verdicts (tbls_verify_each) on the same points equal the oracle's."""
    bls = hip[0]
    pks, msgs, sigs = sets
    bk, bs = list(bad_keys().values()), list(bad_sigs().values())
    rows = [(pks[i], 1, msgs[i], sigs[i]) for i in range(4)]
    rows += [(k, 1, msgs[0], sigs[0]) for k in bk] + [(pks[1], 1, msgs[1], s) for s in bs]
    got = bls.verify_each_raw(rows)
    assert got == [True] * 4 + [False] * (len(bk) + len(bs))


def test_dev_batch_uneven_sets_fallback(hip, sets):
    """As many keys as sets, one set empty and one of two keys: the kernel's
    one-lane fallback.  The partial record's invalid-set count is exactly the
    empty set (the two-key set verifies), then 2 with a bad key in it."""
    import torch

    bls, native, L = hip
    pks, msgs, sigs = sets
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    m = b"\x42" * 32
    agg = O.aggregate_sigs([O.sign(interop_sk(i), m) for i in range(2)])
    n = 6

    def run(k1):
        keys = [pks[0], k1] + [pks[i] for i in range(2, 6)]  # set 0: none, set 1: keys 0, 1, sets 2..5: one each
        off = [0, 0, 2, 3, 4, 5, 6]
        ms = [msgs[0], m] + [msgs[i] for i in range(2, 6)]
        sg = [sigs[0], agg] + [sigs[i] for i in range(2, 6)]
        u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731
        t = dict(pks=u8(b"".join(keys)), msgs=u8(b"".join(ms)), sigs=u8(b"".join(sg)),
                 pk_off=torch.tensor(off, dtype=torch.int32, device=dev),
                 msg_off=torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=dev),
                 rand=torch.tensor([random.getrandbits(62) | 1 for _ in range(n)], dtype=torch.int64, device=dev))
        d = native.TblsDevBatch(t["pks"].data_ptr(), t["pk_off"].data_ptr(), n, t["msgs"].data_ptr(), t["msg_off"].data_ptr(),
                                t["sigs"].data_ptr(), t["rand"].data_ptr(), n)
        out = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=dev)
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(d), stream, out.data_ptr()), "partial")
        torch.cuda.synchronize()
        return int.from_bytes(bytes(out[576:580].cpu().numpy()), "little")

    assert run(pks[1]) == 1
    assert run(bad_keys()["order 11"]) == 2


def test_multi_key_batch_keys_outside_g1_quad(hip):
    """Multi-key batches (k_pk_decompress, then the multi-key aggregation):
    every outside-G1 key -- random non-G1 points and points of order 3, 11,
    33, whose multiples meet the exceptional addition cases of the [x^2]
    chain -- at several positions of a 16 sets x 20 keys batch makes the
    batch fail, and the clean batch verifies.  (Round 4 measured a
    quad-per-key decompression kernel here: configs 2/3 p50 5.48 -> 5.80 ms,
    its 4 x 31,232 lanes fill the chip where the one-lane kernel's chains
    run a quarter-full GPU, so it was removed.)"""
    from teku_amd import synth

    bls = hip[0]
    keys, msgs, sigs = synth.multi_key(16, 20, first_key=3000, seed=9)
    rands = [random.getrandbits(64) | 1 for _ in sigs]

    def run(ks):
        return bls.batch_verify_raw([(b"".join(k), len(k), m, s) for k, m, s in zip(ks, msgs, sigs)], rands)

    assert run(keys) is True
    for name, bad in bad_keys().items():
        for s_i, k_i in ((0, 0), (3, 1), (7, 2), (15, 19)):
            ks = [list(k) for k in keys]
            ks[s_i][k_i] = bad
            assert run(ks) is False, (name, s_i, k_i)
