"""Per-set verdicts of a failed batch from the batch's own work
(tbls_batch_verify_each; tb_lib.hip settle_sets):
per-set Miller values from the batch's lines, group tests over 256- and
16-set groups, then single sets.  Verdicts must equal the C oracle's
fastAggregateVerify per set (the reference's BLS.batchVerify per task,
AggregatingSignatureVerificationService.java:206-233), at every size class:
settled in place (no bucket sums, split Miller kernels: 2,048-16,384 sets) and
re-staged in the settle layout (<= 1,024 sets: wave Miller loops; >= 20,480:
bucket sums)."""

import pytest

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu
THREADS = 16


@pytest.fixture(scope="module")
def S():
    import torch  # noqa: F401

    from teku_amd import native, synth

    native.lib()
    return synth


def _run(S, pk, ms, sg, n_pks=None):
    from teku_amd import native

    if n_pks is None:
        arr = S.SetArray(b"".join(pk), [1] * len(sg), b"".join(ms), [len(m) for m in ms], b"".join(sg))
    else:
        arr = S.SetArray(b"".join(pk), n_pks, b"".join(ms), [len(m) for m in ms], b"".join(sg))
    native.stats(reset=True)
    ok, each = arr.batch_verify_each(S.fast_multipliers(len(sg)))
    return ok, each, native.stats()


def _sets(S, n, seed):
    pks, msgs, sigs = S.single_signer(0, n, seed=seed)
    return ([pks[48 * i : 48 * i + 48] for i in range(n)], [msgs[32 * i : 32 * i + 32] for i in range(n)],
            [sigs[96 * i : 96 * i + 96] for i in range(n)])


@pytest.mark.parametrize("n", [16384, 4096, 2049])
def test_settle_in_place(S, n):
    pk, ms, sg = _sets(S, n, seed=4)
    ok, each, st = _run(S, pk, ms, sg)
    assert ok and all(each) and st["settled"] == 0 and st["partials"] == 1
    bad = {11: sg[12], n // 3: bytes(96), n // 2: S.NOT_IN_G2, n - 1: sg[0], 17 % n: sg[16]}
    for j, b in bad.items():
        sg[j] = b
    ok, each, st = _run(S, pk, ms, sg)
    assert not ok and st["settled"] == 1 and st["partials"] == 1 and st["each_passes"] == 0, st
    assert [i for i, v in enumerate(each) if not v] == sorted(bad)
    if n == 16384:
        assert each == C.verify_each([[p] for p in pk], ms, sg, threads=THREADS)


@pytest.mark.parametrize("n", [128, 1000])
def test_settle_restaged_small(S, n):
    """Wave Miller loops (no lines): the sets are re-staged in the settle layout."""
    pk, ms, sg = _sets(S, n, seed=6)
    sg[5] = sg[6]
    pk[n - 2] = pk[0]
    ok, each, st = _run(S, pk, ms, sg)
    assert not ok and st["settled"] == 1 and st["partials"] == 2, st
    assert each == C.verify_each([[p] for p in pk], ms, sg, threads=THREADS)


def test_settle_restaged_bucket_sums(S):
    """24,576 sets ran the bucket-sum signature side: re-staged per chunk."""
    n = 24576
    pk, ms, sg = _sets(S, n, seed=7)
    bad = {0: sg[1], 12345: bytes([0xC0]) + bytes(95), 24575: S.NOT_IN_G2}
    for j, b in bad.items():
        sg[j] = b
    ok, each, st = _run(S, pk, ms, sg)
    assert not ok and st["settled"] == 1 and st["partials"] == 2, st
    assert [i for i, v in enumerate(each) if not v] == sorted(bad)
    for j in bad:
        lo, hi = max(0, j - 2), min(n, j + 3)
        assert each[lo:hi] == C.verify_each([[p] for p in pk[lo:hi]], ms[lo:hi], sg[lo:hi], threads=THREADS)


def test_settle_multi_key_and_empty(S):
    """Sets of 8 keys, one with a wrong key, one aggregate over a swapped
    message, and a set with no keys (false, left out of the batch)."""
    keys, msgs, sigs = S.multi_key(40, 8, first_key=300, seed=8)
    keys = [list(k) for k in keys]
    keys[3][5] = keys[4][5]
    msgs = list(msgs)
    msgs[30] = msgs[31]
    keys[20] = []
    flat = [k for ks in keys for k in ks]
    ok, each, st = _run(S, flat, msgs, sigs, n_pks=[len(k) for k in keys])
    assert not ok
    assert [i for i, v in enumerate(each) if not v] == [3, 20, 30]
    assert each == C.verify_each(keys, msgs, sigs, threads=THREADS)
