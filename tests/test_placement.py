"""Device placement of batches (tb_lib.hip place_plan through tbls_place_plan;
pure host logic, no device): small batches go whole to the least-loaded
device, large ones shard over every device with key-balanced cuts, and
concurrent callers land on different devices (SURVEY.md 8(e);
AggregatingSignatureVerificationService.java:121-132, 202-205)."""

import random

import pytest

from teku_amd import dist, native


def test_shard_min_default():
    assert native.load_library().tbls_shard_min() == 2048


@pytest.mark.parametrize("D", [1, 2, 4, 8])
def test_config1_batch_stays_on_one_device(D):
    for rr in range(2 * D):
        devs, cuts = native.place_plan(128, n_devices=D, rr=rr, shard_min=2048)
        assert devs == [rr % D] and cuts == [0, 128]


@pytest.mark.parametrize("D", [1, 2, 4, 8])
def test_config4_batch_uses_every_device(D):
    devs, cuts = native.place_plan(16384, n_devices=D, shard_min=2048)
    assert devs == list(range(D))
    assert cuts == [16384 * k // D for k in range(D + 1)]


@pytest.mark.parametrize("n,D,G", [(2047, 8, 1), (2048, 8, 1), (4095, 8, 1), (4096, 8, 2), (6144, 8, 3), (16383, 8, 7),
                                   (1048576, 8, 8), (131072, 4, 4), (5, 8, 1)])
def test_device_count_follows_shard_min(n, D, G):
    devs, cuts = native.place_plan(n, n_devices=D, shard_min=2048)
    assert len(devs) == G and cuts[0] == 0 and cuts[-1] == n
    assert all(cuts[k] <= cuts[k + 1] for k in range(G))
    if G > 1:
        assert min(cuts[k + 1] - cuts[k] for k in range(G)) >= 2048 - 1


def test_n_gpus_caps_and_shard_min_zero():
    devs, _ = native.place_plan(1048576, n_devices=8, n_gpus=2, shard_min=2048)
    assert len(devs) == 2
    devs, cuts = native.place_plan(6, n_devices=8, shard_min=0)
    assert len(devs) == 6 and cuts == list(range(7))  # never more devices than sets
    devs, _ = native.place_plan(100, n_devices=4, shard_min=0)
    assert devs == [0, 1, 2, 3]


def test_least_loaded_devices_chosen():
    devs, _ = native.place_plan(128, n_devices=4, load=[1, 0, 2, 0], rr=0, shard_min=2048)
    assert devs == [1]
    devs, _ = native.place_plan(128, n_devices=4, load=[1, 0, 2, 0], rr=2, shard_min=2048)
    assert devs == [3]  # equal loads: round-robin from rr
    devs, _ = native.place_plan(4096, n_devices=4, load=[3, 0, 2, 1], rr=0, shard_min=2048)
    assert devs == [1, 3]  # the two least loaded, ascending (lock order, root first)


def test_concurrent_workers_spread_over_devices():
    """N workers each holding one small batch: the live library counts a
    placed batch as load until it returns, so the next placement avoids it."""
    for D in (2, 4, 8):
        load = [0] * D
        got = []
        for w in range(D):
            devs, _ = native.place_plan(250, n_devices=D, load=load, rr=7 * w, shard_min=2048)
            assert len(devs) == 1
            load[devs[0]] += 1
            got.append(devs[0])
        assert sorted(got) == list(range(D))


def test_cuts_are_key_balanced_like_dist():
    rng = random.Random(5)
    n_pks = [rng.choice([1, 1, 1, 488, 512]) for _ in range(9000)]
    for D in (2, 4, 8):
        devs, cuts = native.place_plan(len(n_pks), n_pks=n_pks, n_devices=D, shard_min=1)
        assert len(devs) == D
        for r in range(D):
            assert (cuts[r], cuts[r + 1]) == dist.shard_bounds(len(n_pks), D, r, n_pks)


def test_bad_arguments():
    L = native.load_library()
    import ctypes

    dev = (ctypes.c_int * 1)()
    cut = (ctypes.c_size_t * 2)()
    assert L.tbls_place_plan(10, None, 0, 0, None, 0, 2048, dev, cut) < 0


@pytest.mark.parametrize("n,plan", [(131072, (16, 8)), (16384, (8, 16)), (1048576, (16, 4)), (3000, (2, 16))])
def test_accumulator_plan(n, plan):
    """tb_lib.hip acc_plan (tbls_acc_plan, no device): the segmented Miller
    accumulator's pairs per thread x loop segments for the bench batch
    (131,072 sets: one 65,536-thread wave round of 16 x 8), config 4
    (16,384 sets, per-set signature pairs: 32,768 pairs, 8 x 16), 1,048,576 sets (262,144-pair
    chunks: 16 x 4) and 3,000 sets (6,000 pairs: 2 x 16)."""
    per, nseg, split = native.acc_plan(n)
    assert split == 1 and (per, nseg) == plan
