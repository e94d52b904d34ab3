"""Device placement of batches (tb_lib.hip place_plan through tbls_place_plan;
pure host logic, no device): a batch is sharded only over IDLE devices and
only into shards of at least shard_min = 32,768 sets (where one device's
partial stops being a latency chain, profiles/r04_stage_sweep_final.json);
with no idle device it goes whole to the least-loaded one, so concurrent
callers land on different devices (SURVEY.md 8(e);
AggregatingSignatureVerificationService.java:121-132, 202-205).  On an idle
node (every device idle) a lone batch shards down to the latency knee of
4,096 sets per device; a service with more batches
waiting passes n_gpus = 1 (teku_amd/service.py)."""

import random

import pytest

from teku_amd import dist, native

SMIN = 32768
KNEE = 4096


def test_shard_min_default():
    assert native.load_library().tbls_shard_min() == SMIN
    assert native.load_library().tbls_shard_knee() == KNEE


@pytest.mark.parametrize("D", [1, 2, 4, 8])
def test_config1_batch_stays_on_one_device(D):
    for rr in range(2 * D):
        devs, cuts = native.place_plan(128, n_devices=D, rr=rr, shard_min=SMIN)
        assert devs == [rr % D] and cuts == [0, 128]


@pytest.mark.parametrize("D", [1, 2, 4, 8])
def test_config4_batch_takes_one_device(D):
    """16,384 sets is below shard_min: one device when any device is busy
    (here device (rr + 1) % D holds a batch), or with no knee."""
    for rr in range(D):
        devs, cuts = native.place_plan(16384, n_devices=D, rr=rr, shard_min=SMIN, shard_knee=0)
        assert devs == [rr % D] and cuts == [0, 16384]
        if D > 1:
            load = [0] * D
            load[(rr + 1) % D] = 1
            devs, cuts = native.place_plan(16384, n_devices=D, load=load, rr=rr, shard_min=SMIN)
            assert devs == [rr % D] and cuts == [0, 16384]


@pytest.mark.parametrize("D,G", [(1, 1), (2, 2), (4, 4), (8, 4)])
def test_lone_config4_batch_on_idle_node_shards_to_the_knee(D, G):
    """a lone 16,384-set batch on an idle node runs as
    shards of 4,096 sets (modelled device latency 8.6 -> 5.8 ms plus the 0.8 ms
    final exponentiation, profiles/r04_stage_sweep_final.json)."""
    devs, cuts = native.place_plan(16384, n_devices=D, shard_min=SMIN)
    assert len(devs) == G and cuts[0] == 0 and cuts[-1] == 16384
    assert all(cuts[k + 1] - cuts[k] >= KNEE for k in range(G))
    # 8 idle devices, but the caller allows one (a service with batches waiting)
    devs, cuts = native.place_plan(16384, n_devices=D, n_gpus=1, shard_min=SMIN)
    assert len(devs) == 1 and cuts == [0, 16384]


@pytest.mark.parametrize("n,G", [(128, 1), (8191, 1), (8192, 2), (12288, 3), (16384, 4), (32768, 8), (131072, 8)])
def test_idle_node_knee_counts(n, G):
    devs, cuts = native.place_plan(n, n_devices=8, shard_min=SMIN)
    assert len(devs) == G and cuts[-1] == n


def test_eight_concurrent_config4_batches_get_eight_devices():
    """8 simulated devices, 8 service workers each
    placing a 16,384-set batch while the earlier ones are still in flight ->
    8 distinct single devices (round 4: every batch took all 8).  The first
    seven see more batches waiting in the service queue and pass n_gpus = 1;
    the last finds the queue empty (n_gpus = 0) but the node busy."""
    load = [0] * 8
    got = []
    for w in range(8):
        devs, cuts = native.place_plan(16384, n_devices=8, n_gpus=1 if w < 7 else 0, load=load, rr=3 * w + 1, shard_min=SMIN)
        assert len(devs) == 1 and cuts == [0, 16384]
        load[devs[0]] += 1
        got.append(devs[0])
    assert sorted(got) == list(range(8))
    # a ninth caller shares the least-loaded device (all hold one batch)
    devs, _ = native.place_plan(16384, n_devices=8, load=load, rr=5, shard_min=SMIN)
    assert devs == [5]


@pytest.mark.parametrize("n,D,G", [(32767, 8, 1), (65535, 8, 1), (65536, 8, 2), (131072, 8, 4), (131072, 4, 4), (131072, 2, 2),
                                   (262144, 8, 8), (1048576, 8, 8), (5, 8, 1)])
def test_device_count_follows_shard_min(n, D, G):
    """The shard_min rule alone (no knee, as on a node with a device busy):
    131,072 sets still shard (4 x 32,768), config 5's 1,048,576 sets use all 8
    devices."""
    devs, cuts = native.place_plan(n, n_devices=D, shard_min=SMIN, shard_knee=0)
    assert len(devs) == G and cuts[0] == 0 and cuts[-1] == n
    assert all(cuts[k] <= cuts[k + 1] for k in range(G))
    if G > 1:
        assert min(cuts[k + 1] - cuts[k] for k in range(G)) >= SMIN - 1


def test_sharding_uses_idle_devices_only():
    # 1M sets with 3 devices busy: the 5 idle ones, ascending
    devs, cuts = native.place_plan(1048576, n_devices=8, load=[1, 0, 2, 0, 0, 1, 0, 0], rr=0, shard_min=SMIN)
    assert devs == [1, 3, 4, 6, 7] and cuts[-1] == 1048576
    # every device busy: whole batch on the least loaded one
    devs, cuts = native.place_plan(1048576, n_devices=4, load=[2, 1, 3, 1], rr=0, shard_min=SMIN)
    assert devs == [1] and cuts == [0, 1048576]
    devs, _ = native.place_plan(1048576, n_devices=4, load=[2, 1, 3, 1], rr=2, shard_min=SMIN)
    assert devs == [3]  # equal loads: round-robin from rr


def test_n_gpus_caps_and_shard_min_zero():
    devs, _ = native.place_plan(1048576, n_devices=8, n_gpus=2, shard_min=SMIN)
    assert len(devs) == 2
    devs, _ = native.place_plan(16384, n_devices=8, n_gpus=2, shard_min=SMIN)
    assert len(devs) == 2  # the knee on an idle node, capped by n_gpus
    devs, cuts = native.place_plan(6, n_devices=8, shard_min=0)
    assert len(devs) == 6 and cuts == list(range(7))  # never more devices than sets
    devs, _ = native.place_plan(100, n_devices=4, shard_min=0)
    assert devs == [0, 1, 2, 3]
    devs, _ = native.place_plan(100, n_devices=4, load=[0, 1, 0, 0], shard_min=0)
    assert devs == [0, 2, 3]


def test_least_loaded_devices_chosen():
    devs, _ = native.place_plan(128, n_devices=4, load=[1, 0, 2, 0], rr=0, shard_min=SMIN)
    assert devs == [1]
    devs, _ = native.place_plan(128, n_devices=4, load=[1, 0, 2, 0], rr=2, shard_min=SMIN)
    assert devs == [3]  # equal loads: round-robin from rr
    devs, _ = native.place_plan(4 * SMIN, n_devices=4, load=[3, 0, 2, 0], rr=0, shard_min=SMIN)
    assert devs == [1, 3]  # the two idle ones, ascending (lock order, root first)


def test_concurrent_workers_spread_over_devices():
    """N workers each holding one small batch: the live library counts a
    placed batch as load until it returns, so the next placement avoids it."""
    for D in (2, 4, 8):
        load = [0] * D
        got = []
        for w in range(D):
            devs, _ = native.place_plan(250, n_devices=D, load=load, rr=7 * w, shard_min=SMIN)
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
    assert L.tbls_place_plan(10, None, 0, 0, None, 0, 2048, 0, dev, cut) < 0


@pytest.mark.parametrize("n,plan", [(131072, (16, 8)), (16384, (8, 16)), (1048576, (16, 4)), (3000, (2, 16))])
def test_accumulator_plan(n, plan):
    """tb_lib.hip acc_plan (tbls_acc_plan, no device): the segmented Miller
    accumulator's pairs per thread x loop segments for the bench batch
    (131,072 sets: one 65,536-thread wave round of 16 x 8), config 4
    (16,384 sets, per-set signature pairs: 32,768 pairs, 8 x 16), 1,048,576 sets (262,144-pair
    chunks: 16 x 4) and 3,000 sets (6,000 pairs: 2 x 16)."""
    per, nseg, split = native.acc_plan(n)
    assert split == 1 and (per, nseg) == plan
