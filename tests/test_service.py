"""Host logic of the GPU-aware AggregatingSignatureVerificationService
(teku_amd/service.py), with the C oracle as the
verification backend (CPU; the device backend is covered by
tests/test_gpu_bls.py::test_verify_each_and_service).

Mirrors the reference's AggregatingSignatureVerificationServiceTest
(statetransition/src/test/.../signatures/AggregatingSignatureVerificationServiceTest.java):
valid batches complete true, one invalid task among valid ones completes
false alone, a full queue fails the future, verify before start raises."""

import random

import pytest

from oracle import c_oracle as C
from oracle.keys import interop_sk
from teku_amd.service import AggregatingSignatureVerificationService, ServiceCapacityExceededException


@pytest.fixture(scope="module")
def keyset():
    sks = [interop_sk(i) for i in range(12)]
    pks = [C.sk_to_pk(s) for s in sks]
    msgs = [bytes([i + 7]) * 32 for i in range(12)]
    sigs = [C.sign(s, m) for s, m in zip(sks, msgs)]
    return pks, msgs, sigs


def _oracle_batch(sets):
    assert all(npk == 1 for _, npk, _, _ in sets)
    rng = random.Random(len(sets))
    if len(sets) == 1:
        sets = sets * 2  # the oracle's batch takes n >= 2; (s, s) is valid iff s is
    return C.batch_verify([s[0] for s in sets], [s[2] for s in sets], [s[3] for s in sets], [rng.getrandbits(63) | 1 for _ in sets])


def _oracle_each(sets):
    return [_oracle_batch([s]) for s in sets]


def _svc(**kw):
    calls = {"batch": 0, "each": 0}

    def b(sets):
        calls["batch"] += 1
        return _oracle_batch(sets)

    def e(sets):
        calls["each"] += 1
        return _oracle_each(sets)

    s = AggregatingSignatureVerificationService(batch_fn=b, each_fn=e, **kw)
    return s, calls


def test_valid_and_invalid_tasks_one_batch(keyset):
    pks, msgs, sigs = keyset
    svc, calls = _svc(max_batch_size=64)
    bad = {3, 8}
    tasks = []
    for i in range(12):
        sig = sigs[(i + 1) % 12] if i in bad else sigs[i]
        tasks.append(SignatureTaskArgs(pks[i], msgs[i], sig))
    # drive one batch directly (deterministic batching)
    from teku_amd.service import SignatureTask, _set_tuple

    ts = [SignatureTask([_set_tuple([t.pk], t.msg, t.sig)]) for t in tasks]
    svc.batch_verify_signatures(ts)
    assert [t.result.result() for t in ts] == [i not in bad for i in range(12)]
    assert calls == {"batch": 1, "each": 1}  # one failed batch -> one per-set pass, no halving
    m = svc.metrics()  # the reference's executor metrics (AggregatingSignatureVerificationService.java:76-98)
    assert m["signature_verifications_batch_count_total"] == 1 and m["signature_verifications_task_count_total"] == 12
    assert m["signature_verifications_batch_size"] == [12] and m["device_passes_total"] == 2
    assert m["device_sets_per_s"] is None  # a custom batch_fn has no device timing
    assert svc.batch_count == 1 and svc.task_count == 12


def test_split_fallback_matches_reference_halving(keyset):
    pks, msgs, sigs = keyset
    from teku_amd.service import SignatureTask, _set_tuple

    svc, calls = _svc(split_fallback=True, min_batch_size_to_split=4)
    ts = [SignatureTask([_set_tuple([pks[i]], msgs[i], sigs[i] if i != 5 else sigs[6])]) for i in range(12)]
    svc.batch_verify_signatures(ts)
    assert [t.result.result() for t in ts] == [i != 5 for i in range(12)]
    assert calls["batch"] > 1  # halving re-verifies sub-batches


def test_multi_set_task_and_threads(keyset):
    pks, msgs, sigs = keyset
    svc, _ = _svc(max_batch_size=5)
    svc.start()
    try:
        good = svc.verify_many([[pks[0]], [pks[1]]], [msgs[0], msgs[1]], [sigs[0], sigs[1]])
        mixed = svc.verify_many([[pks[2]], [pks[3]]], [msgs[2], msgs[3]], [sigs[2], sigs[2]])
        single = [svc.verify([pks[i]], msgs[i], sigs[i]) for i in range(4, 12)]
        empty = svc.verify_many([], [], [])
        assert good.result(timeout=60) is True
        assert mixed.result(timeout=60) is False
        assert all(f.result(timeout=60) for f in single)
        assert empty.result(timeout=60) is False
        with pytest.raises(Exception):
            svc.verify_many([[pks[0]]], [msgs[0], msgs[1]], [sigs[0]]).result(timeout=5)
    finally:
        svc.stop()


def test_queue_full_and_not_running(keyset):
    pks, msgs, sigs = keyset
    svc, _ = _svc(queue_capacity=1)
    with pytest.raises(RuntimeError):
        svc.verify([pks[0]], msgs[0], sigs[0])
    svc._running = True  # accept without workers draining
    f1 = svc.verify([pks[0]], msgs[0], sigs[0])
    f2 = svc.verify([pks[1]], msgs[1], sigs[1])
    assert not f1.done()
    with pytest.raises(ServiceCapacityExceededException):
        f2.result(timeout=1)
    assert svc.queue_size() == 1


class SignatureTaskArgs:
    def __init__(self, pk, msg, sig):
        self.pk, self.msg, self.sig = pk, msg, sig


class _SimNode:
    """8 simulated devices behind the service's device call: each batch is
    placed by the library's own placement (tbls_place_plan, no device) with
    the n_gpus the service passes and the live load of the batches still in
    flight, holds its devices until `hold` batches are in flight at once (a
    barrier), then completes valid."""

    def __init__(self, hold, D=8):
        import threading

        self.D, self.load, self.placed, self.rr = D, [0] * D, [], 0
        self.lock = threading.Lock()
        self.barrier = threading.Barrier(hold, timeout=60) if hold > 1 else None

    def __call__(self, sets, n_gpus, timing):
        from teku_amd import native

        with self.lock:
            devs, cuts = native.place_plan(len(sets), n_devices=self.D, n_gpus=n_gpus, load=self.load, rr=self.rr)
            self.rr += 1
            for d in devs:
                self.load[d] += 1
            self.placed.append((len(sets), n_gpus, devs))
        if self.barrier is not None:
            self.barrier.wait()
        with self.lock:
            for d in devs:
                self.load[d] -= 1
        timing.n_devices = len(devs)
        return True, [True] * len(sets)


def _gossip_tasks(n, k):
    from teku_amd.service import SignatureTask

    return [SignatureTask([(bytes([i % 251]) * 48, 1, (i).to_bytes(32, "little"), bytes(96))]) for i in range(n * k)]


def test_concurrent_config4_batches_on_eight_simulated_devices():
    """8 workers drain 8 x 16,384 queued gossip tasks;
    a batch that leaves tasks waiting asks for one device, one that drains
    the queue finds the node busy: the 8 concurrent batches run on 8
    distinct devices, one each (the library's placement, tbls_place_plan)."""
    node = _SimNode(hold=8)
    svc = AggregatingSignatureVerificationService(num_threads=8, max_batch_size=16384, queue_capacity=8 * 16384, batch_each_fn=node)
    tasks = _gossip_tasks(8, 16384)
    svc._running = True
    for t in tasks:
        svc.batch_signature_tasks.put_nowait(t)
    svc.start()
    try:
        assert all(t.result.result(timeout=120) for t in tasks)
    finally:
        svc.stop()
    assert sorted(n for n, _, _ in node.placed) == [16384] * 8
    assert all(len(devs) == 1 for _, _, devs in node.placed)
    assert sorted(devs[0] for _, _, devs in node.placed) == list(range(8))
    assert sum(g for _, g, _ in node.placed) >= 1  # batches that left tasks waiting asked for one device


def test_lone_config4_batch_shards_on_idle_simulated_node():
    """a lone 16,384-task batch that drains the queue
    passes n_gpus = 0, and on an idle node the library shards it to the
    latency knee: 4 devices of 4,096 sets."""
    node = _SimNode(hold=1)
    svc = AggregatingSignatureVerificationService(num_threads=8, max_batch_size=16384, batch_each_fn=node)
    tasks = _gossip_tasks(1, 16384)
    svc.batch_verify_signatures(tasks)
    assert all(t.result.result(timeout=5) for t in tasks)
    (n, g, devs), = node.placed
    assert n == 16384 and g == 0 and len(devs) == 4
    assert svc.last_batch_timing["n_devices"] == 4


def test_task_future_interface():
    import threading

    from teku_amd.service import TaskFuture

    f = TaskFuture()
    seen = []
    f.add_done_callback(lambda x: seen.append(x.result()))
    assert not f.done()
    with pytest.raises(TimeoutError):
        f.result(timeout=0.01)
    threading.Timer(0.05, f.set_result, args=(True,)).start()
    assert f.result(timeout=5) is True and f.done() and f.exception() is None and seen == [True]
    g = TaskFuture()
    g.set_exception(ValueError("x"))
    with pytest.raises(ValueError):
        g.result()
    assert isinstance(g.exception(), ValueError)
    cond = threading.Condition()
    fs = [TaskFuture(cond) for _ in range(5)]
    TaskFuture.complete_all(fs, [True, False, True, True, False])
    assert [x.result(timeout=0) for x in fs] == [True, False, True, True, False]
