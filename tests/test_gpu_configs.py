"""GPU parity at every BASELINE.json config size, checked against the C oracle
(oracle/c/bls_oracle.c, pinned by the reference's KATs in tests/test_oracle_c.py).

  config 1  BLS.batchVerify of 128 single-signer interop-key sets on distinct
            messages (BLSBenchmark.java:41-57), valid and every SURVEY.md 8(d)
            tamper, through tbls_batch_verify
  config 2  64 sync-committee sets x 512 keys, fastAggregateVerify per set
            (BLS.java:185-207) through tbls_fast_aggregate_verify_many, 3 tampered
  config 3  64 attestation sets x 488 keys, randomized batchVerify, valid / one
            bad key / one bad signature (BlstPublicKey.java:55-71)
  config 4  16,384 single-signer sets through the service semantics
            (AggregatingSignatureVerificationService.java:171-227), 4 bad, per-task
            verdicts
  config 5  one GPU's 131,072-set shard of the 1,048,576-set batch, valid and
            tampered in the first, middle and last MSM chunk

Inputs are the synthetic sets of SURVEY.md 8(d) (teku_amd/synth.py: interop keys,
sha256 messages, GPU-signed); the oracle verifies the same bytes.
"""

import ctypes
import os

import pytest

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


@pytest.fixture(scope="module")
def S():
    import torch  # noqa: F401  (share torch's HIP runtime)

    from teku_amd import native, synth

    native.lib()
    return synth


def _split(pks, msgs, sigs):
    n = len(sigs) // 96
    return [pks[48 * i : 48 * i + 48] for i in range(n)], [msgs[32 * i : 32 * i + 32] for i in range(n)], [sigs[96 * i : 96 * i + 96] for i in range(n)]


def _tampers(S, pk, ms, sg, j, sk_j):
    """SURVEY.md 8(d) tampered-set list at position j (each expects false)."""
    out = {}
    s = list(sg)
    s[j] = S.sign_blob([sk_j], [bytes([ms[j][0] ^ 1]) + ms[j][1:]])
    out["sig on m^1"] = (pk, ms, s)
    m = list(ms)
    m[j], m[j + 1] = m[j + 1], m[j]
    out["two messages swapped"] = (pk, m, sg)
    for name, bad in [("zero sig", bytes(96)), ("infinity sig", S.INFINITY_G2), ("non-G2 sig", S.NOT_IN_G2)]:
        s = list(sg)
        s[j] = bad
        out[name] = (pk, ms, s)
    for name, bad in [("infinity key", S.INFINITY_G1), ("0x9378a6 key", S.BAD_PK)]:
        p = list(pk)
        p[j] = bad
        out[name] = (p, ms, sg)
    return out


def test_config1_128_sets(S):
    pks, msgs, sigs = S.single_signer(0, 128)
    pk, ms, sg = _split(pks, msgs, sigs)
    r = S.random_multipliers(128)
    assert S.SetArray.single(pks, msgs, sigs).batch_verify(r) is True
    assert C.batch_verify(pk, ms, sg, r, threads=THREADS) is True
    for j in (0, 77, 126):
        for name, (p, m, s) in _tampers(S, pk, ms, sg, j, S.interop_sk(j)).items():
            got = S.SetArray.single(b"".join(p), b"".join(m), b"".join(s)).batch_verify(r)
            exp = C.batch_verify(p, m, s, r, threads=THREADS)
            assert got is exp is False, (name, j)


def test_config2_64x512_fast_aggregate_verify(S):
    keys, msgs, sigs = S.multi_key(64, 512, first_key=0, seed=2)
    arr = S.SetArray.from_lists(keys, msgs, sigs)
    assert arr.fast_aggregate_verify_many() == [True] * 64
    # three tampered sets: a signature over another message, a key swapped for
    # a non-signer, an infinity key (BlstPublicKey.aggregate -> infinity)
    k2, m2, s2 = [list(k) for k in keys], list(msgs), list(sigs)
    s2[5] = sigs[6]
    k2[20][100] = S.pubkeys([S.interop_sk(40000)])[0]
    k2[63][511] = S.INFINITY_G1
    got = S.SetArray.from_lists(k2, m2, s2).fast_aggregate_verify_many()
    exp = C.verify_each(k2, m2, s2, threads=THREADS)
    assert got == exp
    assert [i for i, v in enumerate(got) if not v] == [5, 20, 63]


def test_config3_64x488_randomized_batch(S):
    keys, msgs, sigs = S.multi_key(64, 488, first_key=1000, seed=3)
    r = S.random_multipliers(64)
    assert S.SetArray.from_lists(keys, msgs, sigs).batch_verify(r) is True
    assert C.batch_verify_sets(keys, msgs, sigs, r, threads=THREADS) is True
    k2 = [list(k) for k in keys]
    k2[31][7] = S.pubkeys([S.interop_sk(50000)])[0]  # one bad key
    assert S.SetArray.from_lists(k2, msgs, sigs).batch_verify(r) is False
    assert C.batch_verify_sets(k2, msgs, sigs, r, threads=THREADS) is False
    s2 = list(sigs)
    s2[40] = sigs[41]  # one bad signature
    assert S.SetArray.from_lists(keys, msgs, s2).batch_verify(r) is False
    assert C.batch_verify_sets(keys, msgs, s2, r, threads=THREADS) is False


def test_config4_16k_through_service(S):
    from teku_amd.service import AggregatingSignatureVerificationService, SignatureTask

    n = 16384
    pks, msgs, sigs = S.single_signer(0, n, seed=4)
    pk, ms, sg = _split(pks, msgs, sigs)
    bad = {11: sg[12], 5000: bytes(96), 9999: S.NOT_IN_G2, 16383: sg[0]}
    for j, b in bad.items():
        sg[j] = b
    svc = AggregatingSignatureVerificationService(max_batch_size=n)
    tasks = [SignatureTask([(pk[i], 1, ms[i], sg[i])]) for i in range(n)]
    svc.batch_verify_signatures(tasks)
    got = [t.result.result() for t in tasks]
    exp = C.verify_each([[p] for p in pk], ms, sg, threads=THREADS)
    assert got == exp
    assert [i for i, v in enumerate(got) if not v] == sorted(bad)
    assert svc.device_passes == 1 and svc.last_batch_timing["settled"]  # batch + in-place settle: one call
    m = svc.metrics()  # device metrics from the library's tbls_timing
    assert m["device_sets_verified_total"] == n and m["device_sets_per_s"] > 0 and m["last_batch"]["n_devices"] >= 1


N5, SHARD5 = 1048576, 131072  # config 5: 8 GPUs x 131,072 sets


@pytest.fixture(scope="module")
def cfg5(S):
    """Config 5 at its stated size: 1,048,576 single-signer sets (keys cyclic
    over the first 65,536 interop keys, distinct messages)."""
    return S.single_signer(0, N5, seed=5)


def _dev_partial(native, L, torch, dev, stream, pks, msgs, sigs, rands):
    n = len(sigs) // 96
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731
    t = dict(pks=u8(pks), msgs=u8(msgs), sigs=u8(sigs), pk_off=torch.arange(0, n + 1, dtype=torch.int32, device=dev),
             msg_off=torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=dev),
             rand=torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in rands], dtype=torch.int64, device=dev))
    d = native.TblsDevBatch(t["pks"].data_ptr(), t["pk_off"].data_ptr(), n, t["msgs"].data_ptr(), t["msg_off"].data_ptr(), t["sigs"].data_ptr(),
                            t["rand"].data_ptr(), n)
    out = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=dev)
    native.check(L.tbls_dev_batch_partial(0, ctypes.byref(d), stream, out.data_ptr()), "partial")
    torch.cuda.synchronize()
    return out


def test_config5_1m_as_8_simulated_shards(S, cfg5):
    """SURVEY.md 8(e) at config 5's stated size on one GPU: 8 shards of
    131,072 sets -> 8 partial records -> one gathered final exponentiation
    (tbls_dev_final_verify with g = 8), valid, then with one tampered set in
    shard 0 and in shard 7 (the oracle decides each tampered set alone)."""
    import torch

    from teku_amd import native

    L = native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    pks, msgs, sigs = cfg5
    rands = S.random_multipliers(N5)

    def shard(g, sg=None):
        lo, hi = g * SHARD5, (g + 1) * SHARD5
        return _dev_partial(native, L, torch, dev, stream, pks[48 * lo : 48 * hi], msgs[32 * lo : 32 * hi],
                            (sg if sg is not None else sigs)[96 * lo : 96 * hi], rands[lo:hi])

    recs = [shard(g) for g in range(8)]

    def final(rs):
        ok = ctypes.c_int(7)
        allr = torch.cat(rs)
        native.check(L.tbls_dev_final_verify(0, allr.data_ptr(), len(rs), stream, ctypes.byref(ok)), "final")
        return ok.value

    assert final(recs) == 1
    for g, j in ((0, 17), (7, 7 * SHARD5 + 100000)):
        bad = bytearray(sigs)
        bad[96 * j : 96 * j + 96] = sigs[96 * (j + 1) : 96 * (j + 2)]  # set j carries set j+1's signature
        assert C.verify_each([[pks[48 * j : 48 * j + 48]]], [msgs[32 * j : 32 * j + 32]], [bytes(bad[96 * j : 96 * j + 96])])[0] is False
        rs = list(recs)
        rs[g] = shard(g, bytes(bad))
        assert final(rs) == 0, (g, j)
    assert final(recs) == 1  # the untouched records still verify


def test_config5_1m_one_device_batch(S, cfg5):
    """One tbls_batch_verify of all 1,048,576 sets on one device (offsets, the
    bucket MSM and the chunked line buffers at 1M), valid and one tampered."""
    pks, msgs, sigs = cfg5
    r = S.random_multipliers(N5)
    assert S.SetArray.single(pks, msgs, sigs).batch_verify(r, n_gpus=1) is True
    j = N5 - 5
    bad = bytearray(sigs)
    bad[96 * j : 96 * j + 96] = bytes(96)  # the all-zero signature (BlstSignatureTest.java:54-57)
    assert C.verify_each([[pks[48 * j : 48 * j + 48]]], [msgs[32 * j : 32 * j + 32]], [bytes(96)])[0] is False
    assert S.SetArray.single(pks, msgs, bytes(bad)).batch_verify(r, n_gpus=1) is False


def test_config5_131k_shard(S):
    n = 131072
    pks, msgs, sigs = S.single_signer(0, n, seed=0)
    r = S.random_multipliers(n)
    arr = S.SetArray.single(pks, msgs, sigs)
    assert arr.batch_verify(r) is True
    pk, ms, sg = _split(pks, msgs, sigs)
    assert C.batch_verify(pk, ms, sg, r, threads=THREADS) is True
    # tampered sets in the first, middle and last chunk of the MSM bucket lists
    for j in (3, n // 2 + 1, n - 2):
        for name, (p, m, s) in _tampers(S, pk, ms, sg, j, S.interop_sk(j % 65536)).items():
            got = S.SetArray.single(b"".join(p), b"".join(m), b"".join(s)).batch_verify(r)
            # the oracle's verdict on the tampered set alone decides the batch
            assert C.verify_each([[p[j]]], [m[j]], [s[j]])[0] is False, (name, j)
            assert got is False, (name, j)


def test_multi_key_exceptional_sums(S):
    """Multi-key sets whose aggregation meets P == +-Q (k_set_pk_agg_coop's
    one-lane fallback): a repeated key in one coop row (keys 0 and 16), a key
    beside its negation in one row, keys cancelling to infinity
    (PK_IS_INFINITY -> the set fails), and a repeated key across rows.  Verdicts
    of the randomized batch and of fastAggregateVerify per set vs the C oracle."""
    R = S.R_ORDER
    base = [S.interop_sk(60000 + i) for i in range(40)]
    sets_sk = []
    sets_sk.append(list(base))                                  # plain
    s1 = list(base); s1[16] = s1[0]; sets_sk.append(s1)          # repeated key, same row
    s2 = list(base); s2[17] = R - s2[1]; sets_sk.append(s2)      # key and its negation, same row
    s3 = []
    for k in base[:20]:
        s3 += [k, R - k]
    sets_sk.append(s3)                                          # aggregate = infinity
    s4 = list(base); s4[1] = s4[0]; sets_sk.append(s4)           # repeated key, different rows
    s5 = list(base[:18]); s5[2] = s5[17]; sets_sk.append(s5)     # short set, keys 2 == 17 (rows 2 and 1)
    msgs = [S.bench_message(77, s) for s in range(len(sets_sk))]
    keys = [S.pubkeys(sk) for sk in sets_sk]
    agg = [sum(sk) % R for sk in sets_sk]
    sig = S.sign_blob([a if a else 1 for a in agg], msgs)
    sigs = [sig[96 * s : 96 * s + 96] for s in range(len(sets_sk))]
    sigs[3] = S.INFINITY_G2  # the infinity aggregate's "signature"
    got = S.SetArray.from_lists(keys, msgs, sigs).fast_aggregate_verify_many()
    exp = C.verify_each(keys, msgs, sigs, threads=THREADS)
    assert got == exp == [True, True, True, False, True, True]
    valid = [s for s in range(len(sets_sk)) if s != 3]
    r = S.random_multipliers(len(valid))
    kv, mv, sv = [keys[s] for s in valid], [msgs[s] for s in valid], [sigs[s] for s in valid]
    assert S.SetArray.from_lists(kv, mv, sv).batch_verify(r) is True
    assert S.SetArray.from_lists(keys, msgs, sigs).batch_verify(S.random_multipliers(len(keys))) is False
