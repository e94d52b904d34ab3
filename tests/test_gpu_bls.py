"""GPU parity of the BLS hot path through the C ABI / SPI mirror vs the oracle.

Mirrors the reference's own tests:
  infrastructure/bls/src/test/java/tech/pegasys/teku/bls/BLSTest.java
  infrastructure/bls/src/test/java/tech/pegasys/teku/bls/impl/AbstractBLS12381Test.java
  infrastructure/bls/src/test/java/tech/pegasys/teku/bls/BLSSecretKeyTest.java
and the tampered-set list of SURVEY.md 8(d).
"""

import base64
import ctypes
import random

import pytest

from oracle import bls12_381 as O
from oracle.keys import blstestutil_sk, interop_sk
from tests.test_oracle_kats import (
    KAT_AGGSLOT_SIG,
    KAT_FAV4_MSG,
    KAT_FAV4_PKS,
    KAT_FAV4_SIG,
    KAT_RANDAO_SIG,
    KAT_REAL_PK,
    KAT_REAL_ROOT,
    KAT_REAL_SIG,
    KAT_SK_PK,
    local_signer_roots,
)

pytestmark = pytest.mark.gpu

NOT_IN_G2 = bytes.fromhex("80" + "00" * 94 + "04")
BAD_PK = bytes.fromhex("9378a6e3984e96d2cd50450c76ca14732f1300efa04aecdb805b22e6d6926a85ef409e8f3acf494a1481090bf32ce3bd")
NUL_DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"


@pytest.fixture(scope="module")
def hip():
    import torch  # noqa: F401

    from teku_amd import bls, native

    L = native.lib()
    impl = bls.HipBLS12381()
    bls.BLS.set_bls_implementation(impl)
    return bls, native, L, impl


@pytest.fixture(scope="module")
def sets8():
    sks = [interop_sk(i) for i in range(8)]
    msgs = [bytes([i + 1]) * 32 for i in range(8)]
    pks = [O.sk_to_pk(s) for s in sks]
    sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
    return sks, pks, msgs, sigs


def _raw(bls, pks, msgs, sigs, rands=None, n_gpus=0):
    sets = [(b"".join(p) if isinstance(p, list) else p, len(p) if isinstance(p, list) else 1, m, s) for p, m, s in zip(pks, msgs, sigs)]
    rands = rands or [random.getrandbits(63) | 1 for _ in sets]
    return bls.batch_verify_raw(sets, rands, n_gpus)


def test_batch_valid_and_tampered(hip, sets8):
    bls = hip[0]
    sks, pks, msgs, sigs = sets8
    assert _raw(bls, pks, msgs, sigs) is True
    assert O.batch_verify([[p] for p in pks], msgs, sigs) is True
    cases = {}
    s2 = list(sigs)
    s2[3] = O.sign(sks[3], bytes([msgs[3][0] ^ 1]) + msgs[3][1:])
    cases["sig on m^1"] = (pks, msgs, s2)
    m2 = list(msgs)
    m2[1], m2[2] = m2[2], m2[1]
    cases["swapped msgs"] = (pks, m2, sigs)
    for name, bad in [("zero sig", bytes(96)), ("inf sig", O.INFINITY_G2), ("non-G2 sig", NOT_IN_G2)]:
        s3 = list(sigs)
        s3[5] = bad
        cases[name] = (pks, msgs, s3)
    for name, bad in [("inf pk", O.INFINITY_G1), ("0x9378 pk", BAD_PK), ("zero pk", bytes(48))]:
        p3 = list(pks)
        p3[6] = bad
        cases[name] = (p3, msgs, sigs)
    for name, (p, m, s) in cases.items():
        got = _raw(bls, p, m, s)
        exp = O.batch_verify([[x] for x in p], m, s)
        assert got == exp is False, name


def test_batch_multikey_sets(hip):
    """fastAggregateVerify-style sets (configs 2/3 shape, scaled down)."""
    bls = hip[0]
    pks_l, msgs, sigs = [], [], []
    for j in range(4):
        sks = [interop_sk(10 * j + i) for i in range(5)]
        m = bytes([0xA0 + j]) * 32
        pks_l.append([O.sk_to_pk(s) for s in sks])
        msgs.append(m)
        sigs.append(O.aggregate_sigs([O.sign(s, m) for s in sks]))
    assert _raw(bls, pks_l, msgs, sigs) is True
    pks_l[2] = pks_l[2][:-1]
    assert _raw(bls, pks_l, msgs, sigs) is False


def test_simulated_shards_equal_single_device(hip, sets8):
    """G logical shards on one GPU -> gather of partial records -> one final exp."""
    import torch

    bls, native, L, _ = hip
    sks, pks, msgs, sigs = sets8
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def shard(lo, hi):
        n = hi - lo
        u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731
        t = dict(
            pks=u8(b"".join(pks[lo:hi])),
            msgs=u8(b"".join(msgs[lo:hi])),
            sigs=u8(b"".join(sigs[lo:hi])),
            pk_off=torch.arange(0, n + 1, dtype=torch.int32, device=dev),
            msg_off=torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=dev),
            rand=torch.randint(1, 1 << 62, (n,), dtype=torch.int64, device=dev),
        )
        d = native.TblsDevBatch(
            t["pks"].data_ptr(), t["pk_off"].data_ptr(), n, t["msgs"].data_ptr(), t["msg_off"].data_ptr(), t["sigs"].data_ptr(), t["rand"].data_ptr(), n
        )
        out = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=dev)
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(d), stream, out.data_ptr()), "partial")
        torch.cuda.synchronize()
        return out

    for G in (1, 2, 4):
        cuts = [len(pks) * g // G for g in range(G + 1)]
        recs = torch.cat([shard(cuts[g], cuts[g + 1]) for g in range(G)])
        ok = ctypes.c_int(0)
        native.check(L.tbls_dev_final_verify(0, recs.data_ptr(), G, stream, ctypes.byref(ok)), "final")
        assert ok.value == 1, G
    # one bad shard poisons the gathered result
    sigs_bad = list(sigs)
    sigs_bad[7] = sigs[6]
    pks_bak = pks
    recs = torch.cat([shard(0, 4)])
    sigs[:] = sigs_bad
    recs = torch.cat([recs, shard(4, 8)])
    sigs[:] = [O.sign(s, m) for s, m in zip(sks, msgs)]
    ok = ctypes.c_int(1)
    native.check(L.tbls_dev_final_verify(0, recs.data_ptr(), 2, stream, ctypes.byref(ok)), "final")
    assert ok.value == 0
    assert pks_bak is pks
    # the asynchronous form (pipelined services): verdicts in device memory,
    # the same as the synchronous call's, on a second stream
    s2 = torch.cuda.Stream(dev)
    good = torch.cat([shard(0, 4), shard(4, 8)])
    oks = torch.full((2,), 7, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    native.check(L.tbls_dev_final_verify_async(0, good.data_ptr(), 2, s2.cuda_stream, oks[0:1].data_ptr()), "final_async")
    native.check(L.tbls_dev_final_verify_async(0, recs.data_ptr(), 2, s2.cuda_stream, oks[1:2].data_ptr()), "final_async")
    torch.cuda.synchronize()
    assert oks.tolist() == [1, 0]


def test_async_final_pipelined_two_streams(hip):
    """The shape that rejected a valid batch in round 2 (bench_r02ab): batch k's
    tbls_dev_final_verify_async on stream B runs beside batch k+1's
    tbls_dev_batch_partial on stream A, with double-buffered records; valid
    and tampered batches alternate.  Also two finals on two streams at once
    (the library keeps no scratch for them).  Verdicts must alternate 1, 0."""
    import torch

    from teku_amd import synth

    bls, native, L, _ = hip
    dev = torch.device("cuda", 0)
    n = 96
    pks, msgs, sigs = synth.single_signer(3000, n, seed=31)
    bad_sigs = bytearray(sigs)
    bad_sigs[96 * 40 : 96 * 41] = sigs[96 * 41 : 96 * 42]  # set 40 carries set 41's signature
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731

    def batch(sg):
        t = dict(pks=u8(pks), msgs=u8(msgs), sigs=u8(sg), pk_off=torch.arange(0, n + 1, dtype=torch.int32, device=dev),
                 msg_off=torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=dev),
                 rand=torch.randint(1, 1 << 62, (n,), dtype=torch.int64, device=dev))
        t["desc"] = native.TblsDevBatch(t["pks"].data_ptr(), t["pk_off"].data_ptr(), n, t["msgs"].data_ptr(), t["msg_off"].data_ptr(),
                                        t["sigs"].data_ptr(), t["rand"].data_ptr(), n)
        return t

    batches = [batch(sigs), batch(bytes(bad_sigs))]
    K = 8
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    recs = [torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=dev) for _ in range(2)]
    oks = torch.full((K,), 7, dtype=torch.int32, device=dev)
    done = [torch.cuda.Event() for _ in range(K)]
    torch.cuda.synchronize()
    for k in range(K):
        slot = k % 2
        if k >= 2:  # the record slot is free once batch k-2's final has run
            sa.wait_event(done[k - 2])
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(batches[k % 2]["desc"]), sa.cuda_stream, recs[slot].data_ptr()), "partial")
        ready = torch.cuda.Event()
        ready.record(sa)
        sb.wait_event(ready)
        native.check(L.tbls_dev_final_verify_async(0, recs[slot].data_ptr(), 1, sb.cuda_stream, oks[k : k + 1].data_ptr()), "final_async")
        done[k].record(sb)
    torch.cuda.synchronize()
    assert oks.tolist() == [1, 0] * (K // 2)
    # two finals at once on two streams, over the two (now stable) records
    oks2 = torch.full((2,), 7, dtype=torch.int32, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for _ in range(3):
        native.check(L.tbls_dev_final_verify_async(0, recs[0].data_ptr(), 1, s1.cuda_stream, oks2[0:1].data_ptr()), "final_async")
        native.check(L.tbls_dev_final_verify_async(0, recs[1].data_ptr(), 1, s2.cuda_stream, oks2[1:2].data_ptr()), "final_async")
    torch.cuda.synchronize()
    assert oks2.tolist() == [1, 0]


def test_partials_alternating_streams(hip):
    """Device-resident partials alternating two streams with no host wait
    between them, each followed on its own stream by
    tbls_dev_final_verify_async (the shape of a service with two batches
    queued on a device; the shared workspace orders them by its last-use
    event).  Valid and tampered batches alternate at a bucket-sum size (split
    Miller loop, LDS accumulator) and a small one (coop kernels), so the
    workspace is re-carved between sizes.  (Two workspace slots with batch
    k+1's per-set stages under batch k's final exponentiation measured slower,
    profiles/r06_ab_inflight.json.)"""
    import torch

    from teku_amd import synth

    bls, native, L, _ = hip
    dev = torch.device("cuda", 0)
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731

    def batch(n, seed, tamper):
        pks, msgs, sigs = synth.single_signer(5000, n, seed=seed)
        if tamper:
            sigs = bytearray(sigs)
            i = n // 2
            sigs[96 * i : 96 * (i + 1)], sigs[96 * (i + 1) : 96 * (i + 2)] = sigs[96 * (i + 1) : 96 * (i + 2)], sigs[96 * i : 96 * (i + 1)]
        t = dict(pks=u8(pks), msgs=u8(msgs), sigs=u8(bytes(sigs)), pk_off=torch.arange(0, n + 1, dtype=torch.int32, device=dev),
                 msg_off=torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=dev),
                 rand=torch.randint(1, 1 << 62, (n,), dtype=torch.int64, device=dev))
        t["desc"] = native.TblsDevBatch(t["pks"].data_ptr(), t["pk_off"].data_ptr(), n, t["msgs"].data_ptr(), t["msg_off"].data_ptr(),
                                        t["sigs"].data_ptr(), t["rand"].data_ptr(), n)
        return t

    big = [batch(40960, 7, False), batch(40960, 8, True)]
    small = [batch(96, 9, False), batch(96, 10, True)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    recs = [torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=dev) for _ in range(2)]
    # the expected verdicts: 1 for the valid batches, 0 for the tampered ones
    plan = [big[0], big[1], big[0], big[1], small[0], big[1], small[1], big[0], big[0], small[1]]
    want = [1, 0, 1, 0, 1, 0, 0, 1, 1, 0]
    oks = torch.full((len(plan),), 7, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for k, b in enumerate(plan):
        st = streams[k % 2]
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(b["desc"]), st.cuda_stream, recs[k % 2].data_ptr()), "partial")
        native.check(L.tbls_dev_final_verify_async(0, recs[k % 2].data_ptr(), 1, st.cuda_stream, oks[k : k + 1].data_ptr()), "final_async")
    torch.cuda.synchronize()
    assert oks.tolist() == want
    # and back to one stream: the same slot each time, same verdicts
    for k, b in enumerate(plan[:4]):
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(b["desc"]), streams[0].cuda_stream, recs[0].data_ptr()), "partial")
        native.check(L.tbls_dev_final_verify_async(0, recs[0].data_ptr(), 1, streams[0].cuda_stream, oks[k : k + 1].data_ptr()), "final_async")
    torch.cuda.synchronize()
    assert oks[:4].tolist() == want[:4]


def test_hash_sign_keys_bit_exact(hip):
    bls, native, L, _ = hip
    for msg, dst in [(b"", O.ETH2_DST), (b"abc", O.ETH2_DST), (b"\x42" * 32, O.ETH2_DST), (b"abc", NUL_DST), (bytes(range(200)), O.ETH2_DST)]:
        out = ctypes.create_string_buffer(96)
        native.check(L.tbls_hash_to_g2(msg, len(msg), dst, len(dst), out), "h2g")
        assert out.raw == O.g2_compress(O.hash_to_g2(msg, dst))
    for sk, pk in KAT_SK_PK:
        out = ctypes.create_string_buffer(48)
        native.check(L.tbls_sk_to_pk(sk.to_bytes(32, "big"), out), "sk2pk")
        assert out.raw.hex() == pk
    sk = blstestutil_sk(1234)
    randao, aggslot = local_signer_roots()
    for root, exp in [(randao, KAT_RANDAO_SIG), (aggslot, KAT_AGGSLOT_SIG)]:
        out = ctypes.create_string_buffer(96)
        native.check(L.tbls_sign(sk.to_bytes(32, "big"), root, 32, O.ETH2_DST, len(O.ETH2_DST), out), "sign")
        assert out.raw == base64.b64decode(exp)
    assert L.tbls_sign(bytes(32), b"x", 1, O.ETH2_DST, len(O.ETH2_DST), ctypes.create_string_buffer(96)) == native.BAD_SCALAR


def test_aggregation_bit_exact(hip):
    bls, native, L, impl = hip
    sks = [interop_sk(i) for i in range(7)]
    pks = [O.sk_to_pk(s) for s in sks]
    sigs = [O.sign(s, b"agg") for s in sks]
    assert impl.aggregate_public_keys([bls.HipPublicKey(p) for p in pks]).to_bytes_compressed() == O.aggregate_pks(pks)
    assert impl.aggregate_signatures([bls.HipSignature(s) for s in sigs]).to_bytes_compressed() == O.aggregate_sigs(sigs)
    # any invalid key -> infinity (BlstPublicKey.java:58-65)
    assert impl.aggregate_public_keys([bls.HipPublicKey(p) for p in pks[:3] + [BAD_PK]]).to_bytes_compressed() == O.INFINITY_G1
    # P + (-P) -> infinity; empty signature list -> infinity
    assert impl.aggregate_signatures([]).to_bytes_compressed() == O.INFINITY_G2
    with pytest.raises(bls.BlsException):
        impl.aggregate_signatures([bls.HipSignature(sigs[0]), bls.HipSignature(NOT_IN_G2)])


# ---- BLSTest.java mirrors (through the facade) -------------------------------
def test_blstest_sign_verify(hip):
    bls = hip[0]
    B = bls.BLS
    kp = bls.BLSKeyPair(bls.BLSSecretKey.from_bytes_mod_r(blstestutil_sk(42).to_bytes(32, "big")))
    msg = b"Hello, world!"
    sig = B.sign(kp.secret_key, msg)
    assert B.verify(kp.public_key, msg, sig)
    assert not B.verify(kp.public_key, msg, bls.BLSSignature.empty())  # l.43-51
    # DST variants (l.375-391)
    s2 = B.sign(kp.secret_key, msg, NUL_DST)
    assert B.verify(kp.public_key, msg, s2, NUL_DST)
    assert not B.verify(kp.public_key, msg, s2)


def test_blstest_kats(hip):
    bls = hip[0]
    B = bls.BLS
    pks = [bls.BLSPublicKey.from_bytes_compressed_validate(p) for p in KAT_FAV4_PKS]
    assert B.fast_aggregate_verify(pks, KAT_FAV4_MSG, bls.BLSSignature.from_bytes_compressed(KAT_FAV4_SIG))  # l.106-126
    assert B.verify(bls.BLSPublicKey(KAT_REAL_PK), KAT_REAL_ROOT, bls.BLSSignature(KAT_REAL_SIG))  # l.359-373


def test_blstest_invalid_key_batches(hip):
    """anyVerify_invalidPublicKeyShouldNotThrowAndReturnFalse (l.128-167)."""
    bls = hip[0]
    B = bls.BLS
    kp = bls.BLSKeyPair(bls.BLSSecretKey.from_bytes_mod_r(blstestutil_sk(1).to_bytes(32, "big")))
    msg = KAT_FAV4_MSG
    invalid = bls.BLSPublicKey.from_bytes_compressed(bytes(48))
    valid = bls.BLSPublicKey.from_bytes_compressed(kp.public_key.to_bytes_compressed())
    sig = B.sign(kp.secret_key, msg)
    assert not B.verify(invalid, msg, sig)
    assert not B.aggregate_verify([invalid], [msg], sig)
    assert not B.aggregate_verify([valid, invalid], [msg, msg], sig)
    assert not B.fast_aggregate_verify([invalid], msg, sig)
    assert not B.fast_aggregate_verify([valid, valid, invalid], msg, sig)
    assert not B.batch_verify([[valid], [invalid]], [msg, msg], [sig, sig])
    many = [[valid]] * 63 + [[invalid]]
    assert not B.batch_verify(many, [msg] * 64, [sig] * 64)
    assert B.batch_verify([[valid]] * 64, [msg] * 64, [sig] * 64)


def test_blstest_infinity_and_aggregate(hip):
    bls = hip[0]
    B = bls.BLS
    inf_pk = bls.BLSPublicKey.from_bytes_compressed(O.INFINITY_G1)
    inf_sig = bls.BLSSignature.from_bytes_compressed(O.INFINITY_G2)
    assert not B.verify(inf_pk, b"Hello, world!", inf_sig)  # l.262-266
    zero = bls.BLSSecretKey.from_bytes(bytes(32))
    assert zero.to_public_key().to_bytes_compressed() == O.INFINITY_G1  # l.268-271
    with pytest.raises(ValueError):
        B.sign(zero, b"Hello, world!")  # l.273-277
    kp1 = bls.BLSKeyPair(bls.BLSSecretKey.from_bytes_mod_r(blstestutil_sk(1).to_bytes(32, "big")))
    sig1 = B.sign(kp1.secret_key, b"Hello, world!")
    agg_pk = bls.BLSPublicKey.aggregate([kp1.public_key, zero.to_public_key()])
    agg_sig = B.aggregate([sig1, inf_sig])
    assert not B.verify(agg_pk, b"Hello, world!", agg_sig)  # l.279-292
    with pytest.raises(ValueError):
        B.aggregate([bls.BLSSignature(NOT_IN_G2)])  # l.294-297
    with pytest.raises(ValueError):
        B.aggregate([])  # l.212-216
    with pytest.raises(ValueError):
        B.aggregate([sig1, bls.BLSSignature.empty(), sig1])  # l.76-85
    assert B.aggregate([sig1]) == sig1  # l.69-73
    # prepare(inf pk, inf sig) x2 -> complete false (l.299-312); valid + inf (l.342-357)
    a = B.prepare_batch_verify(0, [zero.to_public_key()], b"Hello, world!", inf_sig)
    b = B.prepare_batch_verify(1, [zero.to_public_key()], b"Hello, world!", inf_sig)
    assert not B.complete_batch_verify([a, b])
    c = B.prepare_batch_verify(0, [kp1.public_key], b"Hello, world!", sig1)
    assert not B.complete_batch_verify([c, b])
    assert B.complete_batch_verify([c])
    assert not B.fast_aggregate_verify([], b"", bls.BLSSignature.empty())  # l.218-228
    assert not B.aggregate_verify([], [], bls.BLSSignature.empty())


def test_blstest_odd_double_pairing(hip):
    """batchVerifyWithPairingOddNumberOfVerifications (l.314-340)."""
    bls = hip[0]
    B = bls.BLS
    kp = bls.BLSKeyPair(bls.BLSSecretKey.from_bytes_mod_r(blstestutil_sk(1).to_bytes(32, "big")))
    m = [b"Hello, 1!", b"Hello, 2!", b"Hello, 3!"]
    s = [B.sign(kp.secret_key, x) for x in m]
    bad = B.sign(kp.secret_key, m[1])
    pks = [[kp.public_key]] * 3
    assert not B.batch_verify(pks, m, [s[0], s[1], bad], True, False)
    assert B.batch_verify(pks, m, s, True, False)


def test_aggregate_verify_distinct(hip):
    """succeedsWhenAggregateVerifyWithDistinctMessagesReturnsTrue (l.170-189) and the infinite-pair case (l.191-210)."""
    bls = hip[0]
    B = bls.BLS
    kps = [bls.BLSKeyPair(bls.BLSSecretKey.from_bytes_mod_r(blstestutil_sk(i).to_bytes(32, "big"))) for i in (1, 2, 3)]
    msgs = [b"Hello, world 1!", b"Hello, world 2!", b"Hello, world 3!"]
    sigs = [B.sign(k.secret_key, m) for k, m in zip(kps, msgs)]
    agg = B.aggregate(sigs)
    assert B.aggregate_verify([k.public_key for k in kps], msgs, agg)
    inf = bls.BLSPublicKey.from_bytes_compressed(O.INFINITY_G1)
    agg2 = B.aggregate(sigs[:2] + [bls.BLSSignature.infinity()])
    assert not B.aggregate_verify([kps[0].public_key, kps[1].public_key, inf], msgs, agg2)


def test_spi_prepare_complete_combinatorics(hip):
    """AbstractBLS12381Test.java:189-229: n = 0..7 positive; one invalid at each position."""
    bls, native, L, impl = hip
    sks = [interop_sk(100 + i) for i in range(7)]
    pks = [bls.HipPublicKey(O.sk_to_pk(s)) for s in sks]
    msgs = [bytes([i]) * 32 for i in range(7)]
    sigs = [bls.HipSignature(O.sign(s, m)) for s, m in zip(sks, msgs)]
    for n in range(0, 8):
        prep = [impl.prepare_batch_verify(i, [pks[i]], msgs[i], sigs[i]) for i in range(n)]
        assert impl.complete_batch_verify(prep) is True
    for bad in range(6):
        prep = [impl.prepare_batch_verify(i, [pks[i]], msgs[i], sigs[(i + 1) % 6 if i == bad else i]) for i in range(6)]
        assert impl.complete_batch_verify(prep) is False
    assert impl.complete_batch_verify([object()]) is False  # ClassCastException path (BlstBLS12381.java:185-188)
    eager = bls.HipBLS12381(eager=True)
    with pytest.raises(ValueError):  # BlstTest.succeedsWhenPrepareBatchVerifyNotInG2ThrowsException
        eager.prepare_batch_verify(0, [pks[0]], msgs[0], bls.HipSignature(NOT_IN_G2))


@pytest.mark.parametrize("n", [20480, 24576, 32768])
def test_large_batch_msm_path(hip, n):
    """Batches of >= 20,480 sets take the bucket-MSM path for sum r_i sig_i
    (k_sig_check + k_msm_*) instead of per-set [r_i] sig_i, and from 32,768
    sets the two-wave per-set kernels (k_set_pk_w2: [r] pk with the window
    table in LDS); 20,480 and 24,576 are the bucket-sum sizes below the
    two-wave kernels: valid -> True; a signature on the wrong message, an
    infinity signature, a non-G2 point, another signer's key and the
    infinity key -> False; a duplicated signature pair (bucket doubling
    case) -> True.
    Keys / signatures come from the GPU generators (interop keys), which
    test_hash_sign_keys_bit_exact pins to the oracle."""
    bls, native, L, impl = hip
    nk = 512
    sks = b"".join(interop_sk(i % nk).to_bytes(32, "big") for i in range(n))
    pk_out = ctypes.create_string_buffer(48 * nk)
    native.check(L.tbls_sk_to_pk_many(sks[: 32 * nk], nk, pk_out), "sk_to_pk_many")
    msgs = [i.to_bytes(4, "little") * 8 for i in range(n)]
    off = (ctypes.c_uint32 * (n + 1))(*[32 * j for j in range(n + 1)])
    sig_out = ctypes.create_string_buffer(96 * n)
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    native.check(L.tbls_sign_many(sks, b"".join(msgs), off, n, dst, len(dst), sig_out), "sign_many")
    pks = [pk_out.raw[48 * (i % nk) : 48 * (i % nk) + 48] for i in range(n)]
    sigs = [sig_out.raw[96 * i : 96 * i + 96] for i in range(n)]
    rng = random.Random(7)
    rands = [rng.getrandbits(64) | 1 for _ in range(n)]
    assert _raw(bls, pks, msgs, sigs, rands)
    bad = list(sigs)
    bad[12345] = sigs[12346]
    assert not _raw(bls, pks, msgs, bad, rands)
    bad = list(sigs)
    bad[777] = bytes([0xC0]) + bytes(95)
    assert not _raw(bls, pks, msgs, bad, rands)
    bad = list(sigs)
    bad[5] = NOT_IN_G2
    assert not _raw(bls, pks, msgs, bad, rands)
    bad = list(pks)
    bad[3] = pks[4]
    assert not _raw(bls, bad, msgs, sigs, rands)
    bad = list(pks)
    bad[n * 11 // 12] = bytes([0xC0]) + bytes(47)
    assert not _raw(bls, bad, msgs, sigs, rands)
    # the same (pk, msg, sig) twice with the same randomizer: equal points in one bucket
    dup_p, dup_m, dup_s, dup_r = list(pks), list(msgs), list(sigs), list(rands)
    dup_p[1], dup_m[1], dup_s[1], dup_r[1] = pks[0], msgs[0], sigs[0], rands[0]
    assert _raw(bls, dup_p, dup_m, dup_s, dup_r)


@pytest.mark.parametrize("n", [24576, 32768])
def test_key_table_bucket_sum_batches(hip, n):
    """Key-table batches large enough for the bucket-sum signature side: the
    library starts their hash after the signature checks (tb_lib.hip
    sig_first, keys from the table) instead of beside them.  Verdicts equal
    the same batches by key bytes (test_large_batch_msm_path's order) for a
    valid batch, a swapped signature, a non-G2 signature and a wrong key
    index."""
    bls, native, L, impl = hip
    nk = 512
    sks = b"".join(interop_sk(i % nk).to_bytes(32, "big") for i in range(n))
    pk_out = ctypes.create_string_buffer(48 * nk)
    native.check(L.tbls_sk_to_pk_many(sks[: 32 * nk], nk, pk_out), "sk_to_pk_many")
    msgs = [i.to_bytes(4, "little") * 8 for i in range(n)]
    off = (ctypes.c_uint32 * (n + 1))(*[32 * j for j in range(n + 1)])
    sig_out = ctypes.create_string_buffer(96 * n)
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    native.check(L.tbls_sign_many(sks, b"".join(msgs), off, n, dst, len(dst), sig_out), "sign_many")
    keys = [pk_out.raw[48 * k : 48 * k + 48] for k in range(nk)]
    sigs = [sig_out.raw[96 * i : 96 * i + 96] for i in range(n)]
    table = bls.ValidatorKeyTable(keys)
    assert table.codes == [0] * nk
    rng = random.Random(11)
    rands = [rng.getrandbits(64) | 1 for _ in range(n)]
    sets = [([i % nk], msgs[i], sigs[i]) for i in range(n)]

    def both(batch):
        by_idx = table.batch_verify(batch, rands)
        by_bytes = _raw(bls, [keys[ks[0]] for ks, _, _ in batch], [m for _, m, _ in batch], [sg for _, _, sg in batch], rands)
        assert by_idx is by_bytes
        return by_idx

    assert both(sets) is True
    bad = list(sets)
    bad[12345] = (bad[12345][0], msgs[12345], sigs[12346])
    assert both(bad) is False
    bad = list(sets)
    bad[5] = (bad[5][0], msgs[5], NOT_IN_G2)
    assert both(bad) is False
    bad = list(sets)
    bad[n - 7] = ([(n - 6) % nk], msgs[n - 7], sigs[n - 7])
    assert both(bad) is False


def test_validator_key_table(hip, sets8):
    """Device-resident key table (tbls_pk_table_load / tbls_batch_verify_idx,
    SURVEY.md 8(f) rank 1): per-key codes as tbls_pk_validate; batches by key
    index give the same booleans as the same batches by key bytes, including
    multi-key sets, an invalid table key (infinity / 0x9378a6... / not on the
    curve) and a tampered signature; out-of-range index -> ValueError."""
    bls, native, L, impl = hip
    sks, pks, msgs, sigs = sets8
    pkb = list(pks)  # compressed 48-byte keys
    inf_pk = bytes([0xC0]) + bytes(47)
    table = bls.ValidatorKeyTable(pkb + [inf_pk, BAD_PK])
    assert table.size == 10 and L.tbls_pk_table_size() == 10
    assert table.codes[:8] == [0] * 8
    assert table.codes[8] == native.PK_IS_INFINITY and table.codes[9] != 0
    tab_keys = pkb + [inf_pk, BAD_PK]

    def oracle(batch):  # the pinned oracle on the same sets, keys by bytes
        return O.batch_verify([[tab_keys[k] for k in ks] for ks, _, _ in batch], [m_ for _, m_, _ in batch], [s_ for _, _, s_ in batch])

    sets = [([i], msgs[i], sigs[i]) for i in range(8)]
    rands = [random.getrandbits(64) | 1 for _ in sets]
    assert table.batch_verify(sets, rands) is oracle(sets) is True
    assert _raw(bls, pkb, msgs, sigs, rands)
    bad = list(sets)
    bad[3] = ([3], msgs[3], sigs[4])
    assert table.batch_verify(bad, rands) is oracle(bad) is False
    for k in (8, 9):
        bad = list(sets)
        bad[2] = ([2, k], msgs[2], sigs[2])
        assert table.batch_verify(bad, rands) is oracle(bad) is False
    # one set signed by keys 0..3 on one message (fastAggregateVerify shape)
    m = b"\x42" * 32
    agg = O.aggregate_sigs([O.sign(sks[i], m) for i in range(4)])
    good4 = sets + [([0, 1, 2, 3], m, agg)]
    bad4 = sets + [([0, 1, 2, 5], m, agg)]
    assert table.batch_verify(good4, rands + [12345]) is oracle(good4) is True
    assert table.batch_verify(bad4, rands + [12345]) is oracle(bad4) is False
    with pytest.raises(ValueError):
        table.batch_verify([([10], msgs[0], sigs[0])], [1])


def test_verify_each_and_service(hip, sets8):
    """Per-set verdicts in one device pass (tbls_verify_each, SURVEY.md 8(f)
    rank 2) equal the oracle's fastAggregateVerify per set on a mix of valid
    and tampered sets (wrong message, swapped signature, zero / infinity /
    non-G2 signature, infinity / invalid / zero key, empty key list,
    multi-key set); tbls_fast_aggregate_verify_many agrees; the service
    settles a failed batch with one per-set pass."""
    from teku_amd.service import AggregatingSignatureVerificationService

    bls, native, L, impl = hip
    sks, pks, msgs, sigs = sets8
    m = b"\x42" * 32
    agg = O.aggregate_sigs([O.sign(sks[i], m) for i in range(3)])
    sets, exp = [], []
    for i in range(8):
        sets.append((pks[i], 1, msgs[i], sigs[i]))
        exp.append(True)
    sets += [
        (pks[0], 1, msgs[1], sigs[0]),
        (pks[1], 1, msgs[1], sigs[2]),
        (pks[2], 1, msgs[2], bytes(96)),
        (pks[3], 1, msgs[3], O.INFINITY_G2),
        (pks[4], 1, msgs[4], NOT_IN_G2),
        (O.INFINITY_G1, 1, msgs[5], sigs[5]),
        (BAD_PK, 1, msgs[6], sigs[6]),
        (bytes(48), 1, msgs[7], sigs[7]),
        (b"", 0, msgs[0], sigs[0]),
        (b"".join(pks[:3]), 3, m, agg),
        (b"".join(pks[:2]), 2, m, agg),
        (O.INFINITY_G1, 1, msgs[0], O.INFINITY_G2),
    ]
    exp += [False] * 9 + [True, False, False]
    # oracle per set (non-empty key lists): BLS.batchVerify of (s, s) == fastAggregateVerify(s)
    for (blob, npk, msg, sig), e in zip(sets, exp):
        if npk == 0:
            continue
        keys = [blob[48 * j : 48 * j + 48] for j in range(npk)]
        assert O.batch_verify([keys, keys], [msg, msg], [sig, sig]) == e
    got = bls.verify_each_raw(sets)
    assert got == exp
    arr = (native.TblsSet * len(sets))()
    keep = []
    for i, (blob, npk, msg, sig) in enumerate(sets):
        bb, mb, sb = (ctypes.create_string_buffer(bytes(x), max(1, len(x))) for x in (blob, msg, sig))
        keep += [bb, mb, sb]
        arr[i].pks = ctypes.cast(bb, ctypes.c_void_p)
        arr[i].n_pks = npk
        arr[i].msg = ctypes.cast(mb, ctypes.c_void_p)
        arr[i].msg_len = len(msg)
        arr[i].sig = ctypes.cast(sb, ctypes.c_void_p)
    ok = (ctypes.c_int * len(sets))()
    native.check(L.tbls_fast_aggregate_verify_many(arr, len(sets), ok), "fav_many")
    assert [v == 1 for v in ok] == exp
    # the service on the device backend: one call (batch, settled per set in place)
    svc = AggregatingSignatureVerificationService(max_batch_size=64)
    from teku_amd.service import SignatureTask

    tasks = [SignatureTask([s]) for s in sets if s[1] > 0]
    svc.batch_verify_signatures(tasks)
    assert [t.result.result() for t in tasks] == [e for s, e in zip(sets, exp) if s[1] > 0]
    assert svc.device_passes == 1 and svc.last_batch_timing["settled"]


def test_batched_deserialization_and_aggregation(hip, sets8):
    """Batched key / signature validation and grouped signature aggregation
     equal the one-at-a-time C ABI calls item by item
    and the oracle's aggregate bytes: valid keys / sigs, infinity, zero bytes,
    0x9378a6... key, non-G2 signature, an empty group (-> infinity) and a
    group holding a non-G2 signature (-> BlsException)."""
    bls, native, L, impl = hip
    sks, pks, msgs, sigs = sets8
    keys = list(pks) + [O.INFINITY_G1, BAD_PK, bytes(48), bytes([0x80]) + bytes(47)]
    codes = bls.validate_public_keys(keys)
    assert codes == [L.tbls_pk_validate(k) for k in keys]
    assert codes[:8] == [0] * 8 and all(c != 0 for c in codes[8:])
    ss = list(sigs) + [O.INFINITY_G2, bytes(96), NOT_IN_G2]
    codes, infs = bls.validate_signatures(ss)
    for s, c, f in zip(ss, codes, infs):
        inf = ctypes.c_int(0)
        assert c == L.tbls_sig_validate(s, ctypes.byref(inf)) and f == bool(inf.value)
    assert codes[:9] == [0] * 9 and infs[8] and codes[9] != 0 and codes[10] != 0
    groups = [sigs[:3], sigs[3:4], [], sigs[4:8] + [O.INFINITY_G2], [sigs[0], NOT_IN_G2], list(sigs)]
    got = bls.aggregate_signature_groups(groups)
    for g, r in zip(groups, got):
        if NOT_IN_G2 in g:
            assert isinstance(r, bls.BlsException)
            continue
        assert r == (O.aggregate_sigs(g) if g else O.INFINITY_G2)
        one = ctypes.create_string_buffer(96)
        if g:
            native.check(L.tbls_aggregate_sigs(b"".join(g), len(g), one), "aggregate_sigs")
            assert one.raw == r


def test_concurrent_callers_threads(hip, sets8):
    """Service workers call batchVerify side by side (the reference's numThreads
    workers, AggregatingSignatureVerificationService.java:121-132, 202-205):
    each batch is placed on the least-loaded device and holds only that
    device's lock, and every caller gets its own verdict (valid and tampered
    batches interleaved from 4 threads)."""
    import threading

    bls = hip[0]
    sks, pks, msgs, sigs = sets8
    bad = list(sigs)
    bad[6] = O.sign(sks[6], msgs[5])
    results, errors = {}, []

    def worker(w):
        try:
            for k in range(6):
                tampered = (w + k) % 2 == 1
                results[(w, k)] = (_raw(bls, pks, msgs, bad if tampered else sigs), not tampered)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(w,)) for w in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    assert len(results) == 24
    for key, (got, want) in results.items():
        assert got is want, key
