"""Config 4 through the SPI facade with FRESH objects:
16,384 gossip attestations arrive as new BLSPublicKey / BLSSignature wrappers
(bls/BLSSignature.java:83-87 decodes lazily, once per object), go through
BLS.batchVerify (BLS.java:230-336) on HipBLS12381, and must cost exactly one
device batch and no single-object device call.  The facade's batch path
hands the bytes to the device, which decodes and group-checks every point
inside the batch; objects decoded one by one (the Java facade's
getSignature() per set) are decoded on the host (tbls_*_decode,
blst_p1/p2_uncompress's contract), never on the device.  Verdicts are the C
oracle's."""

import pytest

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

N = 16384
THREADS = 16


@pytest.fixture(scope="module")
def env():
    import torch  # noqa: F401

    from teku_amd import bls, native, synth

    native.lib()
    bls.BLS.set_bls_implementation(bls.HipBLS12381())
    pks, msgs, sigs = synth.single_signer(0, N, seed=4)
    pk = [pks[48 * i : 48 * i + 48] for i in range(N)]
    ms = [msgs[32 * i : 32 * i + 32] for i in range(N)]
    sg = [sigs[96 * i : 96 * i + 96] for i in range(N)]
    return bls, native, synth, pk, ms, sg


def fresh(bls, pk, sg):
    return [[bls.BLSPublicKey.from_bytes_compressed(p)] for p in pk], [bls.BLSSignature.from_bytes_compressed(s) for s in sg]


def test_fresh_objects_one_device_batch(env):
    bls, native, synth, pk, ms, sg = env
    keys, sigs = fresh(bls, pk, sg)
    native.stats(reset=True)
    assert bls.BLS.batch_verify(keys, ms, sigs) is True
    st = native.stats()
    assert st["partials"] == 1 and st["finals"] == 1, st
    assert st["one_validate"] == 0 and st["helpers"] == 0 and st["each_passes"] == 0, st
    assert st["host_decodes"] == 0, st  # the device decodes inside the batch


def test_fresh_objects_per_object_decode_like_java(env):
    """The Java facade decodes each object through getSignature() /
    getPublicKey() (one JNI host decode each): still no device call until the
    batch."""
    bls, native, synth, pk, ms, sg = env
    keys, sigs = fresh(bls, pk[:2048], sg[:2048])
    native.stats(reset=True)
    for k, s in zip(keys, sigs):
        k[0].get_public_key()
        s.get_signature()
    st = native.stats()
    assert st["host_decodes"] == 2 * 2048 and st["partials"] == 0 and st["one_validate"] == 0, st
    assert bls.BLS.batch_verify(keys, ms[:2048], sigs) is True
    st = native.stats()
    assert st["partials"] == 1 and st["one_validate"] == 0 and st["host_decodes"] == 2 * 2048, st


@pytest.mark.parametrize("kind", ["swapped", "not_in_g2", "bad_encoding", "off_curve", "wrong_key"])
def test_fresh_objects_tampered(env, kind):
    bls, native, synth, pk, ms, sg = env
    pk2, sg2 = list(pk), list(sg)
    j = {"swapped": 11, "not_in_g2": 9999, "bad_encoding": 5000, "off_curve": 7, "wrong_key": 16383}[kind]
    if kind == "swapped":
        sg2[j] = sg[j + 1]
    elif kind == "not_in_g2":
        sg2[j] = synth.NOT_IN_G2
    elif kind == "bad_encoding":
        sg2[j] = bytes(96)
    elif kind == "off_curve":
        sg2[j] = bytes([0xA0]) + bytes(95)  # x = 0 with the sign flag: 4(1 + u) has no root
    else:
        pk2[j] = pk[0]
    keys, sigs = fresh(bls, pk2, sg2)
    native.stats(reset=True)
    got = bls.BLS.batch_verify(keys, ms, sigs)
    st = native.stats()
    assert got is False
    assert st["one_validate"] == 0, st
    # a set that does not decode is an InvalidBatchSemiAggregate in the reference; here the
    # device's decode in the batch gives the same false
    assert st["partials"] == 1 and st["host_decodes"] == 0, st
    lo, hi = max(0, j - 2), min(N, j + 3)
    exp = C.verify_each([[p] for p in pk2[lo:hi]], ms[lo:hi], sg2[lo:hi], threads=THREADS)
    assert exp == [i != j for i in range(lo, hi)]


def test_fresh_objects_through_service(env):
    """AggregatingSignatureVerificationService.verify with BLSPublicKey /
    BLSSignature objects (its callers' types): per-task verdicts equal the
    oracle's, no single-object device call."""
    bls, native, synth, pk, ms, sg = env
    from teku_amd.service import AggregatingSignatureVerificationService

    sg2 = list(sg)
    bad = {11: sg[12], 5000: bytes(96), 9999: synth.NOT_IN_G2, 16383: sg[0]}
    for j, b in bad.items():
        sg2[j] = b
    keys, sigs = fresh(bls, pk, sg2)
    svc = AggregatingSignatureVerificationService(max_batch_size=N).start()
    try:
        native.stats(reset=True)
        futs = [svc.verify(keys[i], ms[i], sigs[i]) for i in range(N)]
        got = [f.result(timeout=120) for f in futs]
    finally:
        svc.stop()
    st = native.stats()
    assert [i for i, v in enumerate(got) if not v] == sorted(bad)
    assert st["one_validate"] == 0, st
    exp = C.verify_each([[p] for p in pk[:64]], ms[:64], sg2[:64], threads=THREADS)
    assert got[:64] == exp


def test_empty_key_list_units(env):
    """BLS.batchVerify with double pairing (BLS.java:306-322): a unit (pair of
    sets) with an empty key list raises (BlsException from the
    IllegalArgumentException), unless an object of the same unit does not
    decode -- then the unit is invalid and the batch is false, no raise."""
    bls, native, synth, pk, ms, sg = env
    keys, sigs = fresh(bls, pk[:6], sg[:6])
    keys[2] = []
    with pytest.raises(bls.BlsException):
        bls.BLS.batch_verify(keys, ms[:6], sigs)
    keys, sigs = fresh(bls, pk[:6], sg[:6])
    keys[2] = []
    sigs[3] = bls.BLSSignature.from_bytes_compressed(bytes(96))  # same unit (2, 3): undecodable
    native.stats(reset=True)
    assert bls.BLS.batch_verify(keys, ms[:6], sigs) is False
    assert native.stats()["partials"] == 0
    keys, sigs = fresh(bls, pk[:6], sg[:6])
    keys[2] = []
    sigs[5] = bls.BLSSignature.from_bytes_compressed(bytes(96))  # another unit: still raises
    with pytest.raises(bls.BlsException):
        bls.BLS.batch_verify(keys, ms[:6], sigs)
