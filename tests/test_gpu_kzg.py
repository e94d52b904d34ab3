"""EIP-4844 KZG on the GPU (teku_amd/kzg.py -> include/tekukzg.h ->
k_kzg.hip) against the C oracle (oracle/c/kzg_oracle.c) and the committed
vectors (tests/golden/kzg/vectors.json).  The cases mirror the reference's
CKZG4844Test (infrastructure/kzg/src/test/java/tech/pegasys/teku/kzg/
CKZG4844Test.java:67-259): load twice, free twice, usage without a setup,
batch / single / batch-of-one prove+verify with the three kinds of mismatch,
empty batch, size mismatches, wrong blob lengths, broken setup files.
Bit-exact: commitments, proofs, per-blob z and y, the batch r."""

import json

import pytest

from oracle import kzg_oracle as K
from teku_amd import kzg
from tests.kzg_util import BLS_MODULUS, SETUP, VECTORS, blob_of, broken_setups, sample_blob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ckzg():
    c = kzg.CKZG4844.get_instance()
    c.load_trusted_setup(SETUP)
    yield c


@pytest.fixture(scope="module")
def orc():
    s = K.Setup.from_file(SETUP)
    yield s
    s.close()


@pytest.fixture(scope="module")
def vectors():
    v = json.load(open(VECTORS))
    blobs = {f"seed{s}": sample_blob(s) for s in v["seeds"]}
    blobs.update({"zero": blob_of([0] * 4096), "const7": blob_of([7] * 4096), "ramp": blob_of(range(4096))})
    return v, blobs


def test_commitments_and_proofs_match_vectors(ckzg, vectors):
    v, blobs = vectors
    names = [c["blob"] for c in v["cases"]]
    got = ckzg.blobs_to_kzg_commitments([blobs[n] for n in names])
    for case, c in zip(v["cases"], got):
        assert c.hex() == case["commitment"], case["blob"]
        assert ckzg.blob_to_kzg_commitment(blobs[case["blob"]]).hex() == case["commitment"]
        assert ckzg.compute_blob_kzg_proof(blobs[case["blob"]], c).hex() == case["proof"], case["blob"]


def test_transcript_matches_oracle(ckzg, vectors):
    v, blobs = vectors
    seeds = v["batch"]["blobs"]
    cases = {c["blob"]: c for c in v["cases"]}
    bl = [blobs[s] for s in seeds]
    cs = [bytes.fromhex(cases[s]["commitment"]) for s in seeds]
    ps = [bytes.fromhex(cases[s]["proof"]) for s in seeds]
    assert ckzg.verify_blob_kzg_proof_batch(bl, cs, ps) is True
    zs, ys, r = ckzg.last_transcript(len(seeds))
    assert [z.hex() for z in zs] == [cases[s]["z"] for s in seeds]
    assert [y.hex() for y in ys] == [cases[s]["y"] for s in seeds]
    assert r.hex() == v["batch"]["r"]


def test_monomial_points_from_lagrange(ckzg):
    ts = kzg.parse_trusted_setup_file(SETUP)
    roots = K.roots_brp()
    ks = [0, 1, 2, 4095]
    got = ckzg.blobs_to_kzg_commitments([blob_of(pow(w, k, BLS_MODULUS) for w in roots) for k in ks])
    assert got == [ts.g1_monomial[k] for k in ks]


def _prove_all(ckzg, blobs):
    cs = ckzg.blobs_to_kzg_commitments(blobs)
    return cs, [ckzg.compute_blob_kzg_proof(b, c) for b, c in zip(blobs, cs)]


@pytest.mark.parametrize("n", [4, 1])
def test_computing_and_verifying_batch_proofs(ckzg, orc, n):
    blobs = [sample_blob(100 + i) for i in range(n)]
    cs, ps = _prove_all(ckzg, blobs)
    assert ckzg.verify_blob_kzg_proof_batch(blobs, cs, ps) is True
    other = [sample_blob(200 + i) for i in range(n)]
    assert ckzg.verify_blob_kzg_proof_batch(other, cs, ps) is False
    ocs, ops = _prove_all(ckzg, other)
    assert ckzg.verify_blob_kzg_proof_batch(blobs, ocs, ps) is False
    assert ckzg.verify_blob_kzg_proof_batch(blobs, cs, ops) is False
    # the oracle agrees on every verdict
    assert orc.verify_blob_kzg_proof_batch(blobs, cs, ps) is True
    assert orc.verify_blob_kzg_proof_batch(blobs, cs, ops) is False


def test_single_proof(ckzg):
    blob, other = sample_blob(300), sample_blob(301)
    c = ckzg.blob_to_kzg_commitment(blob)
    p = ckzg.compute_blob_kzg_proof(blob, c)
    assert ckzg.verify_blob_kzg_proof(blob, c, p) is True
    assert ckzg.verify_blob_kzg_proof(other, c, p) is False
    oc = ckzg.blob_to_kzg_commitment(other)
    assert ckzg.verify_blob_kzg_proof(blob, oc, p) is False
    assert ckzg.verify_blob_kzg_proof(blob, c, ckzg.compute_blob_kzg_proof(other, oc)) is False


def test_verifying_empty_batch(ckzg):
    assert ckzg.verify_blob_kzg_proof_batch([], [], []) is True


def test_batch_size_mismatch_raises(ckzg):
    blobs = [sample_blob(400 + i) for i in range(4)]
    cs, ps = _prove_all(ckzg, blobs)
    for args in [(blobs, cs, ps[:1]), (blobs, cs[:1], ps), (blobs[:1], cs, ps)]:
        with pytest.raises(kzg.KZGException) as ei:
            ckzg.verify_blob_kzg_proof_batch(*args)
        cause = ei.value.__cause__
        assert isinstance(cause, kzg.CKZGException)
        assert __import__("re").fullmatch(r"Invalid .+ size. Expected \d+ bytes but got \d+. \(C_KZG_BADARGS\)", str(cause)), str(cause)


@pytest.mark.parametrize("blob_hex", ["0d2024ece3e004271319699b8b00cc010628b6bc0be5457f031fb1db0afd3ff8", "", "925668a49d06f4"])
def test_incorrect_length_blob(ckzg, blob_hex):
    blob = bytes.fromhex(blob_hex)
    with pytest.raises(kzg.KZGException) as ei:
        ckzg.compute_blob_kzg_proof(blob, ckzg.blob_to_kzg_commitment(blob))
    cause = ei.value.__cause__
    assert cause.error == kzg.C_KZG_BADARGS
    assert "Invalid blob size. Expected 131072 bytes but got" in cause.error_message


def test_badargs_noncanonical_and_bad_points(ckzg, vectors):
    v, blobs = vectors
    case = v["cases"][0]
    blob, c, p = blobs[case["blob"]], bytes.fromhex(case["commitment"]), bytes.fromhex(case["proof"])
    bad_blob = blob[:32 * 9] + BLS_MODULUS.to_bytes(32, "big") + blob[32 * 10:]
    for call in [lambda: ckzg.blob_to_kzg_commitment(bad_blob), lambda: ckzg.verify_blob_kzg_proof(bad_blob, c, p),
                 lambda: ckzg.verify_blob_kzg_proof(blob, bytes([c[0] & 0x7F]) + c[1:], p),
                 lambda: ckzg.verify_blob_kzg_proof_batch([blob, blob], [c, c], [p, bytes(48)])]:
        with pytest.raises(kzg.KZGException) as ei:
            call()
        assert ei.value.__cause__.error == kzg.C_KZG_BADARGS


def test_in_domain_points(ckzg, orc):
    blob = sample_blob(21)
    roots = K.roots_brp()
    c = ckzg.blob_to_kzg_commitment(blob)
    for i in (0, 7, 4095):
        z = roots[i].to_bytes(32, "big")
        proof, y = ckzg.compute_kzg_proof(blob, z)
        assert y == blob[32 * i:32 * i + 32]
        assert (proof, y) == orc.compute_kzg_proof(blob, z)
        assert ckzg.verify_kzg_proof(c, z, y, proof) is True
    z = (12345).to_bytes(32, "big")
    proof, y = ckzg.compute_kzg_proof(blob, z)
    assert (proof, y) == orc.compute_kzg_proof(blob, z)
    assert ckzg.verify_kzg_proof(c, z, y, proof) is True
    y_bad = ((int.from_bytes(y, "big") + 1) % BLS_MODULUS).to_bytes(32, "big")
    assert ckzg.verify_kzg_proof(c, z, y_bad, proof) is False


def test_load_free_lifecycle(ckzg, tmp_path):
    ckzg.load_trusted_setup(SETUP)  # same file twice: no-op
    ckzg.free_trusted_setup()
    with pytest.raises(kzg.KZGException):
        ckzg.free_trusted_setup()
    blob = sample_blob(1)
    for call in [lambda: ckzg.verify_blob_kzg_proof_batch([blob], [bytes(48)], [bytes(48)]),
                 lambda: ckzg.blob_to_kzg_commitment(b""), lambda: ckzg.compute_blob_kzg_proof(b"", bytes(48))]:
        with pytest.raises(kzg.KZGException) as ei:
            call()
        assert str(ei.value.__cause__) == "Trusted Setup is not loaded."
    for path in broken_setups(tmp_path).values():
        with pytest.raises(kzg.KZGException) as ei:
            ckzg.load_trusted_setup(path)
        assert "Failed to parse trusted setup file" in str(ei.value.__cause__)
    ckzg.load_trusted_setup(SETUP)
    c = ckzg.blob_to_kzg_commitment(blob)
    assert ckzg.verify_blob_kzg_proof(blob, c, ckzg.compute_blob_kzg_proof(blob, c)) is True


def test_many_blobs_batch(ckzg, orc):
    """A 64-blob batch, one tampered proof: the GPU and oracle verdicts agree."""
    blobs = [sample_blob(500 + i) for i in range(64)]
    cs, ps = _prove_all(ckzg, blobs)
    assert ckzg.verify_blob_kzg_proof_batch(blobs, cs, ps) is True
    zs, ys, r = ckzg.last_transcript(64)
    ok, ozs, oys, orr = orc.verify_blob_kzg_proof_batch(blobs, cs, ps, detail=True)
    assert ok is True and zs == ozs and ys == oys and r == orr
    ps2 = list(ps)
    ps2[17], ps2[18] = ps[18], ps[17]
    assert ckzg.verify_blob_kzg_proof_batch(blobs, cs, ps2) is False
