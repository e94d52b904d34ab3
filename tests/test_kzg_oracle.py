"""The C KZG oracle (oracle/c/kzg_oracle.c) against the ceremony data the
reference ships (tests/golden/kzg/trusted_setup.txt) and against the committed
regression vectors.  CPU only.

Pinning: a commitment to the evaluations of x^k over the bit-reversed domain
must equal the file's own k-th G1 monomial point (this holds only when the
Lagrange points, their bit-reversal order, the roots of unity and the MSM all
match the ceremony), and proofs must satisfy the pairing equation against the
file's [tau]_2.  The Fiat-Shamir transcript layouts are restated from the spec
and not pinned by any reference vector ("transcript parity unpinned")."""

import json

import pytest

from tests.kzg_util import BLS_MODULUS, SETUP, VECTORS, blob_of, sample_blob
from oracle import kzg_oracle as K


@pytest.fixture(scope="module")
def setup():
    s = K.Setup.from_file(SETUP)
    yield s
    s.close()


@pytest.fixture(scope="module")
def parsed():
    return K.parse_setup_text(SETUP)


def test_setup_shape_and_generators(parsed):
    g1l, g2m, g1m = parsed
    assert len(g1l) == 48 * 4096 and len(g2m) == 96 * 65 and len(g1m) == 48 * 4096
    assert K.g2_generator() == g2m[:96]  # [tau^0]_2 is the G2 generator
    assert g1m[:48].hex().startswith("97f1d3a73197d794")  # [tau^0]_1 is the G1 generator


@pytest.mark.parametrize("k", [0, 1, 2, 3, 255, 4095])
def test_monomial_points_from_lagrange(setup, parsed, k):
    roots = K.roots_brp()
    blob = blob_of(pow(w, k, BLS_MODULUS) for w in roots)
    assert setup.blob_to_kzg_commitment(blob) == parsed[2][48 * k:48 * k + 48]


def test_roots_of_unity():
    roots = K.roots_brp()
    assert len(set(roots)) == 4096
    assert all(pow(w, 4096, BLS_MODULUS) == 1 for w in roots[:64])
    assert roots[0] == 1 and roots[1] == BLS_MODULUS - 1  # brp order: w^0, w^2048


def test_prove_verify_and_negatives(setup):
    blob, other = sample_blob(11), sample_blob(12)
    c = setup.blob_to_kzg_commitment(blob)
    p = setup.compute_blob_kzg_proof(blob, c)
    assert setup.verify_blob_kzg_proof(blob, c, p) is True
    assert setup.verify_blob_kzg_proof(other, c, p) is False
    c2 = setup.blob_to_kzg_commitment(other)
    assert setup.verify_blob_kzg_proof(blob, c2, p) is False
    p2 = setup.compute_blob_kzg_proof(other, c2)
    assert setup.verify_blob_kzg_proof(blob, c, p2) is False
    assert setup.verify_blob_kzg_proof_batch([blob, other], [c, c2], [p, p2]) is True
    assert setup.verify_blob_kzg_proof_batch([blob, other], [c, c2], [p2, p]) is False
    assert setup.verify_blob_kzg_proof_batch([], [], []) is True


def test_badargs(setup):
    blob = sample_blob(11)
    c = setup.blob_to_kzg_commitment(blob)
    p = setup.compute_blob_kzg_proof(blob, c)
    bad_blob = BLS_MODULUS.to_bytes(32, "big") + blob[32:]  # element == r: non-canonical
    assert setup.blob_to_kzg_commitment(bad_blob) == K.KZG_BADARGS
    assert setup.verify_blob_kzg_proof(bad_blob, c, p) == K.KZG_BADARGS
    bad_point = bytes([c[0] & 0x7F]) + c[1:]  # compression flag cleared
    assert setup.verify_blob_kzg_proof(blob, bad_point, p) == K.KZG_BADARGS
    assert setup.verify_blob_kzg_proof_batch([blob, blob], [c, c], [p, bad_point]) == K.KZG_BADARGS


def test_in_domain_point(setup):
    blob = sample_blob(21)
    roots = K.roots_brp()
    c = setup.blob_to_kzg_commitment(blob)
    for i in (0, 7, 4095):
        z = roots[i].to_bytes(32, "big")
        proof, y = setup.compute_kzg_proof(blob, z)
        assert y == blob[32 * i:32 * i + 32]
        assert setup.verify_kzg_proof(c, z, y, proof) is True
        y_bad = ((int.from_bytes(y, "big") + 1) % BLS_MODULUS).to_bytes(32, "big")
        assert setup.verify_kzg_proof(c, z, y_bad, proof) is False


def test_committed_vectors(setup):
    v = json.load(open(VECTORS))
    blobs = {f"seed{s}": sample_blob(s) for s in v["seeds"]}
    blobs.update({"zero": blob_of([0] * 4096), "const7": blob_of([7] * 4096), "ramp": blob_of(range(4096))})
    for case in v["cases"][:3] + v["cases"][-3:]:
        blob = blobs[case["blob"]]
        assert setup.blob_to_kzg_commitment(blob).hex() == case["commitment"]
    zero = next(c for c in v["cases"] if c["blob"] == "zero")
    assert zero["commitment"] == "c0" + "00" * 47 and zero["proof"] == "c0" + "00" * 47
    const7 = next(c for c in v["cases"] if c["blob"] == "const7")
    assert int(const7["y"], 16) == 7  # a constant polynomial evaluates to its constant
