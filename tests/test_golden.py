"""Golden fixtures (tests/golden/vectors.json, made by tests/golden/gen_golden.py).

CPU: the oracle still reproduces every fixture (regression of the pinned oracle).
GPU: the HIP path reproduces every fixture bit-exactly (points) / exactly (booleans).
"""

import ctypes
import json
import os

import pytest

from oracle import bls12_381 as O

V = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")))


def b(x):
    return bytes.fromhex(x[2:])


def test_oracle_reproduces_fixtures():
    for c in V["hash_to_G2"][:4]:
        assert O.g2_compress(O.hash_to_g2(b(c["input"]["msg"]), b(c["input"]["dst"]))) == b(c["output"])
    for c in V["sk_to_pk"]:
        assert O.sk_to_pk(int.from_bytes(b(c["input"]), "big")) == b(c["output"])
    for c in V["deserialization_G1"]:
        assert O.pk_decode_validate(b(c["input"]["pubkey"]))[0] == c["code"]
    for c in V["deserialization_G2"]:
        assert O.sig_decode_validate(b(c["input"]["signature"]))[0] == c["code"]


@pytest.fixture(scope="module")
def hip():
    import torch  # noqa: F401

    from teku_amd import bls, native

    return bls, native, native.lib()


@pytest.mark.gpu
def test_gpu_points(hip):
    bls, native, L = hip
    for c in V["hash_to_G2"]:
        m, d = b(c["input"]["msg"]), b(c["input"]["dst"])
        out = ctypes.create_string_buffer(96)
        native.check(L.tbls_hash_to_g2(m, len(m), d, len(d), out), "h2g")
        assert out.raw == b(c["output"])
    for c in V["sign"]:
        m = b(c["input"]["message"])
        out = ctypes.create_string_buffer(96)
        native.check(L.tbls_sign(b(c["input"]["privkey"]), m, len(m), O.ETH2_DST, len(O.ETH2_DST), out), "sign")
        assert out.raw == b(c["output"])
    for c in V["sk_to_pk"]:
        out = ctypes.create_string_buffer(48)
        native.check(L.tbls_sk_to_pk(b(c["input"]), out), "sk2pk")
        assert out.raw == b(c["output"])
    for c in V["deserialization_G1"]:
        assert L.tbls_pk_validate(b(c["input"]["pubkey"])) == c["code"]
    for c in V["deserialization_G2"]:
        inf = ctypes.c_int(0)
        assert L.tbls_sig_validate(b(c["input"]["signature"]), ctypes.byref(inf)) == c["code"]


@pytest.mark.gpu
def test_gpu_aggregate_and_verify(hip):
    bls, native, L = hip
    impl = bls.HipBLS12381()
    for c in V["aggregate"]:
        sigs = [bls.HipSignature(b(x)) for x in c["input"]]
        if c["output"] is None:
            with pytest.raises(bls.BlsException):
                impl.aggregate_signatures(sigs)
        else:
            assert impl.aggregate_signatures(sigs).to_bytes_compressed() == b(c["output"])
    for c in V["eth_aggregate_pubkeys"]:
        assert impl.aggregate_public_keys([bls.HipPublicKey(b(x)) for x in c["input"]]).to_bytes_compressed() == b(c["output"])
    for c in V["verify"]:
        i = c["input"]
        got = bls.BLS.verify(bls.BLSPublicKey(b(i["pubkey"])), b(i["message"]), bls.BLSSignature(b(i["signature"])))
        assert got == c["output"]
    for c in V["fast_aggregate_verify"]:
        i = c["input"]
        got = bls.BLS.fast_aggregate_verify([bls.BLSPublicKey(b(x)) for x in i["pubkeys"]], b(i["message"]), bls.BLSSignature(b(i["signature"])))
        assert got == c["output"]
    for c in V["batch_verify"]:
        i = c["input"]
        pks = [[bls.BLSPublicKey(b(x)) for x in ps] for ps in i["pubkeys"]]
        got = bls.BLS.batch_verify(pks, [b(x) for x in i["messages"]], [bls.BLSSignature(b(x)) for x in i["signatures"]])
        assert got == c["output"]
