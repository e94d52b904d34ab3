"""The C restatement of the oracle (oracle/c/bls_oracle.c) pinned by the same
reference KATs as the Python oracle, and cross-checked against it.

KATs: BLSSecretKeyTest.java:56-75, MockStartValidatorKeyPairFactoryTest.java:28-52,
LocalSignerTest.java:89-104/125-141, BLSTest.java:359-373, BlstPublicKeyTest.java:52-63,
BLSTest.java:248-256."""

import base64
import random
import subprocess

import pytest

from oracle import bls12_381 as O
from oracle.keys import blstestutil_sk, interop_sk
from tests.test_oracle_kats import (
    KAT_FAV4_MSG,
    KAT_FAV4_PKS,
    KAT_FAV4_SIG,
    KAT_AGGSLOT_SIG,
    KAT_INTEROP_PK,
    KAT_INTEROP_SK,
    KAT_RANDAO_SIG,
    KAT_REAL_PK,
    KAT_REAL_ROOT,
    KAT_REAL_SIG,
    KAT_SK_PK,
    local_signer_roots,
)

NOT_IN_G2 = bytes.fromhex("80" + "00" * 94 + "04")
BAD_PK = bytes.fromhex("9378a6e3984e96d2cd50450c76ca14732f1300efa04aecdb805b22e6d6926a85ef409e8f3acf494a1481090bf32ce3bd")


@pytest.fixture(scope="module")
def C():
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "oracle", "c")])
    from oracle import c_oracle

    return c_oracle


@pytest.mark.parametrize("sk,pk", KAT_SK_PK)
def test_sk_to_pk_kat(C, sk, pk):
    assert C.sk_to_pk(sk).hex() == pk


def test_interop_keys_kat(C):
    for sk, pk in zip(KAT_INTEROP_SK[:4], KAT_INTEROP_PK[:4]):
        assert C.sk_to_pk(sk) == base64.b64decode(pk)
    assert KAT_INTEROP_SK[0] == interop_sk(0)


def test_local_signer_sign_kats(C):
    randao, aggslot = local_signer_roots()
    sk = blstestutil_sk(1234)
    assert C.sign(sk, randao) == base64.b64decode(KAT_RANDAO_SIG)
    assert C.sign(sk, aggslot) == base64.b64decode(KAT_AGGSLOT_SIG)


def test_hash_to_g2_matches_python_oracle(C):
    nul = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
    for m in [b"", b"abc", bytes(range(256))]:
        assert C.hash_to_g2(m) == O.g2_compress(O.hash_to_g2(m))
    assert C.hash_to_g2(b"abc", nul) == O.g2_compress(O.hash_to_g2(b"abc", nul))


def test_validation_codes(C):
    assert C.pk_validate(KAT_REAL_PK) == O.SUCCESS
    assert C.pk_validate(BAD_PK) != O.SUCCESS
    assert C.pk_validate(bytes(48)) == O.BAD_ENCODING
    assert C.pk_validate(O.INFINITY_G1) == O.PK_IS_INFINITY
    assert C.sig_validate(KAT_REAL_SIG) == (O.SUCCESS, False)
    assert C.sig_validate(O.INFINITY_G2) == (O.SUCCESS, True)
    assert C.sig_validate(NOT_IN_G2)[0] == O.POINT_NOT_IN_GROUP
    assert C.sig_validate(bytes(96))[0] == O.BAD_ENCODING


def test_batch_verify_real_values_and_tampered(C):
    rng = random.Random(7)
    sks = [interop_sk(i) for i in range(5)]
    msgs = [bytes([i + 1]) * 32 for i in range(5)]
    pks = [C.sk_to_pk(s) for s in sks] + [KAT_REAL_PK]
    sigs = [C.sign(s, m) for s, m in zip(sks, msgs)] + [KAT_REAL_SIG]
    msgs = msgs + [KAT_REAL_ROOT]
    r = [rng.getrandbits(64) | 1 for _ in pks]
    assert C.batch_verify(pks, msgs, sigs, r) is True
    assert C.batch_verify(pks, msgs, sigs, r, threads=3) is True
    bad = list(sigs)
    bad[1], bad[2] = bad[2], bad[1]
    assert C.batch_verify(pks, msgs, bad, r) is False
    assert C.batch_verify(pks, msgs, sigs[:5] + [NOT_IN_G2], r) is False
    assert C.batch_verify(pks[:5] + [BAD_PK], msgs, sigs, r) is False


def test_multikey_sets_and_verify_each_match_python_oracle(C):
    """Multi-key sets (configs 2/3 shape: BlstPublicKey.aggregate semantics,
    BlstPublicKey.java:55-71) and per-set fastAggregateVerify verdicts
    (BLS.java:185-207): the C oracle equals the Python restatement on the
    reference's FAV-4 KAT (BLSTest.java:106-126) and on valid / tampered sets
    (wrong key count, swapped signature, infinity / invalid / zero key,
    infinity / non-G2 / zero signature, empty key list)."""
    sks = [interop_sk(20 + i) for i in range(6)]
    pks = [C.sk_to_pk(s) for s in sks]
    m = b"\x42" * 32
    agg3 = O.aggregate_sigs([C.sign(s, m) for s in sks[:3]])
    agg2 = O.aggregate_sigs([C.sign(s, b"two") for s in sks[3:5]])
    sets = [KAT_FAV4_PKS, pks[:3], pks[3:5], [pks[5]]]
    msgs = [KAT_FAV4_MSG, m, b"two", b"one"]
    sigs = [KAT_FAV4_SIG, agg3, agg2, C.sign(sks[5], b"one")]
    assert C.batch_verify_sets(sets, msgs, sigs, [3, 5, 7, 11], threads=2) is True
    assert C.verify_each(sets, msgs, sigs, threads=2) == [True] * 4
    cases = [
        (pks[:2], m, agg3),
        (pks[:3], m, agg2),
        (pks[:2] + [O.INFINITY_G1], m, agg3),
        (pks[:2] + [BAD_PK], m, agg3),
        (pks[:2] + [bytes(48)], m, agg3),
        ([pks[0]], b"x", O.INFINITY_G2),
        ([pks[0]], b"x", NOT_IN_G2),
        ([pks[0]], b"x", bytes(96)),
        ([], b"x", sigs[3]),
    ]
    got = C.verify_each([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases], threads=3)
    assert got == [O.fast_aggregate_verify(*c) for c in cases] == [False] * len(cases)
    for c in cases[:-1]:
        assert C.batch_verify_sets(sets + [c[0]], msgs + [c[1]], sigs + [c[2]], [3, 5, 7, 11, 13]) is False
