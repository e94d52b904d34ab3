"""Pin the oracle against every known-answer test the reference holds for this path.

Each test cites the reference test it reproduces.  These run on CPU only.
"""

import base64
import hashlib
import random

import pytest

from oracle import bls12_381 as O
from oracle.keys import JavaRandom, interop_sk, blstestutil_sk

# BLSTest.fastAggregateVerify_verify4Signers (BLSTest.java:106-126)
KAT_FAV4_MSG = bytes.fromhex("999bb85f3690c2ccb1607dd3e11a7e114038eb4044bdbdd340bc81aa3e5e0c9e")
KAT_FAV4_PKS = [
    bytes.fromhex(h)
    for h in [
        "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb",
        "a572cbea904d67468808c8eb50a9450c9721db309128012543902d0ac358a62ae28f75bb8f1c7c42c39a8c5529bf0f4e",
        "89ece308f9d1f0131765212deca99697b112d61f9be9a5f1f3780a51335b3ff981747a0b2ca2179b96d2c0c9024e5224",
        "ac9b60d5afcbd5663a8a44b7c5a02f19e9a77ab0a35bd65809bb5c67ec582c897feb04decc694b13e08587f3ff9b5b60",
    ]
]
KAT_FAV4_SIG = bytes.fromhex(
    "b2550663aa862b2741c9abc94f7b0b8a725b6f12b8f214d833e214e87c64235e4b1fb1e1ee64e5ae942cb3e0392699fc"
    "0524ae6f35072d1f243668de730be8745ab5be3314f90c107e246cefd1f1b97cd7241cfe97f4c80aeb354e8fac2ea720"
)

# BLSTest.testSignatureVerifyForSomeRealValues (BLSTest.java:359-373)
KAT_REAL_ROOT = bytes.fromhex("95b8e2ba063ab62f68ebe7db0a9669ab9e7906aa4e060e1cc0b67b294ce8c5e4")
KAT_REAL_SIG = bytes.fromhex(
    "ab51f352e90509ca5085ec43af9ad3ea4ae42bf30c91af7dcdc113ef79cfc8601b756f18d8cf634436d8b6b0095fc568"
    "0066f382eb3728a7090c55c9afb66e8f94b44d2682db8ef5de4b89928d1744824df174e0c800b9e934b0ad14e6388163"
)
KAT_REAL_PK = bytes.fromhex(
    "b5e8f551c28abd6ef8253581ffad0834bfd8fafa9948d09b337c9c5f21d6e7fd6065a1ee35ac5146ac17344f97490301"
)

# BLSSecretKeyTest.getSecretKeysToPubKeys (BLSSecretKeyTest.java:56-75)
KAT_SK_PK = [
    (0, "c0" + "00" * 47),
    (1, "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"),
    (
        0x72FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF,
        "b5d2c2f45a9d8429e2fc28ffe844601b3d87490682f5dab702ac090fd3d1ec3fe3cc3e5ffb63ca36bc640a2b9f73cc3f",
    ),
    (
        0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000000,
        "b7f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb",
    ),
]

# MockStartValidatorKeyPairFactoryTest (MockStartValidatorKeyPairFactoryTest.java:28-52)
KAT_INTEROP_SK = [
    16808672146709759238327133555736750089977066230599028589193936481731504400486,
    37006103240406073079686739739280712467525465637222501547219594975923976982528,
    22330876536127119444572216874798222843352868708084730796787004036811744442455,
    17048462031355941381150076874414096388968985457797372268770826099852902060945,
    28647806952216650698330424381872693846361470773871570637461872359310549743691,
    2416304019107052589452838695606585506736351107897780798170812672519914514344,
    7300215445567548136411883691093515822872548648751398235557229381530420545683,
    26495790445032093722332687600112008700915252495659977774957922313678954054133,
    2908643403277969554503670470854573663206729491025062456164283925661321952518,
    19554639423851580804889717218680781396599791537051606512605582393920758869044,
]
KAT_INTEROP_PK = [
    "qZp27XeW974i1bfoXe63xWd+iOUR4LM3YY+MTrYTSbS/LRU/ZJ97UzWf6LlKOORM",
    "uJvrxpl2lyajGMjplxvTFxKXxhrqSmV4p6T5S1R9y6W6wWqJEItrah/jaV0ah0oL",
    "o6MrD4tN24PxoKhT2B3XJd/ld9T0w9uOzlLOKwJuyoSBXBp+jpKk3j11VzO/fkqb",
    "iMFB33fNnY16cadcgmxBqcnwPG7hsYDz54UvaigAmd7TUbWNZuZTr45CgWpNj1Mu",
    "gSg7eiDhykYOvZu9dwBdVXNwyrsfmkT1MMTExmIw9nX434tMKBiFGqfXeoDKWkpe",
    "qwvdoPhfhC9DG+rM8SUL8f17pRtBAP1kNktkAf2oW7AGmz5xW1iBloTn/AsQpyo0",
    "mXfxyLcxqNVVgUa/uGyuomQ088WHi1ib8oCkLJFZ5wDp3w5AhilsILAR0ueMJ9Nz",
    "qNTHwneVpyWWExfvWVOnAy7W2Dc524sOinI1PRuLRDlCf376LInKoDzJ8o+Muris",
    "ptMQ27+rmiJFD1mZP4ekzl22Ij87Xx8w0sTscYki1ADgs8d0HejlmWD3JBGg7hCn",
    "mJNBPAAoOj+e2f2YRd2hzqOCKNIlZ/lUHczDV+VKLWpuIEEDySVky8BfSQWsfEk6",
]

# LocalSignerTest.shouldCreateRandaoReveal / shouldSignAggregationSlot
# (ethereum/spec/src/test/java/tech/pegasys/teku/spec/signatures/LocalSignerTest.java:89-104, 125-141)
KAT_RANDAO_SIG = "j7vOT7GQBnv+aIqxb0byMWNvMCXhQwAfj38UcMne7pNGXOvNZKnXQ9Knma/NOPUyAvLcRBDtew23vVtzWcm7naaTRJVvLJS6xiPOMIHOw6wNtGggzc20heZAXZAMdaKi"
KAT_AGGSLOT_SIG = "hnCLCZlbEyzMFq2JLHl6wk4W6gpbFGoQA2N4WB+CpgqVg3gcxJpRKOswtSTU4XdSEU2x3Hf0oTlxer/gVaFwAh84Mm4VLH67LNUxVO4+o2Q5TxOD1sArnvMcOJdGMGp2"


def local_signer_roots():
    """Signing roots of LocalSignerTest: fork info from DataStructureUtil(seed 92892824)
    (DataStructureUtil.java:219-257, 1760-1766), domain per BeaconStateAccessors.java:351-361
    and MiscHelpers.java:321-360, minimal spec (8 slots/epoch)."""
    seed = 92892824
    prev = JavaRandom(seed).next_bytes(4)
    cur = JavaRandom(seed + 1).next_bytes(4)
    fork_epoch = JavaRandom(seed + 2).next_long() & ((1 << 64) - 1)
    gvr = JavaRandom(seed + 3).next_bytes(32)

    def domain(dt, epoch):
        fv = prev if epoch < fork_epoch else cur
        return dt + hashlib.sha256(fv + bytes(28) + gvr).digest()[:28]

    def sroot(num, dom):
        return hashlib.sha256(num.to_bytes(8, "little") + bytes(24) + dom).digest()

    randao = sroot(7, domain(bytes.fromhex("02000000"), 7))
    aggslot = sroot(7, domain(bytes.fromhex("05000000"), 7 // 8))
    return randao, aggslot


def test_fast_aggregate_verify_4_signers():
    assert O.fast_aggregate_verify(KAT_FAV4_PKS, KAT_FAV4_MSG, KAT_FAV4_SIG)
    assert not O.fast_aggregate_verify(KAT_FAV4_PKS[:3], KAT_FAV4_MSG, KAT_FAV4_SIG)


def test_verify_real_values():
    assert O.core_verify(KAT_REAL_PK, KAT_REAL_ROOT, KAT_REAL_SIG)
    assert not O.core_verify(KAT_REAL_PK, bytes([KAT_REAL_ROOT[0] ^ 1]) + KAT_REAL_ROOT[1:], KAT_REAL_SIG)


@pytest.mark.parametrize("sk,pk", KAT_SK_PK)
def test_sk_to_pk(sk, pk):
    assert O.sk_to_pk(sk).hex() == pk


def test_interop_keys():
    for i in range(10):
        assert interop_sk(i) == KAT_INTEROP_SK[i]
    for i in range(3):
        assert O.sk_to_pk(interop_sk(i)) == base64.b64decode(KAT_INTEROP_PK[i])


def test_local_signer_sign_kats():
    sk = blstestutil_sk(1234)
    randao, aggslot = local_signer_roots()
    assert O.sign(sk, randao) == base64.b64decode(KAT_RANDAO_SIG)
    assert O.sign(sk, aggslot) == base64.b64decode(KAT_AGGSLOT_SIG)


@pytest.mark.parametrize(
    "hexsk",
    [
        "73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001",
        "e7db4ea6533afa906673b0101343b00aa77b4805fffcb7fdfffffffe00000002",
        "ff" * 32,
    ],
)
def test_sk_out_of_range_rejected(hexsk):
    # BLSSecretKeyTest.secretKeyFromBytes_shouldThrowWhenInvalidBytes (l.26-45)
    with pytest.raises(ValueError):
        O.sk_from_bytes(bytes.fromhex(hexsk))


def test_rejection_vectors():
    # BlstPublicKeyTest.java:52-63
    bad = bytes.fromhex(
        "9378a6e3984e96d2cd50450c76ca14732f1300efa04aecdb805b22e6d6926a85ef409e8f3acf494a1481090bf32ce3bd"
    )
    assert O.pk_decode_validate(bad)[0] != O.SUCCESS
    # BLSTest.notInG2 (l.248-256): on curve, not in G2
    nig2 = bytes.fromhex("80" + "00" * 94 + "04")
    code, a = O.g2_decompress(nig2)
    assert code == O.SUCCESS and a is not None
    assert O.sig_decode_validate(nig2)[0] == O.POINT_NOT_IN_GROUP
    # BlstSignatureTest.java:54-57: 96 zero bytes do not decode
    assert O.g2_decompress(bytes(96))[0] == O.BAD_ENCODING
    # infinity encodings (BlstSignatureTest.java:40-52, BlstPublicKeyTest.java:39-50)
    assert O.g2_decompress(O.INFINITY_G2) == (O.SUCCESS, None)
    assert O.g1_decompress(O.INFINITY_G1) == (O.SUCCESS, None)
    assert O.pk_decode_validate(O.INFINITY_G1)[0] == O.PK_IS_INFINITY


def test_subgroup_checks_match_order_check():
    rng = random.Random(7)
    # random curve points (mostly not in the subgroup) vs the slow [r]P test
    n_in = n_out = 0
    while n_out < 3:
        x = rng.randrange(O.P)
        y = O.fp_sqrt(x * x * x + 4)
        if y is None:
            continue
        p = O.jac_from_affine(O.FP, (x, y))
        fast, slow = O.g1_in_group(p), O.g1_in_group_slow(p)
        assert fast == slow
        n_out += not slow
    g = O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), rng.randrange(O.R))
    assert O.g1_in_group(g)
    n_out = 0
    while n_out < 2:
        x = (rng.randrange(O.P), rng.randrange(O.P))
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(x), x), O.B_G2))
        if y is None:
            continue
        p = O.jac_from_affine(O.FP2, (x, y))
        assert O.g2_in_group(p) == O.g2_in_group_slow(p)
        n_out += 1
    q = O.jac_mul(O.FP2, O.jac_from_affine(O.FP2, O.G2_GEN), rng.randrange(O.R))
    assert O.g2_in_group(q)


def test_hash_to_g2_structure():
    rng = random.Random(3)
    for _ in range(3):
        u = (rng.randrange(O.P), rng.randrange(O.P))
        q = O.map_to_curve_sswu_g2(u)
        assert O.on_curve_iso(q)
        assert O.on_curve_g2(O.iso_map_g2(q))
    u = (rng.randrange(O.P), rng.randrange(O.P))
    p = O.jac_from_affine(O.FP2, O.iso_map_g2(O.map_to_curve_sswu_g2(u)))
    assert O.jac_eq(O.FP2, O.clear_cofactor_g2(p), O.jac_mul(O.FP2, p, O.H_EFF_G2))
    h = O.hash_to_g2_jac(b"abc")
    assert O.g2_in_group_slow(h)


def test_pairing_bilinear():
    e = O.pairing(O.G1_GEN, O.G2_GEN)
    g1x2 = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), 2))
    assert O.f12_mul(e, e) == O.pairing(g1x2, O.G2_GEN)
    assert e != O.F12_ONE


def test_sign_verify_dst_variants():
    # BLSTest.succeedsWhenWeCanSignAndVerifyWithValidDST / verifyWithDifferentDSTFails (l.375-391)
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
    sk = blstestutil_sk(42)
    pk = O.sk_to_pk(sk)
    msg = b"Hello, world!"
    s = O.sign(sk, msg, dst)
    assert O.core_verify(pk, msg, s, dst)
    assert not O.core_verify(pk, msg, s)
