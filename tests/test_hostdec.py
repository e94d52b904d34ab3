"""Host decoding (tb_hostdec.h, include/tekubls.h tbls_pk_decode / tbls_sig_decode
and their _many forms): blst_p1/p2_uncompress's verdict -- flags, x < p, the
curve equation has a root, x != 0, no subgroup check -- as BlstPublicKey /
BlstSignature.fromBytes throw it (BlstPublicKey.java:38-45,
BlstSignature.java:35-47).  CPU only: no device, no tbls_init.

Pinned against the golden deserialization vectors (tests/golden/vectors.json,
whose `code` is the full device validation: decode + subgroup check), the
oracle's points, and Euler's criterion in Python integers on random x."""

import ctypes
import json
import os
import random

import pytest

from oracle import bls12_381 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))
P = O.P


@pytest.fixture(scope="module")
def L():
    from teku_amd import native

    return native.host()


def is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def g1_expected(b):
    """Python restatement of blst_p1_uncompress's verdict."""
    if not b[0] & 0x80:
        return 1
    if b[0] & 0x40:
        return 0 if (b[0] & 0x3F) == 0 and not any(b[1:]) else 1
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        return 1
    if not is_square(x**3 + 4):
        return 2
    return 3 if x == 0 else 0


def g2_expected(b):
    if not b[0] & 0x80:
        return 1
    if b[0] & 0x40:
        return 0 if (b[0] & 0x3F) == 0 and not any(b[1:]) else 1
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    if x0 >= P or x1 >= P:
        return 1
    a0, a1 = (x0 * x0 - x1 * x1) % P, (2 * x0 * x1) % P
    c0, c1 = (a0 * x0 - a1 * x1 + 4) % P, (a0 * x1 + a1 * x0 + 4) % P
    if not is_square(c0 * c0 + c1 * c1):  # a square in Fp2 iff its norm is a square in Fp
        return 2
    return 3 if x0 == 0 and x1 == 0 else 0


def dec(L, b):
    inf = ctypes.c_int(-1)
    fn = L.tbls_pk_decode if len(b) == 48 else L.tbls_sig_decode
    return fn(bytes(b), ctypes.byref(inf)), inf.value


def test_golden_deserialization_vectors(L):
    # golden `code` = decode + subgroup check; the decoder stops before the group
    for c in V["deserialization_G1"]:
        b = bytes.fromhex(c["input"]["pubkey"][2:])
        code, inf = dec(L, b)
        assert code == g1_expected(b)
        if c["code"] in (1, 2):
            assert code == c["code"]
        elif c["code"] == 6:  # the infinity key decodes (isValid is false)
            assert (code, inf) == (0, 1)
        elif c["code"] == 3:  # off the subgroup: decodes, unless x = 0
            assert code == (3 if int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big") == 0 else 0)
        else:
            assert code == 0
    for c in V["deserialization_G2"]:
        b = bytes.fromhex(c["input"]["signature"][2:])
        code, inf = dec(L, b)
        assert code == g2_expected(b)
        if c["code"] in (1, 2):
            assert code == c["code"]
        elif c["code"] == 0:
            assert code == 0 and inf == (b == bytes([0xC0]) + bytes(95))


def test_oracle_points_decode(L):
    rng = random.Random(11)
    for i in range(12):
        sk = rng.randrange(1, O.R)
        assert dec(L, O.sk_to_pk(sk)) == (0, 0)
        assert dec(L, O.sign(sk, bytes([i]) * 7)) == (0, 0)
    assert dec(L, O.g2_compress(O.hash_to_g2(b"abc"))) == (0, 0)


def test_random_x_against_euler(L):
    rng = random.Random(7)
    for i in range(1500):
        x = rng.randrange(P) if i % 5 else rng.randrange(64)
        b = bytearray(x.to_bytes(48, "big"))
        b[0] |= 0x80 | (0x20 if i & 1 else 0)
        assert dec(L, b)[0] == g1_expected(bytes(b)), x
        x0, x1 = rng.randrange(P), (rng.randrange(P) if i % 3 else 0)
        b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
        b[0] |= 0x80 | (0x20 if i & 2 else 0)
        assert dec(L, b)[0] == g2_expected(bytes(b)), (x0, x1)


def test_encoding_edge_cases(L):
    pk = O.sk_to_pk(12345)
    sig = O.sign(12345, b"m")
    p_be = P.to_bytes(48, "big")
    cases = [
        bytes(48),  # no compression flag
        bytes([pk[0] & 0x7F]) + pk[1:],
        bytes([0xC0]) + bytes(46) + b"\x01",  # infinity with payload
        bytes([0xE0]) + bytes(47),  # infinity with the sign flag
        bytes([0x80 | p_be[0]]) + p_be[1:],  # x = p
        bytes([0x9F]) + b"\xff" * 47,  # x = 2^381 - 1
        bytes([0x80]) + bytes(47),  # x = 0: on the curve, (0, +-2), not in group
        bytes([0xA0]) + bytes(47),
    ]
    for b in cases:
        assert dec(L, b)[0] == g1_expected(b), b.hex()
    assert dec(L, bytes([0x80]) + bytes(47))[0] == 3
    g2 = [
        bytes(96),
        bytes([sig[0] & 0x7F]) + sig[1:],
        bytes([0xC0]) + bytes(94) + b"\x01",
        bytes([0x80 | p_be[0]]) + p_be[1:] + bytes(48),  # x1 = p
        bytes([0x80]) + bytes(47) + p_be,  # x0 = p
        bytes([0x80]) + bytes(95),  # x = 0: 4(1 + u) is not a square
        bytes([0xA0]) + bytes(95),
        bytes.fromhex("80" + "00" * 94 + "04"),  # on E2, outside G2: decodes
    ]
    for b in g2:
        assert dec(L, b)[0] == g2_expected(b), b.hex()
    assert dec(L, bytes.fromhex("80" + "00" * 94 + "04"))[0] == 0


def test_many_equals_single_and_counts(L):
    from teku_amd import native

    rng = random.Random(3)
    pks, sigs = [], []
    for i in range(1300):  # several host threads
        if i % 4 == 0:
            pks.append(O.sk_to_pk(rng.randrange(1, O.R)) if i % 40 == 0 else bytes([0x80 | rng.randrange(32)]) + rng.randbytes(47))
        else:
            pks.append(bytes([rng.choice([0x80, 0xA0, 0x00, 0xC0])]) + rng.randbytes(47))
        sigs.append(bytes([rng.choice([0x80, 0xA0, 0x8F, 0x40])]) + rng.randbytes(95))
    native.stats(reset=True)
    for items, many in ((pks, "tbls_pk_decode_many"), (sigs, "tbls_sig_decode_many")):
        n = len(items)
        codes, inf = ctypes.create_string_buffer(n), ctypes.create_string_buffer(n)
        assert getattr(L, many)(b"".join(items), n, codes, inf) == 0
        for i, b in enumerate(items):
            assert (codes.raw[i], inf.raw[i]) == dec(L, b), i
    st = native.stats()
    assert st["host_decodes"] == 4 * 1300 and st["partials"] == 0 and st["one_validate"] == 0
    assert L.tbls_sig_decode_many(None, 0, None, None) == 0
