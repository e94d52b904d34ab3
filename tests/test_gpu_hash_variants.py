"""Byte-level parity of the batch hash_to_G2 kernels.

batchVerify hashes with one of five kernels by batch size (tb_lib.hip
launch_partial, hash_plan(): TB_HASH_ROW_MAX / TB_HASH_QUAD_MAX /
TB_HASH_DUO_MAX): k_set_hash_w2 + k_set_hash_fix (> 32,768 sets;
k_set_hash is its one-wave A/B twin), k_set_hash_duo + k_set_hash_fix
(8,193 - 32,768),
k_set_hash_quad + k_set_hash_fix (1,025 - 8,192), the row pipeline k_hrow_*
(513 - 1,024) and k_set_hash_coop (<= 512; k_set_hash_wave is its
fall-back).  Each one runs here on the same 640
messages -- empty, 200-byte, 768-byte, random lengths up to 256 bytes -- under the
Ethereum POP DST and the NUL DST (BLSTest.java:375-391), through the test
library's hook (tests/native/k_test_hash.hip), which launches the PRODUCT
library's kernels, and its compressed H(m) is compared byte for byte with the
C oracle (oracle/c: hash_to_G2, RFC 9380) and with the committed golden
vectors (tests/golden/vectors.json "hash_to_G2").  The row pipeline, the
two-wave kernel and the lane-group kernels also run with every set forced through their one-lane exact
fall-backs (k_hrow_fix, k_set_hash_fix: the path a Z = 0 cofactor chain
takes)."""

import ctypes
import json
import os
import random

import pytest

from oracle import bls12_381 as O
from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NUL_DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
RINV = pow(1 << 406, -1, O.P)  # Montgomery R = 2^406 (tb_fp.h)
VARIANTS = {0: "k_set_hash", 2: "k_hrow_*", 3: "k_set_hash_coop", 4: "k_set_hash_wave", 5: "k_set_hash_w2 + k_set_hash_fix", 6: "k_set_hash_quad + k_set_hash_fix", 7: "k_set_hash_duo + k_set_hash_fix"}


def messages():
    rng = random.Random(2024)
    # 768 bytes: past k_set_hash_coop's LDS message words (XW0_MAX blocks), its byte path
    ms = [b"", bytes(200), bytes(range(200)), b"abc", bytes([0xFF]) * 256, bytes(range(256)) * 3]
    while len(ms) < 640:
        ms.append(bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 31, 32, 33, 55, 56, 63, 64, 65, 119, 120, 200, 256]))))
    return ms


def compress(q192):
    """g2a (x.c0, x.c1, y.c0, y.c1: 12 LE u32 limbs each, Montgomery) -> ZCash bytes."""
    limbs = [int.from_bytes(q192[48 * k:48 * k + 48], "little") for k in range(4)]
    x0, x1, y0, y1 = (v * RINV % O.P for v in limbs)
    return O.g2_compress(((x0, x1), (y0, y1)))


@pytest.fixture(scope="module")
def hook():
    from teku_amd import native
    from tests.opcodec import load_test_lib

    L = load_test_lib()
    fn = L.tbls_test_hash_variant
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]

    def run(variant, msgs, dst, force_fix=0):
        off = [0]
        for m in msgs:
            off.append(off[-1] + len(m))
        offs = (ctypes.c_uint32 * len(off))(*off)
        n = len(msgs)
        q = ctypes.create_string_buffer(192 * n)
        sk = ctypes.create_string_buffer(n)
        rc = fn(native.LIB_PATH.encode(), variant, b"".join(msgs) or b"\0", offs, n, dst, len(dst), force_fix, q, sk)
        assert rc == 0, (VARIANTS[variant], rc)
        return [None if sk.raw[i] else compress(q.raw[192 * i:192 * i + 192]) for i in range(n)]

    return run


@pytest.fixture(scope="module")
def expected():
    ms = messages()
    return ms, {dst: [C.hash_to_g2(m, dst) for m in ms] for dst in (O.ETH2_DST, NUL_DST)}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("dst", [O.ETH2_DST, NUL_DST], ids=["POP", "NUL"])
def test_hash_kernel_bytes(hook, expected, variant, dst):
    ms, exp = expected
    got = hook(variant, ms, dst)
    bad = [i for i, (g, e) in enumerate(zip(got, exp[dst])) if g != e]
    assert not bad, (VARIANTS[variant], len(bad), bad[:5])


@pytest.mark.parametrize("variant", [2, 5, 6, 7])
def test_hash_fallback_bytes(hook, expected, variant):
    """Every set through the exact fall-back kernel (k_hrow_fix; k_set_hash_fix)."""
    ms, exp = expected
    got = hook(variant, ms, O.ETH2_DST, force_fix=1)
    assert got == exp[O.ETH2_DST]


def test_golden_vectors_every_kernel(hook):
    vec = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))["hash_to_G2"]
    by_dst = {}
    for v in vec:
        by_dst.setdefault(bytes.fromhex(v["input"]["dst"][2:]), []).append((bytes.fromhex(v["input"]["msg"][2:]), bytes.fromhex(v["output"][2:])))
    for dst, items in by_dst.items():
        for variant in VARIANTS:
            got = hook(variant, [m for m, _ in items], dst)
            assert got == [o for _, o in items], (VARIANTS[variant], dst)


def test_oracles_agree_on_sample(expected):
    """The C oracle used above against the pure-Python restatement on a sample."""
    ms, exp = expected
    for i in (0, 1, 2, 3, 4, 100, 639):
        assert exp[O.ETH2_DST][i] == O.g2_compress(O.hash_to_g2(ms[i])), i
        assert exp[NUL_DST][i] == O.g2_compress(O.hash_to_g2(ms[i], NUL_DST)), i
