"""Host logic of the KZG mirror (teku_amd/kzg.py) and the C ABI of
include/tekukzg.h, on CPU: the trusted-setup parser and its failure cases
(CKZG4844Test.incorrectTrustedSetupFilesShouldThrow, CKZG4844Test.java:237-251;
testInvalidLengthG2PointInNewTrustedSetup, l.253-259), flattening, the
exported symbols, and that without a device the calls fail loudly."""

import ctypes
import os
import re

import pytest

from tests.kzg_util import SETUP, broken_setups
from teku_amd import kzg, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_trusted_setup():
    ts = kzg.parse_trusted_setup_file(SETUP)
    assert len(ts.g1_lagrange) == 4096 and len(ts.g2_monomial) == 65 and len(ts.g1_monomial) == 4096
    assert ts.g2_monomial[0].hex().startswith("93e02b6052719f607dacd3a0")


@pytest.mark.parametrize("name", ["trusted_setup_g1_length.txt", "trusted_setup_g2_length.txt", "trusted_setup_g2_bytesize.txt"])
def test_broken_setup_files_fail_to_parse(tmp_path, name):
    path = broken_setups(tmp_path)[name]
    with pytest.raises(IOError, match="Failed to parse trusted setup file"):
        kzg.parse_trusted_setup_file(path)


def test_invalid_length_g2_point():
    with pytest.raises(ValueError, match="Expected G2 point to be 96 bytes"):
        kzg.TrustedSetup([], [b""], [])


def test_flatten_limits():
    with pytest.raises(ValueError, match="Maximum of 100663296 bytes"):
        kzg._flatten([b""], 769 * kzg.BYTES_PER_BLOB)
    with pytest.raises(ValueError, match="was not the same"):
        kzg._flatten([b"\0" * 47], 48)


def declared_kzg_symbols():
    txt = open(os.path.join(ROOT, "include", "tekukzg.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tkzg_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_kzg_header():
    if not os.path.exists(native.LIB_PATH):
        import __graft_entry__ as ge

        ge.build_hip_lib()
    L = ctypes.CDLL(native.LIB_PATH)
    syms = declared_kzg_symbols()
    assert len(syms) >= 13
    assert not [s for s in syms if not hasattr(L, s)]
    assert set(syms) == set(kzg.EXPORTED)


def test_without_device_or_setup_fails_loudly():
    L = kzg.lib()
    ok = ctypes.c_int(7)
    rc = L.tkzg_verify_blob_kzg_proof_batch(ctypes.byref(ok), b"", 0, b"", 0, b"", 0, 0)
    assert rc == kzg.C_KZG_ERROR and ok.value == 7
    assert L.tkzg_last_error() == b"Trusted Setup is not loaded."
    if native.load_library().tbls_device_count() == 0:
        c = kzg.CKZG4844()
        with pytest.raises(kzg.KZGException):
            c.load_trusted_setup(SETUP)


def test_host_sha256_challenge_digest():
    """tb_sha256_host.h (the host-side Fiat-Shamir challenge hash of small
    host-API batches, tb_kzg.hip verify_host): SHA-NI and portable rounds vs
    hashlib at block-boundary lengths, and compute_challenge's transcript
    layout (FSBLOBVERIFY_V1_ || 4096 as 16 bytes BE || blob || commitment)."""
    import hashlib

    import __graft_entry__ as ge

    L = ctypes.CDLL(ge.build_hostsim())
    L.tbls_hostsim_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p]
    L.tbls_hostsim_kzg_digest.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p]
    rnd = __import__("random").Random(7)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 1000, 131152):
        d = bytes(rnd.getrandbits(8) for _ in range(n))
        for ni in (0, 1):
            out = ctypes.create_string_buffer(32)
            L.tbls_hostsim_sha256(d, len(d), ni, out)
            assert out.raw == hashlib.sha256(d).digest(), (n, ni)
    blob = bytes(rnd.getrandbits(8) for _ in range(131072))
    com = bytes(rnd.getrandbits(8) for _ in range(48))
    out = ctypes.create_string_buffer(32)
    L.tbls_hostsim_kzg_digest(blob, len(blob), com, out)
    assert out.raw == hashlib.sha256(b"FSBLOBVERIFY_V1_" + (4096).to_bytes(16, "big") + blob + com).digest()
