"""ctypes binding of the C KZG oracle (oracle/c/kzg_oracle.c).  TEST
INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the teku_amd product path.

The trusted-setup text parser here restates CKZG4844Utils.parseTrustedSetupFile
(infrastructure/kzg/src/main/java/tech/pegasys/teku/kzg/CKZG4844Utils.java:62-100)
for the oracle's own use; the product-side parser is teku_amd/kzg.py."""

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "c", "_build", "libkzg_oracle.so")
FIELD_ELEMENTS_PER_BLOB = 4096
BYTES_PER_BLOB = 32 * FIELD_ELEMENTS_PER_BLOB
BLS_MODULUS = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
KZG_OK, KZG_BADARGS = 0, 1
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("KZG oracle not built: make -C oracle/c")
        L = ctypes.CDLL(LIB_PATH)
        cp, sz, vp, ip = ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
        L.orc_kzg_load_setup.argtypes = [cp, cp, sz, cp, sz]
        L.orc_kzg_load_setup.restype = vp
        L.orc_kzg_free_setup.argtypes = [vp]
        L.orc_kzg_free_setup.restype = None
        L.orc_kzg_monomial.argtypes = [vp, ctypes.c_int, cp]
        L.orc_kzg_monomial.restype = None
        L.orc_kzg_g2_gen.argtypes = [cp]
        L.orc_kzg_g2_gen.restype = None
        L.orc_kzg_roots_brp.argtypes = [cp]
        L.orc_kzg_roots_brp.restype = None
        L.orc_kzg_blob_to_commitment.argtypes = [vp, cp, cp]
        L.orc_kzg_compute_blob_proof.argtypes = [vp, cp, cp, cp]
        L.orc_kzg_compute_proof.argtypes = [vp, cp, cp, cp, cp]
        L.orc_kzg_verify_proof.argtypes = [vp, cp, cp, cp, cp, ip]
        L.orc_kzg_verify_blob_proof.argtypes = [vp, cp, cp, cp, ip]
        L.orc_kzg_verify_blob_proof_batch.argtypes = [vp, cp, cp, cp, sz, ip, cp, cp, cp]
        _lib = L
    return _lib


def parse_setup_text(path):
    """(g1_lagrange, g2_monomial, g1_monomial) byte strings of a trusted_setup.txt."""
    with open(path) as f:
        n1, n2 = int(f.readline()), int(f.readline())
        rd = lambda k, size: b"".join(bytes.fromhex(f.readline().strip()).rjust(size, b"\0") for _ in range(k))  # noqa: E731
        g1l = rd(n1, 48)
        g2m = rd(n2, 96)
        g1m = rd(n1, 48)
    return g1l, g2m, g1m


class Setup:
    def __init__(self, g1_lagrange, g2_monomial, g1_monomial):
        n1, n2 = len(g1_lagrange) // 48, len(g2_monomial) // 96
        self.h = lib().orc_kzg_load_setup(g1_lagrange, g1_monomial, n1, g2_monomial, n2)
        if not self.h:
            raise ValueError("oracle: bad trusted setup")

    @classmethod
    def from_file(cls, path):
        return cls(*parse_setup_text(path))

    def close(self):
        if self.h:
            lib().orc_kzg_free_setup(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def monomial(self, k):
        out = ctypes.create_string_buffer(48)
        lib().orc_kzg_monomial(self.h, k, out)
        return out.raw

    def blob_to_kzg_commitment(self, blob):
        out = ctypes.create_string_buffer(48)
        rc = lib().orc_kzg_blob_to_commitment(self.h, blob, out)
        return out.raw if rc == KZG_OK else rc

    def compute_blob_kzg_proof(self, blob, commitment):
        out = ctypes.create_string_buffer(48)
        rc = lib().orc_kzg_compute_blob_proof(self.h, blob, commitment, out)
        return out.raw if rc == KZG_OK else rc

    def compute_kzg_proof(self, blob, z):
        p, y = ctypes.create_string_buffer(48), ctypes.create_string_buffer(32)
        rc = lib().orc_kzg_compute_proof(self.h, blob, z, p, y)
        return (p.raw, y.raw) if rc == KZG_OK else rc

    def verify_kzg_proof(self, commitment, z, y, proof):
        ok = ctypes.c_int(0)
        rc = lib().orc_kzg_verify_proof(self.h, commitment, z, y, proof, ctypes.byref(ok))
        return bool(ok.value) if rc == KZG_OK else rc

    def verify_blob_kzg_proof(self, blob, commitment, proof):
        ok = ctypes.c_int(0)
        rc = lib().orc_kzg_verify_blob_proof(self.h, blob, commitment, proof, ctypes.byref(ok))
        return bool(ok.value) if rc == KZG_OK else rc

    def verify_blob_kzg_proof_batch(self, blobs, commitments, proofs, detail=False):
        """-> bool (or the error code); with detail=True also (zs, ys, r) bytes."""
        n = len(blobs)
        ok = ctypes.c_int(0)
        zs, ys, r = ctypes.create_string_buffer(32 * max(n, 1)), ctypes.create_string_buffer(32 * max(n, 1)), ctypes.create_string_buffer(32)
        rc = lib().orc_kzg_verify_blob_proof_batch(self.h, b"".join(blobs), b"".join(commitments), b"".join(proofs), n, ctypes.byref(ok), zs, ys, r)
        res = bool(ok.value) if rc == KZG_OK else rc
        if detail:
            return res, [zs.raw[32 * i:32 * i + 32] for i in range(n)], [ys.raw[32 * i:32 * i + 32] for i in range(n)], r.raw
        return res


def g2_generator():
    out = ctypes.create_string_buffer(96)
    lib().orc_kzg_g2_gen(out)
    return out.raw


def roots_brp():
    out = ctypes.create_string_buffer(32 * FIELD_ELEMENTS_PER_BLOB)
    lib().orc_kzg_roots_brp(out)
    return [int.from_bytes(out.raw[32 * i:32 * i + 32], "big") for i in range(FIELD_ELEMENTS_PER_BLOB)]
