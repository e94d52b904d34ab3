"""EIP-4844 KZG on MI355X: the host-side mirror of the reference's KZG
interface over the C ABI of include/tekukzg.h.

Mirrors, name for name (snake_case) and with the same argument meaning and
error behaviour:
  KZG.java             the interface (loadTrustedSetup, freeTrustedSetup,
                       verifyBlobKzgProof, verifyBlobKzgProofBatch,
                       blobToKzgCommitment, computeBlobKzgProof)
  CKZG4844.java:40-150 the implementation: one trusted setup at a time, the
                       same file loaded twice is a no-op, another file frees
                       the current one first; every failure is a KZGException
                       whose cause is the native error
  CKZG4844Utils.java   flattening (MAX_BYTES_TO_FLATTEN) and the trusted-setup
                       text parser ("Failed to parse trusted setup file")
  TrustedSetup.java    point-size validation ("Expected G2 point to be 96 bytes")
Every computation runs in the HIP kernels of teku_amd/csrc/k_kzg.hip; with no
device the calls raise (no CPU fallback).
"""

import ctypes
import os
import threading

from . import native

BYTES_PER_G1 = 48
BYTES_PER_G2 = 96
FIELD_ELEMENTS_PER_BLOB = 4096
BYTES_PER_FIELD_ELEMENT = 32
BYTES_PER_BLOB = FIELD_ELEMENTS_PER_BLOB * BYTES_PER_FIELD_ELEMENT
BYTES_PER_COMMITMENT = BYTES_PER_PROOF = 48
BLS_MODULUS = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
MAX_BYTES_TO_FLATTEN = 100_663_296  # CKZG4844Utils.java:36 (768 blobs)
PRECOMPUTE_DEFAULT = 0

C_KZG_OK, C_KZG_BADARGS, C_KZG_ERROR, C_KZG_MALLOC = 0, 1, 2, 3
_ERROR_NAMES = {1: "C_KZG_BADARGS", 2: "C_KZG_ERROR", 3: "C_KZG_MALLOC"}

_u8p, _sz, _ip = ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)
_SIGS = {
    "tkzg_load_trusted_setup": (ctypes.c_int, [_u8p, _sz, _u8p, _sz, _u8p, _sz, ctypes.c_uint64]),
    "tkzg_free_trusted_setup": (ctypes.c_int, []),
    "tkzg_blob_to_kzg_commitment": (ctypes.c_int, [_u8p, _u8p, _sz]),
    "tkzg_blobs_to_kzg_commitments": (ctypes.c_int, [_u8p, _u8p, _sz, _sz]),
    "tkzg_compute_blob_kzg_proof": (ctypes.c_int, [_u8p, _u8p, _sz, _u8p]),
    "tkzg_verify_blob_kzg_proof": (ctypes.c_int, [_ip, _u8p, _sz, _u8p, _u8p]),
    "tkzg_verify_blob_kzg_proof_batch": (ctypes.c_int, [_ip, _u8p, _sz, _u8p, _sz, _u8p, _sz, _sz]),
    "tkzg_compute_kzg_proof": (ctypes.c_int, [_u8p, _u8p, _u8p, _sz, _u8p]),
    "tkzg_verify_kzg_proof": (ctypes.c_int, [_ip, _u8p, _u8p, _u8p, _u8p]),
    "tkzg_dev_verify_blob_kzg_proof_batch": (ctypes.c_int, [_ip, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p]),
    "tkzg_dev_verify_blob_kzg_proof_batch_profiled": (ctypes.c_int, [_ip, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p]),
    "tkzg_last_stage_ms": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float)]),
    "tkzg_last_transcript": (ctypes.c_int, [_u8p, _u8p, _sz, _u8p]),
    "tkzg_last_error": (ctypes.c_char_p, []),
}
EXPORTED = tuple(_SIGS)
STAGES = ("challenge", "eval", "points", "transcript_r", "terms", "pairing")

_lib = None
_lib_lock = threading.Lock()


def lib():
    global _lib
    with _lib_lock:
        if _lib is None:
            path = native.LIB_PATH
            if not os.path.exists(path):
                raise KZGException(f"Failed to load the KZG library: {path} not built (run __graft_entry__.build())")
            L = ctypes.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype, fn.argtypes = res, args
            _lib = L
        return _lib


class CKZGException(Exception):
    """The native error (c-kzg's C_KZG_RET plus the JNI wrapper's message)."""

    def __init__(self, error, message):
        self.error = error
        self.error_name = _ERROR_NAMES.get(error, str(error))
        self.error_message = message
        # the JNI wrapper reports argument errors as "<message> (C_KZG_BADARGS)";
        # "Trusted Setup is not loaded." comes through verbatim
        super().__init__(message if message.startswith("Trusted Setup is not loaded") else f"{message} ({self.error_name})")


class KZGException(Exception):
    pass


def _check(rc):
    if rc != C_KZG_OK:
        raise CKZGException(rc, lib().tkzg_last_error().decode(errors="replace"))


class TrustedSetup:
    """TrustedSetup.java:23-42: g1Lagrange, g2Monomial, g1Monomial, sizes validated."""

    def __init__(self, g1_lagrange, g2_monomial, g1_monomial):
        for p in g1_lagrange:
            if len(p) != BYTES_PER_G1:
                raise ValueError(f"Expected G1 point to be {BYTES_PER_G1} bytes")
        for p in g2_monomial:
            if len(p) != BYTES_PER_G2:
                raise ValueError(f"Expected G2 point to be {BYTES_PER_G2} bytes")
        for p in g1_monomial:
            if len(p) != BYTES_PER_G1:
                raise ValueError(f"Expected G1 point to be {BYTES_PER_G1} bytes")
        self.g1_lagrange, self.g2_monomial, self.g1_monomial = list(g1_lagrange), list(g2_monomial), list(g1_monomial)


def _hex_fixed(line, size):
    """Bytes.fromHexString(line, size): strict (even length, a line must be
    there: readLine() null at EOF fails), optional 0x, left-padded to size,
    error if longer."""
    if line == "":
        raise ValueError("unexpected end of file")
    s = line.strip()
    if s.startswith(("0x", "0X")):
        s = s[2:]
    if len(s) % 2:
        raise ValueError("odd-length hex string")
    b = bytes.fromhex(s)
    if len(b) > size:
        raise ValueError("hex longer than the expected size")
    return b.rjust(size, b"\0")


def parse_trusted_setup_file(trusted_setup_file):
    """CKZG4844Utils.parseTrustedSetupFile (CKZG4844Utils.java:62-100)."""
    if not os.path.exists(trusted_setup_file):
        raise FileNotFoundError(f"{trusted_setup_file} is not found")
    try:
        with open(trusted_setup_file, encoding="utf-8") as f:
            rd = f.readline
            g1_size = int(rd())
            g2_size = int(rd())
            g1_lagrange = [_hex_fixed(rd(), BYTES_PER_G1) for _ in range(g1_size)]
            g2_monomial = [_hex_fixed(rd(), BYTES_PER_G2) for _ in range(g2_size)]
            g1_monomial = [_hex_fixed(rd(), BYTES_PER_G1) for _ in range(g1_size)]
        return TrustedSetup(g1_lagrange, g2_monomial, g1_monomial)
    except Exception as ex:
        raise IOError(f"Failed to parse trusted setup file\n: {trusted_setup_file}") from ex


def _flatten(items, expected):
    """CKZG4844Utils.flattenBytes (CKZG4844Utils.java:102-127)."""
    if expected > MAX_BYTES_TO_FLATTEN:
        raise ValueError(f"Maximum of {MAX_BYTES_TO_FLATTEN} bytes can be flattened, but {expected} were requested")
    out = b"".join(bytes(x) for x in items)
    if len(out) != expected:
        raise ValueError(f"The actual bytes to flatten ({len(out)}) was not the same as the expected size specified ({expected})")
    return out


class CKZG4844:
    """CKZG4844.java: the KZG implementation, one instance per process."""

    _instance = None
    _instance_lock = threading.Lock()

    @classmethod
    def get_instance(cls):
        with cls._instance_lock:
            if cls._instance is None:
                cls._instance = cls()
            return cls._instance

    def __init__(self):
        try:
            lib()
        except Exception as ex:
            raise KZGException("Failed to load C-KZG-4844 library") from ex
        self._loaded_file = None
        self._lock = threading.RLock()

    # -- trusted setup --------------------------------------------------------
    def load_trusted_setup(self, trusted_setup_file):
        with self._lock:
            if self._loaded_file is not None and self._loaded_file == trusted_setup_file:
                return
            try:
                if self._loaded_file is not None:
                    self.free_trusted_setup()
                ts = parse_trusted_setup_file(trusted_setup_file)
                g1l = _flatten(ts.g1_lagrange, BYTES_PER_G1 * len(ts.g1_lagrange))
                g2m = _flatten(ts.g2_monomial, BYTES_PER_G2 * len(ts.g2_monomial))
                g1m = _flatten(ts.g1_monomial, BYTES_PER_G1 * len(ts.g1_monomial))
                _check(lib().tkzg_load_trusted_setup(g1m, len(g1m), g1l, len(g1l), g2m, len(g2m), PRECOMPUTE_DEFAULT))
                self._loaded_file = trusted_setup_file
            except Exception as ex:
                raise KZGException(f"Failed to load trusted setup from {trusted_setup_file}") from ex

    def free_trusted_setup(self):
        with self._lock:
            try:
                _check(lib().tkzg_free_trusted_setup())
                self._loaded_file = None
            except Exception as ex:
                raise KZGException("Failed to free trusted setup") from ex

    # -- the four operations --------------------------------------------------
    def verify_blob_kzg_proof(self, blob, kzg_commitment, kzg_proof):
        try:
            ok = ctypes.c_int(0)
            blob = bytes(blob)
            _check(lib().tkzg_verify_blob_kzg_proof(ctypes.byref(ok), blob, len(blob), _b48(kzg_commitment), _b48(kzg_proof)))
            return bool(ok.value)
        except Exception as ex:
            raise KZGException(f"Failed to verify blob and commitment against KZG proof {bytes(kzg_proof).hex()}") from ex

    def verify_blob_kzg_proof_batch(self, blobs, kzg_commitments, kzg_proofs):
        try:
            b = _flatten(blobs, BYTES_PER_BLOB * len(blobs))
            c = _flatten(kzg_commitments, BYTES_PER_COMMITMENT * len(kzg_commitments))
            p = _flatten(kzg_proofs, BYTES_PER_PROOF * len(kzg_proofs))
            ok = ctypes.c_int(0)
            _check(lib().tkzg_verify_blob_kzg_proof_batch(ctypes.byref(ok), b, len(b), c, len(c), p, len(p), len(blobs)))
            return bool(ok.value)
        except Exception as ex:
            raise KZGException(f"Failed to verify blobs and commitments against KZG proofs {[bytes(x).hex() for x in kzg_proofs]}") from ex

    def blob_to_kzg_commitment(self, blob):
        try:
            out = ctypes.create_string_buffer(48)
            blob = bytes(blob)
            _check(lib().tkzg_blob_to_kzg_commitment(out, blob, len(blob)))
            return out.raw
        except Exception as ex:
            raise KZGException("Failed to produce KZG commitment from blob") from ex

    def compute_blob_kzg_proof(self, blob, kzg_commitment):
        try:
            out = ctypes.create_string_buffer(48)
            blob = bytes(blob)
            _check(lib().tkzg_compute_blob_kzg_proof(out, blob, len(blob), _b48(kzg_commitment)))
            return out.raw
        except Exception as ex:
            raise KZGException(f"Failed to compute KZG proof for blob with commitment {bytes(kzg_commitment).hex()}") from ex

    # -- beyond the interface: batched commitments, explicit-z proofs ---------
    def blobs_to_kzg_commitments(self, blobs):
        out = ctypes.create_string_buffer(48 * max(len(blobs), 1))
        b = b"".join(bytes(x) for x in blobs)
        _check(lib().tkzg_blobs_to_kzg_commitments(out, b, len(b), len(blobs)))
        return [out.raw[48 * i:48 * i + 48] for i in range(len(blobs))]

    def compute_kzg_proof(self, blob, z):
        p, y = ctypes.create_string_buffer(48), ctypes.create_string_buffer(32)
        blob = bytes(blob)
        _check(lib().tkzg_compute_kzg_proof(p, y, blob, len(blob), bytes(z)))
        return p.raw, y.raw

    def verify_kzg_proof(self, commitment, z, y, proof):
        ok = ctypes.c_int(0)
        _check(lib().tkzg_verify_kzg_proof(ctypes.byref(ok), _b48(commitment), bytes(z), bytes(y), _b48(proof)))
        return bool(ok.value)

    def last_transcript(self, n):
        """(zs, ys, r) of the last verify of n blobs, 32-byte big-endian each (test hook)."""
        zs, ys, r = ctypes.create_string_buffer(32 * n), ctypes.create_string_buffer(32 * n), ctypes.create_string_buffer(32)
        _check(lib().tkzg_last_transcript(zs, ys, n, r))
        return [zs.raw[32 * i:32 * i + 32] for i in range(n)], [ys.raw[32 * i:32 * i + 32] for i in range(n)], r.raw


def _b48(x):
    b = bytes(x)
    if len(b) != 48:
        raise CKZGException(C_KZG_BADARGS, f"Invalid point size. Expected 48 bytes but got {len(b)}.")
    return b


KZG = CKZG4844  # KZG.getInstance() -> CKZG4844.getInstance() (KZG.java)
