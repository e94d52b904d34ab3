"""The C-ABI set array the Python binding hands to tbls_batch_verify /
tbls_batch_verify_each (teku_amd/synth.py SetArray): every tbls_set entry
points into the caller's blobs in place (no copy since round 5) with the
right key count, message span and signature -- checked by reading the
memory back through the pointers, no device needed.  Also the facade's
marshalling of fresh value objects (teku_amd/bls.py _hip_facade_batch, the
C-level map / join) reaching the same array."""

import ctypes
import os

import numpy as np

from teku_amd import bls, native, synth


def _read(arr):
    out = []
    for i in range(arr.n):
        s = arr.ptr[i]
        out.append((ctypes.string_at(s.pks, 48 * s.n_pks), s.n_pks, ctypes.string_at(s.msg, s.msg_len), ctypes.string_at(s.sig, 96)))
    return out


def test_setarray_points_into_blobs():
    rng = np.random.default_rng(3)
    n_pks = [1, 3, 0, 2, 1]
    lens = [32, 0, 7, 200, 1]
    pks = [bytes(rng.integers(0, 256, 48 * k, dtype=np.uint8)) for k in n_pks]
    msgs = [bytes(rng.integers(0, 256, m, dtype=np.uint8)) for m in lens]
    sigs = [bytes(rng.integers(0, 256, 96, dtype=np.uint8)) for _ in n_pks]
    arr = synth.SetArray(b"".join(pks), n_pks, b"".join(msgs), lens, b"".join(sigs))
    assert arr.n == len(n_pks)
    assert _read(arr) == [(pks[i], n_pks[i], msgs[i], sigs[i]) for i in range(len(n_pks))]
    # numpy length arrays (the facade's form) give the same entries
    arr2 = synth.SetArray(b"".join(pks), np.asarray(n_pks, dtype=np.uint64), b"".join(msgs), np.asarray(lens, dtype=np.uint64),
                          b"".join(sigs))
    assert _read(arr2) == _read(arr)


def test_setarray_empty():
    arr = synth.SetArray(b"", [], b"", [], b"")
    assert arr.n == 0


def test_facade_marshalling(monkeypatch):
    """BLS.batch_verify on HipBLS12381 with fresh objects builds one set
    array holding every object's bytes in order (the device call replaced by
    a recorder)."""
    seen = {}

    def fake_batch_verify(self, rands, n_gpus=0, timing=None):
        seen["sets"] = _read(self)
        seen["rands"] = len(rands)
        return True

    monkeypatch.setattr(synth.SetArray, "batch_verify", fake_batch_verify)
    impl = bls.HipBLS12381.__new__(bls.HipBLS12381)  # no device: the facade only marshals here
    impl.eager = False
    impl.n_gpus = 0
    prev = bls.BLS._impl  # not get_bls_impl(): that initialises the device
    bls.BLS.set_bls_implementation(impl)
    try:
        n = 37
        pk = [os.urandom(48) for _ in range(n)]
        sg = [os.urandom(96) for _ in range(n)]
        ms = [os.urandom(32) for _ in range(n)]
        keys = [[bls.BLSPublicKey.from_bytes_compressed(p)] for p in pk]
        so = [bls.BLSSignature.from_bytes_compressed(s) for s in sg]
        assert bls.BLS.batch_verify(keys, ms, so) is True
        assert seen["rands"] == n
        assert seen["sets"] == [(pk[i], 1, ms[i], sg[i]) for i in range(n)]
        # multi-key sets and bytearray messages take the general path
        keys2 = [[bls.BLSPublicKey.from_bytes_compressed(p) for p in pk[i : i + 2]] for i in range(0, 6, 2)]
        ms2 = [bytearray(m) for m in ms[:3]]
        assert bls.BLS.batch_verify(keys2, ms2, so[:3]) is True
        assert seen["sets"] == [(pk[2 * i] + pk[2 * i + 1], 2, ms[i], sg[i]) for i in range(3)]
    finally:
        bls.BLS._impl = prev
    assert native.PARTIAL_BYTES > 0
