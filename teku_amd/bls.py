"""Host-side mirror of Teku's BLS SPI and facade, backed by libtekubls_hip.so.

Mirrors (same names in snake_case, same argument meaning, same error
behaviour):

* ``tech.pegasys.teku.bls.impl.BLS12381`` (impl/BLS12381.java:34-157)
  -> :class:`HipBLS12381`, with the value types ``HipPublicKey``,
  ``HipSignature``, ``HipSecretKey`` and the opaque ``HipSemiAggregate``;
  the drop-in sibling of ``BlstBLS12381`` (impl/blst/BlstBLS12381.java).
* ``tech.pegasys.teku.bls.BLS`` (BLS.java:40-458) -> :class:`BLS`, and the
  wrappers ``BLSPublicKey`` / ``BLSSignature`` / ``BLSSecretKey`` with their
  lazy, memoised decoding (BLSPublicKey.java:116-120, BLSSignature.java:83-87).
* ``BlsException extends IllegalArgumentException`` (impl/BlsException.java:16)
  -> :class:`BlsException` (a ``ValueError``).

Deferred work: ``prepare_batch_verify`` captures the set and
does only cheap checks; all curve work happens in ``complete_batch_verify``,
which runs one GPU batch.  The boolean results are identical to blst's
(an invalid or throwing prepare also ends in ``False`` there).  Pass
``eager=True`` to :class:`HipBLS12381` to run the G2 group check inside
prepare as ``BlstTest.succeedsWhenPrepareBatchVerifyNotInG2ThrowsException``
(BlstTest.java:93-103) expects.
"""

from __future__ import annotations

import ctypes
import hashlib
import hmac
import operator
import secrets
import threading
from typing import List, Optional, Sequence

import numpy as np

from . import native

ETH2_DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"  # HashToCurve.java:22
CURVE_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001  # BLSConstants.java:25-28
INFINITY_G1 = bytes([0xC0]) + bytes(47)
INFINITY_G2 = bytes([0xC0]) + bytes(95)
BATCH_RANDOM_BYTES = 8  # BlstBLS12381.java:39


class BlsException(ValueError):
    """tech.pegasys.teku.bls.impl.BlsException (an IllegalArgumentException)."""


def _dst(dst) -> bytes:
    if dst is None:
        return ETH2_DST
    if isinstance(dst, str):
        dst = dst.encode()
    if len(dst) > 255:  # RFC 9380 §5.3.3 oversize DST
        dst = hashlib.sha256(b"H2C-OVERSIZE-DST-" + dst).digest()
    return bytes(dst)


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), max(1, len(b)))


# ---------------------------------------------------------------------------
# SPI value types
# ---------------------------------------------------------------------------
def java_bytes_hash(b: bytes) -> int:
    """tuweni Bytes.hashCode (31 * h + signed byte, int32): the hash BlstPublicKey
    / BlstSignature return (BlstPublicKey.java:115-118, BlstSignature.java:152-155)."""
    h = 1
    for x in b:
        h = (31 * h + (x - 256 if x > 127 else x)) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


class PublicKey:
    """impl/PublicKey.java:20-82: the SPI interface every implementation's key
    type implements (a foreign implementation's key subclasses or registers)."""

    __slots__ = ()

    def to_bytes_compressed(self) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError

    # BlstPublicKey.java:115-130: equal to ANY PublicKey with the same
    # compressed bytes; the compressed bytes' hash
    def __eq__(self, o):
        if self is o:
            return True
        return isinstance(o, PublicKey) and self.to_bytes_compressed() == o.to_bytes_compressed()

    def __hash__(self):
        return java_bytes_hash(self.to_bytes_compressed())

    def hash_code(self) -> int:
        return java_bytes_hash(self.to_bytes_compressed())


class Signature:
    """impl/Signature.java:20-91: the SPI interface of signatures."""

    __slots__ = ()

    def to_bytes_compressed(self) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError

    # BlstSignature.java:152-165
    def __eq__(self, o):
        if self is o:
            return True
        return isinstance(o, Signature) and self.to_bytes_compressed() == o.to_bytes_compressed()

    def __hash__(self):
        return java_bytes_hash(self.to_bytes_compressed())

    def hash_code(self) -> int:
        return java_bytes_hash(self.to_bytes_compressed())


def _decode_failed(what: str, b: bytes) -> BlsException:
    return BlsException(f"Deserialization of {what} bytes failed: 0x" + bytes(b).hex())


class HipPublicKey(PublicKey):
    """impl/PublicKey.java:20-82 (BlstPublicKey.java analogue).  Holds the
    compressed bytes.  from_bytes decodes on the host (tbls_pk_decode: flags,
    x < p, on the curve, x != 0 -- blst_p1_uncompress's contract, no device
    call); validity (!infinity && in G1) is computed on the GPU when first
    asked and memoised (BlstPublicKey.java:74-75)."""

    __slots__ = ("_b", "_valid", "_inf")

    def __init__(self, compressed: bytes, _checked_code: Optional[int] = None):
        self._b = bytes(compressed)
        self._valid = None if _checked_code is None else (_checked_code == native.SUCCESS)
        self._inf = self._b == INFINITY_G1

    @staticmethod
    def from_bytes(compressed: bytes) -> "HipPublicKey":
        # BlstPublicKey.fromBytes: decode failures throw (l.38-45)
        if len(compressed) != 48:
            raise BlsException("Deserialization of public key bytes failed")
        b = bytes(compressed)
        if native.host().tbls_pk_decode(b, None) != native.SUCCESS:
            raise _decode_failed("public key", b)
        return HipPublicKey(b)

    def to_bytes_compressed(self) -> bytes:
        return self._b

    def is_infinity(self) -> bool:
        return self._inf

    def is_valid(self) -> bool:
        if self._valid is None:
            rc = native.lib().tbls_pk_validate(self._b)
            if rc == native.DEVICE_ERROR:
                raise native.NativeError(rc, "tbls_pk_validate")
            self._valid = rc == native.SUCCESS
        return self._valid

    def is_in_group(self) -> bool:
        return self._inf or self.is_valid()

    def force_validation(self):
        if not self.is_valid():
            raise BlsException("Invalid PublicKey: 0x" + self._b.hex())

    def verify_signature(self, signature: "HipSignature", message: bytes) -> bool:
        return signature.verify(self, message)



class HipSignature(Signature):
    """impl/Signature.java:20-91 (BlstSignature.java analogue).  from_bytes
    decodes on the host (tbls_sig_decode: blst_p2_uncompress's contract, no
    device call); the G2 subgroup check runs on the GPU when first asked
    (is_in_group, memoised) or inside the batch."""

    __slots__ = ("_b", "_in_group")

    def __init__(self, compressed: bytes):
        self._b = bytes(compressed)
        self._in_group = None

    @staticmethod
    def from_bytes(compressed: bytes) -> "HipSignature":
        # BlstSignature.fromBytes: size check + decode, failures -> BlsException (l.35-47)
        if len(compressed) != 96:
            raise BlsException(f"Expected 96 bytes of input but got {len(compressed)}")
        b = bytes(compressed)
        if native.host().tbls_sig_decode(b, None) != native.SUCCESS:
            raise _decode_failed("signature", b)
        return HipSignature(b)

    def to_bytes_compressed(self) -> bytes:
        return self._b

    def is_infinity(self) -> bool:
        return self._b == INFINITY_G2

    def is_in_group(self) -> bool:
        # BlstSignature.isInGroup (l.147-149): ec2Point.in_group(); the infinity
        # point is in the group
        if self._in_group is None:
            if self.is_infinity():
                self._in_group = True
            else:
                rc = native.lib().tbls_sig_validate(self._b, None)
                if rc == native.DEVICE_ERROR:
                    raise native.NativeError(rc, "tbls_sig_validate")
                self._in_group = rc == native.SUCCESS
        return self._in_group

    # Signature.verify overloads (Signature.java:36-68)
    def verify(self, public_key_or_keys, message: bytes = None, dst=None) -> bool:
        if isinstance(public_key_or_keys, list) and message is None:
            return self.verify_pairs(public_key_or_keys)
        if isinstance(public_key_or_keys, (list, tuple)):
            agg = HipBLS12381.aggregate_public_keys_static(public_key_or_keys)
            return self._core_verify(agg, message, dst)
        return self._core_verify(public_key_or_keys, message, dst)

    def _core_verify(self, pk: "HipPublicKey", message: bytes, dst=None) -> bool:
        ok = ctypes.c_int(0)
        d = _dst(dst)
        m = bytes(message)
        rc = native.lib().tbls_verify(pk.to_bytes_compressed(), _buf(m), len(m), self._b, d, len(d), ctypes.byref(ok))
        if rc == native.DEVICE_ERROR:
            raise native.NativeError(rc, "tbls_verify")
        return rc == native.SUCCESS and ok.value == 1

    def verify_pairs(self, pairs) -> bool:
        """aggregateVerify over (public key, message) pairs (BlstSignature.java:104-122)."""
        if any(pk.is_infinity() for pk, _ in pairs):
            return False
        n = len(pairs)
        pks = b"".join(pk.to_bytes_compressed() for pk, _ in pairs)
        msgs = [bytes(m) for _, m in pairs]
        arr = (ctypes.c_char_p * n)(*[_buf(m).raw for m in msgs])
        lens = (ctypes.c_uint32 * n)(*[len(m) for m in msgs])
        ok = ctypes.c_int(0)
        rc = native.lib().tbls_aggregate_verify(pks, arr, lens, n, self._b, ctypes.byref(ok))
        if rc == native.DEVICE_ERROR:
            raise native.NativeError(rc, "tbls_aggregate_verify")
        return rc == native.SUCCESS and ok.value == 1



class HipSecretKey:
    """impl/SecretKey.java:20-59 (BlstSecretKey.java analogue)."""

    __slots__ = ("_k",)

    def __init__(self, k: int):
        self._k = k % CURVE_ORDER

    def to_bytes(self) -> bytes:
        return self._k.to_bytes(32, "big")

    def is_zero(self) -> bool:
        return self._k == 0

    def derive_public_key(self) -> HipPublicKey:
        out = ctypes.create_string_buffer(48)
        native.check(native.lib().tbls_sk_to_pk(self.to_bytes(), out), "tbls_sk_to_pk")
        return HipPublicKey(out.raw)

    def sign(self, message: bytes, dst=None) -> HipSignature:
        if self.is_zero():  # BlstBLS12381.java:54-56
            raise ValueError("Signing with zero private key is prohibited")
        d = _dst(dst)
        m = bytes(message)
        out = ctypes.create_string_buffer(96)
        native.check(native.lib().tbls_sign(self.to_bytes(), _buf(m), len(m), d, len(d), out), "tbls_sign")
        return HipSignature(out.raw)

    def destroy(self):
        self._k = 0


class KeyPair:
    def __init__(self, secret_key: HipSecretKey):
        self.secret_key = secret_key
        self.public_key = secret_key.derive_public_key()


class HipSemiAggregate:
    """Opaque BatchSemiAggregate (bls/BatchSemiAggregate.java:16): the captured
    sets; the pairing work is deferred to complete_batch_verify."""

    __slots__ = ("sets", "valid")

    def __init__(self, sets, valid=True):
        self.sets = sets  # list of (pk_bytes_concat, n_pks, msg, sig_bytes)
        self.valid = valid

    def merge_with(self, other: "HipSemiAggregate"):
        self.sets.extend(other.sets)
        self.valid = self.valid and other.valid


def _keygen_ikm(ikm: bytes) -> int:
    """KeyGen (draft-irtf-cfrg-bls-signature-04 §2.3) as used by
    BlstSecretKey.generateNew (BlstSecretKey.java:41-47).  Host-side; not on
    the verification path."""
    salt = b"BLS-SIG-KEYGEN-SALT-"
    sk = 0
    while sk == 0:
        salt = hashlib.sha256(salt).digest()
        prk = hmac.new(salt, ikm + b"\x00", hashlib.sha256).digest()
        okm, t = b"", b""
        i = 1
        while len(okm) < 48:
            t = hmac.new(prk, t + (48).to_bytes(2, "big") + bytes([i]), hashlib.sha256).digest()
            okm += t
            i += 1
        sk = int.from_bytes(okm[:48], "big") % CURVE_ORDER
    return sk


class HipBLS12381:
    """impl/BLS12381.java:34-157 on libtekubls_hip.so."""

    def __init__(self, eager: bool = False, n_gpus: int = 0, rng=None):
        self.eager = eager
        self.n_gpus = n_gpus
        self._rng = rng or secrets.SystemRandom()  # BlstBLS12381.java:42 (SecureRandom)
        self._rng_lock = threading.Lock()
        native.lib()

    # -- keys -------------------------------------------------------------
    def generate_key_pair(self, random_or_seed) -> KeyPair:
        if isinstance(random_or_seed, int):
            from random import Random  # BLS12381.java:54-56 default(seed)

            random_or_seed = Random(random_or_seed)
        ikm = bytes(random_or_seed.getrandbits(8) for _ in range(128))
        return KeyPair(HipSecretKey(_keygen_ikm(ikm)))

    def public_key_from_compressed(self, b48: bytes) -> HipPublicKey:
        return HipPublicKey.from_bytes(b48)

    def signature_from_compressed(self, b: bytes) -> HipSignature:
        return HipSignature.from_bytes(b)

    def secret_key_from_bytes(self, b32: bytes) -> HipSecretKey:
        return HipSecretKey(int.from_bytes(bytes(b32), "big"))

    # -- aggregation ------------------------------------------------------
    @staticmethod
    def aggregate_public_keys_static(public_keys: Sequence[HipPublicKey]) -> HipPublicKey:
        if len(public_keys) == 0:  # checkArgument (BlstPublicKey.java:56)
            raise ValueError("empty public key list")
        blob = b"".join(_as_pk(pk).to_bytes_compressed() for pk in public_keys)
        out = ctypes.create_string_buffer(48)
        rc = native.lib().tbls_aggregate_pks(blob, len(public_keys), out)
        if rc in (native.BAD_ENCODING, native.POINT_NOT_ON_CURVE):
            raise BlsException("Deserialization of public key bytes failed")
        native.check(rc, "tbls_aggregate_pks")
        return HipPublicKey(out.raw)

    def aggregate_public_keys(self, public_keys) -> HipPublicKey:
        return self.aggregate_public_keys_static(public_keys)

    def aggregate_signatures(self, signatures) -> HipSignature:
        blob = b"".join(_as_sig(s).to_bytes_compressed() for s in signatures)
        out = ctypes.create_string_buffer(96)
        rc = native.lib().tbls_aggregate_sigs(_buf(blob), len(signatures), out)
        if rc == native.DEVICE_ERROR:
            raise native.NativeError(rc, "tbls_aggregate_sigs")
        if rc != native.SUCCESS:  # BlstSignature.java:64-67
            raise BlsException("Failed to aggregate signatures")
        return HipSignature(out.raw)

    # -- batch verification ------------------------------------------------
    def prepare_batch_verify(self, index: int, public_keys, message: bytes, signature) -> HipSemiAggregate:
        pks = [_as_pk(pk) for pk in public_keys]
        if len(pks) == 0:
            raise ValueError("empty public key list")  # checkArgument, not a BlsException
        sig = _as_sig(signature)
        if self.eager and not sig.is_infinity() and not sig.is_in_group():
            raise BlsException("Error in Blst, error code: BLST_POINT_NOT_IN_GROUP")
        blob = b"".join(pk.to_bytes_compressed() for pk in pks)
        return HipSemiAggregate([(blob, len(pks), bytes(message), sig.to_bytes_compressed())])

    def prepare_batch_verify2(self, index, public_keys1, message1, signature1, public_keys2, message2, signature2):
        a = self.prepare_batch_verify(index, public_keys1, message1, signature1)
        a.merge_with(self.prepare_batch_verify(index + 1, public_keys2, message2, signature2))
        return a

    def next_batch_random_multiplier(self) -> int:
        """BlstBLS12381.nextBatchRandomMultiplier (l.191-195): 8 random bytes + 1.
        The value 2^64 (probability 2^-64) is redrawn to fit the u64 ABI."""
        with self._rng_lock:
            while True:
                r = int.from_bytes(bytes(self._rng.getrandbits(8) for _ in range(BATCH_RANDOM_BYTES)), "big") + 1
                if r < (1 << 64):
                    return r

    def complete_batch_verify(self, prepared_list) -> bool:
        if len(prepared_list) == 0:  # BlstBLS12381.java:163-165
            return True
        sets = []
        for p in prepared_list:
            if not isinstance(p, HipSemiAggregate) or not p.valid:  # l.169-177, 185-188
                return False
            sets.extend(p.sets)
        rands = [self.next_batch_random_multiplier() for _ in sets]
        return batch_verify_raw(sets, rands, self.n_gpus)

    def random_signature(self, seed: int) -> HipSignature:
        return self.generate_key_pair(seed).secret_key.sign(b"Hello, world!")


def batch_verify_raw(sets, rands, n_gpus=0, timing=None) -> bool:
    """One tbls_batch_verify over [(pk_blob, n_pks, msg, sig96)] with randomizers."""
    n = len(sets)
    arr = (native.TblsSet * n)()
    keep = []
    for i, (blob, npk, msg, sig) in enumerate(sets):
        bb, mb, sb = _buf(blob), _buf(msg), _buf(sig)
        keep += [bb, mb, sb]
        arr[i].pks = ctypes.cast(bb, ctypes.c_void_p)
        arr[i].n_pks = npk
        arr[i].msg = ctypes.cast(mb, ctypes.c_void_p)
        arr[i].msg_len = len(msg)
        arr[i].sig = ctypes.cast(sb, ctypes.c_void_p)
    rr = (ctypes.c_uint64 * max(1, n))(*rands)
    ok = ctypes.c_int(0)
    t = native.TblsTiming()
    rc = native.lib().tbls_batch_verify(arr, n, rr, n_gpus, ctypes.byref(ok), ctypes.byref(t))
    if rc == native.BAD_ARGUMENT:
        raise ValueError("empty public key list in batch")
    native.check(rc, "tbls_batch_verify")
    if timing is not None:
        timing.update(total_ms=t.total_ms, device_ms=t.device_ms, n_devices=t.n_devices)
    return ok.value == 1


def verify_each_raw(sets, n_gpus=0) -> List[bool]:
    """Per-set fastAggregateVerify verdicts of [(pk_blob, n_pks, msg, sig96)]
    in one device pass (tbls_verify_each)."""
    n = len(sets)
    if n == 0:
        return []
    arr = (native.TblsSet * n)()
    keep = []
    for i, (blob, npk, msg, sig) in enumerate(sets):
        bb, mb, sb = _buf(blob), _buf(msg), _buf(sig)
        keep += [bb, mb, sb]
        arr[i].pks = ctypes.cast(bb, ctypes.c_void_p)
        arr[i].n_pks = npk
        arr[i].msg = ctypes.cast(mb, ctypes.c_void_p)
        arr[i].msg_len = len(msg)
        arr[i].sig = ctypes.cast(sb, ctypes.c_void_p)
    ok = (ctypes.c_int * n)()
    native.check(native.lib().tbls_verify_each(arr, n, n_gpus, ok), "tbls_verify_each")
    return [v == 1 for v in ok]


def validate_public_keys(pks) -> List[int]:
    """Per-key status (0 = valid; else as tbls_pk_validate) of 48-byte keys in
    one device pass (tbls_pk_validate_many)."""
    n = len(pks)
    if n == 0:
        return []
    codes = ctypes.create_string_buffer(n)
    native.check(native.lib().tbls_pk_validate_many(b"".join(bytes(p) for p in pks), n, codes), "tbls_pk_validate_many")
    return list(codes.raw[:n])


def validate_signatures(sigs):
    """(codes, is_infinity) of 96-byte signatures in one device pass
    (tbls_sig_validate_many): decode + G2 check, as tbls_sig_validate."""
    n = len(sigs)
    if n == 0:
        return [], []
    codes, inf = ctypes.create_string_buffer(n), ctypes.create_string_buffer(n)
    native.check(native.lib().tbls_sig_validate_many(b"".join(bytes(s) for s in sigs), n, codes, inf), "tbls_sig_validate_many")
    return list(codes.raw[:n]), [b == 1 for b in inf.raw[:n]]


def aggregate_signature_groups(groups):
    """BlstSignature.aggregate (BlstSignature.java:57-68) over many groups of
    96-byte signatures in one device pass (tbls_aggregate_sigs_many).  Returns
    per group the 96-byte aggregate, or a BlsException for a group holding an
    undecodable / non-G2 signature."""
    G = len(groups)
    if G == 0:
        return []
    off = [0]
    for g in groups:
        off.append(off[-1] + len(g))
    offs = (ctypes.c_uint32 * (G + 1))(*off)
    out = ctypes.create_string_buffer(96 * G)
    status = (ctypes.c_int * G)()
    blob = b"".join(bytes(s) for g in groups for s in g) or b"\0"
    native.check(native.lib().tbls_aggregate_sigs_many(blob, offs, G, out, status), "tbls_aggregate_sigs_many")
    return [
        BlsException(f"Failed to aggregate signatures (code {status[g]})") if status[g] else out.raw[96 * g : 96 * g + 96]
        for g in range(G)
    ]


class ValidatorKeyTable:
    """Device-resident validator public-key table (SURVEY.md 8(f) rank 1;
    C ABI tbls_pk_table_load / tbls_batch_verify_idx).

    Teku memoizes each key's decompression and validity per BLSPublicKey
    (BlstPublicKey.java:38-45, 74-75, 93-104) and fetches keys by validator
    index (BeaconStateAccessors.getValidatorPubKey, BeaconStateAccessors.java:
    78-97); this keeps that memo in HBM on every device, so batches name keys
    by index.  `codes[i]` is key i's status (0 = valid, as tbls_pk_validate)."""

    def __init__(self, pks):
        blob = b"".join(bytes(p) for p in pks)
        self.size = len(pks)
        codes = ctypes.create_string_buffer(max(1, self.size))
        rc = native.lib().tbls_pk_table_load(blob, self.size, codes)
        if rc == native.BAD_ARGUMENT:
            raise ValueError("empty key table")
        native.check(rc, "tbls_pk_table_load")
        self.codes = list(codes.raw[: self.size])

    def batch_verify(self, sets, rands, n_gpus=0) -> bool:
        """BLS.batchVerify over [(key_indices, msg, sig96)] (same semantics as
        batch_verify_raw with the keys' bytes)."""
        n = len(sets)
        arr = (native.TblsSetIdx * max(1, n))()
        keep = []
        for i, (idx, msg, sig) in enumerate(sets):
            ib = (ctypes.c_uint32 * max(1, len(idx)))(*idx)
            mb, sb = _buf(msg), _buf(sig)
            keep += [ib, mb, sb]
            arr[i].key_idx = ctypes.cast(ib, ctypes.c_void_p)
            arr[i].n_pks = len(idx)
            arr[i].msg = ctypes.cast(mb, ctypes.c_void_p)
            arr[i].msg_len = len(msg)
            arr[i].sig = ctypes.cast(sb, ctypes.c_void_p)
        rr = (ctypes.c_uint64 * max(1, n))(*rands)
        ok = ctypes.c_int(0)
        rc = native.lib().tbls_batch_verify_idx(arr, n, rr, n_gpus, ctypes.byref(ok), None)
        if rc == native.BAD_ARGUMENT:
            raise ValueError("key index out of range / empty key list")
        native.check(rc, "tbls_batch_verify_idx")
        return ok.value == 1


def _as_pk(pk) -> HipPublicKey:
    if isinstance(pk, HipPublicKey):
        return pk
    if isinstance(pk, BLSPublicKey):
        return pk.get_public_key()
    if hasattr(pk, "to_bytes_compressed"):  # foreign implementation (BlstPublicKey.fromPublicKey)
        return HipPublicKey.from_bytes(pk.to_bytes_compressed())
    return HipPublicKey.from_bytes(bytes(pk))


def _as_sig(sig) -> HipSignature:
    if isinstance(sig, HipSignature):
        return sig
    if isinstance(sig, BLSSignature):
        return sig.get_signature()
    if hasattr(sig, "to_bytes_compressed"):
        return HipSignature.from_bytes(sig.to_bytes_compressed())
    return HipSignature.from_bytes(bytes(sig))


# ---------------------------------------------------------------------------
# bls/ wrappers and the static facade
# ---------------------------------------------------------------------------
class BLSPublicKey:
    """bls/BLSPublicKey.java: bytes + lazily decoded impl key."""

    def __init__(self, compressed: bytes = None, impl: HipPublicKey = None):
        self._b = bytes(compressed) if compressed is not None else impl.to_bytes_compressed()
        self._impl = impl

    @staticmethod
    def from_bytes_compressed(b48: bytes) -> "BLSPublicKey":
        return BLSPublicKey(b48)

    @staticmethod
    def from_bytes_compressed_validate(b48: bytes) -> "BLSPublicKey":
        k = BLSPublicKey(b48)
        k.get_public_key().force_validation()  # BLSPublicKey.java:84-89
        return k

    @staticmethod
    def aggregate(keys: List["BLSPublicKey"]) -> "BLSPublicKey":
        return BLSPublicKey(impl=BLS.get_bls_impl().aggregate_public_keys([k.get_public_key() for k in keys]))

    def get_public_key(self) -> HipPublicKey:
        if self._impl is None:
            self._impl = BLS.get_bls_impl().public_key_from_compressed(self._b)
        return self._impl

    def to_bytes_compressed(self) -> bytes:
        return self._b

    def __eq__(self, o):
        return isinstance(o, BLSPublicKey) and o._b == self._b

    def __hash__(self):
        return hash(self._b)


class BLSSignature:
    """bls/BLSSignature.java: bytes + lazily decoded impl signature."""

    def __init__(self, compressed: bytes = None, impl: HipSignature = None):
        self._b = bytes(compressed) if compressed is not None else impl.to_bytes_compressed()
        self._impl = impl

    @staticmethod
    def from_bytes_compressed(b: bytes) -> "BLSSignature":
        return BLSSignature(b)

    @staticmethod
    def empty() -> "BLSSignature":  # 96 zero bytes, invalid (BLSSignature.java:46-48)
        return BLSSignature(bytes(96))

    @staticmethod
    def infinity() -> "BLSSignature":
        return BLSSignature(INFINITY_G2)

    def get_signature(self) -> HipSignature:
        if self._impl is None:
            self._impl = BLS.get_bls_impl().signature_from_compressed(self._b)
        return self._impl

    def to_bytes_compressed(self) -> bytes:
        return self._b

    def is_infinity(self) -> bool:
        try:
            return self.get_signature().is_infinity()
        except BlsException:
            return False

    def __eq__(self, o):
        return isinstance(o, BLSSignature) and o._b == self._b

    def __hash__(self):
        return hash(self._b)


class BLSSecretKey:
    """bls/BLSSecretKey.java."""

    def __init__(self, impl: HipSecretKey):
        self._impl = impl

    @staticmethod
    def from_bytes(b32: bytes) -> "BLSSecretKey":
        if int.from_bytes(bytes(b32), "big") >= CURVE_ORDER:  # BLSSecretKey.java:30-40
            raise ValueError("Invalid bytes for secret key (0 <= SK < r)")
        return BLSSecretKey(BLS.get_bls_impl().secret_key_from_bytes(b32))

    @staticmethod
    def from_bytes_mod_r(b32: bytes) -> "BLSSecretKey":
        v = int.from_bytes(bytes(b32), "big") % CURVE_ORDER
        return BLSSecretKey.from_bytes(v.to_bytes(32, "big"))

    def get_secret_key(self) -> HipSecretKey:
        return self._impl

    def to_public_key(self) -> BLSPublicKey:
        return BLSPublicKey(impl=self._impl.derive_public_key())

    def to_bytes(self) -> bytes:
        return self._impl.to_bytes()


class BLSKeyPair:
    def __init__(self, secret_key: BLSSecretKey):
        self.secret_key = secret_key
        self.public_key = secret_key.to_public_key()


class _InvalidBatchSemiAggregate:
    """BLS.InvalidBatchSemiAggregate (BLS.java:457)."""


class BLS:
    """Static facade (bls/BLS.java)."""

    _impl = None
    verification_disabled = False  # BLSConstants.verificationDisabled

    @classmethod
    def set_bls_implementation(cls, impl):  # BLS.java:51-53
        cls._impl = impl

    @classmethod
    def get_bls_impl(cls):
        if cls._impl is None:
            cls._impl = HipBLS12381()
        return cls._impl

    @staticmethod
    def sign(secret_key: BLSSecretKey, message: bytes, dst=None) -> BLSSignature:
        return BLSSignature(impl=secret_key.get_secret_key().sign(message, dst))

    @staticmethod
    def verify(public_key: BLSPublicKey, message: bytes, signature: BLSSignature, dst=None) -> bool:
        if BLS.verification_disabled:
            return True
        try:
            return signature.get_signature().verify(public_key.get_public_key(), message, dst)
        except ValueError:  # IllegalArgumentException (BLS.java:99-101)
            if dst is not None:
                raise
            return False

    @staticmethod
    def aggregate(signatures: List[BLSSignature]) -> BLSSignature:
        try:
            if len(signatures) == 0:
                raise ValueError("Aggregating zero signatures is invalid.")
            return BLSSignature(impl=BLS.get_bls_impl().aggregate_signatures([s.get_signature() for s in signatures]))
        except ValueError as e:
            raise BlsException("Failed to aggregate signatures") from e

    @staticmethod
    def aggregate_verify(public_keys, messages, signature: BLSSignature) -> bool:
        try:
            if len(public_keys) != len(messages):
                raise ValueError("Number of public keys and number of messages differs.")
            if len(public_keys) == 0:
                return False
            try:
                pairs = [(pk.get_public_key(), m) for pk, m in zip(public_keys, messages)]
                return signature.get_signature().verify_pairs(pairs)
            except BlsException:
                return False
        except ValueError as e:
            raise BlsException("Failed to aggregateVerify") from e

    @staticmethod
    def fast_aggregate_verify(public_keys, message: bytes, signature: BLSSignature) -> bool:
        if BLS.verification_disabled:
            return True
        try:
            if len(public_keys) == 0:
                return False
            try:
                return signature.get_signature().verify([pk.get_public_key() for pk in public_keys], message)
            except BlsException:
                return False
        except ValueError as e:
            raise BlsException("Failed to fastAggregateVerify") from e

    @staticmethod
    def batch_verify(public_keys, messages, signatures, double_pairing=None, parallel=None) -> bool:
        """3-arg (BLS.java:230-254) and 5-arg (275-336) forms."""
        if double_pairing is None:
            try:
                if not (len(public_keys) == len(messages) == len(signatures)):
                    raise ValueError("Different collection sizes")
                count = len(public_keys)
                if count == 0:
                    return False
                if count == 1:
                    return BLS.fast_aggregate_verify(public_keys[0], messages[0], signatures[0])
                return BLS.batch_verify(public_keys, messages, signatures, True, True)
            except ValueError as e:
                raise BlsException("Failed to batchVerify") from e
        if BLS.verification_disabled:
            return True
        try:
            if not (len(public_keys) == len(messages) == len(signatures)):
                raise ValueError("Different collection sizes")
            count = len(public_keys)
            if count == 0:
                return False
            impl = BLS.get_bls_impl()
            if type(impl) is HipBLS12381 and not impl.eager:
                return _hip_facade_batch(impl, public_keys, messages, signatures, double_pairing)
            prepared = []
            if double_pairing:
                for i in range(0, count, 2):
                    if i + 1 < count:
                        prepared.append(
                            BLS._prepare2(i, public_keys[i], messages[i], signatures[i], public_keys[i + 1], messages[i + 1], signatures[i + 1])
                        )
                    else:
                        prepared.append(BLS.prepare_batch_verify(i, public_keys[i], messages[i], signatures[i]))
            else:
                prepared = [BLS.prepare_batch_verify(i, public_keys[i], messages[i], signatures[i]) for i in range(count)]
            return BLS.complete_batch_verify(prepared)
        except ValueError as e:
            if isinstance(e, BlsException) and e.__cause__ is not None:
                raise
            raise BlsException("Failed to batchVerify") from e

    @staticmethod
    def prepare_batch_verify(index, public_keys, message, signature):
        try:
            return BLS.get_bls_impl().prepare_batch_verify(
                index, [pk.get_public_key() for pk in public_keys], message, signature.get_signature()
            )
        except BlsException:
            return _InvalidBatchSemiAggregate()

    @staticmethod
    def _prepare2(index, pks1, m1, s1, pks2, m2, s2):
        try:
            return BLS.get_bls_impl().prepare_batch_verify2(
                index, [pk.get_public_key() for pk in pks1], m1, s1.get_signature(), [pk.get_public_key() for pk in pks2], m2, s2.get_signature()
            )
        except BlsException:
            return _InvalidBatchSemiAggregate()

    @staticmethod
    def complete_batch_verify(prepared) -> bool:
        if BLS.verification_disabled:
            return True
        return BLS.get_bls_impl().complete_batch_verify(prepared)


# ---------------------------------------------------------------------------
# The facade's batch path on HipBLS12381
# ---------------------------------------------------------------------------
def predecode(public_keys=(), signatures=()) -> None:
    """Decode every not-yet-decoded BLSPublicKey / BLSSignature in two host
    calls (tbls_pk_decode_many / tbls_sig_decode_many, spread over host
    threads, no device call): the verdicts and memoisation of calling
    get_public_key() / get_signature() on each (BLSSignature.java:83-87,
    BLSPublicKey.java:116-120) when the installed implementation is
    HipBLS12381, whose from_bytes is that host decode.  Objects that do not
    decode stay undecoded: get_*() raises for them as before."""
    for objs, many, width, make in (
        (signatures, "tbls_sig_decode_many", 96, HipSignature),
        (public_keys, "tbls_pk_decode_many", 48, HipPublicKey),
    ):
        todo = [o for o in objs if type(o) in (BLSSignature, BLSPublicKey) and o._impl is None and len(o._b) == width]
        if not todo:
            continue
        codes = ctypes.create_string_buffer(len(todo))
        native.check(getattr(native.host(), many)(b"".join(o._b for o in todo), len(todo), codes, None), many)
        for o, c in zip(todo, codes.raw):
            if c == native.SUCCESS:
                o._impl = make(o._b)


_get_b = operator.attrgetter("_b")
_first = operator.itemgetter(0)


def _hip_facade_batch(impl, public_keys, messages, signatures, double_pairing) -> bool:
    """BLS.batchVerify's 5-argument body (BLS.java:297-336) on HipBLS12381,
    without per-set semi-aggregate objects and without decoding on the host:
    HipBLS12381.prepareBatchVerify only captures bytes, and the device
    decodes every key and signature inside the batch with the same rules
    (tb_codec.h = tbls_*_decode's), so the verdict is the prepare / complete
    loop's -- a unit (a pair of sets with double_pairing, BLS.java:306-322,
    else one set) holding an undecodable key or signature is an
    InvalidBatchSemiAggregate (the batch is false), which the device's batch
    also returns.  The one case where the host must decode: a unit with an
    empty key list raises (BlstPublicKey.aggregate's checkArgument) unless an
    object of that unit fails to decode first (then it is invalid, no raise),
    so only such units' objects are decoded here.  One device batch, no
    single-object device call, no per-object decode for fresh objects."""
    from .synth import SetArray, fast_multipliers

    # The marshalling runs per object, so it is written as C-level map / join
    # over the lists (a Python loop per object cost ~5 ms of host time per
    # 16,384-set batch on the GPU box: bench.py cfg4_facade).
    key_lists = public_keys if set(map(type, public_keys)) == {list} else [list(ks) for ks in public_keys]
    n = len(key_lists)
    lens = set(map(len, key_lists))
    empty = [i for i in range(n) if not key_lists[i]] if 0 in lens else None
    if empty:
        step = 2 if double_pairing else 1

        def decodes(o):
            try:
                (o.get_public_key() if isinstance(o, BLSPublicKey) else o.get_signature() if isinstance(o, BLSSignature)
                 else _as_pk(o) if isinstance(o, PublicKey) else _as_sig(o))
                return True
            except BlsException:
                return False

        for u in sorted({i - i % step for i in empty}):
            unit = range(u, min(n, u + step))
            if all(decodes(k) for j in unit for k in key_lists[j]) and all(decodes(signatures[j]) for j in unit):
                raise ValueError("empty public key list")
        return False  # every empty-key unit holds an undecodable object: InvalidBatchSemiAggregate

    def raw(o):
        return o._b if type(o) in (BLSPublicKey, BLSSignature) else bytes(o.to_bytes_compressed())

    def blob(objs, cls):
        return b"".join(map(_get_b, objs) if set(map(type, objs)) <= {cls} else map(raw, objs))

    if lens == {1}:
        pk_blob = blob(list(map(_first, key_lists)), BLSPublicKey)
        n_pks = np.ones(n, dtype=np.uint64)
    else:
        pk_blob = blob([k for ks in key_lists for k in ks], BLSPublicKey)
        n_pks = list(map(len, key_lists))
    msgs = messages if set(map(type, messages)) <= {bytes} else [bytes(m) for m in messages]
    sig_blob = blob(signatures, BLSSignature)
    if len(sig_blob) != 96 * n or len(pk_blob) != 48 * int(np.sum(n_pks)):  # a wrong-size encoding never decodes
        return False
    arr = SetArray(pk_blob, n_pks, b"".join(msgs), np.fromiter(map(len, msgs), dtype=np.uint64, count=n), sig_blob)
    return arr.batch_verify(fast_multipliers(n), impl.n_gpus)
