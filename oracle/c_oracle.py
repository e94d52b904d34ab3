"""ctypes binding of the C oracle (oracle/c/bls_oracle.c).  TEST INFRASTRUCTURE
ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg;
never by the teku_amd product path."""

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "c", "_build", "libbls_oracle.so")
ETH2_DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("C oracle not built: make -C oracle/c")
        L = ctypes.CDLL(LIB_PATH)
        cp, sz = ctypes.c_char_p, ctypes.c_size_t
        L.orc_hash_to_g2.argtypes = [cp, sz, cp, sz, cp]
        L.orc_sk_to_pk.argtypes = [cp, cp]
        L.orc_sign.argtypes = [cp, cp, sz, cp, sz, cp]
        L.orc_pk_validate.argtypes = [cp]
        L.orc_sig_validate.argtypes = [cp, ctypes.POINTER(ctypes.c_int)]
        u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
        L.orc_batch_verify.argtypes = [cp, cp, u32p, cp, u64p, sz, cp, sz, ctypes.c_int]
        L.orc_batch_verify_sets.argtypes = [cp, u32p, cp, u32p, cp, u64p, sz, cp, sz, ctypes.c_int]
        L.orc_verify_each.argtypes = [cp, u32p, cp, u32p, cp, sz, cp, sz, ctypes.c_int, ctypes.c_void_p]
        L.orc_verify_each.restype = None
        _lib = L
    return _lib


def hash_to_g2(msg, dst=ETH2_DST):
    out = ctypes.create_string_buffer(96)
    lib().orc_hash_to_g2(msg, len(msg), dst, len(dst), out)
    return out.raw


def sk_to_pk(sk: int):
    out = ctypes.create_string_buffer(48)
    lib().orc_sk_to_pk(sk.to_bytes(32, "big"), out)
    return out.raw


def sign(sk: int, msg, dst=ETH2_DST):
    out = ctypes.create_string_buffer(96)
    lib().orc_sign(sk.to_bytes(32, "big"), msg, len(msg), dst, len(dst), out)
    return out.raw


def pk_validate(pk):
    return lib().orc_pk_validate(pk)


def sig_validate(sig):
    inf = ctypes.c_int(0)
    code = lib().orc_sig_validate(sig, ctypes.byref(inf))
    return code, bool(inf.value)


def batch_verify(pks, msgs, sigs, rands, threads=1, dst=ETH2_DST):
    """Randomized batch verification of n >= 2 single-key sets (BLS.batchVerify)."""
    n = len(pks)
    off = (ctypes.c_uint32 * (n + 1))()
    acc = 0
    for i, m in enumerate(msgs):
        off[i] = acc
        acc += len(m)
    off[n] = acc
    rr = (ctypes.c_uint64 * n)(*rands)
    return lib().orc_batch_verify(b"".join(pks), b"".join(msgs) or b"\0", off, b"".join(sigs), rr, n, dst, len(dst), threads) == 1


def _offsets(items, size_of):
    off = (ctypes.c_uint32 * (len(items) + 1))()
    acc = 0
    for i, x in enumerate(items):
        off[i] = acc
        acc += size_of(x)
    off[len(items)] = acc
    return off


def batch_verify_sets(pks_list, msgs, sigs, rands, threads=1, dst=ETH2_DST):
    """Randomized batch verification of n >= 2 sets, set i signed by the keys
    pks_list[i] (a list of 48-byte keys: BlstPublicKey.aggregate semantics)."""
    n = len(pks_list)
    pk_off = _offsets(pks_list, len)
    m_off = _offsets(msgs, len)
    rr = (ctypes.c_uint64 * n)(*rands)
    blob = b"".join(b"".join(p) for p in pks_list)
    return (
        lib().orc_batch_verify_sets(blob or b"\0", pk_off, b"".join(msgs) or b"\0", m_off, b"".join(sigs), rr, n, dst, len(dst), threads)
        == 1
    )


def verify_each(pks_list, msgs, sigs, threads=1, dst=ETH2_DST):
    """Per-set fastAggregateVerify verdicts (BLS.java:185-207) as a list of bools."""
    n = len(pks_list)
    if n == 0:
        return []
    pk_off = _offsets(pks_list, len)
    m_off = _offsets(msgs, len)
    out = (ctypes.c_uint8 * n)()
    blob = b"".join(b"".join(p) for p in pks_list)
    lib().orc_verify_each(blob or b"\0", pk_off, b"".join(msgs) or b"\0", m_off, b"".join(sigs), n, dst, len(dst), threads, out)
    return [bool(v) for v in out]
