"""ctypes binding of libtekubls_hip.so (include/tekubls.h).

The product path: every call goes to the HIP library.  If the library or a
HIP device is missing this module raises -- there is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TBLS_LIB") or os.path.join(_HERE, "lib", "libtekubls_hip.so")

SUCCESS = 0
BAD_ENCODING = 1
POINT_NOT_ON_CURVE = 2
POINT_NOT_IN_GROUP = 3
AGGR_TYPE_MISMATCH = 4
VERIFY_FAIL = 5
PK_IS_INFINITY = 6
BAD_SCALAR = 7
DEVICE_ERROR = 8
BAD_ARGUMENT = 9

PARTIAL_BYTES = 580


class TblsSet(ctypes.Structure):
    _fields_ = [
        ("pks", ctypes.c_void_p),
        ("n_pks", ctypes.c_uint32),
        ("msg", ctypes.c_void_p),
        ("msg_len", ctypes.c_uint32),
        ("sig", ctypes.c_void_p),
    ]


class TblsSetIdx(ctypes.Structure):
    """tbls_set_idx: a set whose keys are indices into the resident key table."""

    _fields_ = [
        ("key_idx", ctypes.c_void_p),
        ("n_pks", ctypes.c_uint32),
        ("msg", ctypes.c_void_p),
        ("msg_len", ctypes.c_uint32),
        ("sig", ctypes.c_void_p),
    ]


class TblsTiming(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("device_ms", ctypes.c_double), ("n_devices", ctypes.c_uint32)]


class TblsDevBatch(ctypes.Structure):
    _fields_ = [
        ("pks", ctypes.c_void_p),
        ("pk_off", ctypes.c_void_p),
        ("n_keys", ctypes.c_uint32),
        ("msgs", ctypes.c_void_p),
        ("msg_off", ctypes.c_void_p),
        ("sigs", ctypes.c_void_p),
        ("rand", ctypes.c_void_p),
        ("n", ctypes.c_uint32),
    ]


class NativeError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what}: tbls status {code}")
        self.code = code


_lib = None
_lock = threading.Lock()

_SIGS = {
    "tbls_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32]),
    "tbls_shutdown": (None, []),
    "tbls_device_count": (ctypes.c_int, []),
    "tbls_pk_validate": (ctypes.c_int, [ctypes.c_char_p]),
    "tbls_sig_validate": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "tbls_pk_decode": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "tbls_sig_decode": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "tbls_pk_decode_many": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p]),
    "tbls_sig_decode_many": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p]),
    "tbls_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int]),
    "tbls_aggregate_pks": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "tbls_aggregate_sigs": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "tbls_hash_to_g2": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "tbls_sign": (
        ctypes.c_int,
        [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p],
    ),
    "tbls_sk_to_pk": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "tbls_verify": (
        ctypes.c_int,
        [
            ctypes.c_char_p,
            ctypes.c_char_p,
            ctypes.c_size_t,
            ctypes.c_char_p,
            ctypes.c_char_p,
            ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_int),
        ],
    ),
    "tbls_batch_verify": (
        ctypes.c_int,
        [
            ctypes.POINTER(TblsSet),
            ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_uint64),
            ctypes.c_int,
            ctypes.POINTER(ctypes.c_int),
            ctypes.POINTER(TblsTiming),
        ],
    ),
    "tbls_fast_aggregate_verify_many": (ctypes.c_int, [ctypes.POINTER(TblsSet), ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]),
    "tbls_batch_verify_each": (
        ctypes.c_int,
        [ctypes.POINTER(TblsSet), ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(TblsTiming)],
    ),
    "tbls_verify_each": (ctypes.c_int, [ctypes.POINTER(TblsSet), ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "tbls_pk_validate_many": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "tbls_sig_validate_many": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p]),
    "tbls_aggregate_sigs_many": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "tbls_aggregate_verify": (
        ctypes.c_int,
        [
            ctypes.c_char_p,
            ctypes.POINTER(ctypes.c_char_p),
            ctypes.POINTER(ctypes.c_uint32),
            ctypes.c_size_t,
            ctypes.c_char_p,
            ctypes.POINTER(ctypes.c_int),
        ],
    ),
    "tbls_dev_batch_partial": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(TblsDevBatch), ctypes.c_void_p, ctypes.c_void_p]),
    "tbls_pk_table_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]),
    "tbls_pk_table_size": (ctypes.c_size_t, []),
    "tbls_batch_verify_idx": (
        ctypes.c_int,
        [
            ctypes.POINTER(TblsSetIdx),
            ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_uint64),
            ctypes.c_int,
            ctypes.POINTER(ctypes.c_int),
            ctypes.POINTER(TblsTiming),
        ],
    ),
    "tbls_dev_batch_partial_idx": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.POINTER(TblsDevBatch), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "tbls_dev_final_verify": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)],
    ),
    "tbls_dev_final_verify_async": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "tbls_dev_batch_partial_timed": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.POINTER(TblsDevBatch), ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)],
    ),
    "tbls_dev_batch_stage_profile": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.POINTER(TblsDevBatch), ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)],
    ),
    "tbls_acc_plan": (ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int)]),
    "tbls_place_plan": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_size_t)]),
    "tbls_shard_min": (ctypes.c_uint32, []),
    "tbls_shard_knee": (ctypes.c_uint32, []),
    "tbls_sk_to_pk_many": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "tbls_sign_many": (
        ctypes.c_int,
        [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p],
    ),
}

EXPORTED = tuple(_SIGS)


def _loaded_hip_runtimes():
    """Paths of the libamdhip64 copies mapped into this process."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({line.split()[-1] for line in f if "libamdhip64" in line and "/" in line})
    except OSError:
        return []


def _preload_process_hip_runtime():
    """One HIP runtime per process.

    libtekubls_hip.so needs libamdhip64.so.7; PyTorch-ROCm ships its own copy
    (torch/lib/libamdhip64.so, same soname) and its libraries ask for it as
    "libamdhip64.so".  If this library is loaded first, the loader takes
    /opt/rocm's copy for it and torch later maps its own beside it: two HIP
    and two HSA runtimes in one process, and torch's initialisation failed
    with "No HIP GPUs are available" once the library had used the device
    (round 4).  Loading torch's runtime first, by path
    and RTLD_GLOBAL, makes every later request resolve to that one copy: this
    library's soname request matches it, and torch's own load finds the same
    file already mapped.  A process without torch keeps the system runtime.
    The library is built against /opt/rocm's HIP: torch's copy is taken only
    when its ROCm major version (the "+rocmX.Y" of torch's package version,
    read from its metadata, nothing loaded) equals the build's (/opt/rocm/.info/
    version), or when torch is already imported (its runtime is then the
    process's in any case); otherwise the system runtime stays.
    TBLS_HIP_PRELOAD=0 disables this (diagnostics)."""
    if os.environ.get("TBLS_HIP_PRELOAD", "1") == "0" or _loaded_hip_runtimes():
        return
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    if "torch" not in sys.modules and not _same_rocm_major():
        return
    rt = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(rt):
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)


def _rocm_major(version: str):
    """Major version from "7.2.0" or a "+rocm7.0" local version tag (None if absent)."""
    import re

    m = re.search(r"(?:rocm)?(\d+)\.\d+", version.split("+rocm", 1)[1] if "+rocm" in version else version)
    return int(m.group(1)) if m else None


def _same_rocm_major() -> bool:
    """torch's ROCm major version equals /opt/rocm's (the build's)."""
    try:
        import importlib.metadata

        t = importlib.metadata.version("torch")
        tv = _rocm_major(t) if "+rocm" in t else None  # a CUDA or CPU build of torch: no HIP runtime to share
        with open(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), ".info", "version")) as f:
            sv = _rocm_major(f.read().strip())
    except (OSError, ImportError, ValueError):
        return False
    return tv is not None and tv == sv


def load_library(path: str = LIB_PATH):
    """dlopen the library and bind every entry point (no device initialisation)."""
    if not os.path.exists(path):
        raise NativeError(DEVICE_ERROR, f"HIP library not built: {path} (run __graft_entry__.build())")
    _preload_process_hip_runtime()
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_host_lib = None


def host():
    """The library for its host-only entry points (tbls_*_decode*, tbls_stats,
    tbls_place_plan): loaded, never initialised -- no device needed."""
    global _host_lib
    with _lock:
        if _lib is not None:
            return _lib
        if _host_lib is None:
            _host_lib = load_library()
        return _host_lib


def stats(reset=False):
    """tbls_stats as a dict (what the device and the host decoders did)."""
    out = (ctypes.c_uint64 * 8)()
    check(host().tbls_stats(out, 8, 1 if reset else 0), "tbls_stats")
    names = ("partials", "one_validate", "helpers", "each_passes", "finals", "host_decodes", "settled")
    return dict(zip(names, out[: len(names)]))


def lib():
    """The initialised library (raises NativeError when no HIP device is present)."""
    global _lib
    with _lock:
        if _lib is None:
            L = load_library()
            rc = L.tbls_init(-1, 0)
            if rc != SUCCESS:
                raise NativeError(rc, "tbls_init (no usable HIP device)")
            _lib = L
        return _lib


def check(rc, what):
    if rc != SUCCESS:
        raise NativeError(rc, what)


def acc_plan(n_sets):
    """The Miller accumulator plan the library runs for a batch of n_sets
    single-key sets (tbls_acc_plan; no device needed): (per, nseg, split)."""
    L = load_library() if _lib is None else _lib
    per, nseg, split = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
    check(L.tbls_acc_plan(n_sets, ctypes.byref(per), ctypes.byref(nseg), ctypes.byref(split)), "acc_plan")
    return per.value, nseg.value, split.value


def place_plan(n, n_pks=None, n_devices=8, n_gpus=0, load=None, rr=0, shard_min=None, shard_knee=None):
    """The library's device placement of a batch (tbls_place_plan; no device
    needed): returns (devices, cuts) -- device devices[k] verifies sets
    [cuts[k], cuts[k+1]).  shard_knee: the shard floor on an idle node
    (default the library's; 0 = none)."""
    L = load_library() if _lib is None else _lib
    pk = (ctypes.c_uint32 * n)(*n_pks) if n_pks is not None else None
    ld = (ctypes.c_int * n_devices)(*load) if load is not None else None
    dev = (ctypes.c_int * n_devices)()
    cut = (ctypes.c_size_t * (n_devices + 1))()
    smin = L.tbls_shard_min() if shard_min is None else shard_min
    knee = L.tbls_shard_knee() if shard_knee is None else shard_knee
    G = L.tbls_place_plan(n, pk, n_devices, n_gpus, ld, rr, smin, knee, dev, cut)
    if G < 1:
        raise NativeError(-G, "tbls_place_plan")
    return list(dev[:G]), list(cut[: G + 1])
