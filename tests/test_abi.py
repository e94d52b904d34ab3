"""The C-ABI library loads and exports every symbol include/tekubls.h declares
(no compute calls: this container has no GPU)."""

import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "tekubls.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tbls_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from teku_amd import native

    if not os.path.exists(native.LIB_PATH):  # normally built by __graft_entry__.build()
        import __graft_entry__ as ge

        ge.build_hip_lib()
    lib = ctypes.CDLL(native.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from teku_amd import native

    assert set(declared_symbols()) == set(native.EXPORTED)
    native.load_library()


def test_no_device_fails_loudly():
    """Without a HIP device the product path raises instead of falling back."""
    import pytest

    from teku_amd import native

    L = native.load_library()
    if L.tbls_device_count() == 0 and L.tbls_init(-1, 0) != native.SUCCESS:
        native._lib = None
        with pytest.raises(native.NativeError):
            native.lib()
