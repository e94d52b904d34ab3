"""No outlined device function in the built libraries branches through its own
return address (tools/check_long_branches.py): a function whose loop exceeds
the short-branch range got a long branch through s[30:31] from ROCm 7.2's
clang, and its return then never came back (a GPU hang)."""

import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_check_finds_the_hazard_in_a_known_bad_object(tmp_path):
    """The checker itself: a function built to need a long branch is reported."""
    import shutil
    import subprocess

    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    src = tmp_path / "bad.hip"
    # one function whose loop body is > 256 KB of straight-line code
    body = "\n".join(f"    x = x * 0x9e3779b9u + {k}u; x ^= x >> 13;" for k in range(40000))
    src.write_text(f"""#include <hip/hip_runtime.h>
__device__ __attribute__((noinline)) unsigned f(unsigned x, int n) {{
  for (int i = 0; i < n; i++) {{
{body}
  }}
  return x;
}}
extern "C" __global__ void k(unsigned* o, int n) {{ o[threadIdx.x] = f(o[threadIdx.x], n); }}
""")
    obj = tmp_path / "bad.o"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-c", str(src), "-o", str(obj)], capture_output=True, timeout=600)
    if r.returncode:
        pytest.skip("test object did not build")
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_long_branches as C

    import tempfile

    with tempfile.TemporaryDirectory() as d:
        found = [f for co in C.code_objects(str(obj), d) for f in C.findings(co)]
    if not found:
        pytest.skip("this compiler did not expand the test loop into a long branch through s[30:31]")
    assert any("f" in name for name in found)


@pytest.mark.parametrize("lib", ["teku_amd/lib/libtekubls_hip.so", "tests/native/_build/libtekubls_test.so"])
def test_built_libraries_have_no_return_address_long_branch(lib):
    import sys

    path = os.path.join(ROOT, lib)
    if not os.path.exists(path):
        pytest.skip(f"{lib} not built")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_long_branches as C

    assert C.main([path]) == 0
