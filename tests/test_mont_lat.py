"""mont29_lat, the latency form of the Montgomery product used by the wave
kernels (tb_fp.h), computes exactly mont29's limbs: host build of
tests/native/mont_lat_check.cpp (200k random and top-of-range operands)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mont29_lat_matches(tmp_path):
    exe = str(tmp_path / "mont_lat_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "teku_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "mont_lat_check.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "mismatches 0" in out.stdout, out.stdout + out.stderr
