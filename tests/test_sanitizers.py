"""Sanitizer runs of the host-side code (SURVEY.md 5 "Race detection /
sanitizers"; VERDICT r1 hygiene): the host build of the kernel arithmetic
(tb_*.h) and the C oracle, linked into tests/native/sanitize_main.cpp, built
and run under AddressSanitizer + UndefinedBehaviorSanitizer, and the oracle's
pthreaded batch verification under ThreadSanitizer.  GPU sanitizers are not
available on this pool; the product library's host code (tb_lib.hip) runs
under the -m gpu tests only."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BUILD = os.path.join(NATIVE, "_build")


def _build_and_run(tag, flags, threads):
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, f"sanitize_{tag}")
    oc = os.path.join(BUILD, f"bls_oracle_{tag}.o")
    subprocess.check_call(["gcc", "-O1", "-g", "-std=gnu11", "-c", os.path.join(ROOT, "oracle", "c", "bls_oracle.c"), "-o", oc] + flags)
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", os.path.join(NATIVE, "sanitize_main.cpp"), oc, "-o", exe, "-pthread"] + flags)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, str(threads)], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_asan_ubsan_kernel_code_and_oracle():
    _build_and_run("asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"], 4)


def test_tsan_oracle_threads():
    _build_and_run("tsan", ["-fsanitize=thread"], 4)
