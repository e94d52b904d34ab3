"""The BLS JNI glue (integration/native/tekubls_jni.c) compiled with gcc
against a stub JNI environment (tests/native/jni_stub/jni.h) and a recording
fake of the C ABI, under ASan/UBSan: malformed Java arguments (short or
non-monotone message offsets, too few keys / signatures / randomizers, short
fixed-size arrays, small output arrays) return TBLS_BAD_ARGUMENT without
reaching the library or reading past a copied array; well-formed ones reach it
with the sets as the Java side flattened them (tests/native/jni_glue_test.c).
No JDK is needed."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_jni_glue_validates_arguments(tmp_path):
    exe = str(tmp_path / "jni_glue_test")
    cmd = ["gcc", "-std=c11", "-O1", "-g", "-Wall", "-Werror", "-Wno-unused-function", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "tests", "native", "jni_stub"), "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "integration", "native", "tekubls_jni.c"), os.path.join(ROOT, "tests", "native", "jni_glue_test.c"), "-o", exe]
    subprocess.check_call(cmd)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    env.pop("LD_PRELOAD", None)
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("ok")
