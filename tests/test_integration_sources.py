"""Consistency of the Java/JNI integration sources (integration/) with the C
ABI: every `native` method of TekuBlsHip / TekuKzgHip has its JNI definition
in the glue and vice versa, and the glue calls only functions the headers
declare.  The image has no JDK, so this is the check that stands in for
compiling them."""

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
J = os.path.join(ROOT, "integration", "java", "tech", "pegasys", "teku")
N = os.path.join(ROOT, "integration", "native")


def _read(*p):
    with open(os.path.join(*p)) as f:
        return f.read()


def _natives(java):
    return set(re.findall(r"static native \w+(?:\[\])? (\w+)\(", java))


def _jni(c):
    return set(re.findall(r"JNICALL JNAME\((\w+)\)", c))


def _declared(header):
    return set(re.findall(r"\b(t(?:bls|kzg)_\w+)\(", header))


def _called(c):
    return set(re.findall(r"\b(t(?:bls|kzg)_\w+)\(", c))


def test_bls_natives_match_glue():
    java = _read(J, "bls", "impl", "hip", "TekuBlsHip.java")
    c = _read(N, "tekubls_jni.c")
    assert _natives(java) == _jni(c)
    assert _called(c) <= _declared(_read(ROOT, "include", "tekubls.h"))


def test_kzg_natives_match_glue():
    java = _read(J, "kzg", "TekuKzgHip.java")
    c = _read(N, "tekukzg_jni.c")
    assert _natives(java) == _jni(c)
    assert _called(c) <= _declared(_read(ROOT, "include", "tekukzg.h"))


def test_spi_classes_present():
    for f in ("HipBLS12381", "HipPublicKey", "HipSignature", "HipSecretKey", "HipSemiAggregate", "HipLoader"):
        src = _read(J, "bls", "impl", "hip", f + ".java")
        assert re.search(r"\b(class|interface|record) " + f + r"\b", src)
    assert "implements KZG" in _read(J, "kzg", "HipKZG.java")


def test_gpu_service_source_wired_to_batch_verify_each():
    """the Java half of the GPU-aware service is a
    committed source (not an INTEGRATION.md snippet): the service's
    batchVerifySignatures makes one HipBatchVerifier.batchVerifyEach call,
    sizes its workers to the device count and asks for one device while tasks
    wait; HipBatchVerifier reaches the C ABI through the TekuBlsHip native
    that the JNI glue binds to tbls_batch_verify_each."""
    svc = _read(J, "statetransition", "validation", "signatures", "HipAggregatingSignatureVerificationService.java")
    assert re.search(r"class HipAggregatingSignatureVerificationService extends SignatureVerificationService\b", svc)
    body = svc[svc.index("void batchVerifySignatures("):]
    assert body.count("HipBatchVerifier.batchVerifyEach(") == 1
    code = svc[svc.index("public class"):]
    assert "BLS.batchVerify" not in code and "splitTasks" not in code  # no halving fallback
    assert "this.numThreads = HipBatchVerifier.deviceCount();" in svc
    assert "queue.isEmpty() ? 0 : 1" in svc
    ver = _read(J, "bls", "impl", "hip", "HipBatchVerifier.java")
    assert "public static boolean batchVerifyEach(" in ver and "TekuBlsHip.batchVerifyEach(" in ver
    assert "batchVerifyEach" in _natives(_read(J, "bls", "impl", "hip", "TekuBlsHip.java"))
    c = _read(N, "tekubls_jni.c")
    assert "batchVerifyEach" in _jni(c) and "tbls_batch_verify_each(" in c
