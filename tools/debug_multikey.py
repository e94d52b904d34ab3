"""Debug: time the multi-key batch (tests/test_gpu_bls.py::test_batch_multikey_sets) per stage."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

from oracle import c_oracle as C  # noqa: E402
from oracle.keys import interop_sk  # noqa: E402
from teku_amd import bls, native  # noqa: E402

L = native.lib()
sets = []
for j in range(4):
    sks = [interop_sk(10 * j + i) for i in range(5)]
    m = bytes([0xA0 + j]) * 32
    pks = b"".join(C.sk_to_pk(s) for s in sks)
    sig = C.sign(sum(sks) % 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001, m)
    sets.append((pks, 5, m, sig))
print("inputs ready", flush=True)
for rep in range(3):
    t = time.time()
    ok = bls.batch_verify_raw(sets, [3 + rep, 5, 7, 9])
    print("rep", rep, ok, "%.3f s" % (time.time() - t), flush=True)

# single-key sets and the MILLER2 primitive
from oracle import bls12_381 as O  # noqa: E402
from tests.opcodec import enc_fp, enc_fp2, dec_fp12, run_ops  # noqa: E402

sks = [interop_sk(i) for i in range(8)]
single = [(C.sk_to_pk(s), 1, bytes([i + 1]) * 32, C.sign(s, bytes([i + 1]) * 32)) for i, s in enumerate(sks)]
print("single-key 8 sets:", bls.batch_verify_raw(single, list(range(3, 11))), flush=True)
for n in (2, 3, 4, 5):
    print("single-key %d sets:" % n, bls.batch_verify_raw(single[:n], list(range(3, 3 + n))), flush=True)
P0, Q0 = O.G1_GEN, O.G2_GEN
P1 = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), 7))
Q1 = O.hash_to_g2(b"second pair")
rec = enc_fp(P0[0]) + enc_fp(P0[1]) + enc_fp2(Q0[0]) + enc_fp2(Q0[1]) + enc_fp(P1[0]) + enc_fp(P1[1]) + enc_fp2(Q1[0]) + enc_fp2(Q1[1])
f = dec_fp12(run_ops(L.tbls_test_ops, "MILLER2", [rec])[0])
print("MILLER2 op:", O.final_exponentiation(f) == O.f12_mul(O.pairing(P0, Q0), O.pairing(P1, Q1)), flush=True)
rec1 = enc_fp(P1[0]) + enc_fp(P1[1]) + enc_fp2(Q1[0]) + enc_fp2(Q1[1])
f1 = dec_fp12(run_ops(L.tbls_test_ops, "MILLER", [rec1])[0])
print("MILLER op (single pair):", O.final_exponentiation(f1) == O.pairing(P1, Q1), flush=True)
hip = bls.HipBLS12381()
pk0, _, m0, s0 = single[0]
out = ctypes.create_string_buffer(96)
native.check(L.tbls_hash_to_g2(m0, len(m0), O.ETH2_DST, len(O.ETH2_DST), out), "h2g2")
print("hash_to_g2:", out.raw == C.hash_to_g2(m0), flush=True)
okv = ctypes.c_int(0)
native.check(L.tbls_verify(pk0, m0, len(m0), s0, O.ETH2_DST, len(O.ETH2_DST), ctypes.byref(okv)), "verify")
print("tbls_verify single:", okv.value, flush=True)
print("sig_validate:", L.tbls_sig_validate(s0, None), "pk_validate:", L.tbls_pk_validate(pk0), flush=True)
