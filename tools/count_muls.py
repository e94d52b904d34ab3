"""Count Fp multiplications (M) per unit of work for each pipeline stage by
running the stage bodies (teku_amd/csrc/tb_stages.h, the code the kernels run)
on the host instrumentation build (-DTB_COUNT_MULS).  Writes tools/mul_counts.json,
read by bench.py for the roofline's algorithmic work.
One M = one 12-limb Montgomery multiplication = 2*12^2 = 288 32x32->64 MACs.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as O  # noqa: E402
from oracle.keys import interop_sk  # noqa: E402
from tests.opcodec import OPS, enc_fp, enc_fp2, enc_fp12, enc_h2c, run_ops  # noqa: E402

OPS.update(STAGE_PK=24, STAGE_SET_PK=25, STAGE_SET_SIG=26, STAGE_SET_HASH=27, G2_JADD=28)


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "_build", "libtbhostsim_count.so"))
    fn = lib.tbls_hostsim_test_ops
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    cnt = lib.tbls_hostsim_mul_count
    cnt.restype = ctypes.c_ulonglong
    cnt.argtypes = [ctypes.c_int]
    N = 8
    sks = [interop_sk(i) for i in range(N)]
    pks = [O.sk_to_pk(s) for s in sks]
    msgs = [O.sha256_msg(i) if hasattr(O, "sha256_msg") else bytes([i]) * 32 for i in range(N)]
    sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
    r = 0xF123456789ABCDEF

    def per_unit(op, recs):
        cnt(1)
        run_ops(fn, op, recs)
        return cnt(1) / len(recs)

    res = {}
    res["pk_decompress"] = per_unit("STAGE_PK", pks)
    aff = [O.g1_decompress(p)[1] for p in pks]
    res["set_pk"] = per_unit("STAGE_SET_PK", [enc_fp(a[0]) + enc_fp(a[1]) + r.to_bytes(8, "little") for a in aff])
    res["set_sig"] = per_unit("STAGE_SET_SIG", [s + r.to_bytes(8, "little") for s in sigs])
    res["set_hash"] = per_unit("STAGE_SET_HASH", [enc_h2c(m) for m in msgs])
    q = [O.g2_decompress(s)[1] for s in sigs]
    res["g2_sum"] = per_unit("G2_JADD", [enc_fp2(a[0]) + enc_fp2(a[1]) + enc_fp2(b[0]) + enc_fp2(b[1]) for a, b in zip(q, q[1:] + q[:1])])
    res["miller"] = per_unit("MILLER", [enc_fp(a[0]) + enc_fp(a[1]) + enc_fp2(b[0]) + enc_fp2(b[1]) for a, b in zip(aff, q)])
    f = [tuple(tuple((i + j + k, 3 * i + 1) for k in range(3)) for j in range(2)) for i in range(2)]
    res["fp12_prod"] = per_unit("FP12_MUL", [enc_fp12(f[0]) + enc_fp12(f[1])])
    res["final_exp"] = per_unit("FINAL_EXP", [enc_fp12(f[0])])
    # per single-signer set (the unit of the headline metric), excluding the once-per-batch final exp
    res["per_set_total"] = sum(res[k] for k in ["pk_decompress", "set_pk", "set_sig", "set_hash", "g2_sum", "miller", "fp12_prod"])
    out = os.path.join(ROOT, "tools", "mul_counts.json")
    json.dump({k: round(v, 1) for k, v in res.items()}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
