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
MADS_MUL, MADS_SQR, MADS_F2 = 392, 301, 980  # v_mad_u64_u32 per 14 x 29-bit Montgomery product / squaring (tb_fp.h), lazy Fp2 product (tb_tower.h)


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "_build", "libtbhostsim_count.so"))
    fn = lib.tbls_hostsim_test_ops
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    cnt = lib.tbls_hostsim_mul_count
    cnt.restype = ctypes.c_ulonglong
    cnt.argtypes = [ctypes.c_int]
    sqc = lib.tbls_hostsim_sqr_count
    sqc.restype = ctypes.c_ulonglong
    sqc.argtypes = [ctypes.c_int]
    f2c = lib.tbls_hostsim_fp2mul_count
    f2c.restype = ctypes.c_ulonglong
    f2c.argtypes = [ctypes.c_int]
    N = 8
    sks = [interop_sk(i) for i in range(N)]
    pks = [O.sk_to_pk(s) for s in sks]
    msgs = [O.sha256_msg(i) if hasattr(O, "sha256_msg") else bytes([i]) * 32 for i in range(N)]
    sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
    r = 0xF123456789ABCDEF

    sq, f2 = {}, {}

    def per_unit(op, recs, units_per_rec=1, name=None):
        cnt(1)
        sqc(1)
        f2c(1)
        run_ops(fn, op, recs)
        u = len(recs) * units_per_rec
        m, s_, f_ = cnt(1) / u, sqc(1) / u, f2c(1) / u
        if name:
            sq[name] = s_
            f2[name] = f_
        return m

    res = {}
    res["pk_decompress"] = per_unit("STAGE_PK", pks, name="pk_decompress")
    aff = [O.g1_decompress(p)[1] for p in pks]
    res["set_pk"] = per_unit("STAGE_SET_PK", [enc_fp(a[0]) + enc_fp(a[1]) + r.to_bytes(8, "little") for a in aff], name="set_pk")
    # k_sig_check: decode + G2 check (r = 1: no scalar loop)
    res["set_sig"] = per_unit("STAGE_SET_SIG", [s + (1).to_bytes(8, "little") for s in sigs], name="set_sig")
    res["set_hash"] = per_unit("STAGE_SET_HASH", [enc_h2c(m) for m in msgs], name="set_hash")
    q = [O.g2_decompress(s)[1] for s in sigs]
    # Large batches: the signature side as bucket sums by randomizer byte
    # (k_msm_bucket_tree: one mixed addition per nonzero byte, 8 windows, and
    # a 32-lane tree per bucket: 31 additions), then 64 bit
    # sums of 128 buckets each (k_msm_bitsum_pairs: 2 + 63 additions, affine)
    # whose 64 extra Miller pairs are spread over the accumulators
    # (k_sigs.hip, k_lines.hip), per set at n = MSM_N.  Point-operation costs in
    # Fp products from the tb_curve.h formulas (Fp2 mul = 3 products, Fp2 sqr =
    # 2): madd-2007-bl 7M+4S = 29, add-2007-bl 11M+5S = 43; the Fp2 affine
    # conversion (binary-GCD inversion ~65 + norm/products) ~81.
    MADD, ADD, AFF2, MSM_N, NSUM, XP = 29, 43, 81, 131072, 2040, 64
    adds = NSUM * 31 + XP * 65
    res["g2_sum"] = 8 * 255 / 256 * MADD + (adds * ADD + XP * AFF2) / MSM_N
    sq["g2_sum"] = 8 * 255 / 256 * 4 * 2 + adds * 5 * 2 / MSM_N
    f2["g2_sum"] = 8 * 255 / 256 * 7 + adds * 11 / MSM_N
    res["pairs_per_set"] = (MSM_N + XP) / MSM_N
    # small batches: the signature pair's G1 point -[r] g1 = sum of <= 8
    # precomputed multiples (k_set_pk: G1 madd 7M+4S = 11) + affine (~70)
    res["set_pk_sigpair"] = 8 * 255 / 256 * 11 + 70
    # k_set_pk_wave (configs 2/3): one wave per set of k keys -- (k - 64) mixed
    # additions (a lane's first key costs nothing), a 63-addition LDS tree, then
    # [r] apk on the Jacobian sum and the affine conversion.  G1 costs from the
    # tb_curve.h formulas: madd-2007-bl 7M+4S = 11, add-2007-bl 11M+5S = 16,
    # [r]P for a 64-bit r: 63 dbl-2009-l (2M+5S = 7) + ~32 additions.
    G1_MADD, G1_ADD, G1_DBL = 11, 16, 7
    finish = 63 * G1_DBL + 32 * G1_ADD + (res["set_pk"] - 63 * G1_DBL - 32 * G1_MADD)  # + inversion/affine as measured
    for k in (488, 512):
        res[f"set_pk_wave_{k}"] = (k - 64) * G1_MADD + 63 * G1_ADD + finish
    # k_miller2: two pairs per Fp12 accumulator -> work per pair = MILLER2 / 2
    pair = [enc_fp(a[0]) + enc_fp(a[1]) + enc_fp2(b[0]) + enc_fp2(b[1]) for a, b in zip(aff, q)]
    res["miller"] = per_unit("MILLER2", [pair[i] + pair[i + 1] for i in range(0, N, 2)], units_per_rec=2, name="miller")
    # The split Miller loop's accumulator part per pair, for a plan of `per`
    # pairs per thread and `nseg` loop segments (k_lines.hip k_miller_accs):
    # fp12_sqr_i = 12 lazy Fp2 products (36 M), fp12_mul_by_line_i = 13 (39 M);
    # a segment skips its first step's squaring (f = 1) and takes its first
    # line as f.  MILLER2 (two pairs per accumulator, 62 squarings) minus its
    # accumulator share plus the plan's; the segment products' Horner tail (<= 49
    # Fp12 squarings per batch, <= 59 at 16 segments) is below 0.01 M per pair at 131,072 pairs.
    X_ABS = 0xD201000000010000
    dbl = []
    for b in range(62, -1, -1):
        dbl.append(1)
        if (X_ABS >> b) & 1:
            dbl.append(0)
    SQR12, LINE12 = 36, 39
    acc2 = (62 * SQR12) / 2 + 68 * LINE12
    for per, nseg in ((1, 4), (2, 4), (4, 2), (4, 4), (8, 2), (8, 4), (1, 16), (2, 16), (4, 16), (8, 16), (16, 4), (16, 8), (16, 16), (32, 8), (32, 16)):
        sq_ = sum(sum(dbl[68 * j // nseg:68 * (j + 1) // nseg]) - dbl[68 * j // nseg] for j in range(nseg))
        accs = (sq_ * SQR12 + (per * 68 - nseg) * LINE12) / per
        res[f"miller_seg_{per}x{nseg}"] = res["miller"] - acc2 + accs
    # k_miller_accs_lds (round 5): the valid pairs' lines of a step multiplied
    # two at a time (line_mul: 6 Fp2 products = 18 M) and f by their product
    # (fp12_mul_line2_lds: 17 = 51 M), an odd line left over by the sparse
    # product (39 M); a segment's first step stores its first product (or line)
    # as f.  miller_seg2_PxS.
    PAIR12, LMUL = 51 + 18, 18
    for per, nseg in ((2, 16), (4, 16), (8, 16), (16, 4), (16, 8), (16, 16), (32, 8)):
        sq_ = sum(sum(dbl[68 * j // nseg:68 * (j + 1) // nseg]) - dbl[68 * j // nseg] for j in range(nseg))
        step = (per // 2) * PAIR12 + (per % 2) * LINE12
        first = (LMUL + ((per - 2) // 2) * PAIR12 + ((per - 2) % 2) * LINE12) if per >= 2 else 0
        accs = (sq_ * SQR12 + (68 - nseg) * step + nseg * first) / per
        res[f"miller_seg2_{per}x{nseg}"] = res["miller"] - acc2 + accs
    f = [tuple(tuple((i + j + k, 3 * i + 1) for k in range(3)) for j in range(2)) for i in range(2)]
    # one Fp12 product per accumulator, i.e. per two pairs
    res["fp12_prod"] = per_unit("FP12_MUL", [enc_fp12(f[0]) + enc_fp12(f[1])], units_per_rec=2, name="fp12_prod")
    res["final_exp"] = per_unit("FINAL_EXP", [enc_fp12(f[0])])
    # per single-signer set (the unit of the headline metric), excluding the once-per-batch final exp
    res["per_set_total"] = sum(res[k] for k in ["pk_decompress", "set_pk", "set_sig", "set_hash", "g2_sum"]) + res["pairs_per_set"] * (
        res["miller"] + res["fp12_prod"])
    res["note"] = ("per set of the large-batch path (n = 131072, the bench config): set_sig = decode + G2 check (k_sig_check), "
                   "g2_sum = bucket sums + bucket pairs' trees/affine; miller per pair (pairs_per_set pairs per set). "
                   "Small batches add set_pk_sigpair per set and one signature pair per set instead of the bucket pairs.")
    res["sqr_per_unit"] = {k: round(v, 1) for k, v in sq.items()}
    res["mads_per_unit"] = {
        k: round((res[k] - sq[k] - 3 * f2.get(k, 0)) * MADS_MUL + sq[k] * MADS_SQR + f2.get(k, 0) * MADS_F2) for k in sq if k in res
    }
    res["fp2_products_per_unit"] = {k: round(v, 1) for k, v in f2.items()}
    res["mads_per_mul"], res["mads_per_sqr"], res["mads_per_fp2_mul"] = MADS_MUL, MADS_SQR, MADS_F2
    out = os.path.join(ROOT, "tools", "mul_counts.json")
    json.dump({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items() if k != "note"} | {"note": res["note"]}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
