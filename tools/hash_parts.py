"""Per-part latency of hash_to_G2 (and the pairing pieces) on the GPU (one thread per record, 128
records, test library ops): wall time of tbls_test_ops per op minus the FP_ADD
baseline (allocation + copies).  Tells where the per-set hash chain goes.

    python tools/hash_parts.py [n]
"""
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from opcodec import enc_fp, enc_fp2, enc_fp12, enc_h2c, load_test_lib, run_ops  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 128
    L = load_test_lib()
    rng = random.Random(3)
    from oracle import bls12_381 as O

    fp2r = lambda: (rng.randrange(O.P), rng.randrange(O.P))  # noqa: E731
    f12r = lambda: tuple(tuple(fp2r() for _ in range(3)) for _ in range(2))  # noqa: E731
    recs = {
        "FP_ADD": [enc_fp(1) + enc_fp(2)] * n,
        "HASH_TO_FIELD": [enc_h2c(b"m%05d" % i + b"\0" * 26) for i in range(n)],
        "SSWU": [enc_fp2(fp2r()) for _ in range(n)],
        "ISO": [enc_fp2(fp2r()) + enc_fp2(fp2r()) for _ in range(n)],
        "CLEAR_COF": [enc_fp2(fp2r()) + enc_fp2(fp2r()) for _ in range(n)],
        "HASH_TO_G2": [enc_h2c(b"m%05d" % i + b"\0" * 26) for i in range(n)],
        "FP_INV": [enc_fp(rng.randrange(1, O.P)) for _ in range(n)],
        "G2_IN_GROUP": [enc_fp2(O.G2_GEN[0]) + enc_fp2(O.G2_GEN[1])] * n,
        "FP12_INV": [enc_fp12(f12r()) for _ in range(n)],
        "FINAL_EXP": [enc_fp12(f12r()) for _ in range(n)],
        "FINAL_EXP_WAVE": [enc_fp12(f12r()) for _ in range(n)],
        "MILLER_PROG": [enc_fp(O.G1_GEN[0]) + enc_fp(O.G1_GEN[1]) + enc_fp2(O.G2_GEN[0]) + enc_fp2(O.G2_GEN[1])] * n,
    }
    out = {}
    for op, r in recs.items():
        ts = []
        for rep in range(7):
            t0 = time.perf_counter()
            run_ops(L.tbls_test_ops, op, r)
            ts.append((time.perf_counter() - t0) * 1e3)
        out[op] = statistics.median(ts[2:])
    base = out["FP_ADD"]
    for op, v in out.items():
        print("%-14s %7.3f ms (minus baseline %6.3f)" % (op, v, v - base))




def wave_timing():
    """clock64 cycles in one 64-lane block (test hook k_test_wave_timing)."""
    L = load_test_lib()
    from oracle import bls12_381 as O

    rec = b"".join(enc_fp(3 + k) for k in range(12))
    out = run_ops(L.tbls_test_ops, "WAVE_TIMING", [rec])[0]
    c = [int.from_bytes(out[8 * i: 8 * i + 8], "little") / 64 for i in range(3)]
    print("cycles: fp_mul lane 0 %.0f, wave cyc_sqr %.0f, Miller-program level %.0f" % tuple(c))


if __name__ == "__main__":
    if "--timing" in sys.argv:
        wave_timing()
    else:
        main()
