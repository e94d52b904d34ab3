"""Phase times of the 128-set coop hash (k_set_hash_coop) from a profiling
build with -DTB_HASH_STAMPS (tools/build_variant.py stamps TB_HASH_STAMPS
--tus k_hwave.hip; run with TBLS_LIB=teku_amd/lib/variants/libtekubls_hip_stamps.so):
128-set batch verifications through the host API, then the median over the
sets of the last call of each phase, in microseconds (wall_clock64, 100 MHz).

    TBLS_LIB=... python tools/hash_stamps_probe.py [n] [reps]
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["start->field (lane 0: expand_message_xmd, hash_to_field)", "field->sswu (rows 0 and 4: two SSWU maps)",
          "sswu->iso (lane 0: E2' addition + 3-isogeny)", "iso->slots (slot setup)", "slots->levels (cofactor program)",
          "levels->to_fp (barrier)", "to_fp->end (lane 0: affine conversion)"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch  # noqa: F401

    from teku_amd import native, synth

    L = native.lib()
    fn = L.tbls_debug_hash_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_uint]
    pks, msgs, sigs = synth.single_signer(0, n, seed=3)
    arr = synth.SetArray.single(pks, msgs, sigs)
    per = {p: [] for p in PHASES}
    tot, inv = [], []
    buf = (ctypes.c_ulonglong * (16 * n))()
    for _ in range(reps):
        assert arr.batch_verify(synth.fast_multipliers(n))
        assert fn(buf, n) == 0
        for i in range(n):
            t = [buf[16 * i + k] for k in range(8)]
            for k, p in enumerate(PHASES):
                per[p].append((t[k + 1] - t[k]) / 100.0)  # 100 MHz ticks -> us
            tot.append((t[7] - t[0]) / 100.0)
            inv.append((buf[16 * i + 8] - t[6]) / 100.0)
    out = {"n": n, "reps": reps, "phase_us_median": {p: statistics.median(v) for p, v in per.items()}, "total_us_median": statistics.median(tot),
           "to_fp->affine (row 0: row inversion + 2 coop products)": statistics.median(inv)}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
