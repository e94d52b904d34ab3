"""Small-batch (config 1) stage breakdown on the GPU: exclusive per-stage
kernel times (every stage alone on the stream), the overlapped partial, and
the final verification, for n single-signer sets on device-resident inputs.

    python tools/stage_small.py [n ...]      (default 128)
"""

import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from teku_amd import native, synth  # noqa: E402


def main():
    ns = [int(x) for x in sys.argv[1:]] or [128]
    device = torch.device("cuda", 0)
    L = native.lib()
    stream = torch.cuda.current_stream(device).cuda_stream
    out = {}
    for n in ns:
        pks, msgs, sigs = synth.single_signer(0, n)
        db = bench.DevBatch(pks, [1] * n, msgs, [32] * n, sigs, device)
        part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
        st = (ctypes.c_float * 8)()
        ok = ctypes.c_int(0)
        excl, over, fin, tot = [], [], [], []
        for rep in range(12):
            native.check(L.tbls_dev_batch_stage_profile(0, ctypes.byref(db.desc), stream, part.data_ptr(), st), "profile")
            excl.append(list(st)[:7])
            native.check(L.tbls_dev_batch_partial_timed(0, ctypes.byref(db.desc), stream, part.data_ptr(), st), "timed")
            over.append(list(st)[:7])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            native.check(L.tbls_dev_batch_partial(0, ctypes.byref(db.desc), stream, part.data_ptr()), "partial")
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            native.check(L.tbls_dev_final_verify(0, part.data_ptr(), 1, stream, ctypes.byref(ok)), "final")
            t2 = time.perf_counter()
            assert ok.value == 1
            if rep >= 2:
                tot.append((t1 - t0) * 1e3)
                fin.append((t2 - t1) * 1e3)
        med = lambda rows: {k: statistics.median(r[i] for r in rows[2:]) for i, k in enumerate(bench.STAGES)}  # noqa: E731
        out[n] = {"stage_ms_exclusive": med(excl), "stage_ms_overlapped": med(over), "partial_wall_ms": statistics.median(tot),
                  "final_wall_ms": statistics.median(fin)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
