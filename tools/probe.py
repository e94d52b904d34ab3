"""Device-resident timing probes for A/B runs under rocprofv3 (tuning env vars
are read once per process):

    python tools/probe.py partial N [reps]      tbls_dev_batch_partial of N single-signer sets
    python tools/probe.py multikey S K [reps]   tbls_dev_batch_partial of S sets x K keys
    python tools/probe.py stages N [reps]       one warm partial, then only the stage profile (every
                                                stage alone on the stream: per-kernel exclusive times
                                                under rocprofv3 --kernel-trace --stats)
"""

import ctypes
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
    what = sys.argv[1]
    device = torch.device("cuda", 0)
    L = native.lib()
    stream = torch.cuda.current_stream(device).cuda_stream
    stages_only = what == "stages"
    if what in ("partial", "stages"):
        n = int(sys.argv[2])
        reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
        pks, msgs, sigs = synth.single_signer(0, n)
        db = bench.DevBatch(pks, [1] * n, msgs, [32] * n, sigs, device)
    else:
        s, k = int(sys.argv[2]), int(sys.argv[3])
        reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
        r1 = len(sys.argv) > 5 and sys.argv[5] == "r1"  # randomizers 1: no [r] apk scalar multiplication
        keys, msgs, sigs = synth.multi_key(s, k, first_key=1000, seed=3)
        db = bench.DevBatch(b"".join(b"".join(x) for x in keys), [k] * s, b"".join(msgs), [32] * s, b"".join(sigs), device,
                            rands=[1] * s if r1 else None)
    part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    st = (ctypes.c_float * 8)()
    ts, stages = [], []
    for rep in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if not (stages_only and rep):
            native.check(L.tbls_dev_batch_partial(0, ctypes.byref(db.desc), stream, part.data_ptr()), "partial")
        torch.cuda.synchronize()
        if rep:
            ts.append((time.perf_counter() - t0) * 1e3)
        native.check(L.tbls_dev_batch_stage_profile(0, ctypes.byref(db.desc), stream, part.data_ptr(), st), "profile")
        if rep:
            stages.append(list(st)[:7])
    ok = ctypes.c_int(0)
    native.check(L.tbls_dev_final_verify(0, part.data_ptr(), 1, stream, ctypes.byref(ok)), "final")
    assert ok.value == 1
    med = {k: round(statistics.median(r[i] for r in stages), 3) for i, k in enumerate(bench.STAGES)}
    print({"what": sys.argv[1:], "env": {k: v for k, v in os.environ.items() if k.startswith("TBLS_")}, "partial_ms": round(statistics.median(ts), 3),
           "stage_ms_exclusive": med}, flush=True)


if __name__ == "__main__":
    main()
