"""The 128-set latency path (BASELINE p50 metric) for a kernel trace: K
randomized batch verifications of 128 single-signer sets through the host
API (tbls_batch_verify, PCIe included) with 20 ms of idle between calls, so
each call's kernels form one group in a rocprofv3 --kernel-trace; prints the
host p50.  tools/critical_path.py turns the trace into the per-stage
critical path (profiles/r06_latency_128.json).

    rocprofv3 --kernel-trace -d DIR -o lat --output-format csv -- python3 tools/latency_probe.py [n] [reps]
"""

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    import torch  # noqa: F401  (one HIP runtime: torch's)

    from teku_amd import native, synth

    native.lib()
    pks, msgs, sigs = synth.single_signer(0, n, seed=3)
    arr = synth.SetArray.single(pks, msgs, sigs)
    for _ in range(5):
        assert arr.batch_verify(synth.fast_multipliers(n))
    lat = []
    for _ in range(reps):
        time.sleep(0.02)
        t0 = time.perf_counter()
        ok = arr.batch_verify(synth.fast_multipliers(n))
        lat.append((time.perf_counter() - t0) * 1e3)
        assert ok
    print(json.dumps({"n": n, "reps": reps, "p50_ms": statistics.median(lat), "min_ms": min(lat)}), flush=True)


if __name__ == "__main__":
    main()
