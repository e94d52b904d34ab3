"""KZG latency by allocation order (VERDICT round 5
item 7): in a fresh process, either the KZG context first (load + one 6-blob
verification) and then a 131k-set BLS partial, or the BLS partial first and
then the KZG context; then the KZG host-API p50 at 1 and 6 blobs and the
device-resident 64-blob batch.  Prints one JSON line.

    python tools/kzg_order_probe.py kzg_first|bls_first [reps]

Run under rocprofv3 --pmc to compare the KZG kernels' counters between the
two orders (tools/gpu_r06c.sh).
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


def bls_partial(device):
    L = native.lib()
    n = 131072
    pks, msgs, sigs = synth.single_signer(0, n)
    db = bench.DevBatch(pks, [1] * n, msgs, [32] * n, sigs, device)
    part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    native.check(L.tbls_dev_batch_partial(0, ctypes.byref(db.desc), torch.cuda.current_stream(device).cuda_stream, part.data_ptr()),
                 "partial")
    torch.cuda.synchronize()
    return db, part


def main():
    order = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    device = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    keep = None
    if order == "kzg_first":
        bench.kzg_warm()
        keep = bls_partial(device)
    else:
        keep = bls_partial(device)
    t0 = time.perf_counter()
    leg = bench.kzg_leg(device, reps, False)
    res = {"order": order, "lib": os.environ.get("TBLS_LIB", "main"), "p50_ms_1": leg["p50_ms_1"], "p50_ms_6": leg["p50_ms_6"],
           "dev_64_ms": leg.get("dev_64", {}).get("ms"), "leg_s": time.perf_counter() - t0}
    del keep
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
