"""131k-set partial time with the library's workspace allocated before the
test data and device batch ("ws_first") or after them (the bench's order):
does allocation order move the BLS kernels as it moved KZG's
?

    python tools/alloc_order_probe.py ws_first|data_first [reps]
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
    mode = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    device = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = native.lib()
    n = 131072
    stream = torch.cuda.current_stream(device).cuda_stream
    part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    if mode == "ws_first":  # size the workspace with a dummy batch of the same shape first
        dummy = bench.DevBatch(bytes(48 * n), [1] * n, bytes(32 * n), [32] * n, bytes(96 * n), device)
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(dummy.desc), stream, part.data_ptr()), "partial")
        torch.cuda.synchronize()
    pks, msgs, sigs = synth.single_signer(0, n)
    db = bench.DevBatch(pks, [1] * n, msgs, [32] * n, sigs, device)
    ts = []
    for r in range(reps + 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(db.desc), stream, part.data_ptr()), "partial")
        torch.cuda.synchronize()
        if r >= 3:
            ts.append((time.perf_counter() - t0) * 1e3)
    print({"mode": mode, "partial_ms_p50": round(statistics.median(ts), 3), "min": round(min(ts), 3)}, flush=True)


if __name__ == "__main__":
    main()
