"""KZG latency right after sustained BLS load in the same process (the
bench's order) vs cold: runs the KZG leg, then ~LOAD_S seconds of 131k-set
device partials, then the KZG leg again; prints both and the SCLK the driver
reports (rocm-smi, read-only) before and after the load.

    python tools/kzg_after_load.py [load_seconds] [bls_first]

bls_first: initialise the BLS library and run one partial before the KZG
context exists (the bench's order).
"""

import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from teku_amd import native, synth  # noqa: E402


def sclk():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True, timeout=20).stdout
        d = json.loads(out)
        return {k: v.get("sclk clock speed:") for k, v in d.items() if isinstance(v, dict)}
    except Exception as e:  # noqa: BLE001 - diagnostics only
        return str(e)


def main():
    load_s = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    bls_first = len(sys.argv) > 2 and sys.argv[2] == "bls_first"
    device = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    res = {"cold": None, "after_load": None, "bls_first": bls_first}
    if bls_first:  # the bench's order: the 131k-set workspace exists before the KZG context
        L0 = native.lib()
        n0 = 131072
        pks, msgs, sigs = synth.single_signer(0, n0)
        db0 = bench.DevBatch(pks, [1] * n0, msgs, [32] * n0, sigs, device)
        part0 = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
        native.check(L0.tbls_dev_batch_partial(0, ctypes.byref(db0.desc), torch.cuda.current_stream(device).cuda_stream,
                                               part0.data_ptr()), "partial")
        torch.cuda.synchronize()
    res["sclk_cold"] = sclk()
    res["cold"] = {k: v for k, v in bench.kzg_leg(device, 20, False).items() if k in ("p50_ms_1", "p50_ms_6")}
    L = native.lib()
    n = 131072
    pks, msgs, sigs = synth.single_signer(0, n)
    db = bench.DevBatch(pks, [1] * n, msgs, [32] * n, sigs, device)
    part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    t0, steps = time.perf_counter(), 0
    while time.perf_counter() - t0 < load_s:
        native.check(L.tbls_dev_batch_partial(0, ctypes.byref(db.desc), stream, part.data_ptr()), "partial")
        torch.cuda.synchronize()
        steps += 1
        if steps % 200 == 0:
            print("load steps", steps, flush=True)
    res["load_steps"] = steps
    res["sclk_after_load"] = sclk()
    res["after_load"] = {k: v for k, v in bench.kzg_leg(device, 20, False).items() if k in ("p50_ms_1", "p50_ms_6")}
    time.sleep(20)
    res["after_20s_idle"] = {k: v for k, v in bench.kzg_leg(device, 20, False).items() if k in ("p50_ms_1", "p50_ms_6")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
