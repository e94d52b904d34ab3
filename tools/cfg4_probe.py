"""Config-4 shaped host-API latency (tbls_batch_verify on host buffers, PCIe
included) against the device-resident partial, at a few batch sizes:

    python tools/cfg4_probe.py [n ...]
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

from teku_amd import native, synth  # noqa: E402


def main():
    ns = [int(x) for x in sys.argv[1:]] or [16384]
    native.lib()
    for n in ns:
        pks, msgs, sigs = synth.single_signer(0, n, seed=4)
        arr = synth.SetArray.single(pks, msgs, sigs)
        assert arr.batch_verify(synth.random_multipliers(n))
        ts = []
        for _ in range(int(os.environ.get("ITERS", "20"))):
            r = synth.fast_multipliers(n)
            t0 = time.perf_counter()
            ok = arr.batch_verify(r)
            ts.append((time.perf_counter() - t0) * 1e3)
            assert ok
        print({"n": n, "p50_ms": round(statistics.median(ts[2:]), 3), "min_ms": round(min(ts), 3)}, flush=True)


if __name__ == "__main__":
    main()
