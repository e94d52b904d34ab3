"""Config 4's failure path, device passes only: 16,384 single-signer sets with
4 bad ones through tbls_batch_verify_each, `reps` times (for rocprofv3 kernel
traces of the settle kernels), and the host-clock p50 of the call.

    python tools/settle_probe.py [reps]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from teku_amd import native, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    native.lib()
    n = 16384
    pks, msgs, sigs = synth.single_signer(0, n, seed=4)
    sg = [sigs[96 * i : 96 * i + 96] for i in range(n)]
    for j, b in {11: sg[12], 5000: bytes(96), 9999: synth.NOT_IN_G2, 16383: sg[0]}.items():
        sg[j] = b
    arr = synth.SetArray.single(pks, msgs, b"".join(sg))
    lat = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ok, each = arr.batch_verify_each(synth.fast_multipliers(n))
        lat.append((time.perf_counter() - t0) * 1e3)
        assert not ok and [i for i, v in enumerate(each) if not v] == [11, 5000, 9999, 16383]
    print(json.dumps({"settle_call_ms": lat, "p50_ms": statistics.median(lat[1:] or lat)}))


if __name__ == "__main__":
    main()
