"""Multi-device paths on one GPU: a fresh process
initialises the library with TBLS_INIT_SHARE_DEVICES -- 2 library devices over
the visible hardware, each with its own streams, workspace and lock -- so a
batch on an idle "node" is sharded (tbls_place_plan: down to 4,096 sets per
device), its partial records are gathered by peer copies, and a failed batch
is settled per shard on its own device, concurrently, at the per-shard verdict
offsets.  Cases: 8,192 sets (2 shards of 4,096, settled in place from the
batch's lines) and 40,960 sets (2 shards of 20,480: bucket sums, re-staged
settle), each with tampered sets at both ends of both shards, an invalid key
(its signature pair masked, k_settle_mask) and a swapped message; verdicts
against the C oracle's fastAggregateVerify per set.  Prints one JSON line.

    python tools/shared_devices_probe.py [n_devices]

Run by tests/test_gpu_shared_devices.py as a child process.
"""

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import torch  # noqa: F401  (one HIP runtime: torch's, teku_amd/native.py)

    from oracle import c_oracle as C
    from teku_amd import native, synth

    L = native.load_library()
    native.check(L.tbls_init(D, 1), "tbls_init(share devices)")
    native._lib = L
    out = {"devices": L.tbls_device_count(), "cases": []}
    for n in (8192, 40960):
        pks, msgs, sigs = synth.single_signer(0, n, seed=21)
        pk = [pks[48 * i : 48 * i + 48] for i in range(n)]
        ms = [msgs[32 * i : 32 * i + 32] for i in range(n)]
        sg = [sigs[96 * i : 96 * i + 96] for i in range(n)]
        arr = synth.SetArray(b"".join(pk), [1] * n, b"".join(ms), [32] * n, b"".join(sg))
        t = native.TblsTiming()
        ok_valid = arr.batch_verify(synth.fast_multipliers(n), timing=t)
        h = n // 2
        bad = {0: ("sig", sg[1]), h - 1: ("sig", bytes(96)), h: ("sig", synth.NOT_IN_G2), n - 1: ("sig", sg[0]),
               h + 7: ("pk", synth.BAD_PK), 5: ("msg", ms[6])}
        for j, (kind, v) in bad.items():
            if kind == "sig":
                sg[j] = v
            elif kind == "pk":
                pk[j] = v
            else:
                ms[j] = v
        arr = synth.SetArray(b"".join(pk), [1] * n, b"".join(ms), [32] * n, b"".join(sg))
        te = native.TblsTiming()
        native.stats(reset=True)
        ok, each = arr.batch_verify_each(synth.fast_multipliers(n), timing=te)
        st = native.stats()
        exp = C.verify_each([[p] for p in pk], ms, sg, threads=16)
        out["cases"].append({"n": n, "valid_batch": ok_valid, "valid_devices": t.n_devices, "failed_batch": ok, "each_devices": te.n_devices,
                             "device_ms": te.device_ms, "bad_expected": sorted(bad), "bad_got": [i for i, v in enumerate(each) if not v],
                             "match_oracle": each == exp, "settled": st["settled"], "partials": st["partials"]})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
