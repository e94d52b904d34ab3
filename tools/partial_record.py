"""Print the partial record (tbls_dev_batch_partial) of a seeded synthetic
batch as JSON: the 12 Fp coordinates of the Miller product canonicalized mod p
(hex) and the invalid count.  The accumulator plan follows the environment
(TBLS_ACC_PLAN), so tests/test_gpu_accseg.py
runs it once per plan and compares the products.

    python tools/partial_record.py N [seed] [tamper_index]
"""

import ctypes
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from teku_amd import native, synth  # noqa: E402

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RINV = pow(1 << 406, -1, P)


def main():
    n = int(sys.argv[1])
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    tamper = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    device = torch.device("cuda", 0)
    pks, msgs, sigs = synth.single_signer(0, n, seed=seed)
    if 0 <= tamper < n:
        sigs = sigs[: 96 * tamper] + sigs[96 * ((tamper + 1) % n) : 96 * ((tamper + 1) % n) + 96] + sigs[96 * (tamper + 1) :]
    rng = random.Random(seed)
    db = bench.DevBatch(pks, [1] * n, msgs, [32] * n, sigs, device, rands=synth.random_multipliers(n, rng))
    part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    native.check(native.lib().tbls_dev_batch_partial(0, ctypes.byref(db.desc), stream, part.data_ptr()), "partial")
    torch.cuda.synchronize()
    raw = bytes(part.cpu().numpy())
    coords = [(int.from_bytes(raw[48 * k : 48 * k + 48], "little") * RINV) % P for k in range(12)]
    ok = ctypes.c_int(0)
    native.check(native.lib().tbls_dev_final_verify(0, part.data_ptr(), 1, stream, ctypes.byref(ok)), "final")
    print(json.dumps({"n": n, "coords": [hex(c) for c in coords], "n_bad": int.from_bytes(raw[576:580], "little"), "ok": ok.value}))


if __name__ == "__main__":
    main()
