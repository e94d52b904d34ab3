"""The failing order of round 4's gpurun_out/r04r_pytest.log, in one fresh process:
the library initialises the device and does real work first (batches, the
1,048,576-set signing of the config-5 fixture), and only then does torch
initialise HIP.  Prints one JSON line: the libamdhip64 copies mapped into the
process, whether torch's initialisation worked, the HIP error state the
library saw.  Exit 0 iff torch initialised and one runtime is mapped.

  python tools/runtime_order_probe.py [preload|nopreload] [sets_to_sign]

`nopreload` sets TBLS_HIP_PRELOAD=0 (teku_amd/native.py): the library binds
the system HIP runtime and torch maps its own beside it (round 4's state).
Run by tests/test_gpu_runtime.py as a child process (one process per order).
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "preload"
    n_sign = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    if mode == "nopreload":
        os.environ["TBLS_HIP_PRELOAD"] = "0"
    sys.path.insert(0, ROOT)
    from teku_amd import native, synth

    out = {"mode": mode, "sets_signed": n_sign}
    t0 = time.time()
    L = native.lib()  # the library initialises HIP first
    pks, msgs, sigs = synth.single_signer(0, 16384, seed=9)
    arr = synth.SetArray.single(pks, msgs, sigs)
    out["batch_16k"] = arr.batch_verify(synth.fast_multipliers(16384))
    small = synth.SetArray.single(pks[: 48 * 128], msgs[: 32 * 128], sigs[: 96 * 128])
    out["batch_128"] = small.batch_verify(synth.fast_multipliers(128))
    native.check(L.tbls_pk_table_load(pks[: 48 * 4096], 4096, None), "pk_table_load")
    big = synth.single_signer(0, n_sign, seed=5)  # the config-5 fixture: tbls_sign_many on the device
    out["signed_bytes"] = len(big[2])
    out["library_s"] = round(time.time() - t0, 2)
    out["runtimes_before_torch"] = native._loaded_hip_runtimes()
    import torch

    try:
        torch.cuda.init()
        x = torch.arange(1024, device="cuda").sum().item()
        out["torch_ok"] = x == 1024 * 1023 // 2
    except RuntimeError as e:
        out["torch_ok"] = False
        out["torch_error"] = str(e)
    out["runtimes"] = native._loaded_hip_runtimes()
    # the library keeps working after torch's initialisation
    out["batch_128_after"] = small.batch_verify(synth.fast_multipliers(128))
    print(json.dumps(out), flush=True)
    return 0 if out["torch_ok"] and len(out["runtimes"]) == 1 and out["batch_128_after"] else 1


if __name__ == "__main__":
    sys.exit(main())
