"""Gossip-flood failure path (config 4 shape): 16384
single-key sets with `--bad` invalid signatures, settled by the service's
per-set pass (tbls_verify_each) vs the reference's recursive halving
(AggregatingSignatureVerificationService.java:208-227, split_fallback=True).
Prints one JSON line: per-set pass throughput and both fallbacks' wall time."""

import argparse
import ctypes
import json
import random
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--bad", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from oracle.keys import interop_sk
    from teku_amd import bls, native
    from teku_amd.service import AggregatingSignatureVerificationService, SignatureTask

    L = native.lib()
    n, nk = a.n, 512
    sks = b"".join(interop_sk(i % nk).to_bytes(32, "big") for i in range(n))
    pk_out = ctypes.create_string_buffer(48 * nk)
    native.check(L.tbls_sk_to_pk_many(sks[: 32 * nk], nk, pk_out), "sk_to_pk_many")
    msgs = [i.to_bytes(4, "little") * 8 for i in range(n)]
    off = (ctypes.c_uint32 * (n + 1))(*[32 * j for j in range(n + 1)])
    sig_out = ctypes.create_string_buffer(96 * n)
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    native.check(L.tbls_sign_many(sks, b"".join(msgs), off, n, dst, len(dst), sig_out), "sign_many")
    sets = [(pk_out.raw[48 * (i % nk) : 48 * (i % nk) + 48], 1, msgs[i], sig_out.raw[96 * i : 96 * i + 96]) for i in range(n)]
    rng = random.Random(1)
    bad = sorted(rng.sample(range(n), a.bad))
    for i in bad:
        sets[i] = (sets[i][0], 1, sets[i][2], sets[(i + 1) % n][3])
    exp = [i not in set(bad) for i in range(n)]

    bls.verify_each_raw(sets[:256])  # warm up
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got = bls.verify_each_raw(sets)
        ts.append(time.perf_counter() - t0)
    assert got == exp, "per-set verdicts differ"
    each_s = min(ts)

    def settle(split):
        svc = AggregatingSignatureVerificationService(max_batch_size=n, split_fallback=split)
        tasks = [SignatureTask([s]) for s in sets]
        t0 = time.perf_counter()
        svc.batch_verify_signatures(tasks)
        dt = time.perf_counter() - t0
        assert [t.result.result() for t in tasks] == exp
        return dt, svc.device_passes

    gpu_s, gpu_passes = settle(False)
    ref_s, ref_passes = settle(True)
    print(
        json.dumps(
            {
                "metric": "per-set verdicts/sec (tbls_verify_each)",
                "n_sets": n,
                "bad": a.bad,
                "verify_each_s": round(each_s, 4),
                "verify_each_sets_per_s": round(n / each_s, 1),
                "service_per_set_fallback_s": round(gpu_s, 4),
                "service_per_set_device_passes": gpu_passes,
                "reference_halving_fallback_s": round(ref_s, 4),
                "reference_halving_device_passes": ref_passes,
            }
        ),
        flush=True,
    )


if __name__ == "__main__":
    main()
