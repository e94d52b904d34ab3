"""Benchmark: randomized BLS batchVerify throughput on 1-8 MI355X.

Workload (one "step"): every rank verifies its own shard of S single-signer
signature sets (interop keys reused cyclically from the first 65,536, distinct
32-byte messages) through the device-resident C ABI: per-GPU partial Miller
product (incl. its (-g1, sum r_i sig_i) pair) -> RCCL all_gather of the 580-byte
partials -> rank 0 multiplies them and runs one final exponentiation.  This is
config 5's per-GPU shard (1,048,576 sets over 8 GPUs = 131,072 per GPU) with
weak scaling; inputs are resident in HBM before the timed region.

Also reported: p50/p99 latency of a 128-set batchVerify (config 1 shape)
through the host C ABI (API entry -> boolean, PCIe upload included), the
per-stage kernel times, the integer-VALU roofline of the dominant kernel, and a
CPU baseline (the oracle, timed on a bounded sample on this host).

python bench.py --gpus N --steps K --warmup W
"""

import argparse
import ctypes
import hashlib
import json
import os
import secrets
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from teku_amd import native  # noqa: E402
from teku_amd.dist import all_gather_partials, shard_bounds  # noqa: E402

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# Algorithmic work per unit: Fp products (and their v_mad_u64_u32 count),
# counted by tools/count_muls.py on the hostsim build of the same stage code.
STAGES = ["pk_decompress", "set_pk", "set_sig", "set_hash", "g2_sum", "miller", "fp12_prod"]
M_PER_UNIT = json.load(open(os.path.join(ROOT, "tools", "mul_counts.json"))) if os.path.exists(
    os.path.join(ROOT, "tools", "mul_counts.json")
) else {}


def interop_sk(i):
    h = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(h, "little") % R_ORDER


def bench_message(seed, j):
    return hashlib.sha256(b"teku-bench" + seed.to_bytes(8, "little") + j.to_bytes(8, "little")).digest()


def make_workload(L, first, count, n_keys_uniq=65536):
    """Synthetic sets [first, first+count): pk/sig generated on the GPU."""
    kidx = [(first + j) % n_keys_uniq for j in range(count)]
    uniq = sorted(set(kidx))
    sk_bytes = {k: interop_sk(k).to_bytes(32, "big") for k in uniq}
    blob = b"".join(sk_bytes[k] for k in uniq)
    pk_out = ctypes.create_string_buffer(48 * len(uniq))
    native.check(L.tbls_sk_to_pk_many(blob, len(uniq), pk_out), "sk_to_pk_many")
    pk_of = {k: pk_out.raw[48 * i : 48 * i + 48] for i, k in enumerate(uniq)}
    msgs = [bench_message(0, first + j) for j in range(count)]
    sks = b"".join(sk_bytes[k] for k in kidx)
    mb = b"".join(msgs)
    off = (ctypes.c_uint32 * (count + 1))(*[32 * j for j in range(count + 1)])
    sig_out = ctypes.create_string_buffer(96 * count)
    CH = 65536
    for s in range(0, count, CH):
        e = min(count, s + CH)
        o2 = (ctypes.c_uint32 * (e - s + 1))(*[32 * j for j in range(e - s + 1)])
        tmp = ctypes.create_string_buffer(96 * (e - s))
        native.check(L.tbls_sign_many(sks[32 * s : 32 * e], mb[32 * s : 32 * e], o2, e - s, DST, len(DST), tmp), "sign_many")
        ctypes.memmove(ctypes.addressof(sig_out) + 96 * s, tmp, 96 * (e - s))
    del off
    pks = b"".join(pk_of[k] for k in kidx)
    return pks, mb, sig_out.raw


class DevBatch:
    """A batch resident in HBM (torch tensors) + its tbls_dev_batch descriptor."""

    def __init__(self, pks, msgs, sigs, n, device):
        u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(device)  # noqa: E731
        self.pks = u8(pks)
        self.msgs = u8(msgs)
        self.sigs = u8(sigs)
        self.pk_off = torch.arange(0, n + 1, dtype=torch.int32, device=device)
        self.msg_off = torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=device)
        r = [secrets.randbits(64) | 1 for _ in range(n)]  # randomizers in [1, 2^64)
        self.rand = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in r], dtype=torch.int64, device=device)
        self.desc = native.TblsDevBatch(
            self.pks.data_ptr(), self.pk_off.data_ptr(), n, self.msgs.data_ptr(), self.msg_off.data_ptr(), self.sigs.data_ptr(), self.rand.data_ptr(), n
        )
        self.n = n


# Integer-MAC roofline.  The bound is the v_mad_u64_u32 issue rate: measured
# 47.6 lane-ops/CU/clk on MI355X (tools/microbench/fp_rates.hip,
# profiles/r01_microbench_fp_rates.json) -> x CUs x 2.4 GHz.  Algorithmic work
# = Fp products per unit (tools/count_muls.py on the same stage code) x 392
# v_mad_u64_u32 per product (301 per squaring), tools/mul_counts.json.
MAD_RATE_PER_CU_CLK = 47.6
CLOCK_HZ = 2.4e9
STAGE_UNITS = {"pk_decompress": "keys", "set_pk": "sets", "set_sig": "sets", "set_hash": "sets", "g2_sum": "sets", "miller": "pairs", "fp12_prod": "pairs"}


def roofline_entry(stage_ms, S, device):
    props = torch.cuda.get_device_properties(device)
    peak = MAD_RATE_PER_CU_CLK * props.multi_processor_count * CLOCK_HZ / 1e12  # T mad/s
    mads = M_PER_UNIT.get("mads_per_unit", {})
    per_stage = {}
    for i, name in enumerate(STAGES):
        if name in mads and stage_ms[i] > 0:
            per_stage[name] = mads[name] * S / (stage_ms[i] * 1e-3) / 1e12
    dom = max(range(len(STAGES)), key=lambda i: stage_ms[i])  # exclusive times
    name = STAGES[dom]
    achieved = per_stage.get(name)
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath)).get("k_" + ("miller2" if name == "miller" else name), {}).get("bytes_per_launch")
    return {
        "bound": "valu-int (v_mad_u64_u32 issue)",
        "kernel": "k_" + ("miller2" if name == "miller" else name),
        "achieved": achieved,
        "peak": peak,
        "unit": "T v_mad_u64_u32/s",
        "frac": (achieved / peak) if achieved else None,
        "traffic": traffic,
        "units_per_launch": S,
        "unit_of_work": STAGE_UNITS[name],
        "mads_per_unit": mads.get(name),
        "fp_products_per_unit": M_PER_UNIT.get(name),
        "kernel_ms": stage_ms[dom],
        "stage_frac": {k: v / peak for k, v in per_stage.items()},
    }


def cpu_baseline_oracle(pks, msgs, sigs, sample_sets=4096, threads=16):
    """The C oracle (oracle/c/bls_oracle.c, 'port') timed on this host over a
    bounded sample of the same workload: the first `sample_sets` sets."""
    from oracle import c_oracle as C

    threads = max(1, min(threads, os.cpu_count() or 1))
    n = sample_sets
    pk = [pks[48 * j : 48 * j + 48] for j in range(n)]
    ms = [msgs[32 * j : 32 * j + 32] for j in range(n)]
    sg = [sigs[96 * j : 96 * j + 96] for j in range(n)]
    rr = [secrets.randbits(64) | 1 for _ in range(n)]
    t0 = time.perf_counter()
    ok = C.batch_verify(pk, ms, sg, rr, threads=threads)
    dt = time.perf_counter() - t0
    assert ok, "C oracle rejected the valid sample"
    return {
        "value": n / dt,
        "unit": "sigs/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle/c batch_verify of the first {n} sets of this workload, {threads} pthreads, {dt:.1f} s; "
        "build's own C restatement (6x64-bit CIOS Montgomery), not blst",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets-per-gpu", type=int, default=int(os.environ.get("TBLS_SETS_PER_GPU", 131072)))
    ap.add_argument("--lat-reps", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    L = native.lib()

    S = args.sets_per_gpu
    t_gen = time.perf_counter()
    lo, hi = shard_bounds(S * world, world, rank)  # weak scaling: S sets per rank
    pks, msgs, sigs = make_workload(L, lo, hi - lo)
    batch = DevBatch(pks, msgs, sigs, S, device)
    gen_s = time.perf_counter() - t_gen
    partial = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    stage_acc = [0.0] * len(STAGES)
    ok = ctypes.c_int(0)
    stage = (ctypes.c_float * 8)()

    def step(timed_stages):
        if timed_stages:
            native.check(L.tbls_dev_batch_partial_timed(local, ctypes.byref(batch.desc), stream, partial.data_ptr(), stage), "partial")
            for i in range(len(STAGES)):
                stage_acc[i] += stage[i]
        else:
            native.check(L.tbls_dev_batch_partial(local, ctypes.byref(batch.desc), stream, partial.data_ptr()), "partial")
        src = all_gather_partials(partial)
        if rank == 0:
            native.check(L.tbls_dev_final_verify(local, src.data_ptr(), world, stream, ctypes.byref(ok)), "final")
            if ok.value != 1:
                raise RuntimeError("valid synthetic batch rejected")

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    total_sets = S * world * args.steps
    value = total_sets / dt

    # Same steps with the keys in the device-resident validator table
    # (tbls_pk_table_load / tbls_dev_batch_partial_idx):
    # keys decompressed and validated once, as Teku memoizes them per
    # BLSPublicKey.  Reported beside `value`, which decodes every key per step.
    T = min(S, 65536)
    native.check(L.tbls_pk_table_load(pks[: 48 * T], T, None), "pk_table_load")
    key_idx = torch.arange(0, S, dtype=torch.int32, device=device) % T

    def step_tab():
        native.check(L.tbls_dev_batch_partial_idx(local, ctypes.byref(batch.desc), key_idx.data_ptr(), stream, partial.data_ptr()), "partial_idx")
        src = all_gather_partials(partial)
        if rank == 0:
            native.check(L.tbls_dev_final_verify(local, src.data_ptr(), world, stream, ctypes.byref(ok)), "final")
            if ok.value != 1:
                raise RuntimeError("valid synthetic batch rejected (key table)")

    step_tab()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_tab()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt_tab = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt_tab], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_tab = float(t.item())
    if rank != 0:
        dist.barrier()
        dist.destroy_process_group()
        return

    stage_ms = [a / args.steps for a in stage_acc]
    # Exclusive per-stage kernel times (every stage alone on the stream): the
    # roofline's denominators.  In the timed steps the stages overlap, so
    # their event brackets include each other's work.
    excl = [0.0] * len(STAGES)
    for _ in range(2):
        native.check(L.tbls_dev_batch_stage_profile(local, ctypes.byref(batch.desc), stream, partial.data_ptr(), stage), "profile")
        for i in range(len(STAGES)):
            excl[i] += stage[i] / 2
    roofline = roofline_entry(excl, S, device)

    # p50 latency of a 128-set batchVerify through the host C ABI (config 1 shape)
    from teku_amd import bls

    lat = []
    if args.lat_reps <= 0:
        lat = [float("nan")]
    sets128 = [(pks[48 * j : 48 * j + 48], 1, msgs[32 * j : 32 * j + 32], sigs[96 * j : 96 * j + 96]) for j in range(128)]
    for _ in range(args.lat_reps + 3 if args.lat_reps > 0 else 0):
        rr = [secrets.randbits(64) | 1 for _ in range(128)]
        t1 = time.perf_counter()
        good = bls.batch_verify_raw(sets128, rr, n_gpus=1)
        lat.append((time.perf_counter() - t1) * 1e3)
        assert good
    lat = sorted(lat[3:]) if args.lat_reps > 0 else lat

    cpu = None if args.no_cpu_baseline else cpu_baseline_oracle(pks, msgs, sigs, min(4096, S))
    line = {
        "metric": "BLS sigs verified/sec (batchVerify), 1-8 GPUs; p50 latency @128-sig batch",
        "value": value,
        "unit": "sigs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery Fp, 14x29-bit limb products)",
        "data": "synthetic: interop keys (first 65,536 reused cyclically), distinct sha256 messages, GPU-signed",
        "config": {
            "workload": "config 5 per-GPU shard: randomized batchVerify of %d single-signer sets per GPU, RCCL Fp12 partial gather, 1 final exp" % S,
            "sets_per_gpu": S,
            "parallelism": "data-parallel shards, dp%d" % world,
        },
        "value_key_table": total_sets / dt_tab,
        "ms_per_step_key_table": dt_tab / args.steps * 1e3,
        "key_table": "value_key_table: same steps with keys from the device-resident validator table (%d keys decompressed "
        "and validated once, as Teku memoizes BLSPublicKey); value decodes and group-checks every key per step" % T,
        "p50_latency_ms_128": statistics.median(lat),
        "p99_latency_ms_128": lat[min(len(lat) - 1, int(0.99 * len(lat)))],
        "stage_ms_overlapped": dict(zip(STAGES, stage_ms)),
        "stage_ms_exclusive": dict(zip(STAGES, excl)),
        "roofline": roofline,
        "cpu_baseline": cpu,
        "workload_gen_s": gen_s,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
