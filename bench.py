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

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# Algorithmic work per unit, in Fp-multiplication equivalents (M), counted by
# tools/count_muls.py on the hostsim build of the same kernel code.
# One M = 12x12 limb Montgomery product = 2*12^2 = 288 32x32->64 MACs.
MACS_PER_M = 288
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


def cpu_baseline_oracle(sample_sets=4):
    """The oracle (pure-Python restatement) timed on a bounded sample."""
    from oracle import bls12_381 as O

    sks = [interop_sk(i) for i in range(sample_sets)]
    msgs = [bench_message(0, j) for j in range(sample_sets)]
    pks = [[O.sk_to_pk(s)] for s in sks]
    sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
    rands = [secrets.randbits(64) | 1 for _ in range(sample_sets)]
    t0 = time.perf_counter()
    ok = O.batch_verify(pks, msgs, sigs, rands)
    dt = time.perf_counter() - t0
    assert ok
    return {
        "value": sample_sets / dt,
        "unit": "sigs/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle.bls12_381.batch_verify of {sample_sets} interop-key sets (pure Python, 1 thread); build CPU path, not blst",
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
    pks, msgs, sigs = make_workload(L, rank * S, S)
    batch = DevBatch(pks, msgs, sigs, S, device)
    gen_s = time.perf_counter() - t_gen
    partial = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    gathered = torch.empty(world * native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
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
        if world > 1:
            dist.all_gather_into_tensor(gathered, partial)
            src = gathered
        else:
            src = partial
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
    if rank != 0:
        dist.barrier()
        dist.destroy_process_group()
        return

    stage_ms = [a / args.steps for a in stage_acc]
    # integer-VALU roofline of the dominant kernel: k_miller (largest single
    # kernel; it runs alone after the three concurrent per-set stages join)
    dom = STAGES.index("miller")
    props = torch.cuda.get_device_properties(device)
    cus = props.multi_processor_count
    peak_tmacs = cus * 128 * 2.4e9 / 1e12  # v_mad_u64_u32: full rate, 4 SIMD32 per CU, 2.4 GHz max clock
    m_unit = M_PER_UNIT.get(STAGES[dom])
    units = S + 1 if STAGES[dom] == "miller" else S
    achieved = None
    if m_unit:
        achieved = m_unit * MACS_PER_M * units / (stage_ms[dom] * 1e-3) / 1e12
    roofline = {
        "bound": "valu-int",
        "kernel": "k_" + STAGES[dom],
        "achieved": achieved,
        "peak": peak_tmacs,
        "unit": "TMAC/s",
        "frac": (achieved / peak_tmacs) if achieved else None,
        "traffic": None,
        "m_per_unit": m_unit,
        "macs_per_m": MACS_PER_M,
        "units_per_launch": units,
        "kernel_ms": stage_ms[dom],
        "stage_tmacs": {
            STAGES[i]: (M_PER_UNIT[STAGES[i]] * MACS_PER_M * (S + 1 if STAGES[i] == "miller" else S) / (stage_ms[i] * 1e-3) / 1e12)
            if M_PER_UNIT.get(STAGES[i]) and stage_ms[i] > 0 else None
            for i in range(len(STAGES))
        },
    }

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

    cpu = None if args.no_cpu_baseline else cpu_baseline_oracle()
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
        "dtype": "u32 (381-bit Montgomery Fp on 12x32-bit limbs)",
        "data": "synthetic: interop keys (first 65,536 reused cyclically), distinct sha256 messages, GPU-signed",
        "config": {
            "workload": "config 5 per-GPU shard: randomized batchVerify of %d single-signer sets per GPU, RCCL Fp12 partial gather, 1 final exp" % S,
            "sets_per_gpu": S,
            "parallelism": "data-parallel shards, dp%d" % world,
        },
        "p50_latency_ms_128": statistics.median(lat),
        "p99_latency_ms_128": lat[min(len(lat) - 1, int(0.99 * len(lat)))],
        "stage_ms": dict(zip(STAGES, stage_ms)),
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
