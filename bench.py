"""Benchmark: randomized BLS batchVerify throughput on 1-8 MI355X.

Workload (one "step"): every rank verifies its own shard of S single-signer
signature sets (interop keys reused cyclically from the first 65,536, distinct
32-byte messages) through the device-resident C ABI: per-GPU partial Miller
product (incl. its (-g1, sum r_i sig_i) pair) -> RCCL all_gather of the 580-byte
partials -> rank 0 multiplies them and runs one final exponentiation.  This is
config 5's per-GPU shard (1,048,576 sets over 8 GPUs = 131,072 per GPU) with
weak scaling; inputs are resident in HBM before the timed region.

Also reported on rank 0 (extra keys of the same JSON line):
  * config 1: p50/p99 latency of a 128-set batchVerify through the host C ABI
    (API entry -> boolean, PCIe upload included), >= 100 repetitions;
  * config 2: 64 x 512-key fastAggregateVerify (tbls_fast_aggregate_verify_many);
  * config 3: 64 x 488-key randomized batchVerify (keys as bytes, and from the
    device-resident key table), with the aggregation kernel's roofline;
  * config 4: 16,384 single-signer sets through the host C ABI (the service's
    batch), and the failure-path settle time with 4 bad signatures;
  * the per-stage kernel times and the integer-MAC roofline of the dominant
    kernel on SURVEY.md 8(d)'s model (300 MAC per Fp product);
  * the CPU baseline: the C oracle timed on this host's cores (N threads and
    1 thread, CPU model stated) on a bounded sample of the same workload.

python bench.py --gpus N --steps K --warmup W
"""

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Hardware queues per process (read by the HIP runtime at its first use,
# before torch or the library touch the device).  The BLS library opens four
# streams per device (the caller's pipeline and three per-set stage streams);
# with the runtime's default of four hardware queues the KZG context's two
# streams, opened after them, share queues with them and the KZG pipeline ran
# 12 % slower (profiles/r06_kzg_hw_queues.json).  A node
# running both contexts on a GPU sets at least 8.  The GPU
# boxes export GPU_MAX_HW_QUEUES=4 (the runtime's default) in the environment,
# so a lower value is raised; TBLS_BENCH_HW_QUEUES sets it explicitly (A/B).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("TBLS_BENCH_HW_QUEUES") or str(max(8, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from teku_amd import native, synth  # noqa: E402
from teku_amd.dist import all_gather_partials, shard_bounds  # noqa: E402

# ---------------------------------------------------------------------------
# Roofline: algorithmic work = Fp products (M) per unit,
# counted by tools/count_muls.py on the host build of the same stage code,
# x 300 32x32->64 MACs per M (12-limb CIOS Montgomery, 2*12^2 + 12).  Peak =
# the measured v_mad_u64_u32 throughput of the whole chip at four waves per
# SIMD (tools/microbench/mad_peak.hip, profiles/r04_microbench_mad_peak.json:
# 3.39e13 MAD/s = 59.1 lane-ops/CU/clk at the 2.24 GHz the box ran; rounds 1-3
# used 47.6 lane-ops/CU/clk x 2.4 GHz = 2.92e13 from a microbenchmark whose
# inline-asm multiply-adds each got a hazard s_nop).  One wave per SIMD -- the
# occupancy of every 512-register kernel -- issues at most 2.65e13 MAD/s
# (47.1 lane-ops/CU/clk): "frac_1wave" reports the dominant kernel against
# that ceiling.  The kernels' own 14 x 29-bit products issue 392
# v_mad_u64_u32 per M (301 per squaring); "issue_frac" reports that
# instruction-level fraction too.
# ---------------------------------------------------------------------------
MAC_PER_M = 300
MAD_PEAK_PER_S = 3.3923e13  # 256 CUs, four waves per SIMD (measured)
MAD_1WAVE_PER_S = 2.6492e13  # one wave per SIMD (measured)
STAGES = ["pk_decompress", "set_pk", "set_sig", "set_hash", "g2_sum", "miller", "fp12_prod"]
STAGE_KERNEL = {
    "pk_decompress": "k_pk_decompress",
    "set_pk": "k_set_pk_w2",
    "set_sig": "k_sig_check_w2",
    "set_hash": "k_set_hash_w2 + k_set_hash_fix",
    "g2_sum": "k_msm_bucket_tree + k_msm_bitsum_pairs + 64 x k_miller_wave",
    "miller": "k_miller_lines_w2 + k_miller_accs_lds",
    "fp12_prod": "k_fp12_prod_wave_seg + k_fp12_seg_combine_coop",
}
# Algorithmic HBM bytes per unit of the Miller stage: a
# pair's G1 point (96 B) and G2 point (192 B) in, its share of the segment
# outputs out (8 segments x 576 B per 16-pair group = 288 B), codes (3 B).
# The split Miller loop adds the line table by design: 68 lines x 3 Fp2 =
# 19,584 B per pair written by the line kernel and read once by the
# accumulator (tb_lines.h).
MILLER_ALG_BYTES_PER_PAIR = 96 + 192 + 288 + 3
MILLER_LINE_BYTES_PER_PAIR = 19584
STAGE_UNITS = {"pk_decompress": "keys", "set_pk": "sets", "set_sig": "sets", "set_hash": "sets", "g2_sum": "sets", "miller": "pairs", "fp12_prod": "pairs"}
_MC = os.path.join(ROOT, "tools", "mul_counts.json")
M_PER_UNIT = json.load(open(_MC)) if os.path.exists(_MC) else {}


def peak_mac_per_s(device, one_wave=False):
    """The measured chip-wide v_mad_u64_u32 rate, scaled to this device's CU count."""
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    return (MAD_1WAVE_PER_S if one_wave else MAD_PEAK_PER_S) * cus / 256


def acc_plan(S):
    """(per, nseg, split) of the library's Miller-accumulator plan at S sets (tbls_acc_plan)."""
    per, nseg, split = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
    native.check(native.lib().tbls_acc_plan(S, ctypes.byref(per), ctypes.byref(nseg), ctypes.byref(split)), "acc_plan")
    return per.value, nseg.value, split.value


def plan_counts(S):
    """M_PER_UNIT with the Miller work of the plan the library runs at S sets:
    the segmented accumulator (k_miller_accs_lds: f in LDS, lines paired)
    shares one f^2 among `per` pairs (tools/count_muls.py miller_seg2_PxS), the
    unsegmented k_miller_acc2 among 2."""
    per, nseg, split = acc_plan(S)
    mc = dict(M_PER_UNIT)
    key = f"miller_seg2_{per}x{nseg}"
    seg = split and (nseg > 1 or per > 2)
    if seg and key in mc:
        d = mc[key] - mc["miller"]
        mc["miller"] = mc[key]
        mc["per_set_total"] = mc["per_set_total"] + mc.get("pairs_per_set", 1.0) * d
        mads = dict(mc.get("mads_per_unit", {}))
        if "miller" in mads:  # the accumulator's products are lazy Fp2 products (3 M, 980 v_mad_u64_u32 each)
            mads["miller"] = round(mads["miller"] + d / 3 * mc.get("mads_per_fp2_mul", 980))
        mc["mads_per_unit"] = mads
    kern = dict(STAGE_KERNEL)
    if os.environ.get("TBLS_W2") == "0":  # the library's kernel selection (tb_lib.hip w2)
        kern.update(set_pk="k_set_pk", set_sig="k_sig_check", set_hash="k_set_hash")
    lines_k = "k_miller_lines_w2"
    acc_k = "k_miller_accs_lds" if seg else f"k_miller_acc{2 if per == 2 else 1}"
    kern["miller"] = f"{lines_k} + {acc_k}"
    return mc, kern, {"per": per, "nseg": nseg, "kernel": acc_k}


def roofline_entry(stage_ms, S, device, ms_per_step):
    peak = peak_mac_per_s(device)
    M_PER_UNIT, STAGE_KERNEL, plan = plan_counts(S)
    mads = M_PER_UNIT.get("mads_per_unit", {})
    per_stage = {}
    pairs = M_PER_UNIT.get("pairs_per_set", 1.0)  # set pairs + the signature side's bucket pairs
    units = {k: S * (pairs if STAGE_UNITS[k] == "pairs" else 1.0) for k in STAGES}
    for i, name in enumerate(STAGES):
        if name in M_PER_UNIT and stage_ms[i] > 0:
            per_stage[name] = M_PER_UNIT[name] * MAC_PER_M * units[name] / (stage_ms[i] * 1e-3)
    dom = max(range(len(STAGES)), key=lambda i: stage_ms[i])  # exclusive times
    name = STAGES[dom]
    achieved = per_stage.get(name)
    kernel = STAGE_KERNEL[name]
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):  # HBM bytes per launch from the PMC passes, summed over the stage's kernels
        tj = json.load(open(tpath))
        parts = [tj.get(k.strip(), {}).get("bytes_per_launch") for k in kernel.split("+")]
        traffic = sum(parts) if all(p is not None for p in parts) else None
    per_set = M_PER_UNIT.get("per_set_total")
    alg = units[name] * MILLER_ALG_BYTES_PER_PAIR if name == "miller" else None
    alg_lines = alg + 2 * units[name] * MILLER_LINE_BYTES_PER_PAIR if alg else None
    return {
        "bound": "valu-int (v_mad_u64_u32 issue)",
        "kernel": kernel,
        "achieved": achieved / 1e12 if achieved else None,
        "peak": peak / 1e12,
        "unit": "T MAC/s (32x32->64)",
        "frac": (achieved / peak) if achieved else None,
        "peak_1wave": peak_mac_per_s(device, True) / 1e12,
        "frac_1wave": (achieved / peak_mac_per_s(device, True)) if achieved else None,
        "traffic": traffic,
        "traffic_unit": "B per launch (profiles/pmc_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE, this round's build)",
        "algorithmic_bytes": alg,
        "traffic_ratio": (traffic / alg) if traffic and alg else None,
        "traffic_ratio_with_line_tables": (traffic / alg_lines) if traffic and alg_lines else None,
        "model": "SURVEY.md 8(d): Fp products per unit (tools/mul_counts.json) x 300 MAC",
        "units_per_launch": round(units[name]),
        "unit_of_work": STAGE_UNITS[name],
        "fp_products_per_unit": M_PER_UNIT.get(name),
        "kernel_ms": stage_ms[dom],
        "issue_frac": (mads[name] * units[name] / (stage_ms[dom] * 1e-3)) / peak if name in mads else None,
        "stage_frac": {k: v / peak for k, v in per_stage.items()},
        "pipeline_frac": (per_set * MAC_PER_M * S / (ms_per_step * 1e-3)) / peak if per_set else None,
        "acc_plan": plan,
    }


class DevBatch:
    """A batch resident in HBM (torch tensors) + its tbls_dev_batch descriptor."""

    def __init__(self, pks, n_pks, msgs, msg_lens, sigs, device, rands=None):
        n = len(n_pks)
        u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(device)  # noqa: E731
        i32 = lambda v: torch.tensor(v, dtype=torch.int64).to(torch.int32).to(device)  # noqa: E731
        self.pks = u8(pks)
        self.msgs = u8(msgs)
        self.sigs = u8(sigs)
        off = [0]
        for k in n_pks:
            off.append(off[-1] + k)
        moff = [0]
        for m in msg_lens:
            moff.append(moff[-1] + m)
        self.pk_off = i32(off)
        self.msg_off = i32(moff)
        r = rands or synth.random_multipliers(n)
        self.rand = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in r], dtype=torch.int64, device=device)
        self.n_keys = off[-1]
        self.desc = native.TblsDevBatch(
            self.pks.data_ptr(), self.pk_off.data_ptr(), self.n_keys, self.msgs.data_ptr(), self.msg_off.data_ptr(), self.sigs.data_ptr(),
            self.rand.data_ptr(), n
        )
        self.n = n


def timed(fn, reps):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        out.append((time.perf_counter() - t0) * 1e3)
    return sorted(out)


def pct(xs, q):
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """(threads, env_cap, quota): the CPUs this process may run on
    (sched_getaffinity -- BASELINE.md's `nproc`), the environment's thread cap
    (OMP_NUM_THREADS / MAX_JOBS: the box's CPU share) and the cgroup CPU quota
    in cores (cpu.max; None when unlimited or unreadable)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    cap = None
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        if os.environ.get(var, "").isdigit():
            cap = min(cap or n, int(os.environ[var]))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return max(1, n), cap, quota


def granted_threads(T, cap, quota):
    """The threads this process is granted: min(affinity, environment cap,
    cgroup quota rounded down) -- on the GPU box affinity names every CPU of
    the machine (256) while the box's share is 16 (OMP_NUM_THREADS / MAX_JOBS,
    cpu.max), and Teku sizes its verifier pool from the cores it may use
    (P2PConfig.java:42-43)."""
    g = T
    if cap:
        g = min(g, cap)
    if quota:
        g = min(g, max(1, int(quota)))
    return max(1, g)


def cpu_baseline_oracle(pks, msgs, sigs, sample_sets=4096, sample_1t=512):
    """The C oracle (oracle/c/bls_oracle.c, 'port') timed on this host over a
    bounded sample of the same workload: the first `sample_sets` sets on the
    threads this process is granted (`granted_threads`: the headline), the
    same sample on every CPU of the affinity mask (oversubscribed beyond the
    grant: secondary), the first `sample_1t` sets on one thread, and the p50
    of a 128-set batch (config 1) on the granted threads."""
    from oracle import c_oracle as C

    T, cap, quota = cpu_threads()
    Tg = granted_threads(T, cap, quota)
    pk = [pks[48 * j : 48 * j + 48] for j in range(sample_sets)]
    ms = [msgs[32 * j : 32 * j + 32] for j in range(sample_sets)]
    sg = [sigs[96 * j : 96 * j + 96] for j in range(sample_sets)]
    rr = synth.random_multipliers(sample_sets)
    t0 = time.perf_counter()
    assert C.batch_verify(pk, ms, sg, rr, threads=Tg), "C oracle rejected the valid sample"
    dt = time.perf_counter() - t0
    t0 = time.perf_counter()
    assert C.batch_verify(pk[:sample_1t], ms[:sample_1t], sg[:sample_1t], rr[:sample_1t], threads=1)
    dt1 = time.perf_counter() - t0
    lat = timed(lambda: C.batch_verify(pk[:128], ms[:128], sg[:128], rr[:128], threads=Tg), 7)
    dt_all = None
    if T > Tg:  # the same sample on every CPU of the affinity mask (beyond the grant)
        t0 = time.perf_counter()
        assert C.batch_verify(pk, ms, sg, rr, threads=T)
        dt_all = time.perf_counter() - t0
    return {
        "value": sample_sets / dt,
        "unit": "sigs/s",
        "cores": Tg,
        "kind": "port",
        "sample": f"oracle/c batch_verify of the first {sample_sets} sets of this workload on {Tg} pthreads ({dt:.1f} s; the "
        f"threads this process is granted: min(affinity {T}, env cap {cap}, cgroup quota {quota})) and of the first "
        f"{sample_1t} on 1 thread ({dt1:.1f} s); the build's own C restatement (6x64-bit CIOS Montgomery), not blst",
        "value_1thread": sample_1t / dt1,
        "threads_granted": Tg,
        "threads_affinity": T,
        "env_thread_cap": cap,
        "cgroup_cpu_quota_cores": quota,
        "value_affinity_oversubscribed": sample_sets / dt_all if dt_all else None,
        "cpu_model": cpu_model(),
        "machine_cpus": os.cpu_count(),
        "p50_latency_ms_128": statistics.median(lat),
    }


def extra_configs(device, stream, reps):
    """Configs 2, 3, 4 (BASELINE.json) on this rank's GPU; see the module doc."""
    out = {}
    peak = peak_mac_per_s(device)
    # config 2: 64 sync-committee sets x 512 keys, fastAggregateVerify per set
    keys, msgs, sigs = synth.multi_key(64, 512, first_key=0, seed=2)
    arr = synth.SetArray.from_lists(keys, msgs, sigs)
    assert arr.fast_aggregate_verify_many() == [True] * 64
    lat = timed(arr.fast_aggregate_verify_many, reps)
    out["cfg2"] = {
        "what": "64 sets x 512 keys, fastAggregateVerify per set (tbls_fast_aggregate_verify_many, keys as bytes, PCIe included)",
        "p50_ms": statistics.median(lat),
        "p99_ms": pct(lat, 0.99),
        "sets_per_s": 64 / (statistics.median(lat) * 1e-3),
        "reps": reps,
    }
    # config 3: 64 attestation sets x 488 keys, randomized batchVerify
    keys, msgs, sigs = synth.multi_key(64, 488, first_key=1000, seed=3)
    arr = synth.SetArray.from_lists(keys, msgs, sigs)
    assert arr.batch_verify(synth.random_multipliers(64))
    lat = timed(lambda: arr.batch_verify(synth.random_multipliers(64)), reps)
    L = native.lib()
    flat = [k for ks in keys for k in ks]
    native.check(L.tbls_pk_table_load(b"".join(flat), len(flat), None), "pk_table_load")
    idx_arrays, keep = (native.TblsSetIdx * 64)(), []
    for s in range(64):
        ki = (ctypes.c_uint32 * 488)(*range(488 * s, 488 * (s + 1)))
        mb, sb = ctypes.create_string_buffer(msgs[s], 32), ctypes.create_string_buffer(sigs[s], 96)
        keep += [ki, mb, sb]
        idx_arrays[s].key_idx = ctypes.cast(ki, ctypes.c_void_p)
        idx_arrays[s].n_pks = 488
        idx_arrays[s].msg = ctypes.cast(mb, ctypes.c_void_p)
        idx_arrays[s].msg_len = 32
        idx_arrays[s].sig = ctypes.cast(sb, ctypes.c_void_p)

    def idx_verify():
        rr = (ctypes.c_uint64 * 64)(*synth.random_multipliers(64))
        ok = ctypes.c_int(0)
        native.check(L.tbls_batch_verify_idx(idx_arrays, 64, rr, 1, ctypes.byref(ok), None), "batch_verify_idx")
        assert ok.value == 1

    idx_verify()
    lat_tab = timed(idx_verify, reps)
    # the aggregation kernel alone (exclusive stage time on a device-resident batch)
    db = DevBatch(b"".join(flat), [488] * 64, b"".join(msgs), [32] * 64, b"".join(sigs), device)
    part = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    st = (ctypes.c_float * 8)()
    agg_ms = []
    for _ in range(5):
        native.check(L.tbls_dev_batch_stage_profile(device.index, ctypes.byref(db.desc), stream, part.data_ptr(), st), "profile")
        agg_ms.append(st[1])
    agg_ms = statistics.median(agg_ms)
    agg_m = M_PER_UNIT.get("set_pk_wave_488")
    out["cfg3"] = {
        "what": "64 sets x 488 keys, randomized batchVerify (tbls_batch_verify, keys as bytes, PCIe included)",
        "p50_ms": statistics.median(lat),
        "p99_ms": pct(lat, 0.99),
        "sets_per_s": 64 / (statistics.median(lat) * 1e-3),
        "p50_ms_key_table": statistics.median(lat_tab),
        "sets_per_s_key_table": 64 / (statistics.median(lat_tab) * 1e-3),
        "aggregation_kernel": ("k_set_pk_wave (one 64-lane wave per set: strided mixed adds, LDS tree, [r] apk)"
                               if os.environ.get("TBLS_COOP") == "0" else
                               "k_set_pk_agg_coop (32 coop rows per set: row sums of mixed adds, LDS tree, [r] apk by nibbles on "
                               "16 rows, -[r] g1 on row 17; critical path: the 60 doublings to 2^60 apk)"),
        "aggregation_ms": agg_ms,
        "aggregation_frac": (agg_m * MAC_PER_M * 64 / (agg_ms * 1e-3)) / peak if agg_m and agg_ms > 0 else None,
        "aggregation_fp_products_per_set": agg_m,
        "reps": reps,
    }
    # config 4: 16,384 gossip attestations per slot, one service batch (host C ABI)
    n4 = 16384
    pks, msgs, sigs = synth.single_signer(0, n4, seed=4)
    arr = synth.SetArray.single(pks, msgs, sigs)
    assert arr.batch_verify(synth.random_multipliers(n4))
    lat4 = timed(lambda: arr.batch_verify(synth.fast_multipliers(n4)), max(5, reps // 4))
    from teku_amd.service import AggregatingSignatureVerificationService, SignatureTask

    sg = [sigs[96 * i : 96 * i + 96] for i in range(n4)]
    bad = {11: sg[12], 5000: bytes(96), 9999: synth.NOT_IN_G2, 16383: sg[0]}
    for j, b in bad.items():
        sg[j] = b
    # the failure path at the same level as p50_ms: one tbls_batch_verify_each on the
    # staged set array (the batch, then the per-set verdicts settled in place)
    arr_bad = synth.SetArray.single(pks, msgs, b"".join(sg))

    def settle_once():
        ok, each = arr_bad.batch_verify_each(synth.fast_multipliers(n4))
        assert not ok and [i for i, v in enumerate(each) if not v] == sorted(bad)

    settle_once()  # warm: the settle workspace is allocated on first use
    native.stats(reset=True)
    settle = timed(settle_once, max(5, reps // 4))
    st = native.stats()
    # and through the service (tasks in, per-task futures out: the Python glue included), happy and failing
    sets_ok = [(pks[48 * i : 48 * i + 48], 1, msgs[32 * i : 32 * i + 32], sigs[96 * i : 96 * i + 96]) for i in range(n4)]
    sets_bad = [(pks[48 * i : 48 * i + 48], 1, msgs[32 * i : 32 * i + 32], sg[i]) for i in range(n4)]
    svc_ms = {}
    for name, sets in (("happy", sets_ok), ("failure", sets_bad)):
        walls = []
        for _ in range(4):
            svc = AggregatingSignatureVerificationService(max_batch_size=n4)
            tasks = [SignatureTask([s]) for s in sets]
            t0 = time.perf_counter()
            svc.batch_verify_signatures(tasks)
            walls.append((time.perf_counter() - t0) * 1e3)
            assert sum(1 for t in tasks if not t.result.result()) == (0 if name == "happy" else 4)
        svc_ms[name] = statistics.median(walls[1:])
    out["cfg4"] = {
        "what": "16,384 single-signer sets in one batch (tbls_batch_verify on a staged set array, PCIe included); failure path: 4 bad "
        "sets, the batch and every set's verdict settled in place from the batch's own Miller work in one tbls_batch_verify_each",
        "p50_ms": statistics.median(lat4),
        "sigs_per_s": n4 / (statistics.median(lat4) * 1e-3),
        "failure_settle_ms": statistics.median(settle),
        "failure_to_happy": statistics.median(settle) / statistics.median(lat4),
        "failure_device_passes": 1,
        "failure_device_pipelines": st["partials"] / max(1, len(settle)),
        "service_ms": svc_ms,
    }
    out["cfg4_facade"] = facade_cfg4(pks, msgs, sigs, max(5, reps // 4), statistics.median(lat4))
    return out


def facade_cfg4(pks, msgs, sigs, reps, raw_p50):
    """Config 4 through the SPI facade with FRESH objects: BLS.batchVerify
    (BLS.java:230-336) on HipBLS12381 over 16,384 new BLSPublicKey /
    BLSSignature wrappers per rep (created before the clock starts, as gossip
    decoding creates them); the facade hands their bytes to one device batch,
    which decodes and group-checks every point.  Beside it, what a Java
    facade pays per object for getSignature() (BLSSignature.java:83-87 ->
    HipSignature.fromBytes -> tbls_sig_decode on the caller's thread): the
    host decode of the 16,384 signatures one call at a time, and as one
    tbls_sig_decode_many call over the host threads.  Counters from tbls_stats
    of the last rep."""
    import ctypes

    from teku_amd import bls as B

    B.BLS.set_bls_implementation(B.HipBLS12381())
    n = len(sigs) // 96
    pk = [pks[48 * i : 48 * i + 48] for i in range(n)]
    ms = [msgs[32 * i : 32 * i + 32] for i in range(n)]
    sg = [sigs[96 * i : 96 * i + 96] for i in range(n)]
    lat = []
    st = None
    for _ in range(reps + 1):
        keys = [[B.BLSPublicKey.from_bytes_compressed(p)] for p in pk]
        so = [B.BLSSignature.from_bytes_compressed(s) for s in sg]
        native.stats(reset=True)
        t0 = time.perf_counter()
        assert B.BLS.batch_verify(keys, ms, so) is True
        lat.append((time.perf_counter() - t0) * 1e3)
        st = native.stats()
    lat = lat[1:]
    H = native.host()
    t0 = time.perf_counter()
    for s in sg:
        assert H.tbls_sig_decode(s, None) == 0
    one = (time.perf_counter() - t0) * 1e6 / n
    codes = ctypes.create_string_buffer(n)
    many = []
    for _ in range(3):
        t0 = time.perf_counter()
        native.check(H.tbls_sig_decode_many(sigs, n, codes, None), "sig_decode_many")
        many.append((time.perf_counter() - t0) * 1e3)
    p50 = statistics.median(lat)
    return {
        "what": "16,384 fresh BLSPublicKey/BLSSignature objects through BLS.batchVerify on HipBLS12381 (one tbls_batch_verify; "
        "PCIe included); host decode = a Java facade's per-object getSignature() cost",
        "p50_ms": p50,
        "ratio_to_raw_p50": p50 / raw_p50 if raw_p50 else None,
        "device_batches": st["partials"],
        "single_object_device_calls": st["one_validate"],
        "host_decodes_in_batch": st["host_decodes"],
        "sig_host_decode_us_per_object_1thread": one,
        "sig_host_decode_ms_16k_many": statistics.median(many),
        "reps": reps,
    }


def kzg_warm():
    """Load the trusted setup and run one 6-blob verification (the KZG
    context created before the BLS library's: tools/kzg_order_probe.py's
    kzg_first order).  Round 5 called it before the BLS legs to avoid the
    KZG-after-BLS slowdown; round 6 found its cause (hardware queues shared
    with the BLS streams, fixed by GPU_MAX_HW_QUEUES above) and the bench no
    longer calls it."""
    from teku_amd import kzg

    ck = kzg.CKZG4844.get_instance()
    ck.load_trusted_setup(os.path.join(ROOT, "tests", "golden", "kzg", "trusted_setup.txt"))
    import random

    rnd = random.Random(8999)
    blobs = [b"".join(rnd.randrange(kzg.BLS_MODULUS).to_bytes(32, "big") for _ in range(4096)) for _ in range(6)]
    cs = ck.blobs_to_kzg_commitments(blobs)
    ps = [ck.compute_blob_kzg_proof(b, c) for b, c in zip(blobs, cs)]
    assert ck.verify_blob_kzg_proof_batch(blobs, cs, ps)


def kzg_leg(device, reps, cpu_sample):
    """EIP-4844 KZG: verifyBlobKzgProofBatch on the
    reference's trusted setup (tests/golden/kzg/trusted_setup.txt), seeded
    random blobs, commitments and proofs made by the GPU prover.  Reports the
    host-API latency at 1 and 6 blobs (Deneb's per-block maximum, PCIe
    included), device-resident throughput at 64 and 512 blobs with per-stage
    kernel times, and the C oracle's per-blob time (1 thread) on a sample."""
    from teku_amd import kzg

    setup = os.path.join(ROOT, "tests", "golden", "kzg", "trusted_setup.txt")
    ck = kzg.CKZG4844.get_instance()
    ck.load_trusted_setup(setup)
    import random

    def blob(seed):
        rnd = random.Random(seed)
        return b"".join(rnd.randrange(kzg.BLS_MODULUS).to_bytes(32, "big") for _ in range(4096))

    base = [blob(9000 + i) for i in range(64)]
    cs = ck.blobs_to_kzg_commitments(base)
    t0 = time.perf_counter()
    ps = [ck.compute_blob_kzg_proof(b, c) for b, c in zip(base[:8], cs[:8])]
    prove_ms = (time.perf_counter() - t0) * 1e3 / 8
    ps += [ck.compute_blob_kzg_proof(b, c) for b, c in zip(base[8:], cs[8:])]
    t0 = time.perf_counter()
    ck.blobs_to_kzg_commitments(base)
    commit_ms = (time.perf_counter() - t0) * 1e3 / 64
    out = {"what": "verify_blob_kzg_proof_batch (CKZG4844.verifyBlobKzgProofBatch) on the reference trusted setup, seeded blobs",
           "commit_ms_per_blob_64": commit_ms, "prove_ms_per_blob": prove_ms}
    for n in (1, 6):
        assert ck.verify_blob_kzg_proof_batch(base[:n], cs[:n], ps[:n])
        lat = timed(lambda: ck.verify_blob_kzg_proof_batch(base[:n], cs[:n], ps[:n]), reps)
        out[f"p50_ms_{n}"] = statistics.median(lat)
        out[f"p99_ms_{n}"] = pct(lat, 0.99)
    L = kzg.lib()
    ok = ctypes.c_int(0)
    st = (ctypes.c_float * 6)()
    for n in (64, 512):
        reps_n = [i % 64 for i in range(n)]
        db = torch.tensor(bytearray(b"".join(base[i] for i in reps_n)), dtype=torch.uint8, device=device)
        dc = torch.tensor(bytearray(b"".join(cs[i] for i in reps_n)), dtype=torch.uint8, device=device)
        dp = torch.tensor(bytearray(b"".join(ps[i] for i in reps_n)), dtype=torch.uint8, device=device)
        torch.cuda.synchronize()

        def run():
            kzg._check(L.tkzg_dev_verify_blob_kzg_proof_batch(ctypes.byref(ok), db.data_ptr(), dc.data_ptr(), dp.data_ptr(), n, None))
            assert ok.value == 1

        run()
        lat = timed(run, max(3, reps // 4))
        med = statistics.median(lat)
        kzg._check(L.tkzg_dev_verify_blob_kzg_proof_batch_profiled(ctypes.byref(ok), db.data_ptr(), dc.data_ptr(), dp.data_ptr(), n, None))
        stage = dict(zip(kzg.STAGES, list(st) if L.tkzg_last_stage_ms(st) == 0 else []))
        out[f"dev_{n}"] = {"ms": med, "blobs_per_s": n / (med * 1e-3), "stage_ms": stage,
                           # the challenge kernel streams the blobs once: 131,152 B of transcript per blob
                           "challenge_hbm_GBps": n * 131152 / (stage.get("challenge", 0) * 1e-3) / 1e9 if stage.get("challenge") else None}
    if cpu_sample:
        from oracle import kzg_oracle as K

        s = K.Setup.from_file(setup)
        t0 = time.perf_counter()
        assert s.verify_blob_kzg_proof_batch(base[:2], cs[:2], ps[:2]) is True
        cpu_s = time.perf_counter() - t0
        s.close()
        out["cpu_baseline"] = {"value": 2 / cpu_s, "unit": "blobs/s", "cores": 1, "kind": "port",
                               "sample": "2-blob verify_blob_kzg_proof_batch through the C oracle (spec restatement: one Fermat "
                                         "inversion per barycentric term, 8-bit-window Pippenger), one thread"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets-per-gpu", type=int, default=int(os.environ.get("TBLS_SETS_PER_GPU", 131072)))
    ap.add_argument("--lat-reps", type=int, default=100)
    ap.add_argument("--extra-reps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip configs 2/3/4")
    ap.add_argument("--no-1m", action="store_true", help="skip config 5 at its full 1,048,576-set size on this one GPU")
    ap.add_argument("--serial", action="store_true", help="timed steps with every stage alone on the stream (profiling)")
    ap.add_argument("--no-kzg", action="store_true", help="skip the KZG leg (SURVEY.md 8(f) rank 4)")
    ap.add_argument("--kzg-only", action="store_true", help="profiling: run only the KZG leg and print its JSON")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if args.kzg_only:
        print(json.dumps(kzg_leg(device, args.extra_reps, False)), flush=True)
        return
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    L = native.lib()

    S = args.sets_per_gpu
    t_gen = time.perf_counter()
    lo, hi = shard_bounds(S * world, world, rank)  # weak scaling: S sets per rank
    pks, msgs, sigs = synth.single_signer(lo, hi - lo)
    batch = DevBatch(pks, [1] * S, msgs, [32] * S, sigs, device)
    gen_s = time.perf_counter() - t_gen
    partial = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    stage_acc = [0.0] * len(STAGES)
    ok = ctypes.c_int(0)
    stage = (ctypes.c_float * 8)()

    def step(timed_stages):
        if args.serial:
            native.check(L.tbls_dev_batch_stage_profile(local, ctypes.byref(batch.desc), stream, partial.data_ptr(), stage), "profile")
        elif timed_stages:
            native.check(L.tbls_dev_batch_partial_timed(local, ctypes.byref(batch.desc), stream, partial.data_ptr(), stage), "partial")
        else:
            native.check(L.tbls_dev_batch_partial(local, ctypes.byref(batch.desc), stream, partial.data_ptr()), "partial")
        if timed_stages or args.serial:
            for i in range(len(STAGES)):
                stage_acc[i] += stage[i]
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
    for _ in range(args.steps):  # the plain partial: no stage events inside the timed region
        step(args.serial)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stage_steps = 2 if not args.serial else args.steps  # the overlapped stage times from two event-timed steps after it
    if not args.serial:
        for _ in range(stage_steps):
            step(True)
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

    # Config 5 at its stated size (1,048,576 sets) on this one GPU: one device
    # batch of all sets (offsets, the bucket MSM and 4 line-buffer chunks at
    # 1M); single-GPU runs only (the driver's N>1 runs shard config 5 instead).
    one_m = None
    if world == 1 and not args.no_1m:
        n1m = 1 << 20
        del batch
        t_g = time.perf_counter()
        pk1, ms1, sg1 = synth.single_signer(0, n1m, seed=5)
        b1m = DevBatch(pk1, [1] * n1m, ms1, [32] * n1m, sg1, device)
        del pk1, ms1, sg1
        gen1 = time.perf_counter() - t_g

        def step_1m():
            native.check(L.tbls_dev_batch_partial(local, ctypes.byref(b1m.desc), stream, partial.data_ptr()), "partial_1m")
            native.check(L.tbls_dev_final_verify(local, partial.data_ptr(), 1, stream, ctypes.byref(ok)), "final_1m")
            if ok.value != 1:
                raise RuntimeError("valid synthetic 1M batch rejected")

        step_1m()
        torch.cuda.synchronize()
        k1m = 3
        t0 = time.perf_counter()
        for _ in range(k1m):
            step_1m()
        torch.cuda.synchronize()
        dt1m = (time.perf_counter() - t0) / k1m
        one_m = {"value": n1m / dt1m, "unit": "sigs/s", "ms_per_batch": dt1m * 1e3, "steps": k1m, "gen_s": gen1,
                 "what": "config 5 at 1,048,576 sets as ONE device batch on this GPU (partial + final exponentiation, inputs in HBM)"}
        del b1m
        batch = DevBatch(pks, [1] * S, msgs, [32] * S, sigs, device)  # the profiled steps below use the 131k shard

    stage_ms = [a / stage_steps for a in stage_acc]
    # Exclusive per-stage kernel times (every stage alone on the stream): the
    # roofline's denominators.  In the timed steps the stages overlap, so
    # their event brackets include each other's work.
    excl = [0.0] * len(STAGES)
    for _ in range(2):
        native.check(L.tbls_dev_batch_stage_profile(local, ctypes.byref(batch.desc), stream, partial.data_ptr(), stage), "profile")
        for i in range(len(STAGES)):
            excl[i] += stage[i] / 2
    ms_per_step = dt / args.steps * 1e3
    roofline = roofline_entry(excl, S, device, ms_per_step)

    # config 1: latency of a 128-set batchVerify through the host C ABI
    arr128 = synth.SetArray.single(pks[: 48 * 128], msgs[: 32 * 128], sigs[: 96 * 128])
    lat = []
    if args.lat_reps > 0:
        for _ in range(3):
            assert arr128.batch_verify(synth.random_multipliers(128), n_gpus=1)
        lat = timed(lambda: arr128.batch_verify(synth.random_multipliers(128), n_gpus=1), args.lat_reps)
    extra = {} if args.no_extra else extra_configs(device, stream, args.extra_reps)
    kzg_out = None if args.no_kzg else kzg_leg(device, args.extra_reps, not args.no_cpu_baseline)
    if kzg_out is not None:
        kzg_out["context"] = ("trusted setup loaded after the BLS legs (GPU_MAX_HW_QUEUES=%s: the KZG streams get hardware queues of their own)"
                              % os.environ.get("GPU_MAX_HW_QUEUES"))

    cpu = None if args.no_cpu_baseline else cpu_baseline_oracle(pks, msgs, sigs, min(4096, S), min(512, S))
    line = {
        "metric": "BLS sigs verified/sec (batchVerify), 1-8 GPUs; p50 latency @128-sig batch",
        "value": value,
        "unit": "sigs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
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
        "serial_stages": bool(args.serial),
        "value_1m": one_m["value"] if one_m else None,
        "config5_1m": one_m,
        "value_key_table": total_sets / dt_tab,
        "ms_per_step_key_table": dt_tab / args.steps * 1e3,
        "key_table": "value_key_table: same steps with keys from the device-resident validator table (%d keys decompressed "
        "and validated once, as Teku memoizes BLSPublicKey); value decodes and group-checks every key per step" % T,
        "p50_latency_ms_128": statistics.median(lat) if lat else None,
        "p99_latency_ms_128": pct(lat, 0.99) if lat else None,
        "latency_reps_128": len(lat),
        "stage_ms_overlapped": dict(zip(STAGES, stage_ms)),
        "stage_ms_exclusive": dict(zip(STAGES, excl)),
        "roofline": roofline,
        "configs": extra,
        "kzg": kzg_out,
        "cpu_baseline": cpu,
        "workload_gen_s": gen_s,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
