#!/bin/bash
# Round 5: settle-from-batch parity, service with the new failure path, then
# the accumulator A/B: half-LDS (default) vs full-LDS (variant) vs register
# (TBLS_ACC_LDS=0), each with and without TBLS_ACC_JOIN.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05c}
echo "== settle / service parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_settle.py tests/test_gpu_facade.py "tests/test_gpu_configs.py::test_config4_16k_through_service" tests/test_gpu_accseg.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -30; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), round(d['roofline']['frac'], 4), d['roofline'].get('kernel'), round(d['stage_ms_exclusive']['miller'], 2))"
}
run half TBLS_ACC_LDS=1 || exit $?
run half_join TBLS_ACC_LDS=1 TBLS_ACC_JOIN=1 || exit $?
run full TBLS_LIB=teku_amd/lib/ab/libtekubls_hip_ldsfull.so || exit $?
run full_join TBLS_LIB=teku_amd/lib/ab/libtekubls_hip_ldsfull.so TBLS_ACC_JOIN=1 || exit $?
run reg TBLS_ACC_LDS=0 || exit $?
run reg_join TBLS_ACC_LDS=0 TBLS_ACC_JOIN=1 || exit $?
echo "== cfg4 failure settle"
timeout -k 10 300 python - > gpurun_out/settle_$TAG.json 2> gpurun_out/settle_$TAG.err <<'PY' || exit $?
import json, statistics, sys, time
sys.path.insert(0, '.')
import torch
from teku_amd import native, synth
from teku_amd.service import AggregatingSignatureVerificationService, SignatureTask
native.lib()
n = 16384
pks, msgs, sigs = synth.single_signer(0, n, seed=4)
sg = [sigs[96 * i: 96 * i + 96] for i in range(n)]
for j, b in {11: sg[12], 5000: bytes(96), 9999: synth.NOT_IN_G2, 16383: sg[0]}.items():
    sg[j] = b
sets = [(pks[48 * i: 48 * i + 48], 1, msgs[32 * i: 32 * i + 32], sg[i]) for i in range(n)]
out = {}
for mode in ("settle", "each"):
    lat = []
    for _ in range(6):
        svc = AggregatingSignatureVerificationService(max_batch_size=n, batch_fn=(None if mode == "settle" else (lambda s: synth.SetArray.from_tuples(s).batch_verify(synth.fast_multipliers(len(s))))))
        tasks = [SignatureTask([s]) for s in sets]
        t0 = time.perf_counter(); svc.batch_verify_signatures(tasks); lat.append((time.perf_counter() - t0) * 1e3)
        assert sum(1 for t in tasks if not t.result.result()) == 4
    out[mode] = {"p50_ms": statistics.median(lat[1:]), "runs": lat}
arr = synth.SetArray.single(pks, msgs, sigs)
lat = []
for _ in range(8):
    t0 = time.perf_counter(); assert arr.batch_verify(synth.fast_multipliers(n)); lat.append((time.perf_counter() - t0) * 1e3)
out["happy_p50_ms"] = statistics.median(lat[1:])
print(json.dumps(out))
PY
cat gpurun_out/settle_$TAG.json
echo done
