#!/bin/bash
# Round 5: accumulator A/B with the bit-sum pairs on k_miller_wave_g (global
# tables): full-LDS (default) vs half-LDS (variant) vs register (TBLS_ACC_LDS=0);
# kernel trace of the settle path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05d}
echo "== parity (accumulator plans, configs)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_accseg.py tests/test_gpu_settle.py "tests/test_gpu_configs.py::test_config5_131k_shard" "tests/test_gpu_bls.py::test_large_batch_msm_path" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), round(d['roofline']['frac'], 4), d['roofline'].get('kernel'), round(d['stage_ms_exclusive']['miller'], 2))"
}
run full || exit $?
run half TBLS_LIB=teku_amd/lib/ab/libtekubls_hip_ldshalf.so || exit $?
run reg TBLS_ACC_LDS=0 || exit $?
run full2 || exit $?
echo "== settle trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_settle -o run --output-format csv -- python3 tools/settle_probe.py 4 > gpurun_out/settle_${TAG}.log 2>&1 || exit $?
tail -2 gpurun_out/settle_${TAG}.log
echo done
