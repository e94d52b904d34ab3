#!/bin/bash
# Round 5: the LDS accumulator on 960 waves (plan 32 x 15) beside the
# bit-sum pairs' chain instead of joining it (TBLS_ACC_JOIN=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05q}
V="TBLS_ACC_PLAN=32,15 TBLS_ACC_JOIN=0 TBLS_ACC_LDS=1"
env $V timeout -k 10 600 python -u -m pytest "tests/test_gpu_configs.py::test_config5_131k_shard" "tests/test_gpu_bls.py::test_large_batch_msm_path" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), round(d['value_key_table']), {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()})"
}
for r in 1 2; do
  run base$r || exit $?
  run p960_$r $V || exit $?
  run p960join_$r TBLS_ACC_PLAN=32,15 || exit $?
done
env $V timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-1m --no-kzg --no-extra --lat-reps 0 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
echo done
