#!/bin/bash
# Round 5: lean signature check (point parked in LDS, tb_lean.h), shuffle-tree
# bucket sums (k_msm_bucket_tree), sequential SSWU by default.  Full GPU suite,
# bench A/B of the accumulator (register vs LDS) now that the bucket sums use
# no LDS, FETCH/WRITE of the 131k step's kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05g}
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), d['roofline']['kernel'], {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()})"
}
run auto || exit $?
run lds TBLS_ACC_LDS=1 || exit $?
run auto2 || exit $?
run lds2 TBLS_ACC_LDS=1 || exit $?
P="tools/probe.py partial 131072 2"
echo "== pmc" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_write.log 2>&1 || exit $?
echo done
