#!/bin/bash
# Quad kernels: byte parity first, then config-4 stage times (quad vs pair hash),
# the TBLS_W2 A/B at 131k, and the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NOHV" ]; then
  echo "== hash variants"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_hash_variants.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_r04f_hv.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_r04f_hv.log; [ $rc -eq 0 ] || exit $rc
fi
for plan in "4096,16384,32768" "4096,0,32768"; do
  echo "== stage_small 16384 plan=$plan"
  TBLS_HASH_PLAN=$plan timeout -k 10 300 python tools/stage_small.py 16384 > gpurun_out/stage16k_$plan.json 2> gpurun_out/stage16k_$plan.err || exit $?
  tail -c 1500 gpurun_out/stage16k_$plan.json; echo
done
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
for m in 1 3 5 7; do
  echo "== bench W2=$m"
  TBLS_W2=$m timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04f_w$m.json 2> gpurun_out/bench_r04f_w$m.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_r04f_w$m.json'));print('W2=$m', d['value'], d['ms_per_step'], d['stage_ms_exclusive'])" || exit $?
done
K="$K" NOBENCH=1 TAG=r04f bash tools/gpu_r04.sh
