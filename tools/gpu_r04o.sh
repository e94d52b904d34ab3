#!/bin/bash
# Per-set stages side by side at every size: bench, row-vs-quad hash at
# 2,048-4,096 sets, and the product tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
echo "== bench" && timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04o.json 2> gpurun_out/bench_r04o.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04o.json'));print(d['value'], d['ms_per_step'], d['stage_ms_overlapped'])" || exit $?
for plan in "4096,8192,32768" "2048,8192,32768" "1024,8192,32768"; do
  echo "== stage 1024 2048 3072 4096 plan=$plan"
  TBLS_HASH_PLAN=$plan timeout -k 10 300 python tools/stage_small.py 1024 2048 3072 4096 > gpurun_out/stage_row_$plan.json 2> gpurun_out/stage_row_$plan.err || exit $?
  python3 -c "
import json
for n, d in json.load(open('gpurun_out/stage_row_$plan.json')).items():
    print(n, 'partial', round(d['partial_wall_ms'], 2), 'hash excl', round(d['stage_ms_exclusive']['set_hash'], 2), 'over', round(d['stage_ms_overlapped']['set_hash'], 2))" || exit $?
done
K="test_gpu_accseg or test_gpu_hrow or test_gpu_bls or test_gpu_configs" NOBENCH=1 TAG=r04o bash tools/gpu_r04.sh
