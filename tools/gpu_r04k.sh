#!/bin/bash
# Accumulator plans up to 32 x 16: the old plan (8,4) vs the new default at
# 131k, config-4 stages, the accumulator parity tests, the product tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
for pl in default 8,4 16,8; do
  echo "== bench plan=$pl"
  if [ "$pl" = default ]; then E=""; else E="TBLS_ACC_PLAN=$pl"; fi
  env $E timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04k_$pl.json 2> gpurun_out/bench_r04k_$pl.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_r04k_$pl.json'));print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'], d['roofline']['acc_plan'])" || exit $?
done
echo "== stage_small 16384 default / 2,4"
timeout -k 10 300 python tools/stage_small.py 16384 > gpurun_out/stage_r04k.json 2> gpurun_out/stage_r04k.err || exit $?
TBLS_ACC_PLAN=2,4 timeout -k 10 300 python tools/stage_small.py 16384 > gpurun_out/stage_r04k_old.json 2> gpurun_out/stage_r04k_old.err || exit $?
python3 -c "
import json
for f in ['stage_r04k', 'stage_r04k_old']:
    for n, d in json.load(open('gpurun_out/' + f + '.json')).items():
        print(f, n, 'excl', {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()}, 'partial', round(d['partial_wall_ms'], 2))" || exit $?
K="test_gpu_accseg or test_gpu_hrow or test_gpu_bls or test_gpu_configs" NOBENCH=1 TAG=r04k bash tools/gpu_r04.sh
