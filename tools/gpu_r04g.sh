#!/bin/bash
# Lane-group kernels (quad <= 8,192 sets, duo <= 32,768) and the signed-digit
# Fp2 products: stage times at 8,192 / 16,384 sets against the previous plan,
# the 131k bench, the product GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 16384 8192; do
  for plan in "4096,8192,32768,0" "4096,0,0,32768"; do
    echo "== stage_small $n plan=$plan"
    TBLS_HASH_PLAN=$plan timeout -k 10 300 python tools/stage_small.py $n > gpurun_out/stage_${n}_$plan.json 2> gpurun_out/stage_${n}_$plan.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/stage_${n}_$plan.json'))['$n'];print('excl', {k: round(v, 3) for k, v in d['stage_ms_exclusive'].items()}, 'partial', round(d['partial_wall_ms'], 3))" || exit $?
  done
done
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
echo "== bench 131k" && timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04g.json 2> gpurun_out/bench_r04g.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04g.json'));print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'], d['roofline']['frac'])" || exit $?
K="$K" NOBENCH=1 TAG=r04g bash tools/gpu_r04.sh
