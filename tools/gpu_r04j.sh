#!/bin/bash
# Windowed [r] apk + G1 doubling runs + lean two-wave line kernel (A/B), and
# the product tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
for v in 0 1; do
  echo "== bench LINES_W2=$v"
  TBLS_LINES_W2=$v timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04j_l$v.json 2> gpurun_out/bench_r04j_l$v.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_r04j_l$v.json'));print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'])" || exit $?
done
echo "== stage_small 16384"
timeout -k 10 300 python tools/stage_small.py 16384 > gpurun_out/stage_r04j.json 2> gpurun_out/stage_r04j.err || exit $?
python3 -c "
import json
for n, d in json.load(open('gpurun_out/stage_r04j.json')).items():
    print(n, 'excl', {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()}, 'partial', round(d['partial_wall_ms'], 2))" || exit $?
K="test_gpu_hrow or test_gpu_bls or test_gpu_configs or test_gpu_accseg" NOBENCH=1 TAG=r04j bash tools/gpu_r04.sh
