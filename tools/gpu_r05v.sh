#!/bin/bash
# Round 5: accumulators with a wave-uniform segment index (scalar line-row
# bases): parity of every accumulator path, bench x2, FETCH/WRITE.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05v}
timeout -k 10 900 python -u -m pytest tests/test_gpu_accseg.py tests/test_gpu_configs.py tests/test_gpu_settle.py tests/test_gpu_bls.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
for k in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$k.json 2> gpurun_out/bench_${TAG}_$k.err || exit $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$k.json'))
print(round(d['value']), round(d['ms_per_step'], 2), round(d['value_key_table']), {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()})"
done
P="tools/probe.py stages 131072 3"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_write.log 2>&1 || exit $?
echo done
