#!/bin/bash
# Round 5: the LDS-resident accumulator (k_miller_accs_lds) -- parity of the
# partial records under every plan, then the 131k bench A/B against the
# register-resident k_miller_accs, then WRITE_SIZE / SQ counters of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05b}
echo "== parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_accseg.py tests/test_gpu_configs.py tests/test_gpu_hrow.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
for v in 1 0 1; do
  echo "== bench TBLS_ACC_LDS=$v"
  TBLS_ACC_LDS=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_lds$v.json 2> gpurun_out/bench_${TAG}_lds$v.err || exit $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_lds$v.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel'), d['stage_ms_exclusive']['miller'])"
done
P="tools/probe.py partial 131072 2"
for v in 1 0; do
  echo "== pmc WRITE_SIZE lds=$v" && TBLS_ACC_LDS=$v timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write$v -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_write$v.log 2>&1 || exit $?
  echo "== pmc SQ lds=$v" && TBLS_ACC_LDS=$v timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d gpurun_out/pmc_${TAG}_sq$v -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_sq$v.log 2>&1 || exit $?
done
echo done
