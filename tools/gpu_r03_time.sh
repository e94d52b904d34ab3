#!/bin/bash
# BLS parity subset + small-batch stage timing (A/B of the lane-cooperative stages) + bench (timing legs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
TAG=${TAG:-time}
mkdir -p $O
echo "== pytest" && timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_kcoop.py tests/test_gpu_bls.py tests/test_gpu_kzg.py} -x -q --timeout 300 --timeout-method thread > $O/pytest_bls_$TAG.log 2>&1; rc=$?; tail -3 $O/pytest_bls_$TAG.log; [ $rc -eq 0 ] || exit $rc
# variants: "name:ENV=V,ENV=V"
for VAR in ${VARIANTS:-coop: nocoop:TBLS_KEYS_COOP=0,TBLS_SIG_COOP=0}; do
NAME=${VAR%%:*}; ENVS=${VAR#*:}
echo "== stage_small $NAME ($ENVS)" && env ${ENVS//,/ } timeout -k 10 300 python tools/stage_small.py 128 1024 > $O/stage_small_${TAG}_$NAME.json 2> $O/stage_small_${TAG}_$NAME.err || exit $?
python -c "import json; d=json.load(open('$O/stage_small_${TAG}_$NAME.json')); [print(k, {a:round(b,3) for a,b in v['stage_ms_exclusive'].items()}, round(v['partial_wall_ms'],3), round(v['final_wall_ms'],3)) for k,v in d.items()]"
done
echo "== bench" && timeout -k 10 600 python bench.py --no-extra --no-cpu-baseline --no-1m ${BENCH_ARGS} > $O/bench_$TAG.json 2> $O/bench_$TAG.err; rc=$?; python -c "import json; d=json.load(open('$O/bench_$TAG.json')); print({k:d[k] for k in ('value','ms_per_step','value_key_table','p50_latency_ms_128','p99_latency_ms_128')}); print(d['kzg'].get('p50_ms_1'), d['kzg'].get('p50_ms_6'))"; exit $rc
