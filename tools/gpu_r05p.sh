#!/bin/bash
# Round 5: hash after the signature checks (1) / after the whole bucket-sum
# chain (2) / first (0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05p}
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), d['value_key_table'] and round(d['value_key_table']))"
}
for r in 1 2; do
  run chain$r TBLS_SIG_FIRST=2 || exit $?
  run hash$r TBLS_SIG_FIRST=0 || exit $?
  run sig$r TBLS_SIG_FIRST=1 || exit $?
done
TBLS_SIG_FIRST=2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-1m --no-kzg --no-extra --lat-reps 0 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
echo done
