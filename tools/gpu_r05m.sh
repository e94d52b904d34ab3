#!/bin/bash
# Round 5: full bench (configs 1-4, facade, 1M) with and without the
# high-priority signature stream + joined LDS accumulator.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05m}
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-kzg"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json')); c = d['configs']
print('$name', round(d['value']), round(d['ms_per_step'], 2), 'p50', round(d['p50_latency_ms_128'], 3), '1m', round(d['value_1m']), 'kt', round(d['value_key_table']),
      {k: round(v['p50_ms'], 3) for k, v in c.items()}, 'fail', round(c['cfg4']['failure_settle_ms'], 2))"
}
run base || exit $?
run new TBLS_SIG_PRIO=1 TBLS_ACC_JOIN=1 || exit $?
run base2 || exit $?
run new2 TBLS_SIG_PRIO=1 TBLS_ACC_JOIN=1 || exit $?
echo done
