#!/bin/bash
# Round 5: signature / bucket-sum stream at high priority (TBLS_SIG_PRIO=1),
# with the register and the LDS accumulator.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05l}
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), d['roofline']['kernel'], {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()})"
}
for r in 1 2; do
  run base$r || exit $?
  run prio$r TBLS_SIG_PRIO=1 || exit $?
  run prio_lds$r TBLS_SIG_PRIO=1 TBLS_ACC_LDS=1 || exit $?
  run prio_join$r TBLS_SIG_PRIO=1 TBLS_ACC_LDS=1 TBLS_ACC_JOIN=1 || exit $?
done
echo done
