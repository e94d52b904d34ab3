#!/bin/bash
# Round 5: KZG latency after the BLS legs with the signature stream at high
# vs normal priority (TBLS_SIG_PRIO, A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05t}
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-1m --no-extra --lat-reps 20"
for v in 1 0 1 0; do
  TBLS_SIG_PRIO=$v timeout -k 10 400 python bench.py $ARGS > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || exit $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$v.json')); k = d['kzg']
print('prio $v', round(d['value']), round(d['p50_latency_ms_128'], 3), round(k['p50_ms_1'], 3), round(k['p50_ms_6'], 3), round(k['dev_64']['ms'], 2))"
done
echo done
