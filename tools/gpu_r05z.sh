#!/bin/bash
# Round 5: the driver's bench command with the KZG context warmed at start.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05z}
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_$TAG.json')); c = d['configs']; k = d['kzg']
print(round(d['value']), round(d['ms_per_step'], 2), 'p50', round(d['p50_latency_ms_128'], 3), '1m', round(d['value_1m']), 'kt', round(d['value_key_table']),
      {x: round(v['p50_ms'], 3) for x, v in c.items()}, 'fail', round(c['cfg4']['failure_settle_ms'], 2), 'cpu', round(d['cpu_baseline']['value']),
      'kzg', round(k['p50_ms_1'], 3), round(k['p50_ms_6'], 3), round(k['dev_64']['ms'], 2))"
echo done
