#!/bin/bash
# Round 6 checkpoint: GPU suite, the driver's bench command, the 128-set
# latency timeline, and the KZG hardware-queue experiment.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r06h}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_$TAG.log 2>&1; rc=$?
  tail -3 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit $?
python3 -c "
import json; d = json.load(open('$O/bench_$TAG.json')); c = d['configs']; k = d['kzg']
print(round(d['value']), round(d['ms_per_step'], 2), 'p50', round(d['p50_latency_ms_128'], 3), '1m', round(d['value_1m']), 'kt', round(d['value_key_table']),
      {x: round(v['p50_ms'], 3) for x, v in c.items()}, 'fail', round(c['cfg4']['failure_settle_ms'], 2), 'svc', c['cfg4']['service_ms'], 'cpu', round(d['cpu_baseline']['value']),
      'kzg', round(k['p50_ms_1'], 3), round(k['p50_ms_6'], 3), 'frac', round(d['roofline']['frac'], 3), {x: round(v, 3) for x, v in d['stage_ms_exclusive'].items()})"
TAG=$TAG bash tools/gpu_r06d.sh > $O/lat_$TAG.txt 2>&1 || exit $?; tail -3 $O/lat_$TAG.txt
[ -n "$KZGQ" ] && { bash tools/gpu_r06f.sh || exit $?; }
echo done
