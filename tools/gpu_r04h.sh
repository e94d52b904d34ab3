#!/bin/bash
# Mid-size batches on the one-wave per-set kernels: stage times at 16,384 /
# 8,192 sets, then the full default bench (configs, KZG, CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== stage_small 16384 8192"
timeout -k 10 300 python tools/stage_small.py 16384 8192 > gpurun_out/stage_r04h.json 2> gpurun_out/stage_r04h.err || exit $?
python3 -c "
import json
for n, d in json.load(open('gpurun_out/stage_r04h.json')).items():
    print(n, 'excl', {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()}, 'over', {k: round(v, 2) for k, v in d['stage_ms_overlapped'].items()}, 'partial', round(d['partial_wall_ms'], 2))" || exit $?
echo "== bench (default)" && timeout -k 10 900 python bench.py > gpurun_out/bench_r04h.json 2> gpurun_out/bench_r04h.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_r04h.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel'))
print({k: (v.get('p50_ms'), v.get('sigs_per_s') or v.get('sets_per_s')) for k, v in d['configs'].items()})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], 'p50@128', d.get('p50_latency_ms_128'), 'value_1m', d.get('value_1m'), 'key_table', d.get('value_key_table'))" || exit $?
