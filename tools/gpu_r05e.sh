#!/bin/bash
# Round 5 checkpoint: whole GPU suite, smoke, default bench, kernel-trace stats
# of the 131k bench step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05e}
echo "== pytest -m gpu"
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
echo "== bench (default)" && timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_$TAG.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel'), d['stage_ms_exclusive'])
print({k: (v.get('p50_ms'), v.get('sigs_per_s') or v.get('sets_per_s')) for k, v in d['configs'].items()})
print('cfg4', d['configs']['cfg4']); print('facade', d['configs'].get('cfg4_facade'))
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], 'p50@128', d.get('p50_latency_ms_128'), 'value_1m', d.get('value_1m'), 'key_table', d.get('value_key_table'))" || exit $?
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg > gpurun_out/prof_${TAG}.log 2>&1 || exit $?
echo done
