#!/bin/bash
# Round 5: full GPU suite + smoke after build() rebuilt the test library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05u}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}.json'))
print(round(d['value']), round(d['ms_per_step'], 2), round(d['value_key_table']))"
echo done
