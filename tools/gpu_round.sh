#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=${SETS:-16384}
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --sets-per-gpu $SETS > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --sets-per-gpu $SETS --no-cpu-baseline --lat-reps 0 > gpurun_out/prof.log 2>&1; rc=$?; tail -3 gpurun_out/prof.log; exit $rc
fi
