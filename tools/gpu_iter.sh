#!/bin/bash
# One iteration on the GPU box: the GPU parity tests (or the subset in $TESTS),
# the default bench line, and the stage breakdown at the sizes in $STAGES.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
echo "== pytest -m gpu $TESTS"
timeout -k 10 900 python -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
[ -n "$NOBENCH" ] && exit 0
echo "== bench"
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "$STAGES" ]; then
  echo "== stages $STAGES"
  timeout -k 10 300 python tools/stage_small.py $STAGES > gpurun_out/stage_small.json 2> gpurun_out/stage_small.err || exit $?
fi
echo done
