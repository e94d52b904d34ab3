#!/bin/bash
# Round-4 GPU session: parity tests (optionally a -k filter), then the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r04}
if [ -z "$NOTEST" ]; then
  echo "== pytest -m gpu ${K:+-k $K}"
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu ${K:+-k "$K"} --timeout 180 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -6 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  echo "== bench" && timeout -k 10 600 python bench.py $BARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; cat gpurun_out/bench_$TAG.json | head -c 3000; echo; tail -3 gpurun_out/bench_$TAG.err; exit $rc
fi
