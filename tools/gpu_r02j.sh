#!/bin/bash
# Re-entry baseline on the current tree: full GPU parity suite, the default
# bench line, and a kernel trace (per-kernel start/end) of two 131k steps for
# the concurrency timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu_r02j.log 2>&1; rc=$?; tail -4 $O/pytest_gpu_r02j.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 600 python bench.py > $O/bench_r02j.json 2> $O/bench_r02j.err; rc=$?; cat $O/bench_r02j.json; tail -3 $O/bench_r02j.err; [ $rc -eq 0 ] || exit $rc
cd /tmp
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_r02j -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-extra --no-kzg --no-cpu-baseline --lat-reps 5 > $O/trace_r02j.log 2>&1
echo "RC=$?"
