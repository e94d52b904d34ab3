#!/bin/bash
# Coop product parity + timing, then the full GPU suite and the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== coop" && timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -s -k coop --timeout 120 --timeout-method thread > gpurun_out/pytest_coop.log 2>&1; rc=$?; grep -E "coop cycles|passed|failed|Error" gpurun_out/pytest_coop.log | tail -5; [ $rc -eq 0 ] || exit $rc
[ -n "$COOP_ONLY" ] && exit 0
NOPROF=1 bash tools/gpu_full.sh
