#!/bin/bash
# The primitive-op GPU tests (coop products, coop final exponentiation, ...).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v -s --timeout 300 --timeout-method thread ${OPS_K:+-k "$OPS_K"} > gpurun_out/pytest_ops.log 2>&1; rc=$?
grep -E "cycles|PASS|FAIL|Error|error|passed|failed" gpurun_out/pytest_ops.log | tail -30; exit $rc
