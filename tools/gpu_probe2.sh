#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="timeout -k 10 180 python tools/probe.py"
{
$P partial 131072 4 &&
TBLS_ACC_PAIRS=1 $P partial 131072 4 &&
TBLS_ACC_PAIRS=1 TBLS_ACC_PER=4 TBLS_ACC_SEG=2 $P partial 131072 4 &&
TBLS_ACC_PAIRS=1 $P partial 16384 4 &&
$P partial 16384 4 &&
$P multikey 64 488 4
} > gpurun_out/probe2.log 2>&1 || { tail -5 gpurun_out/probe2.log; exit 1; }
grep "^{" gpurun_out/probe2.log
echo "== accseg test"
timeout -k 10 600 python -u -m pytest tests/test_gpu_accseg.py -x -v -m gpu --timeout 500 --timeout-method thread > gpurun_out/pytest_accseg.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_accseg.log; exit $rc
