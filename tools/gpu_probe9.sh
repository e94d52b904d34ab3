#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="timeout -k 10 180 python tools/probe.py"
{
$P partial 131072 4 &&
$P partial 16384 4 &&
$P partial 128 8
} > gpurun_out/probe9.log 2>&1 || { tail -5 gpurun_out/probe9.log; exit 1; }
grep "^{" gpurun_out/probe9.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc9_fetch -o run --output-format csv -- python3 tools/probe.py partial 131072 1 > gpurun_out/pmc9.log 2>&1 || exit 1
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 500 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
