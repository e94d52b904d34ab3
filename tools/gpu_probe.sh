#!/bin/bash
# A/B probes of the accumulator plan and the aggregation kernel, plus a
# kernel-trace profile of the default plan (each step under its own limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="timeout -k 10 180 python tools/probe.py"
{
$P partial 131072 4 &&
TBLS_ACC_SEG=0 $P partial 131072 4 &&
TBLS_ACC_PER=4 TBLS_ACC_SEG=2 $P partial 131072 4 &&
TBLS_ACC_PER=8 TBLS_ACC_SEG=2 $P partial 131072 4 &&
TBLS_ACC_PER=4 TBLS_ACC_SEG=4 $P partial 131072 4 &&
$P partial 16384 4 &&
TBLS_ACC_PER=1 TBLS_ACC_SEG=4 $P partial 16384 4 &&
TBLS_ACC_PER=4 TBLS_ACC_SEG=4 $P partial 16384 4 &&
TBLS_ACC_SEG=0 $P partial 16384 4 &&
$P multikey 64 488 6 &&
TBLS_AGG_COOP=0 $P multikey 64 488 6
} > gpurun_out/probe.log 2>&1 || { tail -5 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log | grep "^{"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_probe -o run --output-format csv -- python3 tools/probe.py partial 131072 2 > gpurun_out/prof_probe.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_probe_mk -o run --output-format csv -- python3 tools/probe.py multikey 64 488 4 > gpurun_out/prof_probe_mk.log 2>&1 || exit $?
echo done
