#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="timeout -k 10 180 python tools/probe.py"
{
$P partial 16384 6 &&
TBLS_HALVES=0 $P partial 16384 6 &&
$P multikey 64 488 6 &&
$P multikey 64 512 6
} > gpurun_out/probe6.log 2>&1 || { tail -5 gpurun_out/probe6.log; exit 1; }
grep "^{" gpurun_out/probe6.log
