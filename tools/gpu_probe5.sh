#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="timeout -k 10 180 python tools/probe.py"
{
$P partial 16384 6 &&
TBLS_HALVES=0 $P partial 16384 6 &&
$P partial 4096 6 &&
TBLS_HALVES=0 $P partial 4096 6
} > gpurun_out/probe5.log 2>&1 || { tail -5 gpurun_out/probe5.log; exit 1; }
grep "^{" gpurun_out/probe5.log
