#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="timeout -k 10 180 python tools/probe.py"
{
$P partial 131072 4 &&
TBLS_DEC2=0 $P partial 131072 4 &&
$P partial 16384 4 &&
TBLS_DEC2=0 $P partial 16384 4
} > gpurun_out/probe3.log 2>&1 || { tail -5 gpurun_out/probe3.log; exit 1; }
grep "^{" gpurun_out/probe3.log
