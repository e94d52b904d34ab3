#!/bin/bash
# Round 5: BLS partial time vs allocation order (workspace first / data first).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in data_first ws_first data_first ws_first; do
  timeout -k 10 300 python tools/alloc_order_probe.py $m 20 >> gpurun_out/alloc_order.log 2>&1 || exit $?
  tail -1 gpurun_out/alloc_order.log
done
echo done
