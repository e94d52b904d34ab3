#!/bin/bash
# Round 6: GPU suite on the new build (coop Miller for small pair counts,
# settle mask, shared-device sharding test, non-temporal line traffic), then
# the NT A/B (main vs TB_LINE_NT=0) and the KZG allocation-order probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${TAG:-r06b}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_$TAG.log 2>&1; rc=$?
  tail -5 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARS" ]; then
  LAT=${LAT:-50} TAG=$TAG VARS="$VARS" bash tools/gpu_ab2.sh || exit $?
fi
if [ -n "$KZG" ]; then
  for o in bls_first kzg_first bls_first kzg_first; do
    timeout -k 10 300 python tools/kzg_order_probe.py $o 30 >> $O/kzg_order_$TAG.log 2>&1 || exit $?
    tail -1 $O/kzg_order_$TAG.log
  done
  for V in $KZGVARS; do
    for o in bls_first kzg_first; do
      TBLS_LIB=$V timeout -k 10 300 python tools/kzg_order_probe.py $o 30 >> $O/kzg_order_$TAG.log 2>&1 || exit $?
      tail -1 $O/kzg_order_$TAG.log
    done
  done
fi
echo done
