#!/bin/bash
# Round 6: is the KZG-after-BLS slowdown the hardware-queue sharing? The
# probe's bls_first / kzg_first orders at GPU_MAX_HW_QUEUES 4 (the box
# default) and 8 / 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for q in 4 8 16; do
  for o in bls_first kzg_first; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/kzg_order_probe.py $o 30 > $O/kzgq_${q}_$o.log 2>&1 || exit $?
    echo "queues $q $(tail -1 $O/kzgq_${q}_$o.log)"
  done
done
echo done
