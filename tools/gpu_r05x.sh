#!/bin/bash
# Round 5: KZG latency cold vs right after 60 s of BLS load (clock check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/kzg_after_load.py 60 > gpurun_out/kzg_after_load.log 2>&1 || exit $?
tail -1 gpurun_out/kzg_after_load.log
echo done
