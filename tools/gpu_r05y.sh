#!/bin/bash
# Round 5: KZG latency when the BLS library is initialised first (bench order).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/kzg_after_load.py 10 bls_first > gpurun_out/kzg_bls_first.log 2>&1 || exit $?
tail -1 gpurun_out/kzg_bls_first.log
echo done
