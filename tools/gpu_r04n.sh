#!/bin/bash
# Per-set stages in sequence (chain) vs side by side from 32,768 sets.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cm in 0 262144; do
  echo "== chain_min=$cm"
  TBLS_CHAIN_MIN=$cm timeout -k 10 600 python tools/stage_small.py 32768 65536 98304 131072 > gpurun_out/stage_chain_$cm.json 2> gpurun_out/stage_chain_$cm.err || exit $?
  python3 -c "
import json
for n, d in json.load(open('gpurun_out/stage_chain_$cm.json')).items():
    print(n, 'partial', round(d['partial_wall_ms'], 2), {k: round(v, 2) for k, v in d['stage_ms_overlapped'].items()})" || exit $?
done
