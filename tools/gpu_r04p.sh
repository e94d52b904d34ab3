#!/bin/bash
# Bucket-sum signature side from 16,384 / 8,192 sets (TBLS_MSM_MIN) vs 32,768.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mm in 32768 16384 8192; do
  echo "== msm_min=$mm"
  TBLS_MSM_MIN=$mm timeout -k 10 600 python tools/stage_small.py 8192 12288 16384 24576 > gpurun_out/stage_msm_$mm.json 2> gpurun_out/stage_msm_$mm.err || exit $?
  python3 -c "
import json
for n, d in json.load(open('gpurun_out/stage_msm_$mm.json')).items():
    print(n, 'partial', round(d['partial_wall_ms'], 2), {k: round(v, 2) for k, v in d['stage_ms_overlapped'].items()})" || exit $?
done
