#!/bin/bash
# Quad key decompression for multi-key batches: its parity tests, then the
# bench's configs 2/3 (and the rest of the line).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
K="test_gpu_kcoop or test_gpu_configs or test_gpu_bls" NOBENCH=1 TAG=r04l bash tools/gpu_r04.sh || exit $?
echo "== bench (no cpu baseline, no kzg)" && timeout -k 10 600 python bench.py --no-cpu-baseline --no-kzg > gpurun_out/bench_r04l.json 2> gpurun_out/bench_r04l.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_r04l.json'))
print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'])
print({k: (v.get('p50_ms'), v.get('aggregation_ms'), v.get('p50_ms_key_table')) for k, v in d['configs'].items()})" || exit $?
