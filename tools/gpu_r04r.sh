#!/bin/bash
# two-wave hash with the parked cofactor chain: hash parity, then a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_hash_variants.py tests/test_gpu_configs.py tests/test_gpu_kcoop.py "tests/test_gpu_bls.py::test_large_batch_msm_path" -m gpu > gpurun_out/r04r_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04r_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg > gpurun_out/bench_r04r.json 2> gpurun_out/bench_r04r.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_r04r.json'))
print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'])
print({k: v.get('p50_ms') for k, v in d['configs'].items()})"
