#!/bin/bash
# two-wave hash (parked cofactor chain) + [r] apk with the LDS window table:
# the >= 32,768-set tests, then a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_configs.py::test_config5_1m_as_8_simulated_shards" "tests/test_gpu_bls.py::test_large_batch_msm_path" tests/test_gpu_kcoop.py tests/test_gpu_accseg.py -m gpu > gpurun_out/r04s_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r04s_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg > gpurun_out/bench_r04s.json 2> gpurun_out/bench_r04s.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_r04s.json'))
print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'])
print({k: v.get('p50_ms') for k, v in d['configs'].items()})"
