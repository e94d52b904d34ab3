#!/bin/bash
# Round 5: the switch cleanup build (priority and join fixed), MSM parity,
# bench; KZG latency with and without the HIP runtime preload.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05s}
timeout -k 10 600 python -u -m pytest "tests/test_gpu_configs.py::test_config5_131k_shard" tests/test_gpu_settle.py "tests/test_gpu_bls.py::test_key_table_bucket_sum_batches" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}.json'))
print(round(d['value']), round(d['ms_per_step'], 2), round(d['value_key_table']), d['roofline']['kernel'])"
for v in 1 0 1 0; do
  TBLS_HIP_PRELOAD=$v timeout -k 10 300 python bench.py --kzg-only > gpurun_out/kzg_${TAG}_$v.json 2> gpurun_out/kzg_${TAG}_$v.err || exit $?
  python3 -c "
import json; d = json.load(open('gpurun_out/kzg_${TAG}_$v.json')); k = d.get('kzg', d)
print('preload $v', round(k['p50_ms_1'], 3), round(k['p50_ms_6'], 3), round(k['dev_64']['ms'], 2))"
done
echo done
