#!/bin/bash
# Round 6 start: carry-chain hazard microbenchmark, then the driver's bench command on the round-5 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/microbench/carry_chain > gpurun_out/r06a_carry_chain.json || exit $?
cat gpurun_out/r06a_carry_chain.json
timeout -k 10 60 tools/microbench/mad_peak > gpurun_out/r06a_mad_peak.json || exit $?
cat gpurun_out/r06a_mad_peak.json
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r06a.json 2> gpurun_out/bench_r06a.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_r06a.json')); c = d['configs']; k = d['kzg']
print(round(d['value']), round(d['ms_per_step'], 2), 'p50', round(d['p50_latency_ms_128'], 3), '1m', round(d['value_1m']), 'kt', round(d['value_key_table']),
      {x: round(v['p50_ms'], 3) for x, v in c.items()}, 'cpu', round(d['cpu_baseline']['value']),
      'kzg', round(k['p50_ms_1'], 3), round(k['p50_ms_6'], 3))"
echo done
