#!/bin/bash
# Timing only: small-batch stage breakdown + bench line (no parity suite).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
TAG=${TAG:-time}
mkdir -p $O
echo "== stage_small" && timeout -k 10 300 python tools/stage_small.py 128 1024 > $O/stage_small_$TAG.json 2> $O/stage_small_$TAG.err; rc=$?; cat $O/stage_small_$TAG.json | python -c "import json,sys; d=json.load(sys.stdin); [print(k, {a:round(b,3) for a,b in v['stage_ms_exclusive'].items()}, round(v['partial_wall_ms'],3), round(v['final_wall_ms'],3)) for k,v in d.items()]"; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 600 python bench.py --no-extra --no-kzg --no-cpu-baseline ${BENCH_ARGS} > $O/bench_$TAG.json 2> $O/bench_$TAG.err; rc=$?; python -c "import json; d=json.load(open('$O/bench_$TAG.json')); print({k:d[k] for k in ('value','ms_per_step','value_key_table','p50_latency_ms_128','p99_latency_ms_128')}); print(d['stage_ms_exclusive'])"; exit $rc
