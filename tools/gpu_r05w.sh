#!/bin/bash
# Round 5 final evidence (last build): full GPU suite, smoke, the default bench (the driver's
# command), rocprof kernel stats of the bench, stage-only trace, FETCH/WRITE.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05w}
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
echo "== bench (driver command)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/bench_$TAG.json')); c = d['configs']
print(round(d['value']), round(d['ms_per_step'], 2), 'p50', round(d['p50_latency_ms_128'], 3), '1m', round(d['value_1m']), 'kt', round(d['value_key_table']),
      {k: round(v['p50_ms'], 3) for k, v in c.items()}, 'fail', round(c['cfg4']['failure_settle_ms'], 2), 'cpu', round(d['cpu_baseline']['value']),
      'frac', round(d['roofline']['frac'], 3), {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()})"
echo "== kernel trace of a short bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-1m --no-kzg --lat-reps 20 --extra-reps 5 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
P="tools/probe.py stages 131072 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_stages -o run --output-format csv -- python3 $P > gpurun_out/prof_${TAG}_stages.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d gpurun_out/pmc_${TAG}_sq -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_sq.log 2>&1 || exit $?
echo done
