#!/bin/bash
# One GPU session: parity tests, the default bench line, rocprofv3 kernel-trace
# stats of the same bench command, then PMC passes (each its own run, as
# MI355X_MICROARCH.md prescribes): FETCH_SIZE, WRITE_SIZE, SQ counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=${SETS:-131072}
PARGS="--steps 1 --warmup 0 --sets-per-gpu $SETS --lat-reps 0 --no-cpu-baseline --no-1m --no-extra --no-kzg"
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 600 python bench.py --sets-per-gpu $SETS > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
[ -n "$NOPROF" ] && exit 0
echo "== kernel trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --sets-per-gpu $SETS --lat-reps 0 --no-cpu-baseline --no-1m > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log
echo "== pmc FETCH_SIZE" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_fetch.log 2>&1 || exit $?
echo "== pmc WRITE_SIZE" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_write.log 2>&1 || exit $?
echo "== pmc SQ" && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_sq.log 2>&1 || exit $?
echo done
