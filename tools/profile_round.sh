#!/bin/bash
# One profiling session on the GPU box: kernel-trace stats of the bench, then
# PMC passes (each in its own run, as MI355X_MICROARCH.md's rocprofv3 section
# prescribes): SQ instruction/cycle counters, FETCH_SIZE, WRITE_SIZE.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=${SETS:-131072}
ARGS="--steps 2 --warmup 1 --sets-per-gpu $SETS --lat-reps 0 --no-cpu-baseline --no-1m"
PARGS="--steps 1 --warmup 0 --sets-per-gpu $SETS --lat-reps 0 --no-cpu-baseline --no-1m --no-extra --no-kzg"
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log
echo "== pmc SQ" && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_sq.log 2>&1 || exit $?
echo "== pmc FETCH_SIZE" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_fetch.log 2>&1 || exit $?
echo "== pmc WRITE_SIZE" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_write.log 2>&1 || exit $?
echo done
