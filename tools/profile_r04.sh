#!/bin/bash
# Round-4 profiling session: kernel-trace stats of the bench (the 131k step,
# no 1M leg), then PMC passes -- each counter set in its own run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes -- over the bench
# workload alone (tools/probe.py partial 131072: the per-set, Miller and
# product kernels of one 131k partial, nothing from the configs), so that
# every launch of a kernel in the CSV has the bench's grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 3 --warmup 1 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg"
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof4.log 2>&1 || exit $?
tail -c 600 gpurun_out/prof4.log; echo
P="tools/probe.py partial 131072 2"
echo "== pmc FETCH_SIZE" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc4_fetch -o run --output-format csv -- python3 $P > gpurun_out/pmc4_fetch.log 2>&1 || exit $?
echo "== pmc WRITE_SIZE" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc4_write -o run --output-format csv -- python3 $P > gpurun_out/pmc4_write.log 2>&1 || exit $?
echo "== pmc SQ" && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU -d gpurun_out/pmc4_sq -o run --output-format csv -- python3 $P > gpurun_out/pmc4_sq.log 2>&1 || exit $?
echo done
