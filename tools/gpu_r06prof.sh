#!/bin/bash
# Round 6: rocprofv3 kernel trace + stats of the driver's exact bench
# command (profiles/r06_kernel_stats_driver_cmd.csv), and the per-size
# durations of the roofline kernels from the same trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
rm -rf $O/prof_drv
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof_drv -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_drv.json 2> $O/prof_drv.err || exit $?
tail -c 300 $O/prof_drv.json
echo done
