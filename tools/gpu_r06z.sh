#!/bin/bash
# Round 6 final evidence: smoke(), the driver's bench command with the
# 128-set latency timeline, then the profiling session (kernel trace stats,
# SQ / FETCH_SIZE / WRITE_SIZE passes) of the same build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r06z}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || exit $?
tail -1 $O/smoke_$TAG.log
TAG=$TAG NOTEST=1 bash tools/gpu_r06h.sh || exit $?
bash tools/profile_round.sh || exit $?
echo done
