#!/bin/bash
# Round 6: the 128-set latency path as a kernel timeline (rocprofv3
# kernel trace of tools/latency_probe.py -> tools/critical_path.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r06d}
mkdir -p $O
rm -rf $O/lat_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/lat_$TAG -o lat --output-format csv -- python3 tools/latency_probe.py 128 40 > $O/lat_$TAG.log 2>&1 || exit $?
tail -1 $O/lat_$TAG.log
f=$(find $O/lat_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/critical_path.py "$f" $O/latency_128_$TAG.json | head -60
echo done
