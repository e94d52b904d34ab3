#!/bin/bash
# Round 6 quick check: the named GPU test files (TESTS), their printed
# cycle counts, then the 128-set latency probe (60 calls).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-chk}
mkdir -p $O
timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -x -v -s -m gpu --timeout 300 --timeout-method thread > $O/pytest_$TAG.log 2>&1; rc=$?
tail -3 $O/pytest_$TAG.log; grep -h "cycles" $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/latency_probe.py 128 60 > $O/lat_probe_$TAG.json 2>&1 || exit $?
tail -1 $O/lat_probe_$TAG.json
echo done
