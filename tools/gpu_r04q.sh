#!/bin/bash
# config-4 host-API latency: bit-sum Miller stream placement and msm threshold A/B
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/cfg4q.log
: > $O
echo "== xw on hash stream (default)" >> $O
timeout -k 10 300 python tools/cfg4_probe.py 12288 16384 24576 32768 >> $O 2>&1 &&
echo "== TBLS_XW=0" >> $O &&
TBLS_XW=0 timeout -k 10 300 python tools/cfg4_probe.py 12288 16384 24576 >> $O 2>&1 &&
echo "== TBLS_MSM_MIN=32768" >> $O &&
TBLS_MSM_MIN=32768 timeout -k 10 300 python tools/cfg4_probe.py 12288 16384 24576 >> $O 2>&1
rc=$?
grep -v amdgpu.ids $O
exit $rc
