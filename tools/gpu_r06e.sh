#!/bin/bash
# Round 6: coop vs wave Miller kernels on the 128-set latency path:
# kernel traces of tools/latency_probe.py with the default plan and with
# TBLS_MILLER_WAVE_MAX=2048,0 (no coop Miller), and the KZG leg each way.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for mode in coop wave; do
  TAG=r06e_$mode
  rm -rf $O/lat_$TAG
  if [ $mode = wave ]; then export TBLS_MILLER_WAVE_MAX=2048,0; else unset TBLS_MILLER_WAVE_MAX; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/lat_$TAG -o lat --output-format csv -- python3 tools/latency_probe.py 128 40 > $O/lat_$TAG.log 2>&1 || exit $?
  tail -1 $O/lat_$TAG.log
  f=$(find $O/lat_$TAG -name "*kernel_trace.csv" | head -1)
  python3 tools/critical_path.py "$f" $O/latency_128_$TAG.json > /dev/null || exit $?
  python3 -c "
import json; d=json.load(open('$O/latency_128_$TAG.json')); print('$mode span', d['device_span_ms_p50']); [print('  %-30s %7.3f %7.3f %6.3f'%(k,v['start_ms'],v['end_ms'],v['ms'])) for k,v in d['kernels'].items()]"
  timeout -k 10 300 python tools/kzg_order_probe.py kzg_first 30 > $O/kzg_$TAG.log 2>&1 || exit $?
  tail -1 $O/kzg_$TAG.log
done
echo done
