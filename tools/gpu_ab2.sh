#!/bin/bash
# A/B, alternating the main build and variant libraries (VARS="path ...",
# each run as TBLS_LIB=path) twice on one box: the 131k step and its
# exclusive stage times (no configs / KZG / CPU leg; LAT=n adds the 128-set p50).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
TAG=${TAG:-ab2}
mkdir -p $O
ARGS="--steps 10 --warmup 3 --no-extra --no-kzg --no-1m --no-cpu-baseline --lat-reps ${LAT:-0}"
show() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step'],3), 'p50', d.get('p50_latency_ms_128'), {k:round(v,3) for k,v in d['stage_ms_exclusive'].items()})"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/ab2_main_${TAG}_$r.json 2> $O/ab2_main_${TAG}_$r.err || exit $?
  show $O/ab2_main_${TAG}_$r.json main
  for V in ${VARS:-$VAR}; do
    b=$(basename $V .so)
    TBLS_LIB=$V timeout -k 10 300 python bench.py $ARGS > $O/ab2_${b}_${TAG}_$r.json 2> $O/ab2_${b}_${TAG}_$r.err || exit $?
    show $O/ab2_${b}_${TAG}_$r.json $b
  done
done
echo done
