#!/bin/bash
# A/B of a variant library (TBLS_LIB=$VAR) against the main build on the bench's
# exclusive stage times, then timings of the main build and the part latencies.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
TAG=${TAG:-ab}
mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-extra --no-kzg --no-cpu-baseline --lat-reps 0"
echo "== variant $VAR" && TBLS_LIB=$VAR timeout -k 10 300 python bench.py $ARGS > $O/ab_var_$TAG.json 2> $O/ab_var_$TAG.err; rc=$?; python -c "import json; d=json.load(open('$O/ab_var_$TAG.json')); print(round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms_exclusive'].items()})"; [ $rc -eq 0 ] || exit $rc
echo "== main" && timeout -k 10 300 python bench.py $ARGS > $O/ab_main_$TAG.json 2> $O/ab_main_$TAG.err; rc=$?; python -c "import json; d=json.load(open('$O/ab_main_$TAG.json')); print(round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms_exclusive'].items()})"; [ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/gpu_time.sh || exit $?
echo "== parts" && timeout -k 10 300 python tools/hash_parts.py 128 > $O/parts_$TAG.txt 2>&1; rc=$?; cat $O/parts_$TAG.txt; exit $rc
