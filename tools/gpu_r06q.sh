#!/bin/bash
# Round 6: hardware queues A/B (TBLS_BENCH_HW_QUEUES=4 against the bench's
# default of at least 8) on one box, alternated twice: the 131k step, its
# stage times and the KZG leg (1 / 6 blobs); then the driver's command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r06q}
mkdir -p $O
ARGS="--steps 10 --warmup 3 --no-extra --no-1m --no-cpu-baseline --lat-reps 0 --extra-reps 20"
show() { python -c "import json; d=json.load(open('$1')); k=d['kzg']; print('$2', round(d['ms_per_step'],3), 'kzg', round(k['p50_ms_1'],3), round(k['p50_ms_6'],3), {x:round(v,3) for x,v in d['stage_ms_exclusive'].items()})"; }
for r in 1 2; do
  for q in 4 8; do
    TBLS_BENCH_HW_QUEUES=$q timeout -k 10 400 python bench.py $ARGS > $O/hwq${q}_${TAG}_$r.json 2> $O/hwq${q}_${TAG}_$r.err || exit $?
    show $O/hwq${q}_${TAG}_$r.json hwq$q
  done
done
[ -n "$FULL" ] || { echo done; exit 0; }
TAG=$TAG NOTEST=1 bash tools/gpu_r06h.sh || exit $?
echo done
