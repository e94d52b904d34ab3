cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in 0 1 2; do
  TBLS_MILLER_VARIANT=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --sets-per-gpu 131072 --no-cpu-baseline --lat-reps 0 > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print($v, d['value'], d['stage_ms_exclusive']['miller'])"
done
