cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fp_bounds" > gpurun_out/pytest_r02b.log 2>&1
rc=$?
echo "PYTEST_RC=$rc" >> gpurun_out/pytest_r02b.log
if [ $rc -le 1 ]; then
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --lat-reps 50 > gpurun_out/bench_r02b_split.json 2>&1 &&
  TBLS_MILLER_SPLIT=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --lat-reps 20 > gpurun_out/bench_r02b_fused.json 2>&1 &&
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-extra --no-cpu-baseline --lat-reps 5 --serial > $GRAFT_REPO_ROOT/gpurun_out/prof_r02b.log 2>&1
fi
