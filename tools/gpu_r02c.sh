cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02c.log 2>&1
rc=$?
echo "PYTEST_RC=$rc" >> gpurun_out/pytest_r02c.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r02c.json 2>&1 &&
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-extra --no-cpu-baseline --lat-reps 5 --serial > $GRAFT_REPO_ROOT/gpurun_out/prof_r02c.log 2>&1
fi
