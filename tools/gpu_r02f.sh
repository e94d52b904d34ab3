cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02f.log 2>&1
rc=$?
echo "PYTEST_RC=$rc" >> gpurun_out/pytest_r02f.log
if [ $rc -le 1 ]; then
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --lat-reps 30 > gpurun_out/bench_r02f_main.json 2>&1 &&
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02f -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-extra --no-cpu-baseline --lat-reps 3 --serial > $GRAFT_REPO_ROOT/gpurun_out/prof_r02f.log 2>&1
fi
