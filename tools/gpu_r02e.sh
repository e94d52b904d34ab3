cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02e.log 2>&1
rc=$?
echo "PYTEST_RC=$rc" >> gpurun_out/pytest_r02e.log
if [ $rc -le 1 ]; then
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --lat-reps 30 > gpurun_out/bench_r02e_main.json 2>&1 &&
  TBLS_LIB=$GRAFT_REPO_ROOT/teku_amd/lib/variants/libtekubls_hip_fence.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --lat-reps 30 > gpurun_out/bench_r02e_fence.json 2>&1 &&
  TBLS_LIB=$GRAFT_REPO_ROOT/teku_amd/lib/variants/libtekubls_hip_fence.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -k "config5 or config1" --timeout 300 --timeout-method thread > gpurun_out/pytest_r02e_fence.log 2>&1
fi
