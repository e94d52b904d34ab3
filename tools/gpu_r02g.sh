cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kzg.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02g_kzg.log 2>&1
rc=$?
echo "PYTEST_RC=$rc" >> gpurun_out/pytest_r02g_kzg.log
if [ $rc -eq 0 ]; then
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-extra --lat-reps 3 --extra-reps 12 > gpurun_out/bench_r02g.json 2> gpurun_out/bench_r02g.err
fi
