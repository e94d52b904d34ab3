set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -x -q -m gpu > gpurun_out/gpu_ops.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_ops.log
exit $rc
