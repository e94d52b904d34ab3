set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K="test_gpu_hash_variants or test_gpu_bls or test_gpu_configs or test_gpu_hrow" NOBENCH=1 TAG=r04c bash tools/gpu_r04.sh &&
NOTEST=1 TAG=r04c BARGS="--no-cpu-baseline" bash tools/gpu_r04.sh &&
timeout -k 10 100 ./tools/microbench/fp2_rates > gpurun_out/fp2_rates2.json 2> gpurun_out/fp2_rates2.err; rc=$?; cat gpurun_out/fp2_rates2.json; tail -3 gpurun_out/fp2_rates2.err; exit $rc
