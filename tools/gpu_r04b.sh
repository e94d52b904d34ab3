set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/mad_peak > gpurun_out/mad_peak.json && cat gpurun_out/mad_peak.json &&
timeout -k 10 120 ./tools/microbench/fp2_rates > gpurun_out/fp2_rates.json && cat gpurun_out/fp2_rates.json &&
K="test_gpu_bls or test_gpu_configs" NOBENCH=1 TAG=r04b bash tools/gpu_r04.sh &&
NOTEST=1 TAG=r04b BARGS="--no-cpu-baseline" bash tools/gpu_r04.sh
