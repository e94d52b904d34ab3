set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
echo "== bench W2=1" && timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04d_w2.json 2> gpurun_out/bench_r04d_w2.err &&
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04d_w2.json'));print('W2', d['value'], d['ms_per_step'], d['stage_ms_exclusive'])" &&
echo "== bench W2=0" && TBLS_W2=0 timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04d_w1.json 2> gpurun_out/bench_r04d_w1.err &&
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04d_w1.json'));print('W1', d['value'], d['ms_per_step'], d['stage_ms_exclusive'])" &&
K="test_gpu_bls or test_gpu_configs" NOBENCH=1 TAG=r04d bash tools/gpu_r04.sh
