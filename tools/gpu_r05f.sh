#!/bin/bash
# Round 5: the two-wave hash with its two SSWU maps in sequence (variant
# TB_HASH_SSWU_SEQ=1) against the interleaved pair: hash parity, bench A/B,
# FETCH/WRITE of k_set_hash_w2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05f}
V=teku_amd/lib/ab/libtekubls_hip_sswuseq.so
echo "== hash parity (variant)"
TBLS_LIB=$V timeout -k 10 600 python -u -m pytest "tests/test_gpu_configs.py::test_config5_131k_shard" "tests/test_gpu_bls.py::test_large_batch_msm_path" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --lat-reps 0 --no-cpu-baseline --no-1m --no-kzg --no-extra"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || return $?
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_${TAG}_$name.json'))
print('$name', round(d['value']), round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in d['stage_ms_exclusive'].items()})"
}
run base || exit $?
run seq TBLS_LIB=$V || exit $?
run base2 || exit $?
run seq2 TBLS_LIB=$V || exit $?
P="tools/probe.py partial 131072 2"
for v in base seq; do
  E=""; [ $v = seq ] && E="TBLS_LIB=$V"
  echo "== pmc $v" && env $E timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch_$v -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_fetch_$v.log 2>&1 || exit $?
  env $E timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write_$v -o run --output-format csv -- python3 $P > gpurun_out/pmc_${TAG}_write_$v.log 2>&1 || exit $?
done
echo done
