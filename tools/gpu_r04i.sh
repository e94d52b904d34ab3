#!/bin/bash
# Hash cofactor clearing with the LDS-parked point: stage times and PMC
# traffic; the TB_G1_XRUNS=1 variant (key subgroup check as doubling runs)
# against the default; then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-extra --no-kzg --lat-reps 0 --steps 5 --warmup 2"
echo "== bench default" && timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04i.json 2> gpurun_out/bench_r04i.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04i.json'));print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'])" || exit $?
echo "== bench g1x" && TBLS_LIB=teku_amd/lib/ab/libtekubls_hip_g1x.so timeout -k 10 300 python bench.py $Q > gpurun_out/bench_r04i_g1x.json 2> gpurun_out/bench_r04i_g1x.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04i_g1x.json'));print(d['value'], d['ms_per_step'], d['stage_ms_exclusive'])" || exit $?
P="--steps 1 --warmup 0 --lat-reps 0 --no-cpu-baseline --no-extra --no-kzg"
echo "== pmc FETCH_SIZE" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_i -o run --output-format csv -- python3 bench.py $P > gpurun_out/pmc_fetch_i.log 2>&1 || exit $?
echo "== pmc WRITE_SIZE" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_i -o run --output-format csv -- python3 bench.py $P > gpurun_out/pmc_write_i.log 2>&1 || exit $?
echo "== pytest -m gpu (all)"
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_r04i.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r04i.log; exit $rc
