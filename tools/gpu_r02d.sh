cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TBLS_LIB=$GRAFT_REPO_ROOT/teku_amd/lib/variants/libtekubls_hip_w2.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --lat-reps 30 > gpurun_out/bench_r02d_w2.json 2>&1 &&
cd /tmp && TBLS_LIB=$GRAFT_REPO_ROOT/teku_amd/lib/variants/libtekubls_hip_w2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-extra --no-cpu-baseline --lat-reps 3 --serial > $GRAFT_REPO_ROOT/gpurun_out/prof_r02d.log 2>&1
