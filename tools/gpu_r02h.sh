cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python tools/stage_small.py 128 1024 > $O/stage_small_r02h.json 2> $O/stage_small_r02h.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r02h_128 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stage_small.py 128 > $O/prof_r02h_128.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r02h_131k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-extra --no-kzg --no-cpu-baseline --lat-reps 3 --serial > $O/prof_r02h_131k.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r02h_kzg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --kzg-only --extra-reps 12 > $O/prof_r02h_kzg.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_r02h -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-extra --no-kzg --no-cpu-baseline --lat-reps 0 > $O/pmc_fetch_r02h.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_r02h -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-extra --no-kzg --no-cpu-baseline --lat-reps 0 > $O/pmc_write_r02h.log 2>&1
echo "RC=$?"
