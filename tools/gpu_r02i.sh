cd /tmp
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS -d $O/pmc_sq_r02i_128 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stage_small.py 128 > $O/pmc_sq_r02i_128.log 2>&1
echo "RC=$?"
