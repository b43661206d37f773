cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
grep -i "TCC_EA0_RD\|TCC_BUBBLE\|TCC_EA0_WR\|FETCH_SIZE\|WRITE_SIZE\|TCC_REQ\|TCC_READ\b" $GRAFT_REPO_ROOT/gpurun_out/counters.txt | head -40
