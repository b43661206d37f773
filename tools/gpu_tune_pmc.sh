# FETCH_SIZE per tuning variant (A0 512^3) -- is the x gather re-read from beyond L2?
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/tunepmc
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P -o run \
   -- python3 $R/tools/tune_spmv.py 512 1 > $P/tune.log 2>&1 || exit $?
echo ok
