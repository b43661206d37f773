set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pv
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pv/fetch -o run -- python3 tools/pmc_variant.py "$1" > gpurun_out/pv/fetch.log 2>&1
st=$?; tail -3 gpurun_out/pv/fetch.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pv/hit -o run -- python3 tools/pmc_variant.py "$1" > gpurun_out/pv/hit.log 2>&1
st=$?; tail -3 gpurun_out/pv/hit.log; exit $st
