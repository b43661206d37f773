# fused-kernel occupancy variants after the 32-bit addressing / interior fast path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py tests/test_gpu_master.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_occ.log 2>&1
st=$?; tail -2 gpurun_out/pytest_occ.log; [ $st -eq 0 ] || exit $st
AMG_RR_OCC=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread -k fused > gpurun_out/pytest_occ5.log 2>&1
st=$?; tail -2 gpurun_out/pytest_occ5.log; [ $st -eq 0 ] || exit $st
for v in 0 5; do
  AMG_RR_OCC=$v timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_occ$v.json 2> gpurun_out/bench_occ$v.log
  st=$?; echo "occ=$v"; grep -E 'it/s|ms,' gpurun_out/bench_occ$v.log; [ $st -eq 0 ] || exit $st
done
