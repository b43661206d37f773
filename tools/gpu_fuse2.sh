# fused residual + restriction variants: parity tests, then the 512^3 bench per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fuse.log 2>&1
st=$?; tail -3 gpurun_out/pytest_fuse.log; [ $st -eq 0 ] || exit $st
AMG_RR_LINES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread -k fused > gpurun_out/pytest_fuse1.log 2>&1
st=$?; tail -3 gpurun_out/pytest_fuse1.log; [ $st -eq 0 ] || exit $st
for v in ${VARS:-1 2}; do
  AMG_RR_LINES=$v timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_rr$v.json 2> gpurun_out/bench_rr$v.log
  st=$?; echo "rr_lines=$v"; tail -2 gpurun_out/bench_rr$v.log; grep -o '"fine_spmv": {[^}]*}' gpurun_out/bench_rr$v.json; [ $st -eq 0 ] || exit $st
done
