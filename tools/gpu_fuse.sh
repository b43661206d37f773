# fused residual + restriction: parity tests, then the 512^3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fuse.log 2>&1
st=$?; tail -5 gpurun_out/pytest_fuse.log; [ $st -eq 0 ] || exit $st
for z in ${ZCS:-16}; do
  AMG_PLANE_MARCH=$z timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_f$z.json 2> gpurun_out/bench_f$z.log
  st=$?; echo "zc=$z"; tail -6 gpurun_out/bench_f$z.log; [ $st -eq 0 ] || exit $st
done
