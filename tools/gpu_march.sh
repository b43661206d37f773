# plane-marching kernel: parity tests, then the 512^3 bench at several chunk lengths
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py tests/test_gpu_master.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_march.log 2>&1
st=$?; tail -5 gpurun_out/pytest_march.log; [ $st -eq 0 ] || exit $st
for z in ${ZCS:-32 16 64}; do
  AMG_PLANE_MARCH=$z timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_z$z.json 2> gpurun_out/bench_z$z.log
  st=$?; echo "zc=$z"; tail -6 gpurun_out/bench_z$z.log; [ $st -eq 0 ] || exit $st
done
AMG_PLANE_MARCH_XCD=0 timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_x0.json 2> gpurun_out/bench_x0.log
st=$?; echo "xcd=0"; tail -6 gpurun_out/bench_x0.log; exit $st
