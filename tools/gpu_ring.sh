# LDS-ring residual + restriction: march tests, bench with ring off / on, then elasticity r = 5, 6
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_march.log 2>&1
st=$?; tail -2 gpurun_out/pytest_march.log; [ $st -eq 0 ] || exit $st
for V in 0 1 0 1; do
  AMG_RR_RING=$V timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_ring$V.json 2> gpurun_out/bench_ring$V.log
  st=$?; echo "ring=$V"; grep -E "steps in|residual_restrict" gpurun_out/bench_ring$V.log; [ $st -eq 0 ] || exit $st
done
RS="5 6" bash tools/gpu_elast.sh
