# round 2: distributed tests (serialised RCCL exchange), 1-rank RCCL bench, default bench with CPU leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
st=$?; tail -3 gpurun_out/pytest_dist.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py --force-dist 1 --cpu-baseline 0 > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.log
st=$?; tail -3 gpurun_out/bench_dist1.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log
st=$?; tail -12 gpurun_out/bench_full.log; exit $st
