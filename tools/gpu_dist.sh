set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py -x -q > gpurun_out/pytest_dist.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_dist.log; tail -30 gpurun_out/pytest_dist.log
[ $st -eq 0 ] || exit $st
timeout -k 10 300 python bench.py --force-dist 1 --steps 10 --warmup 2 > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.log
st=$?; tail -5 gpurun_out/bench_dist1.log; cat gpurun_out/bench_dist1.json; exit $st
