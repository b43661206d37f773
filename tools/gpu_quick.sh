set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_gpu.log; tail -25 gpurun_out/pytest_gpu.log
[ $st -eq 0 ] || exit $st
timeout -k 10 400 python bench.py --cpu-baseline 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.log
st=$?; tail -6 gpurun_out/bench_quick.log; cat gpurun_out/bench_quick.json; exit $st
