set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_gpu.log; tail -25 gpurun_out/pytest_gpu.log
[ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_vi.json 2> gpurun_out/bench_vi.log
st=$?; tail -4 gpurun_out/bench_vi.log; cat gpurun_out/bench_vi.json; [ $st -eq 0 ] || exit $st
AMG_VALUE_INDEX=0 timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.log
st=$?; tail -4 gpurun_out/bench_plain.log; exit $st
