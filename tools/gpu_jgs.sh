# hybrid JGS kernel change: kernel / solve / config tests, then config-3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solve.py tests/test_gpu_async.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_jgs.log 2>&1
st=$?; tail -3 gpurun_out/pytest_jgs.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python tools/bench_async.py > gpurun_out/bench_async.json 2> gpurun_out/bench_async.log
st=$?; cat gpurun_out/bench_async.log; exit $st
