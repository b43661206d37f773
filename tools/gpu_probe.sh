set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 ./tools/_stencil_probe > gpurun_out/stencil_probe.log 2>&1; st=$?; cat gpurun_out/stencil_probe.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
st=$?; tail -2 gpurun_out/pytest_dist.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python bench.py --force-dist 1 --steps 20 --warmup 3 > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.log
st=$?; grep "steps in" gpurun_out/bench_dist1.log; exit $st
