# round-2 re-entry check: GPU tests (verbose, per-test timeout), smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
st=$?; tail -2 gpurun_out/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log
st=$?; tail -4 gpurun_out/bench_full.log; cat gpurun_out/bench_full.json; exit $st
