# quick iteration: the given pytest selection, the SpMV tuning table, then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 600 python -u -m pytest $SEL -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_iter.log; tail -15 gpurun_out/pytest_iter.log
[ $st -eq 0 ] || exit $st
if [ -n "$2" ]; then
timeout -k 10 300 python tools/tune_spmv.py 512 5 $2 > gpurun_out/tune_iter.log 2>&1 || exit $?
cat gpurun_out/tune_iter.log
fi
timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.log
st=$?; tail -4 gpurun_out/bench_iter.log; cat gpurun_out/bench_iter.json; exit $st
