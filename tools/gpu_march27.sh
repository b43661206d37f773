# 27-pt plane march + fused prolongation/post-sweep: march tests, the solve tests,
# the 512^3 bench line, then a rocprofv3 kernel trace of a short bench (step breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_march.log 2>&1
st=$?; tail -3 gpurun_out/pytest_march.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python -u -m pytest tests/test_gpu_solve.py tests/test_gpu_configs.py tests/test_gpu_master.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_solve.log 2>&1
st=$?; tail -3 gpurun_out/pytest_solve.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/bench.json 2> gpurun_out/bench.log
st=$?; tail -8 gpurun_out/bench.log; [ $st -eq 0 ] || exit $st
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run \
   -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P.json 2> $P.err
st=$?; [ $st -eq 0 ] || exit $st
T=$(find $P -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/step_breakdown.py $T > $GRAFT_REPO_ROOT/gpurun_out/step_breakdown.txt
head -60 $GRAFT_REPO_ROOT/gpurun_out/step_breakdown.txt
