# asynchronous additive options (single GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_solve.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_async.log 2>&1
st=$?; grep -E 'PASS|FAIL|Error|passed|failed' gpurun_out/pytest_async.log | tail -25; exit $st
