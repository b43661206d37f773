# run the given GPU test files (default: all) verbosely with per-test timeouts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FILES=${FILES:-tests}
timeout -k 10 1000 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
st=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_sel.log | tail -5; tail -3 gpurun_out/pytest_sel.log; exit $st
