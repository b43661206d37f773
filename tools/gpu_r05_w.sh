#!/bin/bash
# round 5 (w): the update-window test, the async suite, smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py -m "gpu and not slow" -v -s -rf --timeout 200 \
   --timeout-method thread > $O/async.log 2>&1; echo "async exit $?"; grep -E "passed|failed" $O/async.log | tail -1
grep -E "level [0-9]: windows|test_update_windows" $O/async.log | head -12
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo "smoke exit $?"; tail -3 $O/smoke.log
