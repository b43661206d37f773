#!/bin/bash
# round 5 (z): the slow GPU tests on the final tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05z
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/ -m "gpu and slow" -v -s -rf --timeout 500 --timeout-method thread \
   > $O/slow.log 2>&1; echo "slow exit $?"; grep -E "PASSED|FAILED|passed|failed" $O/slow.log | tail -8
