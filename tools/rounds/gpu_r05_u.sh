#!/bin/bash
# round 5 (u): the whole GPU suite (not slow) on the current tree, file by file
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05u
mkdir -p $O
export AMG_SEGV_TRACE=1
fail=0
for f in tests/test_gpu_*.py; do
  n=$(basename $f .py)
  timeout -k 10 600 python -u -m pytest $f -m "gpu and not slow" -q -rf --timeout 200 --timeout-method thread \
     > $O/$n.log 2>&1
  rc=$?
  echo "$n exit $rc: $(grep -E "passed|failed|error" $O/$n.log | tail -1)"
  case $rc in 0|1) ;; *) echo "stopping: $n exit $rc"; exit $rc;; esac
  [ $rc -eq 1 ] && fail=1
done
exit $fail
