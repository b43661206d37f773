#!/bin/bash
# the round-end GPU test tier alone (flakiness check of the async bands)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=gpurun_out/tests_only
mkdir -p $P
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 400 --timeout-method thread > $P/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> $P/pytest_gpu.log; tail -5 $P/pytest_gpu.log; exit $st
