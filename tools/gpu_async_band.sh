#!/bin/bash
# asynchronous solves against the oracle's asynchronous band (SMEM_Async_Add_AMG on OpenMP threads)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=gpurun_out/band
mkdir -p $P
timeout -k 10 1100 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_solve.py tests/test_gpu_dist.py \
   tests/test_gpu_configs.py -k "async or band or config3" -v -s --timeout 600 --timeout-method thread > $P/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "band|PASS|FAIL|passed|failed" $P/pytest.log | tail -40
exit $rc
