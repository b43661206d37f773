#!/bin/bash
# round 5 (q): async Jacobi over 8-slot links (small, accel, 512^3 overlap)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q
mkdir -p $O
export AMG_SEGV_TRACE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -k "async_jacobi or sps" -m "gpu and not slow" -v -s -rf \
   --timeout 150 --timeout-method thread > $O/ajac.log 2>&1; echo "ajac exit $?"; grep -E "passed|failed" $O/ajac.log | tail -2
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -k "async_jacobi_512" -m slow -v -s -rf --timeout 380 \
   --timeout-method thread > $O/ajac512.log 2>&1; echo "ajac512 exit $?"; grep -E "512\^3|passed|failed" $O/ajac512.log | tail -10
