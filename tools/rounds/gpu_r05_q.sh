#!/bin/bash
# round 5 (q): async Jacobi over the device-resident links: small cases, accel, and 512^3 at 8 and
# 2 ranks on one GPU (overlap record per rank)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -k "async_jacobi or sps" -m "gpu and not slow" -v -s -rf \
   --timeout 150 --timeout-method thread > $O/ajac.log 2>&1; echo "ajac exit $?"; grep -E "passed|failed" $O/ajac.log | tail -2
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -k "async_jacobi_512" -m slow -v -s -rf --timeout 500 \
   --timeout-method thread > $O/ajac512.log 2>&1; echo "ajac512 exit $?"; grep -E "512\^3|passed|failed" $O/ajac512.log | tail -12
