#!/bin/bash
# round 4: the full GPU test pass (not slow), then config 4 at size (the 512^3
# asynchronous slab solve: 1 rank over RCCL, 2 and 8 ranks over the channels)
set -o pipefail
mkdir -p gpurun_out/r04d
export AMG_LINK_TIMEOUT_S=120 AMG_SEGV_TRACE=1
timeout -k 10 780 python -u -m pytest tests -m "gpu and not slow" -v -rf --timeout 170 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/r04d/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -12 gpurun_out/r04d/pytest_gpu.log | cut -c1-200
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 380 python -u -m pytest tests/test_gpu_slab_async.py -k 512 -v -s --timeout 360 --timeout-method thread \
   > gpurun_out/r04d/slab512.log 2>&1
rc=$?; echo "slab512 exit $rc"; grep -E "512\^3|PASS|FAIL" gpurun_out/r04d/slab512.log | tail -6
exit $rc
