#!/bin/bash
# round 4 final tree: the slow GPU tests the driver's round-end pass includes
# (512^3 sync slab at 1 / 2 / 8 ranks after the slab_vcycle fix, elasticity at
# size), then the interleaved A/B of the 7-pt march defaults (tools/gpu_r04_o.sh)
set -o pipefail
mkdir -p gpurun_out/r04p
export AMG_SEGV_TRACE=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_classical.py -m "gpu and slow" -v -s -rf \
   --timeout 330 --timeout-method thread > gpurun_out/r04p/slow.log 2>&1
rc=$?; echo "slow exit $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04p/slow.log | tail -6 | cut -c1-160
case $rc in 0|1) ;; *) exit $rc;; esac
./tools/gpu_r04_o.sh
