#!/bin/bash
# round 4: numbers for the failing bands (dist async, grid), the sync slab
# teardown fault in a fresh process with the native backtrace (faulthandler
# off so the library's handler prints), then the remaining test files
set -o pipefail
mkdir -p gpurun_out/r04f
export AMG_LINK_TIMEOUT_S=120 AMG_SEGV_TRACE=1
run() { # name timeout args...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -v -s -rf --timeout 170 --timeout-method thread > gpurun_out/r04f/$name.log 2>&1
   local rc=$?
   echo "$name exit $rc"
   case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
   return 0
}
run slab 420 -p no:faulthandler tests/test_gpu_slab.py -k "not 512"
run dist_band 300 tests/test_gpu_dist.py -k "async_band or async_additive"
run grid 300 tests/test_gpu_grid.py tests/test_gpu_grid_ipc.py
run slab_async 300 tests/test_gpu_slab_async.py -k "not 512"
run late 400 tests/test_gpu_solve.py tests/test_gpu_sps.py tests/test_gpu_tuning.py tests/test_gpu_configs.py
echo done
