#!/bin/bash
# round 4: row-form async schedules bitwise + the widened bands; the sync slab
# file (zero-guess fold off, the default); the LDS-ring fused prolongation tests and
# the level-0 variants under a kernel trace (tools/gpu_r04_h.sh); last (fold
# on) the first two slab cases with kernels serialised so a fault names its launch
set -o pipefail
mkdir -p gpurun_out/r04g
export AMG_LINK_TIMEOUT_S=120 AMG_SEGV_TRACE=1
run() { # name timeout args...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -v -s -rf --timeout 170 --timeout-method thread > gpurun_out/r04g/$name.log 2>&1
   local rc=$?
   echo "$name exit $rc"; grep -E "passed|failed" gpurun_out/r04g/$name.log | tail -1
   case $rc in 0|1) ;; *) echo "stopping after $name"; exit $rc;; esac
   if grep -q "illegal memory access\|Memory access fault" gpurun_out/r04g/$name.log; then echo "GPU fault in $name: stopping"; exit 3; fi
   return 0
}
run dist 400 tests/test_gpu_dist.py -k "async_band or schedule_bitwise"
run grid 300 tests/test_gpu_grid.py -k converges
run slab_nofold 420 -p no:faulthandler tests/test_gpu_slab.py -k "not 512"
./tools/gpu_r04_h.sh || exit $?
AMG_ZG_FOLD_SLAB=1 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 run slab_serial 300 -p no:faulthandler tests/test_gpu_slab.py -k "dims0 or dims1" -x
echo done
