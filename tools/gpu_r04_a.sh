#!/bin/bash
# round 4: schedule-mode parity (single GPU, slab, grid), composed transfers,
# slab fold, per-level channels, coupling
set -o pipefail
mkdir -p gpurun_out/r04a
export AMG_LINK_TIMEOUT_S=60
run() { # name timeout args...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -v -s --timeout 170 --timeout-method thread > gpurun_out/r04a/$name.log 2>&1
   local rc=$?
   echo "$name exit $rc"
   # a fault, abort, segfault or time limit: nothing more on the GPU
   case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
   return 0
}
run slab_async 900 tests/test_gpu_slab_async.py -k "not 512"
run async 900 tests/test_gpu_async.py -k "global or composed"
run grid 600 tests/test_gpu_grid.py
run delay 600 tests/test_gpu_delay.py
run slab 900 tests/test_gpu_slab.py -k "not 512"
echo done
