#!/bin/bash
# round 4, second pass: link event fix (slab async), GLOBAL-residual sequential
# schedules, the coupling child under a kernel trace (queue ids), the slab
# teardown fault with the native backtrace, then the 27-pt march variants
set -o pipefail
mkdir -p gpurun_out/r04c
export AMG_LINK_TIMEOUT_S=60
run() { # name timeout args...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -v -s --timeout 170 --timeout-method thread > gpurun_out/r04c/$name.log 2>&1
   local rc=$?
   echo "$name exit $rc"
   case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
   return 0
}
run slab_async 600 tests/test_gpu_slab_async.py -k "not 512"
run async_gres 300 tests/test_gpu_async.py -k "schedule_bitwise and global-local"
cd /tmp && export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04c/coupling -o run \
   -- python3 $GRAFT_REPO_ROOT/tests/test_gpu_delay.py coupling 1 > $GRAFT_REPO_ROOT/gpurun_out/r04c/coupling1.log 2>&1
rc=$?; echo "coupling trace exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
cd $GRAFT_REPO_ROOT
export AMG_SEGV_TRACE=1
run slab_dims3 300 tests/test_gpu_slab.py -k "test_slab_matches_single_gpu and dims3"
run coupling 400 tests/test_gpu_delay.py -k coupling
./tools/gpu_mz27.sh || exit $?
echo done
