#!/bin/bash
# round 5 (c): batch (b)'s async tests (replay checks), then the bench with the
# new legs (vcycle_general_csr, the config-1 SEQ leg, host info)
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export AMG_SEGV_TRACE=1
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 240 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
run dist_band 400 tests/test_gpu_dist.py -k "band or accel or schedule"
run slab_async 400 tests/test_gpu_slab_async.py
run procs 400 tests/test_gpu_slab_async_procs.py
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; tail -12 $O/bench.err
exit $rc
