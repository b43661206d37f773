#!/bin/bash
# round 5 (b): the timed schedule (AMG_SCHED_TIMED, bitwise vs the oracle's
# schedule 4) and the timed-model checks of the free races that replace the
# wide oracle bands: single GPU (test_gpu_async, test_gpu_solve), the
# row-partitioned distributed solve (test_gpu_dist), slabs as threads and as
# processes; then the 2-process torchrun bench of the async cycle
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export AMG_SEGV_TRACE=1
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 240 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
run async 400 tests/test_gpu_async.py && \
run solve_band 200 tests/test_gpu_solve.py -k "band" && \
run dist_band 400 tests/test_gpu_dist.py -k "band or accel or schedule" && \
run slab_async 400 tests/test_gpu_slab_async.py && \
run procs 400 tests/test_gpu_slab_async_procs.py || exit $?
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
   --master-port=29611 tools/bench_dist_async.py --size 128 --cycles 8 --runs 2 --transport host --rep 4096 \
   > $O/bench_async_procs.json 2> $O/bench_async_procs.err
rc=$?; echo "bench procs exit $rc"; head -c 800 $O/bench_async_procs.json
exit $rc
