#!/bin/bash
# round 5 (d): the free-race checks against the oracle's replays (timed
# schedule with the recorded end times; the sliced replay of distributed runs)
set -o pipefail
O=gpurun_out/r05d
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
run async 300 tests/test_gpu_async.py -k "band or replay"
grep -hE "run [0-9]: device" $O/*.log | sed 's/^ *//' > $O/replay_summary.txt
wc -l $O/replay_summary.txt
