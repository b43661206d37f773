#!/bin/bash
# round 5 (i): the replay checks with torn-update detection (slab threads and
# processes, row-partitioned, elasticity), and the fused post-sweep +
# outer-residual march at 1 and 2 workgroups per CU; the LDS-tile hybrid JGS
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
export AMG_SEGV_TRACE=1
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 240 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
run jgs 300 tests/test_gpu_kernels.py -k hybrid_jgs
for w in 1 3; do
  AMG_JGS_WAVE=$w timeout -k 10 300 python -u tools/bench_async.py --transfers composed > $O/async3_jgs$w.json 2> $O/async3_jgs$w.err
  echo "config 3 jgs_wave $w exit $?: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_jgs$w.json | tr '\n' ' ')"
done
AMG_JGS_WAVE=3 run async_jgs3 400 tests/test_gpu_async.py tests/test_gpu_configs.py -k "hybrid or async"
run slab_async 400 tests/test_gpu_slab_async.py
run procs 400 tests/test_gpu_slab_async_procs.py
run dist_band 400 tests/test_gpu_dist.py -k "band or accel"
run elast 400 tests/test_gpu_elast_async.py
grep -hE "run [0-9]: device" $O/*.log | sed 's/^ *//' > $O/replay_summary.txt
