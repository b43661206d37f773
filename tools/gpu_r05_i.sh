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
run slab_async 400 tests/test_gpu_slab_async.py
run procs 400 tests/test_gpu_slab_async_procs.py
run dist_band 400 tests/test_gpu_dist.py -k "band or accel"
run elast 400 tests/test_gpu_elast_async.py
grep -hE "run [0-9]: device" $O/*.log | sed 's/^ *//' > $O/replay_summary.txt
for occ in 1 2; do
  AMG_FUSE_OUTER_OCC=$occ timeout -k 10 200 python -u bench.py --fuse-outer 2 --cpu-baseline 0 --general 0 \
     > $O/fo2_occ$occ.json 2> $O/fo2_occ$occ.err
  echo "fuse_outer 2 occ $occ exit $?: $(grep -o '"ms_per_step": [0-9.]*' $O/fo2_occ$occ.json)"; grep -E "post_sweep_outer" $O/fo2_occ$occ.err
done
run ajac 300 tests/test_gpu_dist.py -k "async_jacobi or sps"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -k "async_jacobi_512" -m slow -v -s -rf --timeout 560 \
   --timeout-method thread > $O/ajac512.log 2>&1; echo "ajac512 exit $?"; grep -E "512\^3 async|passed|failed" $O/ajac512.log | tail -10
run bsr 200 tests/test_gpu_bsr.py tests/test_gpu_classical.py -k "bsr or elasticity_solve"
for xs in 1 0; do
  AMG_BSR3_XS=$xs timeout -k 10 300 python -u tools/bench_elasticity.py --refine 5 > $O/elast5_xs$xs.json 2> $O/elast5_xs$xs.err
  echo "elast r5 xs=$xs exit $?: $(python3 -c "import json,sys; d=json.load(open('$O/elast5_xs$xs.json')); print(d['it_per_s'], d['fine_spmv'])" 2>&1 | tail -1)"
done
