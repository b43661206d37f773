#!/bin/bash
# round 5 (j): the fused post-sweep + outer-residual march at 1 and 2 workgroups
# per CU, the async Jacobi (links, overlap) small and at 512^3, the bsr3 x-sharing A/B
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
export AMG_SEGV_TRACE=1
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 240 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
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
