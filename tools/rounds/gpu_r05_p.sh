#!/bin/bash
# round 5 (p): async Jacobi over links after the send/receive deadlock fix
# (small cases, accel, and 512^3 with its overlap record), the distributed
# replay checks, config 3 with / without the folded level-0 correction
# (cheap stamps), the fused outer march at 1 / 2 workgroups per CU, bsr3 x sharing
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05p
mkdir -p $O
export AMG_SEGV_TRACE=1
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 150 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
run dist 500 tests/test_gpu_dist.py -k "async_jacobi or sps or band or accel" || exit 1
for v in 1 0 1 0; do
  AMG_JGS_FOLD=$v timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 \
     > $O/async3_fold$v.json 2> $O/async3_fold$v.err
  echo "config 3 fold $v: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_fold$v.json | tr '\n' ' ')"
done
AMG_JGS_WAVE=3 AMG_JGS_TILE_OCC=4 timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 \
   > $O/async3_tile.json 2> $O/async3_tile.err
echo "config 3 tile: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_tile.json | tr '\n' ' ')"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -k "async_jacobi_512" -m slow -v -s -rf --timeout 380 \
   --timeout-method thread > $O/ajac512.log 2>&1; echo "ajac512 exit $?"; grep -E "512\^3|passed|failed" $O/ajac512.log | tail -6
for occ in 1 2; do
  AMG_FUSE_OUTER_OCC=$occ timeout -k 10 200 python -u bench.py --fuse-outer 2 --cpu-baseline 0 --general 0 \
     > $O/fo2_occ$occ.json 2> $O/fo2_occ$occ.err
  echo "fuse_outer 2 occ $occ exit $?: $(grep -o '"ms_per_step": [0-9.]*' $O/fo2_occ$occ.json)"
done
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --general 0 > $O/fo0.json 2> $O/fo0.err
echo "fuse_outer 0: $(grep -o '"ms_per_step": [0-9.]*' $O/fo0.json)"
for xs in 1 0; do
  AMG_BSR3_XS=$xs timeout -k 10 300 python -u tools/bench_elasticity.py --refine 5 > $O/elast5_xs$xs.json 2> $O/elast5_xs$xs.err
  echo "elast r5 xs=$xs exit $?: $(python3 -c "import json; d=json.load(open('$O/elast5_xs$xs.json')); print(d.get('it_per_s'), d.get('fine_spmv'))" 2>&1 | tail -1)"
done
