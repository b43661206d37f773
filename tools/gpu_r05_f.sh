#!/bin/bash
# round 5 (f): the fused post-sweep + outer-residual march (bitwise tests, then
# an interleaved bench A/B of fuse_outer 0 / 1 / 2), the race probe and the
# elasticity async tests
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
export AMG_SEGV_TRACE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -k "fused_sweep_outer" -v -s -rf --timeout 200 \
   --timeout-method thread > $O/fused_outer.log 2>&1
rc=$?; echo "fused_outer tests exit $rc"; grep -E "passed|failed" $O/fused_outer.log | tail -2
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in 0 2 1; do
    timeout -k 10 200 python -u bench.py --fuse-outer $m --cpu-baseline 0 --general 0 > $O/ab_m${m}_r${rep}.json \
       2> $O/ab_m${m}_r${rep}.err
    rc=$?; echo "bench fuse_outer=$m rep $rep exit $rc: $(grep -o '"ms_per_step": [0-9.]*' $O/ab_m${m}_r${rep}.json)"
    grep -E "post_sweep|outer" $O/ab_m${m}_r${rep}.err | head -3
    [ $rc -eq 0 ] || exit $rc
  done
done
bash tools/gpu_r05_e.sh
