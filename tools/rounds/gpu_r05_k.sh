#!/bin/bash
# round 5 (k): config 5's asynchronous additive cycle at size -- the r = 6
# elasticity hierarchy (6.5M DoF, classical DMEM parameters) as 8 and 4
# row-partitioned ranks on one GPU (bench_elasticity --async-ranks)
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export AMG_SEGV_TRACE=1
for R in 8 4; do
  timeout -k 10 540 python -u tools/bench_elasticity.py --refine 6 --steps 5 --warmup 1 --async-ranks $R \
     --async-cycles 10 > $O/elast6_async$R.json 2> $O/elast6_async$R.err
  rc=$?; echo "elast r6 async $R ranks exit $rc"; grep -E "elast async|relres" $O/elast6_async$R.err | tail -4
  [ $rc -eq 0 ] || exit $rc
done
