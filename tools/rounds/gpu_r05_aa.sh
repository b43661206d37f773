#!/bin/bash
# round 5 (aa): bsr3 blocks per batch (AMG_BSR3_U 9 / 14 / 27): parity, elasticity r = 5 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05aa
mkdir -p $O
for u in 2 3; do
  AMG_BSR3_U=$u timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_classical.py -m "gpu and not slow" \
     -x -q --timeout 200 --timeout-method thread > $O/t$u.log 2>&1; echo "bsr tests U=$u exit $?"; tail -1 $O/t$u.log
done
for u in 4 3 2 4 3 2; do
  AMG_BSR3_U=$u timeout -k 10 300 python -u tools/bench_elasticity.py --refine 5 > $O/e$u.json 2> $O/e$u.err
  echo "U=$u: $(python3 -c "import json; d=json.load(open('$O/e$u.json')); print(round(d['it_per_s'],1), round(d['fine_spmv']['ms']*1e3,1), 'us', round(d['fine_spmv']['frac'],3))")"
done
