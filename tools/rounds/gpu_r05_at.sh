#!/bin/bash
# round 5 (at): blocks per batch of the lane-per-block-row 3x3 kernel
# (AMG_BSR3_RU 2 / 4 / 6 / 8): bitwise tests, elasticity r = 6 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05at
mkdir -p $O
for u in 2 6 8; do
  AMG_BSR3_RU=$u timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 200 --timeout-method thread > $O/t$u.log 2>&1
  rc=$?; echo "bsr tests RU=$u: $(tail -1 $O/t$u.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for u in 4 2 6 8; do
    AMG_BSR3_RU=$u timeout -k 10 400 python -u tools/bench_elasticity.py --refine 6 > $O/e${u}_$i.json 2> $O/e${u}_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "elast RU $u exit $rc"; exit $rc; }
    echo "RU $u: $(python3 -c "import json; d=json.load(open('$O/e${u}_$i.json')); print(round(d['it_per_s'],2), round(d['fine_spmv']['ms']*1e3,1), 'us', round(d['roofline']['frac'],3))")"
  done
done
