#!/bin/bash
# round 5 (an): the lane-per-block-row 3x3 block kernel as the default --
# the GPU files that register elasticity operators, then config 5 at r = 5 / 6
# (sync V-cycle with the bsr3 roofline) and r = 6 asynchronous at 8 ranks
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05an
mkdir -p $O
export AMG_SEGV_TRACE=1
for f in test_gpu_bsr test_gpu_classical test_gpu_elast_async test_gpu_sps; do
  timeout -k 10 400 python -u -m pytest tests/$f.py -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread > $O/$f.log 2>&1
  rc=$?; echo "$f: $(tail -1 $O/$f.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 5 6; do
  timeout -k 10 400 python -u tools/bench_elasticity.py --refine $r > $O/elast$r.json 2> $O/elast$r.err
  rc=$?; [ $rc -eq 0 ] || { echo "elast $r exit $rc"; exit $rc; }
  echo "r=$r: $(python3 -c "import json; d=json.load(open('$O/elast$r.json')); print(round(d['it_per_s'],1), round(d['fine_spmv']['ms']*1e3,1), 'us', round(d['roofline']['frac'],3), d['matrix_format'])")"
done
timeout -k 10 540 python -u tools/bench_elasticity.py --refine 6 --steps 5 --warmup 1 --async-ranks 8 \
   --async-cycles 10 > $O/elast6_async8.json 2> $O/elast6_async8.err
rc=$?; echo "elast r6 async 8 ranks exit $rc"; grep -E "elast async|relres" $O/elast6_async8.err | tail -3
exit $rc
