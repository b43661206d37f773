#!/bin/bash
# round 5 (am): the lane-per-block-row 3x3 block kernel (AMG_BSR3=2):
# bitwise tests, then elasticity r = 5 / r = 6 A/B against the default form
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05am
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 200 --timeout-method thread > $O/tbsr.log 2>&1
rc=$?; echo "bsr tests: $(tail -1 $O/tbsr.log)"; [ $rc -eq 0 ] || exit $rc
AMG_BSR3=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_classical.py -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread > $O/tcl.log 2>&1
rc=$?; echo "classical tests (form 2): $(tail -1 $O/tcl.log)"; [ $rc -eq 0 ] || exit $rc
e() { # tag refine env...
  local tag=$1 r=$2; shift 2
  env "$@" timeout -k 10 400 python -u tools/bench_elasticity.py --refine $r > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag exit $rc"; exit $rc; }
  echo "$tag: $(python3 -c "import json; d=json.load(open('$O/$tag.json')); print(round(d['it_per_s'],1), round(d['fine_spmv']['ms']*1e3,1), 'us', round(d['roofline']['frac'],3), d['matrix_format'])")"
}
for i in 1 2 3; do
  e r5_f1_$i 5 AMG_BSR3=1
  e r5_f2_$i 5 AMG_BSR3=2
done
for i in 1 2; do
  e r6_f1_$i 6 AMG_BSR3=1
  e r6_f2_$i 6 AMG_BSR3=2
done
