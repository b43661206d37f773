#!/bin/bash
# round 5 (aj): the halo-ahead march with the right-hand side ahead too
# (AMG_MZ_HPF=3: one plane, 90 VGPRs; 4: two planes, 105 VGPRs or 96 at
# AMG_MZ_WPE=5) against the default, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05aj
mkdir -p $O
for h in 3 4; do
  AMG_MZ_PF=3 AMG_MZ_HPF=$h timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -x -q --timeout 120 --timeout-method thread -k "march_tuning_bitwise" > $O/tests_h$h.log 2>&1
  rc=$?; tail -1 $O/tests_h$h.log; [ $rc -eq 0 ] || exit $rc
done
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --cpu-baseline 0 --general 0 > $O/bench_$tag.json 2> $O/bench_$tag.err
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $tag exit $rc"; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); fk=d['fine_kernels']; print('$tag', round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms'],3) for k,v in fk.items()})"
}
for i in 1 2; do
  run base$i AMG_MZ_PF=1
  run h3_$i AMG_MZ_PF=3 AMG_MZ_HPF=3
  run h4_$i AMG_MZ_PF=3 AMG_MZ_HPF=4
  run h4w5_$i AMG_MZ_PF=3 AMG_MZ_HPF=4 AMG_MZ_WPE=5
done
