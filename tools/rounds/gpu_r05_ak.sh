#!/bin/bash
# round 5 (ak): the fused level-0 residual + restriction with its right-hand
# side a fine plane ahead (AMG_RR_FPF=1: held to 4 waves per SIMD, 3: 136
# VGPRs at 3 waves) and compiled for 5 waves (AMG_RR_OCC=5), bitwise tests
# then an interleaved bench A/B against the default
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ak
mkdir -p $O
for v in "AMG_RR_FPF=1" "AMG_RR_FPF=3" "AMG_RR_OCC=5"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread -k "fused_residual_restrict" > $O/tests_${v}.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_${v}.log)"; [ $rc -eq 0 ] || exit $rc
done
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --cpu-baseline 0 --general 0 > $O/bench_$tag.json 2> $O/bench_$tag.err
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $tag exit $rc"; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); fk=d['fine_kernels']; print('$tag', round(d['value'],1), round(d['ms_per_step'],4), d['parity'].get('iterate_bitwise'), {k: round(v['ms'],3) for k,v in fk.items()})"
}
for i in 1 2; do
  run base$i AMG_RR_FPF=0
  run fpf1_$i AMG_RR_FPF=1
  run fpf3_$i AMG_RR_FPF=3
  run occ5_$i AMG_RR_OCC=5
done
