#!/bin/bash
# round 5 (aq): the halo-ahead march for the SpMV's two-lines-per-lane form
# (the metric's fine SpMV): bitwise tuning tests, then the bench's fine_spmv
# interleaved -- AMG_MZ_PF=1 (no halo-ahead), 3 (halo-ahead, two lines), 3 with
# one line per lane for the SpMV (AMG_MZ_LINES_GEMV=1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05aq
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --cpu-baseline 0 --general 0 > $O/bench_$tag.json 2> $O/bench_$tag.err
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $tag exit $rc"; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); s=d['fine_spmv']; print('$tag', round(d['value'],1), 'spmv', round(s['ms'],4), 'ms', round(s['frac'],4))"
}
for i in 1 2; do
  run pf1_$i AMG_MZ_PF=1
  run pf3_$i AMG_MZ_PF=3
  run pf3l1_$i AMG_MZ_PF=3 AMG_MZ_LINES_GEMV=1
done
