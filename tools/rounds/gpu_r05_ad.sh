#!/bin/bash
# round 5 (ad): hybrid JGS grp kernel at 4 / 6 / 8 waves per SIMD (AMG_JGS_WPE): parity, config 3 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ad
mkdir -p $O
for w in 6 8; do
  AMG_JGS_WPE=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k hybrid_jgs -m "gpu and not slow" -x -q \
     --timeout 200 --timeout-method thread > $O/t$w.log 2>&1; echo "jgs tests WPE=$w exit $?"; tail -1 $O/t$w.log
done
for w in 0 6 8 0 6 8; do
  AMG_JGS_WPE=$w timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 > $O/a$w.json 2> $O/a$w.err
  echo "WPE $w: $(grep -o '"cycles_per_s": [0-9.]*' $O/a$w.json | tr '\n' ' ')"
done
