#!/bin/bash
# round 5 (ab): 7-pt march at 8 waves per SIMD (AMG_MZ_WPE=8): parity, interleaved bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ab
mkdir -p $O
AMG_MZ_WPE=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py tests/test_gpu_solve.py -m "gpu and not slow" -x -q \
   --timeout 200 --timeout-method thread > $O/t.log 2>&1; echo "tests WPE=8 exit $?"; tail -1 $O/t.log
for v in 8 0 8 0 8 0; do
  AMG_MZ_WPE=$v timeout -k 10 200 python -u bench.py --cpu-baseline 0 --general 0 --steps 40 > $O/b$v.json 2> $O/b$v.err
  echo "WPE $v: $(grep -o '"ms_per_step": [0-9.]*' $O/b$v.json) $(grep -E "outer_residual_sweep|post_sweep" $O/b$v.err | tr -s ' ' | cut -c1-60 | tr '\n' ' ')"
done
