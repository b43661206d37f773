#!/bin/bash
# round 5 (t): div_rcp on level 0 and the 27-pt levels: parity + interleaved A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_march.py tests/test_gpu_solve.py tests/test_gpu_classical.py \
   -m "gpu and not slow" -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; echo "tests exit $?"; tail -2 $O/tests.log
for v in 1 0 1 0 1 0; do
  AMG_FAST_DIV=$v timeout -k 10 200 python -u bench.py --cpu-baseline 0 --general 0 --steps 40 > $O/b$v.json 2> $O/b$v.err
  echo "fast_div $v: $(grep -o '"ms_per_step": [0-9.]*' $O/b$v.json) $(grep -o '"iterate_bitwise": [a-z]*' $O/b$v.json)"
done
