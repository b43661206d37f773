#!/bin/bash
# round 5 (ac): 7-pt march occupancy capped by LDS padding (6 -> 5 / 4 / 3 workgroups per CU)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ac
mkdir -p $O
for v in 0 26624 34816 48469 0 26624 34816 48469; do
  AMG_MZ_LDSPAD=$v timeout -k 10 200 python -u bench.py --cpu-baseline 0 --general 0 --steps 40 > $O/b$v.json 2> $O/b$v.err
  echo "pad $v: $(grep -o '"ms_per_step": [0-9.]*' $O/b$v.json) $(grep -o '"iterate_bitwise": [a-z]*' $O/b$v.json) $(grep -E "outer_residual_sweep|post_sweep" $O/b$v.err | tr -s ' ' | cut -c1-48 | tr '\n' ' ')"
done
