#!/bin/bash
# 7-pt march variants on the final tree (kernel trace of a short 512^3 bench
# each): prefetch distance 2 (AMG_MZ_PF), occupancy-sized chunks (AMG_MZ_OCC),
# both; the default alongside
set -o pipefail
R=$(pwd)
P=$R/gpurun_out/r04m
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for v in "AMG_MZ_PF=1" "AMG_MZ_PF=2" "AMG_MZ_OCC=-1" "AMG_MZ_PF=2 AMG_MZ_OCC=-1"; do
  name=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d $P/$name -o run -- python3 $R/bench.py --steps 6 --warmup 2 --cpu-baseline 0 --spmv-reps 2 \
     > $P/$name.json 2> $P/$name.err
  st=$?; echo "$name exit $st"; [ $st -eq 0 ] || exit $st
  f=$(find $P/$name -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/step_breakdown.py $f > $P/$name.steps.txt && grep -E "step wall|EpiResJacobi|EpiJacobi, true, 1" $P/$name.steps.txt | head -4
done
echo done
