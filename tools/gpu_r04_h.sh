#!/bin/bash
# fused residual + restriction chunking (AMG_RR_ZC coarse planes per chunk;
# a chunk re-reads two fine planes of its neighbours) and lines per lane
# (AMG_RR_LINES): kernel trace of a short 512^3 bench per variant
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/r04h
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for v in "0 1" "16 1" "32 1" "16 2"; do
  set -- $v
  name=rrzc$1_lines$2
  AMG_RR_ZC=$1 AMG_RR_LINES=$2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d $P/$name -o run -- python3 $R/bench.py --steps 6 --warmup 2 --cpu-baseline 0 --spmv-reps 2 \
     > $P/$name.json 2> $P/$name.err
  st=$?; echo "$name exit $st"; [ $st -eq 0 ] || exit $st
  f=$(find $P/$name -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/step_breakdown.py $f > $P/$name.steps.txt && grep -E "step wall|res_restrict" $P/$name.steps.txt
done
echo done
