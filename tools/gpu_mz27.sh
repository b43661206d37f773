#!/bin/bash
# march-kernel variants: 27-pt prefetch distance (AMG_MZ27_PF), occupancy-sized
# chunks (AMG_MZ27_OCC / AMG_MZ_OCC: 0 off, -1 the kernel's own occupancy):
# kernel trace of a short 512^3 bench per variant, the step's per-kernel
# timeline (tools/step_breakdown.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/mz27
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for v in "1 0 0" "2 0 0" "2 -1 0" "2 -1 -1"; do
  set -- $v
  name=pf$1_occ27$2_occ7$3
  AMG_MZ27_PF=$1 AMG_MZ27_OCC=$2 AMG_MZ_OCC=$3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d $P/$name -o run -- python3 $R/bench.py --steps 6 --warmup 2 --cpu-baseline 0 --spmv-reps 2 \
     > $P/$name.json 2> $P/$name.err
  st=$?; echo "$name exit $st"; [ $st -eq 0 ] || exit $st
  f=$(find $P/$name -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/step_breakdown.py $f > $P/$name.steps.txt && grep -E "step wall|mz27|res_restrict|csr_mz_kernel" $P/$name.steps.txt
done
