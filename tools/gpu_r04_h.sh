#!/bin/bash
# level-0 kernel variants, kernel trace of a short 512^3 bench each: the fused
# residual + restriction's z-chunk (AMG_RR_ZC coarse planes; a chunk re-reads
# two fine planes of its neighbours) and the prolongation fused into the
# post-sweep with the coarse correction from an LDS ring (AMG_FUSE_PROLONG 4 /
# 5); first the LDS form's bitwise tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/gpurun_out/r04h
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -k fused_prolong -v -rf --timeout 120 \
   --timeout-method thread > $P/fused_prolong.log 2>&1
st=$?; echo "fused_prolong tests exit $st"; tail -3 $P/fused_prolong.log
case $st in 0|1) ;; *) exit $st;; esac
grep -q "illegal memory access\|Memory access fault" $P/fused_prolong.log && exit 3
cd /tmp && export TMPDIR=/tmp
for v in "AMG_RR_ZC=0" "AMG_FUSE_PROLONG=4" "AMG_FUSE_PROLONG=6" "AMG_FUSE_PROLONG=5" "AMG_FUSE_PROLONG=7" "AMG_RR_ZC=16" "AMG_RR_ZC=32"; do
  name=${v//=/_}
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d $P/$name -o run -- python3 $R/bench.py --steps 6 --warmup 2 --cpu-baseline 0 --spmv-reps 2 \
     > $P/$name.json 2> $P/$name.err
  st=$?; echo "$name exit $st"; [ $st -eq 0 ] || exit $st
  f=$(find $P/$name -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/step_breakdown.py $f > $P/$name.steps.txt && grep -E "step wall|res_restrict|prolong|EpiJacobi, true" $P/$name.steps.txt
done
echo done
