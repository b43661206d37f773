# A/B of one environment knob: the fused residual + restriction tests and the
# 512^3 bench (no CPU leg) per value, interleaved.  VAR=name VALS="0 1 0 1"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=${VAR:-AMG_RR_PF}
VALS=${VALS:-"0 1 0 1"}
for V in $(echo $VALS | tr ' ' '\n' | sort -u); do
  env $VAR=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread -k "fused_residual_restrict or hierarchy" > gpurun_out/pytest_ab$V.log 2>&1
  st=$?; echo "$VAR=$V tests:"; tail -1 gpurun_out/pytest_ab$V.log; [ $st -eq 0 ] || exit $st
done
i=0
for V in $VALS; do
  i=$((i+1))
  env $VAR=$V timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_ab${i}_$V.json 2> gpurun_out/bench_ab${i}_$V.log
  st=$?; echo "$VAR=$V"; grep -E "steps in|residual_restrict|post_sweep" gpurun_out/bench_ab${i}_$V.log; [ $st -eq 0 ] || exit $st
done
