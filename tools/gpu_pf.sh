# plane-ahead prefetch A/B: fused residual + restriction (AMG_RR_PF 0 / 1 occ-4 / 2 occ-3)
# and the 7-pt march (AMG_MZ_PF)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AMG_MZ_PF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mzpf.log 2>&1
st=$?; echo "MZ_PF=1 march tests:"; tail -1 gpurun_out/pytest_mzpf.log; [ $st -eq 0 ] || exit $st
VAR=AMG_RR_PF VALS="0 2 1 0 2 1" bash tools/gpu_ab.sh || exit $?
i=0
for V in 0 1 0 1; do
  i=$((i+1))
  AMG_MZ_PF=$V timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_mz${i}_$V.json 2> gpurun_out/bench_mz${i}_$V.log
  st=$?; echo "AMG_MZ_PF=$V"; grep -E "steps in|residual_restrict|post_sweep|outer" gpurun_out/bench_mz${i}_$V.log; [ $st -eq 0 ] || exit $st
done
