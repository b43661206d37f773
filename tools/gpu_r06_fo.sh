# fused post sweep + outer residual (mz_sweep_outer_kernel) with the exact
# reciprocal division and operands one / two planes ahead: its bitwise tests
# under both prefetch depths, then the headline A/B
set -o pipefail
O=${1:-gpurun_out/r06/fo}
mkdir -p $O
for pd in 1 2; do
AMG_FUSE_OUTER_PD=$pd timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread -k "fused_sweep_outer or slab_sweep_outer" > $O/tests_pd$pd.log 2>&1 || { echo tests pd=$pd failed; tail -30 $O/tests_pd$pd.log; exit 1; }
tail -1 $O/tests_pd$pd.log
done
bash tools/gpu_r06_ab.sh $O/ab - "AMG_FUSE_OUTER=2" "AMG_FUSE_OUTER=2 AMG_FUSE_OUTER_PD=2"
