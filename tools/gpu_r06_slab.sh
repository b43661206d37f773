# fuse_outer 3 (slab-blocked post sweep + outer residual): its bitwise tests,
# then the interleaved bench A/B over slab sizes (tools/gpu_r06_ab.sh)
set -o pipefail
O=${1:-gpurun_out/r06/slab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -x -v --timeout 120 --timeout-method thread -k "slab_sweep_outer or fused_sweep_outer" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
shift
bash tools/gpu_r06_ab.sh $O/ab "$@"
