# 27-pt LDS plane ring (AMG_MZ27_PF=3): its bitwise tests, then the headline
# bench A/B against the register march (tools/gpu_r06_ab.sh)
set -o pipefail
O=${1:-gpurun_out/r06/mz27}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py tests/test_gpu_march.py -x -q --timeout 120 --timeout-method thread -k "march27 or plane_march" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_r06_ab.sh $O/ab - "AMG_MZ27_PF=3"
