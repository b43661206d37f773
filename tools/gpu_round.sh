set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_gpu.log; tail -5 gpurun_out/pytest_gpu.log
[ $st -eq 0 ] || exit $st
bash tools/gpu_pmc.sh
