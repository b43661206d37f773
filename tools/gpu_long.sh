set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
st=$?; tail -4 gpurun_out/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 400 python tools/tune_spmv.py -5 5 vi_base,long > gpurun_out/tune_long3.log 2>&1 || exit $?
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" gpurun_out/tune_long3.log | grep "r256\|vi_base"
timeout -k 10 400 python tools/bench_elasticity.py --refine 5 > gpurun_out/bench_elast5.json 2> gpurun_out/bench_elast5.log
st=$?; tail -1 gpurun_out/bench_elast5.log; cat gpurun_out/bench_elast5.json; exit $st
