# Master-pattern kernel: its parity tests, the whole GPU suite, the 512^3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mp
timeout -k 10 300 python -u -m pytest tests/test_gpu_master.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mp/pytest_master.log 2>&1
st=$?; tail -5 gpurun_out/mp/pytest_master.log; [ $st -eq 0 ] || exit $st
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mp/pytest_gpu.log 2>&1
st=$?; tail -3 gpurun_out/mp/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/mp/bench.json 2> gpurun_out/mp/bench.log
st=$?; cat gpurun_out/mp/bench.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u tools/tune_spmv.py 512 5 mp,ABL_mp_f3,ABL_mp_br > gpurun_out/mp/tune.log 2>&1; st=$?; grep "^A0" gpurun_out/mp/tune.log; exit $st
