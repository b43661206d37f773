#!/bin/bash
# hybrid JGS wave kernel: bitwise kernel tests, async solves, config-3 throughput (wave vs lane), kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/jgs
mkdir -p $P
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -k "hybrid or gauss" -q --timeout 400 --timeout-method thread > $P/pytest_kernels.log 2>&1 || exit $?
tail -2 $P/pytest_kernels.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_solve.py tests/test_gpu_async.py tests/test_gpu_configs.py tests/test_gpu_sps.py tests/test_gpu_delay.py -q -s --timeout 400 --timeout-method thread > $P/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $P/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AMG_JGS_WAVE=2 timeout -k 10 600 python tools/bench_async.py --reps 2 > $P/bench_async_wave.json 2> $P/bench_async_wave.log || exit $?
timeout -k 10 600 python tools/bench_async.py --reps 3 > $P/bench_async.json 2> $P/bench_async.log || exit $?
tail -3 $P/bench_async_wave.log; tail -3 $P/bench_async.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/tools/bench_async.py --reps 1 --cycles 10 > $P/trace_async.json 2> $P/trace_async.err || exit $?
head -12 $P/trace/run_kernel_stats.csv
