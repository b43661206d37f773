#!/bin/bash
# round-3 kernel checks: kernel bitwise tests (hybrid JGS forms, long-row dictionary), async bands,
# config-3 throughput (bench_async) and its kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/r03
mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_march.py -q --timeout 300 --timeout-method thread > $P/pytest_kernels.log 2>&1
rc=$?; tail -3 $P/pytest_kernels.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_solve.py tests/test_gpu_async.py tests/test_gpu_configs.py -q -s --timeout 400 --timeout-method thread > $P/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $P/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/bench_async.py --reps 3 > $P/bench_async.json 2> $P/bench_async.log || exit $?
tail -2 $P/bench_async.log
for sm in 0 1; do
  AMG_JGS_SMALL=$sm timeout -k 10 600 python tools/bench_async.py --reps 2 > $P/bench_async_s$sm.json 2> $P/bench_async_s$sm.log || exit $?
  echo "small=$sm"; tail -2 $P/bench_async_s$sm.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/tools/bench_async.py --reps 1 --cycles 10 > $P/trace_async.json 2> $P/trace_async.err || exit $?
head -14 $P/trace/run_kernel_stats.csv | cut -c1-150
echo done
