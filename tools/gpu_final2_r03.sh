#!/bin/bash
# round-3 evidence: every GPU test, smoke(), the default bench line, the one-rank distributed
# line, the rocprofv3 kernel trace + PMC traffic passes of the bench, config-3 throughput
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/final2
mkdir -p $P
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 400 --timeout-method thread > $P/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> $P/pytest_gpu.log; tail -3 $P/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1
st=$?; tail -2 $P/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py > $P/bench_full.json 2> $P/bench_full.log
st=$?; cat $P/bench_full.json; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py --gpus 1 --force-dist 1 > $P/bench_dist1.json 2> $P/bench_dist1.log
st=$?; cat $P/bench_dist1.json; [ $st -eq 0 ] || exit $st
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace_bench.json 2> $P/trace_bench.err || exit $?
cp $P/trace/run_kernel_stats.csv $P/kernel_stats.csv
python3 $R/tools/step_breakdown.py $P/trace/run_kernel_trace.csv > $P/step_breakdown.txt || exit $?
head -3 $P/step_breakdown.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/fetch -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/write -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/write.log 2>&1 || exit $?
F=$(find $P/fetch -name "*counter_collection.csv" | head -1)
W=$(find $P/write -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_fine.py $F $W 512 $P/traffic.json > $P/pmc_fine.log 2>&1 || exit $?
cat $P/pmc_fine.log
cd $R
timeout -k 10 600 python tools/bench_async.py --reps 3 > $P/bench_async.json 2> $P/bench_async.log || exit $?
tail -2 $P/bench_async.log
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/async_trace -o run \
   -- python3 $R/tools/bench_async.py --reps 1 --cycles 10 > $P/async_trace.json 2> $P/async_trace.err || exit $?
cp $P/async_trace/run_kernel_stats.csv $P/kernel_stats_async.csv
echo done
