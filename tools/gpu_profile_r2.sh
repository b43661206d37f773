# round-2 evidence run: every GPU test, smoke, the default bench line (CPU
# baseline + parity), a rocprofv3 kernel trace + stats of the bench with one
# step's breakdown, then the FETCH_SIZE / WRITE_SIZE passes for the traffic
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st" >> gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
st=$?; tail -1 gpurun_out/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log
st=$?; tail -3 gpurun_out/bench_full.log; [ $st -eq 0 ] || exit $st
P=$R/gpurun_out/prof
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace_bench.json 2> $P/trace_bench.err || exit $?
T=$(find $P/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $T > $R/gpurun_out/step_breakdown.txt && head -3 $R/gpurun_out/step_breakdown.txt
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/fetch -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/write -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/write.log 2>&1 || exit $?
echo "write ok"
F=$(find $P/fetch -name "*counter_collection.csv" | head -1)
W=$(find $P/write -name "*counter_collection.csv" | head -1)
cp $R/profiles/traffic.json $R/gpurun_out/traffic.json
cd $R/tools && python3 pmc_fine.py $F $W 512 $R/gpurun_out/traffic.json > $R/gpurun_out/pmc_fine.log 2>&1; tail -30 $R/gpurun_out/pmc_fine.log
