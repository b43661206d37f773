# config 3 throughput (256^3 ASYNC_MULTADD hybrid JGS) and a kernel trace of it
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/async
mkdir -p $P
cd $R
timeout -k 10 600 python tools/bench_async.py > $P/bench_async.json 2> $P/bench_async.log
st=$?; cat $P/bench_async.log; [ $st -eq 0 ] || exit $st
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/tools/bench_async.py --reps 1 --cycles 10 > $P/trace_async.json 2> $P/trace_async.err || exit $?
python3 $R/tools/stream_overlap.py $P/trace/run_kernel_trace.csv | tee $P/overlap.txt
