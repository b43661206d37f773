# rocprofv3 kernel trace + stats of a short 512^3 bench (no PMC); analyse with
# tools/step_breakdown.py gpurun_out/prof/trace/run_kernel_trace.csv
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/prof
rm -rf $P/trace && mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 "$@" > $P/trace_bench.json 2> $P/trace_bench.err || exit $?
tail -3 $P/trace_bench.err
python3 $R/tools/step_breakdown.py $P/trace/run_kernel_trace.csv
