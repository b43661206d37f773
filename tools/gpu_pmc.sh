# rocprofv3 kernel trace + stats of the 512^3 bench, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) over tools/pmc_run.py; never combined with sys/runtime traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/prof
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace_bench.json 2> $P/trace_bench.err || exit $?
echo "trace ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/fetch -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/write -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/write.log 2>&1 || exit $?
echo "write ok"
find $P -name "*.csv" | head -20
