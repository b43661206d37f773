# rocprofv3 kernel trace + stats of the 512^3 bench, then separate PMC passes
# for FETCH_SIZE and WRITE_SIZE (never combined with sys/runtime traces).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $R/gpurun_out/prof/trace_bench.json 2> $R/gpurun_out/prof/trace_bench.err
echo "trace exit $?"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $R/gpurun_out/prof/fetch -o run \
   -- python3 $R/bench.py --steps 4 --warmup 1 --cpu-baseline 0 --spmv-reps 2 > $R/gpurun_out/prof/fetch_bench.json 2> $R/gpurun_out/prof/fetch_bench.err
echo "fetch exit $?"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $R/gpurun_out/prof/write -o run \
   -- python3 $R/bench.py --steps 4 --warmup 1 --cpu-baseline 0 --spmv-reps 2 > $R/gpurun_out/prof/write_bench.json 2> $R/gpurun_out/prof/write_bench.err
echo "write exit $?"
find $R/gpurun_out/prof -name "*.csv" | head -20
