#!/bin/bash
# round 4 final evidence in one call: the headline bench (CPU baseline, parity
# leg), its rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE PMC
# passes (tools/pmc_fine.py -> traffic), config 3's async vs sync additive
# (composed and explicit smoothed transfers), config 4's async additive at
# 512^3 (1 rank over RCCL, 8 ranks over the channels)
set -o pipefail
R=$(pwd)
P=$R/gpurun_out/r04k
mkdir -p $P
export AMG_LINK_TIMEOUT_S=120
step() { # name timeout cmd...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t "$@" > $P/$name.json 2> $P/$name.log
   local rc=$?
   echo "$name exit $rc"; tail -c 400 $P/$name.json; echo
   case $rc in 0) ;; *) echo "stopping after $name"; exit $rc;; esac
}
step bench 420 python -u bench.py
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace_bench.json 2> $P/trace_bench.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $P/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $f > $P/step_breakdown.txt; head -2 $P/step_breakdown.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/fetch -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/write -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/write.log 2>&1
rc=$?; echo "write exit $rc"; [ $rc -eq 0 ] || exit $rc
fc=$(find $P/fetch -name "*counter_collection.csv" | head -1)
wc=$(find $P/write -name "*counter_collection.csv" | head -1)
cd $R && python3 tools/pmc_fine.py $fc $wc 512 $P/traffic.json > $P/pmc_fine.log 2>&1; tail -4 $P/pmc_fine.log
step async3_composed 240 python -u tools/bench_async.py --transfers composed
step async3_explicit 300 python -u tools/bench_async.py --transfers explicit
step async_dist1 300 python -u tools/bench_dist_async.py --ranks 1 --cycles 8
step async_dist8 420 python -u tools/bench_dist_async.py --ranks 8 --cycles 8
echo done
