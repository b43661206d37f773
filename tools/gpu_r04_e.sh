#!/bin/bash
# round 4 profile evidence: rocprofv3 kernel trace + stats of the 512^3 bench
# (kernel_stats.csv, the step's per-kernel timeline), then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) over tools/pmc_run.py for the fine kernels' HBM
# bytes (tools/pmc_fine.py -> traffic.json); never combined with other traces
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/r04e
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace_bench.json 2> $P/trace_bench.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $P/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $f > $P/step_breakdown.txt; head -3 $P/step_breakdown.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/fetch -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/write -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/write.log 2>&1
rc=$?; echo "write exit $rc"; [ $rc -eq 0 ] || exit $rc
fc=$(find $P/fetch -name "*counter_collection.csv" | head -1)
wc=$(find $P/write -name "*counter_collection.csv" | head -1)
cd $R && python3 tools/pmc_fine.py $fc $wc 512 $P/traffic.json > $P/pmc_fine.log 2>&1; cat $P/pmc_fine.log | tail -8
echo done
