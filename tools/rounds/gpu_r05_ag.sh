#!/bin/bash
# round 5 (ag): the SQ wait breakdown done right (SQ_WAIT_ANY = parked on
# s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY),
# plus the L2's hit rate and fabric request mix, per fine kernel of the
# 512^3 step (tools/pmc_run.py).  Each pass is its own rocprofv3 run; a pass
# whose counters the listing does not hold is skipped.
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/gpurun_out/r05ag
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $P/counters.txt 2>&1
echo "listing exit $? lines $(wc -l < $P/counters.txt)"
has() { grep -q -- "$1" $P/counters.txt; }
csvs=""
for pass in "sqw SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES" \
            "tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
            "tcc2 TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum"; do
  set -- $pass; nm=$1; shift
  ok=1
  for c in "$@"; do has "${c%_sum}" || { echo "$nm: no $c in the listing, skipped"; ok=0; }; done
  [ $ok -eq 1 ] || continue
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $P/$nm -o run \
     -- python3 $R/tools/pmc_run.py 512 > $P/$nm.log 2>&1
  rc=$?; echo "$nm exit $rc"; [ $rc -eq 0 ] || exit $rc
  rm -f $(find $P/$nm -name "*kernel_trace.csv")
  c=$(find $P/$nm -name "*counter_collection.csv" | head -1)
  csvs="${csvs:+$csvs,}$c"
done
cd $R && python3 tools/pmc_sq.py $csvs $P/pmc_sq2.json > $P/pmc_sq2.log 2>&1; cat $P/pmc_sq2.log
