#!/bin/bash
# round 6 final evidence: the headline bench (CPU baselines, parity, general-CSR
# leg), its kernel trace + stats and step breakdown, the FETCH_SIZE /
# WRITE_SIZE passes (traffic) and an SQ pass (instruction / wait counters per
# fine kernel); config 3 and the config-4 async bench (threads and torchrun)
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/${1:-gpurun_out/r06final}
mkdir -p $P
export AMG_LINK_TIMEOUT_S=120
step() { # name timeout cmd...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t "$@" > $P/$name.json 2> $P/$name.log
   local rc=$?
   echo "$name exit $rc"; tail -c 300 $P/$name.json; echo
   case $rc in 0) ;; *) echo "stopping after $name"; exit $rc;; esac
}
step bench 500 python -u bench.py
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 --general 0 > $P/trace_bench.json 2> $P/trace_bench.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $P/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $f > $P/step_breakdown.txt; head -2 $P/step_breakdown.txt; rm -f $f
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" \
            "sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES" "tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  set -- $pass; nm=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $P/$nm -o run \
     -- python3 $R/tools/pmc_run.py 512 > $P/$nm.log 2>&1
  rc=$?; echo "$nm exit $rc"; [ $rc -eq 0 ] || exit $rc
  rm -f $(find $P/$nm -name "*kernel_trace.csv")
done
fc=$(find $P/fetch -name "*counter_collection.csv" | head -1)
wc=$(find $P/write -name "*counter_collection.csv" | head -1)
sc=$(find $P/sq -name "*counter_collection.csv" | head -1),$(find $P/tcc -name "*counter_collection.csv" | head -1)
cd $R && python3 tools/pmc_fine.py $fc $wc 512 $P/traffic.json > $P/pmc_fine.log 2>&1; tail -4 $P/pmc_fine.log
python3 tools/pmc_sq.py $sc $P/pmc_sq.json > $P/pmc_sq.log 2>&1; cat $P/pmc_sq.log
step async3_composed 240 python -u tools/bench_async.py --transfers composed
step async_dist8 420 python -u tools/bench_dist_async.py --ranks 8 --cycles 8
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
   --master-port 29533 tools/bench_dist_async.py --size 256 --cycles 8 --transport host > $P/async_dist_torchrun2.json 2> $P/async_dist_torchrun2.log
echo "torchrun 2 exit $?"; tail -c 300 $P/async_dist_torchrun2.json

step elast6 600 python -u tools/bench_elasticity.py --refine 6 --steps 20
echo done2
