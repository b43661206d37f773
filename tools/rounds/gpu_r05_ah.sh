#!/bin/bash
# round 5 (ah): the 7-pt march with its halo operands two planes ahead
# (AMG_MZ_PF=3): bitwise tests, an interleaved bench A/B against the default,
# and the L2 counters of both (tools/pmc_run.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ah
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -x -q --timeout 120 --timeout-method thread -k "march_tuning_bitwise" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for pf in 1 3; do
    AMG_MZ_PF=$pf timeout -k 10 300 python -u bench.py --cpu-baseline 0 --general 0 > $O/bench_pf${pf}_$i.json 2> $O/bench_pf${pf}_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench pf $pf exit $rc"; exit $rc; }
    python3 -c "import json; d=json.load(open('$O/bench_pf${pf}_$i.json')); fk=d.get('fine_kernels',{}); print('pf $pf', d['value'], d['ms_per_step'], {k: round(v.get('ms',0),3) for k,v in fk.items()} if isinstance(fk,dict) else '')"
  done
done
cd /tmp && export TMPDIR=/tmp
for pf in 1 3; do
  AMG_MZ_PF=$pf timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d $O/tcc$pf -o run \
     -- python3 $R/tools/pmc_run.py 512 > $O/tcc$pf.log 2>&1
  rc=$?; echo "tcc pf $pf exit $rc"; [ $rc -eq 0 ] || exit $rc
  rm -f $(find $O/tcc$pf -name "*kernel_trace.csv")
  c=$(find $O/tcc$pf -name "*counter_collection.csv" | head -1)
  (cd $R && python3 tools/pmc_sq.py $c $O/tcc$pf.json)
done
