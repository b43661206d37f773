#!/bin/bash
# round 5 (ai): halo operands ahead at 5 waves per SIMD -- two planes ahead
# held to 5 waves (AMG_MZ_PF=3 AMG_MZ_WPE=5) and one plane ahead
# (AMG_MZ_PF=3 AMG_MZ_HPF=1, 90 VGPRs) -- against the default, interleaved;
# the L2 counters of the one-plane form
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ai
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -x -q --timeout 120 --timeout-method thread -k "march_tuning_bitwise" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AMG_MZ_PF=3 AMG_MZ_HPF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -x -q --timeout 120 --timeout-method thread -k "march_tuning_bitwise" > $O/tests_h1.log 2>&1
rc=$?; tail -1 $O/tests_h1.log; [ $rc -eq 0 ] || exit $rc
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --cpu-baseline 0 --general 0 > $O/bench_$tag.json 2> $O/bench_$tag.err
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $tag exit $rc"; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); fk=d['fine_kernels']; print('$tag', round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms'],3) for k,v in fk.items()})"
}
for i in 1 2; do
  run base$i AMG_MZ_PF=1
  run h2w5_$i AMG_MZ_PF=3 AMG_MZ_WPE=5
  run h1_$i AMG_MZ_PF=3 AMG_MZ_HPF=1
done
cd /tmp && export TMPDIR=/tmp
AMG_MZ_PF=3 AMG_MZ_HPF=1 timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d $O/tcch1 -o run \
   -- python3 $R/tools/pmc_run.py 512 > $O/tcch1.log 2>&1
rc=$?; echo "tcc h1 exit $rc"; [ $rc -eq 0 ] || exit $rc
rm -f $(find $O/tcch1 -name "*kernel_trace.csv")
c=$(find $O/tcch1 -name "*counter_collection.csv" | head -1)
(cd $R && python3 tools/pmc_sq.py $c $O/tcch1.json)
