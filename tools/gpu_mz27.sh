#!/bin/bash
# 27-pt march occupancy variant: bench it/s (default vs waves_per_eu 4) and the per-step kernel timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/mz27
mkdir -p $P
for o in 1 4 1 4; do
  AMG_MZ27_OCC=$o timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > $P/bench_o$o.json 2> $P/bench_o$o.log || exit $?
  echo "occ=$o $(python -c "import json;d=json.load(open('$P/bench_o$o.json'));print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for o in 1 4; do
  AMG_MZ27_OCC=$o timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/trace$o -o run \
     -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace$o.json 2> $P/trace$o.err || exit $?
  python3 $R/tools/step_breakdown.py $P/trace$o/run_kernel_trace.csv > $P/step$o.txt || exit $?
  grep -E "step wall|mz27" $P/step$o.txt
done
echo done
