#!/bin/bash
# marching prolongation: bitwise GPU tests of the geometric paths, then A/B bench and a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/prolong
mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py tests/test_gpu_slab.py tests/test_gpu_configs.py -q -m gpu -x --timeout 300 --timeout-method thread > $P/pytest.log 2>&1
st=$?; echo "pytest exit $st" >> $P/pytest.log; tail -3 $P/pytest.log; [ $st -eq 0 ] || exit $st
AMG_PROLONG_MARCH=0 timeout -k 10 300 python bench.py --cpu-baseline 0 > $P/bench_old.json 2> $P/bench_old.log || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > $P/bench_new.json 2> $P/bench_new.log || exit $?
python -c "
import json
for k in ('old','new'):
    d=json.load(open('$P/bench_'+k+'.json')); print(k, d['value'], d['ms_per_step'], d.get('parity'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace_bench.json 2> $P/trace_bench.err || exit $?
python3 $R/tools/step_breakdown.py $P/trace/run_kernel_trace.csv > $P/step_breakdown.txt || exit $?
grep -i "prolong\|wall" $P/step_breakdown.txt
echo done
