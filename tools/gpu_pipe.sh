#!/bin/bash
# plane-march pipelining: bitwise kernel / march / solve tests, bench it/s and the step timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/pipe
mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_march.py tests/test_gpu_solve.py tests/test_gpu_configs.py -q -s --timeout 400 --timeout-method thread > $P/pytest.log 2>&1
rc=$?; tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > $P/bench$i.json 2> $P/bench$i.log || exit $?
  echo "$(python -c "import json;d=json.load(open('$P/bench$i.json'));print(d['value'], d['ms_per_step'], d['fine_spmv']['frac'], d['roofline']['frac'], d.get('parity'))")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/trace -o run \
   -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/trace.json 2> $P/trace.err || exit $?
python3 $R/tools/step_breakdown.py $P/trace/run_kernel_trace.csv > $P/step.txt || exit $?
head -8 $P/step.txt; grep -E "mz27|prolong|EpiJacobi" $P/step.txt | tail -4
echo done
