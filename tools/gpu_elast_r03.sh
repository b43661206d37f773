#!/bin/bash
# config 5 (elasticity) at size on one GPU: bitwise tests at r = 5, 6; bench lines r = 5, 6 with the
# 3x3 block kernel's roofline; rocprofv3 kernel stats of the r = 6 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/elast
mkdir -p $P
timeout -k 10 900 python -u -m pytest tests/test_gpu_classical.py tests/test_gpu_bsr.py -q -s --timeout 600 --timeout-method thread > $P/pytest.log 2>&1
rc=$?; tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 5 6; do
  timeout -k 10 600 python tools/bench_elasticity.py --refine $r --steps 20 > $P/bench_r$r.json 2> $P/bench_r$r.log || exit $?
  cat $P/bench_r$r.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run \
   -- python3 $R/tools/bench_elasticity.py --refine 6 --steps 5 --warmup 1 > $P/trace.json 2> $P/trace.err || exit $?
head -8 $P/trace/run_kernel_stats.csv | cut -c1-160
echo done
