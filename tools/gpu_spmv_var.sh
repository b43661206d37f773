#!/bin/bash
# fine SpMV under march variants (+ the march bitwise tests and one bench line)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_march.py -q --timeout 300 --timeout-method thread > gpurun_out/march_tests.log 2>&1
rc=$?; tail -2 gpurun_out/march_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "AMG_MZ_LINES_GEMV=1" "" "AMG_MZ_LINES_GEMV=4" "AMG_MZ_LINES_GEMV=2 AMG_PLANE_MARCH=32" "AMG_MZ_LINES_GEMV=4 AMG_PLANE_MARCH=32"; do
  env $v timeout -k 10 120 python tools/spmv_variants.py 512 || exit $?
done
for v in "" "AMG_MZ_LINES=4"; do
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_l.json 2> gpurun_out/bench_l.log || exit $?
  echo "${v:-default}: $(python -c "import json;d=json.load(open('gpurun_out/bench_l.json'));print(d['value'], d['ms_per_step'], d['fine_spmv']['frac'], d['roofline']['frac'])")"
done
