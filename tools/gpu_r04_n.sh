#!/bin/bash
# round 4 final tree: the full GPU test pass (not slow), smoke(), the headline
# bench (7-pt march defaults: prefetch 2, occupancy-sized chunks)
set -o pipefail
mkdir -p gpurun_out/r04n
export AMG_SEGV_TRACE=1
timeout -k 10 780 python -u -m pytest tests -m "gpu and not slow" -v -rf --timeout 170 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/r04n/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r04n/pytest_gpu.log | cut -c1-200
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04n/smoke.log 2>&1
st=$?; echo "smoke exit $st"; [ $st -eq 0 ] || exit $st
timeout -k 10 420 python -u bench.py > gpurun_out/r04n/bench.json 2> gpurun_out/r04n/bench.log
st=$?; echo "bench exit $st"; tail -c 300 gpurun_out/r04n/bench.json; exit $st
