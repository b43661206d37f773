#!/bin/bash
# round 4: confirm the slab async file (band with the sequential members) and
# smoke() on the final tree
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 400 python -u -m pytest tests/test_gpu_slab_async.py -m "gpu and not slow" -v -s -rf --timeout 170 \
   --timeout-method thread > gpurun_out/r04l/slab_async.log 2>&1
rc=$?; echo "slab_async exit $rc"; grep -E "band|passed|failed" gpurun_out/r04l/slab_async.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04l/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/r04l/smoke.log
exit $rc
