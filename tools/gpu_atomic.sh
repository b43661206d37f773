#!/bin/bash
# async additive update form: returning atomics (default) vs the reference's add-then-read
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "" "AMG_ATOMIC_READ=1" "" "AMG_ATOMIC_READ=1"; do
  env $v timeout -k 10 600 python tools/bench_async.py --reps 2 > gpurun_out/ba.json 2> gpurun_out/ba.log || exit $?
  echo "${v:-default}: $(grep '\[async\]' gpurun_out/ba.log | tail -1)"
done
AMG_ATOMIC_READ=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py -q --timeout 300 --timeout-method thread > gpurun_out/async_read.log 2>&1
rc=$?; tail -2 gpurun_out/async_read.log; exit $rc
