#!/bin/bash
# round 4: deterministic async schedules vs the oracle, the async bands, and the
# slab tests with the zero-guess fold re-landed
set -o pipefail
mkdir -p gpurun_out/r04sched
timeout -k 10 900 python -u -m pytest tests/test_gpu_async.py -v -s --timeout 300 --timeout-method thread \
   > gpurun_out/r04sched/pytest_async.log 2>&1
echo "async exit $?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py -v -s --timeout 300 --timeout-method thread \
   > gpurun_out/r04sched/pytest_slab.log 2>&1
echo "slab exit $?"
