#!/bin/bash
# round 4: config 4 at size (512^3 async additive, smoothed transfers, per-level
# channels), config 3 throughput with composed transfers, the headline bench
set -o pipefail
mkdir -p gpurun_out/r04b
export AMG_LINK_TIMEOUT_S=120
step() { # name timeout cmd...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t "$@" > gpurun_out/r04b/$name.log 2>&1
   local rc=$?
   echo "$name exit $rc"
   case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
   return 0
}
step bench 600 python -u bench.py
step async_dist1 600 python -u tools/bench_dist_async.py --ranks 1 --cycles 8
step async_dist8 900 python -u tools/bench_dist_async.py --ranks 8 --cycles 8
step async3_composed 600 python -u tools/bench_async.py --transfers composed
step async3_explicit 900 python -u tools/bench_async.py --transfers explicit
step slab512 1100 python -u -m pytest tests/test_gpu_slab_async.py -k 512 -v -s --timeout 1000 --timeout-method thread
echo done
