#!/bin/bash
# round 4 measurements: the headline bench (with its CPU baseline and parity
# leg), config 4's asynchronous additive line at 512^3 (1 rank over RCCL, 8
# ranks over the channels), config 3's async vs sync additive (composed and
# explicit smoothed transfers)
set -o pipefail
mkdir -p gpurun_out/r04b
export AMG_LINK_TIMEOUT_S=120
step() { # name timeout cmd...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t "$@" > gpurun_out/r04b/$name.json 2> gpurun_out/r04b/$name.log
   local rc=$?
   echo "$name exit $rc"
   case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
   return 0
}
step bench 420 python -u bench.py
step async3_composed 240 python -u tools/bench_async.py --transfers composed
step async3_composed_graphs 240 python -u tools/bench_async.py --transfers composed --graphs 1
step async_dist1 300 python -u tools/bench_dist_async.py --ranks 1 --cycles 8
step async_dist8 420 python -u tools/bench_dist_async.py --ranks 8 --cycles 8
step async_dist8_xfp 420 env AMG_FUSE_XFP_SLAB=1 python -u tools/bench_dist_async.py --ranks 8 --cycles 8
step async3_explicit 300 python -u tools/bench_async.py --transfers explicit
step bench_mzpf2 300 env AMG_MZ_PF=2 python -u bench.py --cpu-baseline 0
step bench_again 300 python -u bench.py --cpu-baseline 0
echo done
