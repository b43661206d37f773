#!/bin/bash
# round 5 (h): what makes the 1-rank slab free race deviate from its replay:
# one hardware queue (no concurrent kernels), the fused transfers off
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
GPU_MAX_HW_QUEUES=1 timeout -k 10 200 python -u tools/race_probe.py --form slab --runs 8 > $O/q1.log 2>&1
echo "q1 exit $?"; grep run $O/q1.log | cut -c1-60
GPU_MAX_HW_QUEUES=16 AMG_FUSE_XFER=0 timeout -k 10 200 python -u tools/race_probe.py --form slab --runs 8 > $O/q16_nofuse.log 2>&1
echo "q16 nofuse exit $?"; grep run $O/q16_nofuse.log | cut -c1-60
GPU_MAX_HW_QUEUES=16 AMG_FUSE_TRANSFER=0 AMG_FUSE_XFER=0 timeout -k 10 200 python -u tools/race_probe.py --form slab --runs 8 > $O/q16_nogeo.log 2>&1
echo "q16 nogeo exit $?"; grep run $O/q16_nogeo.log | cut -c1-60
