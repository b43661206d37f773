#!/bin/bash
# round 5 (e): race probe (1-rank slab async free race vs the oracle's replay)
# with the default 4 hardware queues and with 16
set -o pipefail
O=${O:-gpurun_out/r05e}
mkdir -p $O
timeout -k 10 200 python -u tools/race_probe.py --runs 8 > $O/probe_q4.log 2>&1; echo "q4 exit $?"; cat $O/probe_q4.log | grep run
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u tools/race_probe.py --runs 8 > $O/probe_q16.log 2>&1; echo "q16 exit $?"; grep run $O/probe_q16.log
timeout -k 10 200 python -u tools/race_probe.py --runs 4 --ranks 2 > $O/probe_r2.log 2>&1; echo "r2 exit $?"; grep run $O/probe_r2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_elast_async.py -v -s -rf --timeout 240 --timeout-method thread \
   > $O/elast_async.log 2>&1; echo "elast exit $?"; grep -E "passed|failed" $O/elast_async.log | tail -2
