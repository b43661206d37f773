#!/bin/bash
# round 5 (v): every free-race replay check with its printout (device-clock windows)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_solve.py tests/test_gpu_slab_async.py \
   tests/test_gpu_slab_async_procs.py tests/test_gpu_dist.py tests/test_gpu_elast_async.py -k "band or replay or race" \
   -m "gpu and not slow" -v -s -rf --timeout 200 --timeout-method thread > $O/races.log 2>&1
echo "races exit $?"; grep -E "passed|failed" $O/races.log | tail -1
grep -E "run [0-9]+: device" $O/races.log | sed 's/^.*::[^ ]* *//; s/^ *//' > $O/replay_summary.txt; wc -l $O/replay_summary.txt
grep -c OUTSIDE $O/replay_summary.txt
