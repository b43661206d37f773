#!/bin/bash
# round 5 (g): race probe -- the single-GPU async solve vs the 1-rank slab solve,
# 4 and 16 hardware queues
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
for q in 4 16; do
  for form in single slab; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u tools/race_probe.py --form $form --runs 8 > $O/probe_${form}_q$q.log 2>&1
    echo "$form q$q exit $?"; grep run $O/probe_${form}_q$q.log | cut -c1-60
  done
done
