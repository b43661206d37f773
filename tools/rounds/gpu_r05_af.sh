#!/bin/bash
# round 5 (af): the asynchronous additive cycles with a hardware queue per stream
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05af
mkdir -p $O
for q in 4 16 32 4 16 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 > $O/a$q.json 2> $O/a$q.err
  echo "config 3 queues $q: $(grep -o '"cycles_per_s": [0-9.]*' $O/a$q.json | tr '\n' ' ')"
done
for q in 4 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u tools/bench_dist_async.py --ranks 1 --cycles 8 > $O/d1_$q.json 2> $O/d1_$q.err
  echo "config 4 1 rank queues $q: $(python3 -c "import json; d=json.load(open('$O/d1_$q.json')); print(round(d['value'],2))" 2>&1 | tail -1)"
done
