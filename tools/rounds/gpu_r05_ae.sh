#!/bin/bash
# round 5 (ae): DMEM_AsyncSmooth at 512^3, 2 and 8 ranks, one hardware queue per stream
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ae
mkdir -p $O
for r in 2 8; do
  GPU_MAX_HW_QUEUES=32 timeout -k 10 400 python -u tools/bench_async_jacobi.py --ranks $r > $O/ajac$r.json 2> $O/ajac$r.err
  echo "ranks $r exit $?: $(python3 -c "import json; d=json.load(open('$O/ajac$r.json')); print(d['relres'], round(d['sweeps_per_s'],1))")"
  grep "^rank" $O/ajac$r.err
done
