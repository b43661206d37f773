#!/bin/bash
# round 5 (ap): config 3's level-0 FULL_ASYNC prolongation with its read-backs
# batched per workgroup (AMG_ATOMIC_NORET=2) -- the async test file under it,
# then config 3 interleaved against the per-row add-then-read form (1) and the
# capture form (0)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ap
mkdir -p $O
AMG_ATOMIC_NORET=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread > $O/tasync.log 2>&1
rc=$?; echo "async tests (mode 2): $(tail -1 $O/tasync.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in 1 2 0; do
    AMG_ATOMIC_NORET=$m timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 > $O/a${m}_$i.json 2> $O/a${m}_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench mode $m exit $rc"; exit $rc; }
    echo "mode $m: $(grep -o '"cycles_per_s": [0-9.]*' $O/a${m}_$i.json | tr '\n' ' ')"
  done
done
