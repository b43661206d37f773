#!/bin/bash
# round 5 (o): config 3 with the level-0 FULL_ASYNC correction folded into the
# hybrid JGS or not (AMG_JGS_FOLD), add-then-read vs capture atomics, under a
# kernel trace (stats kept, traces dropped); the distributed replay checks
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05o
mkdir -p $O
export AMG_SEGV_TRACE=1
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 150 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
for v in "1 1 1" "1 0 1" "0 1 1" "0 0 1"; do
  set -- $v
  (cd /tmp && export TMPDIR=/tmp && AMG_JGS_FOLD=$1 AMG_ATOMIC_NORET=$2 timeout -k 10 300 rocprofv3 \
     --kernel-trace --stats --output-format csv -d $O/trace_$1_$2 -o run -- python3 $R/tools/bench_async.py \
     --transfers composed --reps 1 > $O/async3_$1_$2.json 2> $O/async3_$1_$2.err) || exit 1
  rm -f $O/trace_$1_$2/run_kernel_trace.csv
  echo "config 3 fold $1 noret $2: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_$1_$2.json | tr '\n' ' ')"
done
for v in "1 1" "0 1" "1 1" "0 1"; do
  set -- $v
  AMG_JGS_FOLD=$1 AMG_ATOMIC_NORET=$2 timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 \
     > $O/async3_plain_$1_$2.json 2> $O/async3_plain_$1_$2.err
  echo "config 3 (no trace) fold $1 noret $2: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_plain_$1_$2.json | tr '\n' ' ')"
done
run dist_band 500 tests/test_gpu_dist.py -k "band or accel"
grep -hE "run [0-9]+: device" $O/*.log | sed 's/^ *//' > $O/replay_summary.txt
