#!/bin/bash
# round 5 (n): the FULL_ASYNC level-0 correction folded into the hybrid JGS
# (grp and tile forms) in the reference's add-then-read form vs the capture
# form; config 3 under a kernel trace; the replay checks on device windows
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n
mkdir -p $O
export AMG_SEGV_TRACE=1 AMG_REPLAY_DUMP=$O/dump
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 150 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
run jgs 300 tests/test_gpu_kernels.py -k hybrid_jgs || exit 1
run async 400 tests/test_gpu_async.py tests/test_gpu_configs.py -k "hybrid or async"
for v in "1 1 1" "1 0 1" "3 1 4"; do
  set -- $v
  (cd /tmp && export TMPDIR=/tmp && AMG_JGS_WAVE=$1 AMG_ATOMIC_NORET=$2 AMG_JGS_TILE_OCC=$3 timeout -k 10 300 rocprofv3 \
     --kernel-trace --stats --output-format csv -d $O/trace_$1_$2_$3 -o run -- python3 $R/tools/bench_async.py \
     --transfers composed --reps 1 > $O/async3_$1_$2_$3.json 2> $O/async3_$1_$2_$3.err) || exit 1
  echo "config 3 jgs_wave $1 noret $2 occ $3: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_$1_$2_$3.json | tr '\n' ' ')"
  f=$(find $O/trace_$1_$2_$3 -name "*kernel_stats.csv" | head -1); grep -E "jgs|atomic_correct|xfer_prolong" "$f" | cut -d, -f1-4 | cut -c1-150
done
for v in "1 1" "1 0"; do
  set -- $v
  AMG_JGS_WAVE=$1 AMG_ATOMIC_NORET=$2 timeout -k 10 300 python -u tools/bench_async.py --transfers composed --reps 3 \
     > $O/async3_plain_$1_$2.json 2> $O/async3_plain_$1_$2.err
  echo "config 3 (no trace) jgs_wave $1 noret $2: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_plain_$1_$2.json | tr '\n' ' ')"
done
run slab_async 400 tests/test_gpu_slab_async.py
run procs 400 tests/test_gpu_slab_async_procs.py
run elast 400 tests/test_gpu_elast_async.py
run dist_band 500 tests/test_gpu_dist.py -k "band or accel"
grep -hE "run [0-9]+: device" $O/*.log | sed 's/^ *//' > $O/replay_summary.txt
