#!/bin/bash
# round 5 (l): the LDS-tile hybrid JGS (parity, config 3 kernel times under a
# kernel trace for jgs_wave 1 / 3) and the replay checks with the row-time
# model of torn updates (recorded tables dumped for study off the GPU)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l
mkdir -p $O
export AMG_SEGV_TRACE=1 AMG_REPLAY_DUMP=$O/dump
run() { # name timeout files...
   local name=$1 t=$2; shift 2
   timeout -k 10 $t python -u -m pytest "$@" -m "gpu and not slow" -v -s -rf --timeout 240 --timeout-method thread \
      > $O/$name.log 2>&1
   local rc=$?; echo "$name exit $rc"; grep -E "passed|failed" $O/$name.log | tail -2
   return $rc
}
run jgs 300 tests/test_gpu_kernels.py -k hybrid_jgs || exit 1
for w in 1 3; do
  (cd /tmp && export TMPDIR=/tmp && AMG_JGS_WAVE=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/trace_jgs$w -o run -- python3 $R/tools/bench_async.py --transfers composed --reps 1 \
     > $O/async3_jgs$w.json 2> $O/async3_jgs$w.err) || exit 1
  echo "config 3 jgs_wave $w: $(grep -o '"cycles_per_s": [0-9.]*' $O/async3_jgs$w.json | tr '\n' ' ')"
  f=$(find $O/trace_jgs$w -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-4 | cut -c1-150
done
AMG_JGS_WAVE=3 run async_jgs3 400 tests/test_gpu_async.py tests/test_gpu_configs.py -k "hybrid or async"
run slab_async 400 tests/test_gpu_slab_async.py
run procs 400 tests/test_gpu_slab_async_procs.py
run dist_band 400 tests/test_gpu_dist.py -k "band or accel"
run elast 400 tests/test_gpu_elast_async.py
grep -hE "run [0-9]+: device" $O/*.log | sed 's/^ *//' > $O/replay_summary.txt
