# config 3: the FULL_ASYNC update forms without a profiler (concurrent level streams), interleaved
set -o pipefail
O=${1:-gpurun_out/r06/atomic2}
mkdir -p $O
for rep in 1 2 3; do
for v in 0 1; do
  AMG_ATOMIC_NORET=$v timeout -k 10 300 python3 tools/bench_async.py --transfers composed > $O/a_${v}_$rep.json 2> $O/a_${v}_$rep.err || { echo "variant $v failed"; tail -5 $O/a_${v}_$rep.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/a_${v}_$rep.json').read().strip().splitlines()[-1])
print(f\"[NORET=$v] async {d['async']['cycles_per_s']:.1f} sync {d['sync']['cycles_per_s']:.1f} ratio {d['async_over_sync_speed']:.3f}\")"
done
done
