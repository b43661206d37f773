# config 3 throughput across round 6's commits (worktrees bisect_r05 = a6a2c63,
# bisect_a = cd8d89b, bisect_b = b5967d2, this tree), interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r06/bisect4
mkdir -p $O
for rep in 1 2; do
for t in bisect_r05 new; do
  d=$GRAFT_REPO_ROOT/${t%_noret1}; [ $t = new ] && d=$GRAFT_REPO_ROOT
  e=""; [ $t = bisect_a_noret1 ] && e="AMG_ATOMIC_NORET=1"
  (cd $d && env $e timeout -k 10 300 python3 tools/bench_async.py --transfers composed > $O/a_${t}_$rep.json 2> $O/a_${t}_$rep.err) || { echo "$t failed"; tail -5 $O/a_${t}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/a_${t}_$rep.json').read().strip().splitlines()[-1])
print(f\"[$t] async {d['async']['cycles_per_s']:.1f} sync {d['sync']['cycles_per_s']:.1f} ratio {d['async_over_sync_speed']:.3f}\")"
done
done
