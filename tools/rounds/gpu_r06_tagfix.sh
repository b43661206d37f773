# the fused prolongation + update held to 5 waves per SIMD: its bitwise tests,
# then config 4 and config 3 against the round-5 tree (bisect_r05), interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r06/tagfix
mkdir -p $O
export AMG_LINK_TIMEOUT_S=120
for rep in 1; do
for t in bisect_r05 new; do
  d=$GRAFT_REPO_ROOT/$t; [ $t = new ] && d=$GRAFT_REPO_ROOT
  (cd $d && timeout -k 10 400 python3 tools/bench_dist_async.py --ranks 8 --cycles 8 > $O/d_${t}_$rep.json 2> $O/d_${t}_$rep.err) || { echo "$t failed"; tail -5 $O/d_${t}_$rep.err; exit 1; }
  (cd $d && timeout -k 10 300 python3 tools/bench_async.py --transfers composed > $O/a_${t}_$rep.json 2> $O/a_${t}_$rep.err) || { echo "$t failed"; tail -5 $O/a_${t}_$rep.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/d_${t}_$rep.json').read().strip().splitlines()[-1])
a=json.loads(open('$O/a_${t}_$rep.json').read().strip().splitlines()[-1])
print('[$t] config4', round(d['value'], 2), 'config3 async', round(a['async']['cycles_per_s'], 1), 'sync', round(a['sync']['cycles_per_s'], 1))"
done
done
