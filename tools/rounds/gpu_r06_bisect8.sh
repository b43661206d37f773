# config 4 across round 6's commits: a6a2c63 (bisect_r05), cd8d89b (bisect_a),
# f920c31 (bisect_b), this tree with and without the prolongation's NT loads
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r06/bisect8
mkdir -p $O
export AMG_LINK_TIMEOUT_S=120
for rep in 1; do
for t in bisect_r05 bisect_a new; do
  d=$GRAFT_REPO_ROOT/$t; e=""
  case $t in new) d=$GRAFT_REPO_ROOT;; new_pnt0) d=$GRAFT_REPO_ROOT; e="AMG_PROLONG_NT=0";; esac
  (cd $d && env $e timeout -k 10 400 python3 tools/bench_dist_async.py --ranks 8 --cycles 8 > $O/d_${t}_$rep.json 2> $O/d_${t}_$rep.err) || { echo "$t failed"; tail -5 $O/d_${t}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/d_${t}_$rep.json').read().strip().splitlines()[-1])
print('[$t]', round(d['value'], 2), [r['level_finish_ms'] for r in d['runs']][0])"
done
done
