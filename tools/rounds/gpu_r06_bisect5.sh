# config 4 (512^3, 8 thread ranks on one GPU, DMEM async additive): round-5 tree against this tree
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r06/bisect5
mkdir -p $O
export AMG_LINK_TIMEOUT_S=120
for rep in 1 2; do
for t in bisect_r05 new; do
  d=$GRAFT_REPO_ROOT/$t; [ $t = new ] && d=$GRAFT_REPO_ROOT
  (cd $d && timeout -k 10 400 python3 tools/bench_dist_async.py --ranks 8 --cycles 8 > $O/d_${t}_$rep.json 2> $O/d_${t}_$rep.err) || { echo "$t failed"; tail -5 $O/d_${t}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/d_${t}_$rep.json').read().strip().splitlines()[-1])
print('[$t]', {k: v for k, v in d.items() if not isinstance(v, (list, dict))})"
done
done
