# config 3 (256^3 ASYNC_MULTADD hybrid JGS, composed transfers): the FULL_ASYNC
# update forms (AMG_ATOMIC_NORET 0 capture / 1 add-then-read / 2), interleaved,
# with kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06/atomic}
mkdir -p $O
for rep in 1 2; do
for v in 0 1 2; do
  d=$O/p_${v}_$rep
  AMG_ATOMIC_NORET=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/bench_async.py --transfers composed > $O/a_${v}_$rep.json 2> $O/a_${v}_$rep.err || { echo "variant $v failed"; tail -5 $O/a_${v}_$rep.err; exit 1; }
  python3 - $v $O/a_${v}_$rep.json $(find $d -name "*kernel_stats.csv" | head -1) <<'PY'
import csv, json, sys
v, bj, ks = sys.argv[1:4]
d = json.loads(open(bj).read().strip().splitlines()[-1])
print(f"[NORET={v}] async {d['async']['cycles_per_s']:.1f} sync {d['sync']['cycles_per_s']:.1f} cycles/s ratio {d['async_over_sync_speed']:.3f}")
rows = sorted(csv.DictReader(open(ks)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f"   {float(r['TotalDurationNs'])/1e6:8.2f} ms total {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>5} {r['Name'][:70]}")
PY
done
done
