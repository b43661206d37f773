# long-row kernel forms: bitwise tests, then the elasticity r=6 V-cycle per
# form (AMG_LONG_FORM 0 / 1 / 2, AMG_LONG_XCD), interleaved, with rocprof
# kernel stats of each run
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06/long}
R=${2:-6}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_classical.py -x -q --timeout 200 --timeout-method thread -k "long_forms or elasticity_solve or classical_solve or matvec or residual or jacobi" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
for v in "AMG_LONG_FORM=0" "AMG_LONG_FORM=1" "AMG_LONG_FORM=2" "AMG_LONG_FORM=1 AMG_LONG_XCD=0"; do
  tag=$(echo "$v" | tr ' =' '_-')
  d=$O/p_${tag}_$rep
  env $v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/bench_elasticity.py --refine $R --steps 20 > $O/e_${tag}_$rep.json 2> $O/e_${tag}_$rep.err || { echo "variant $v failed"; tail -5 $O/e_${tag}_$rep.err; exit 1; }
  s=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$v" "$O/e_${tag}_$rep.json" "$s" <<'PY'
import csv, json, sys
v, bj, ks = sys.argv[1:4]
d = json.loads(open(bj).read().strip().splitlines()[-1])
rows = list(csv.DictReader(open(ks)))
out = sorted(((float(r["TotalDurationNs"]), r["Name"][:60], float(r["AverageNs"]) / 1e3, int(r["Calls"])) for r in rows), reverse=True)
print(f"[{v}] {d['it_per_s']:.1f} it/s {d['ms_per_step']:.3f} ms/step")
for t, n, a, c in out[:6]:
    print(f"   {t/1e6:8.2f} ms total {a:9.1f} us x{c:5d}  {n}")
PY
done
done
