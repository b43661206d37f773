# interleaved A/B of environment variants on the headline bench under
# rocprofv3 kernel stats: tools/gpu_r06_ab.sh OUT "ENV1" "ENV2" ...
# (each ENV a space-separated list of VAR=value, "-" for the default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$1; shift
mkdir -p $O
i=0
for rep in 1 2; do
for v in "$@"; do
  i=$((i+1))
  tag=$(echo "$v" | tr ' =' '_-')
  envs=""; [ "$v" != "-" ] && envs="$v"
  d=$O/p_${tag}_$rep
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0 --general 0 --spmv-reps 5 > $O/b_${tag}_$rep.json 2> $O/b_${tag}_$rep.err || { echo "variant $v failed"; tail -5 $O/b_${tag}_$rep.err; exit 1; }
  s=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$v" "$O/b_${tag}_$rep.json" "$s" <<'PY'
import csv, json, sys
v, bj, ks = sys.argv[1:4]
d = json.load(open(bj))
rows = list(csv.DictReader(open(ks)))
out = []
for r in rows:
    n = r["Name"]
    for key in ("csr_mz27", "mz_res_restrict", "csr_mz_kernel", "geo_prolong_march", "mz_sweep_outer"):
        if key in n:
            out.append((float(r["TotalDurationNs"]), n[:70], float(r["AverageNs"]) / 1e3, int(r["Calls"])))
out.sort(reverse=True)
print(f"[{v}] {d['value']:.1f} it/s {d['ms_per_step']:.3f} ms/step parity-free")
for t, n, a, c in out[:8]:
    print(f"   {a:9.1f} us x{c:4d}  {n}")
PY
done
done
