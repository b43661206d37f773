#!/bin/bash
# round 5 (ar): kernel time of the elasticity r = 6 V-cycle by kernel
# (rocprofv3 kernel trace summary)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ar
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run \
   -- python3 $R/tools/bench_elasticity.py --refine 6 --steps 10 --warmup 2 > $O/e6.json 2> $O/e6.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
rm -f $(find $O/trace -name "*kernel_trace.csv")
s=$(find $O/trace -name "*kernel_stats.csv" | head -1)
python3 - "$s" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):7d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
PY
