#!/bin/bash
# round 5 (ao): kernel time of config 3's asynchronous additive cycle (composed
# transfers) by kernel, from a rocprofv3 kernel trace (summary only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run \
   -- python3 $R/tools/bench_async.py --transfers composed --reps 1 > $O/async3.json 2> $O/async3.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
rm -f $(find $O/trace -name "*kernel_trace.csv")
s=$(find $O/trace -name "*kernel_stats.csv" | head -1)
python3 - "$s" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):7d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
