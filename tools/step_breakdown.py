"""Per-step kernel timeline of a rocprofv3 kernel trace of bench.py: the
kernels between two consecutive outer-residual launches (one step), with
their durations, the step's wall span and its busy time."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "EpiResJacobi" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
seg = rows[a:b]
wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e6
print(f"step wall {wall:.3f} ms, busy {busy:.3f} ms, {len(seg)} kernels")
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void amgk::", "").replace("amgk::", "")[:64]
    print(f"  {d:8.1f} us  grid {int(r['Grid_Size_X']):>10}  {nm}")
