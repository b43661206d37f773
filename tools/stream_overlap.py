"""Concurrency of the level streams in a rocprofv3 kernel trace: over the
window of the last amg_async_solve (the kernels between the first and last
atomic_correct_k of the final run), the sum of kernel durations divided by
the union of their intervals (1.0 = strictly serial), the peak number of
kernels in flight, and the distinct hardware queues used.

usage: stream_overlap.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ac = [i for i, r in enumerate(rows) if "atomic_correct_k" in r["Kernel_Name"]]
if not ac:
    sys.exit("no atomic_correct_k in the trace")
# the last async solve: walk back from the last atomic_correct to a gap > 5 ms
end = ac[-1]
start = end
while start > 0 and int(rows[start]["Start_Timestamp"]) - int(rows[start - 1]["End_Timestamp"]) < 5_000_000:
    start -= 1
seg = rows[start:end + 1]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg]
tot = sum(b - a for a, b in iv)
union, cur_a, cur_b = 0, None, None
ev = []
for a, b in iv:
    ev += [(a, 1), (b, -1)]
    if cur_b is None or a > cur_b:
        if cur_b is not None:
            union += cur_b - cur_a
        cur_a, cur_b = a, b
    else:
        cur_b = max(cur_b, b)
union += cur_b - cur_a
depth = peak = 0
for _, d in sorted(ev):
    depth += d
    peak = max(peak, depth)
qkey = "Queue_Id" if "Queue_Id" in seg[0] else None
queues = sorted({r[qkey] for r in seg}) if qkey else []
wall = iv[-1][1] - iv[0][0]
print(f"kernels {len(seg)}, wall {wall / 1e6:.3f} ms, busy-union {union / 1e6:.3f} ms, "
      f"sum of durations {tot / 1e6:.3f} ms, concurrency {tot / max(union, 1):.2f}, peak in flight {peak}, "
      f"hardware queues {queues}")
