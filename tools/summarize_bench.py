"""One-line summaries of the JSON outputs of a measurement batch
(tools/rounds/gpu_r05_r.sh): bench.py lines (it/s, ms per step, the fine kernels'
fractions of peak, the parity leg), bench_async.py (async / sync cycles/s) and
bench_dist_async.py (additive cycles/s, relres).  usage:
summarize_bench.py <dir with *.json>"""
import glob
import json
import os
import sys


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    return None


for p in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = last_json(p)
    except Exception as e:  # a truncated run
        print(f"{os.path.basename(p)}: unreadable ({e})")
        continue
    name = os.path.basename(p)
    if d is None:
        print(f"{name}: no JSON line")
    elif "fine_kernels" in d:
        fk = ", ".join(f"{k} {v['ms'] * 1e3:.0f} us ({v['frac']:.2f})" for k, v in d["fine_kernels"].items())
        par = d.get("parity") or {}
        print(f"{name}: {d['value']:.1f} it/s, {d['ms_per_step']:.3f} ms/step; fine SpMV {d['fine_spmv']['ms'] * 1e3:.0f} us "
              f"({d['fine_spmv']['frac']:.3f}); {fk}; bitwise {par.get('iterate_bitwise')}; "
              f"cpu {((d.get('cpu_baseline') or {}).get('value'))}")
    elif "async" in d and "sync" in d:
        print(f"{name}: async {d['async']['cycles_per_s']:.1f} cycles/s, sync {d['sync']['cycles_per_s']:.1f}, "
              f"ratio {d['async_over_sync_speed']:.2f}; relres async {min(d['async']['relres']):.3e} "
              f"sync {d['sync']['relres'][0]:.3e}")
    elif "runs" in d:
        r = max(d["runs"], key=lambda q: q["cycles_per_s"])
        print(f"{name}: {d['value']:.1f} additive cycles/s ({d['ranks']} rank(s)), relres {r['relres']:.3e}, "
              f"level finish ms {r['level_finish_ms']}")
    else:
        print(f"{name}: {list(d)[:6]}")
