"""Per-dispatch PMC values from a rocprofv3 SQLite output (run_results.db):
prints dispatch id, kernel (short), grid size, duration and each counter."""
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    names = {r[0]: r[1] for r in cur.execute("select id, name from rocpd_info_pmc")}
    ksym = {r[0]: r[1] for r in cur.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    vals = defaultdict(dict)
    for ev, pmc, v in cur.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        vals[ev][names.get(pmc, pmc)] = vals[ev].get(names.get(pmc, pmc), 0) + v
    out = []
    for did, kid, st, en, gx, ev in cur.execute(
            "select dispatch_id, kernel_id, start, end, grid_size_x, event_id from rocpd_kernel_dispatch "
            "order by dispatch_id"):
        out.append((did, ksym.get(kid, "?"), gx, (en - st) * 1e-6, vals.get(ev, {})))
    return out


if __name__ == "__main__":
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for did, k, gx, ms, v in rows(sys.argv[1]):
        if filt in k:
            print(did, k[:60], gx, f"{ms:.3f}ms", {a: f"{b:.4g}" for a, b in v.items()})
