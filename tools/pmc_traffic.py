"""HBM traffic of the fine-grid residual kernel from rocprofv3 PMC passes.

FETCH_SIZE and WRITE_SIZE come from separate --pmc passes of tools/pmc_run.py.
On gfx950 FETCH_SIZE under-counts wide streaming reads (MI355X_MICROARCH.md,
HBM: 16-byte lanes are reported at one half), and other access widths are
uncalibrated, so the same run first streams 2 GiB with 16-, 8-, 4- and 1-byte
lanes and writes 2 GiB with 8-byte lanes: factor_w = reported / true bytes.

Residual kernel r = f - A u (one launch over the 512^3 fine grid):
  streams   col (16-byte lanes), value index or val (4- or 16-byte lanes),
            rowptr (4-byte lanes), f (8-byte lanes)          -> known bytes
  gather    x[col] (8-byte elements)                         -> unknown
  writes    r (8-byte lanes)
The gather's true bytes are what FETCH reports beyond the known streams,
divided by the 8-byte factor.  traffic = known reads + gather + writes.

usage: pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <n> <out.json>
"""
import csv
import json
import re
import sys
from collections import defaultdict

CAL = 2 << 30


def load(path):
    rows = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024.0)
    return rows


def pick(rows, pattern, grid=None):
    """per-dispatch values of kernels matching pattern; grid = rows of one launch
    (a dictionary-coded workgroup covers RPL 256-row tiles)"""
    out = []
    for (name, g), vals in rows.items():
        m = re.search(pattern, name)
        if not m:
            continue
        rpl = re.search(r"csr_(dc|rp|rpp)_kernel<\d, \w+, [\w:]+, (\d+)[,>]", name)
        mp = re.search(r"csr_mp_kernel<\d, \w+, [\w:]+, \d+, \w+, \d+, (\d+)>", name)
        # a paired-row-pattern or master-pattern lane owns two rows per slab
        if mp:
            rows_done = g * int(mp.group(1)) * 2
        else:
            rows_done = g * (int(rpl.group(2)) * (2 if rpl.group(1) == "rpp" else 1) if rpl else 1)
        if grid is None or rows_done == grid:
            out += vals
    return out


def main():
    fetch, write, n, out = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    fac = {}
    for w, pat in ((16, r"calib_read_k<16>"), (8, r"calib_read_k<8>"), (4, r"calib_read_k<4>"),
                   (1, r"calib_read_k<1>")):
        v = pick(fetch, pat)
        fac[f"read{w}"] = v[0] / CAL
    fac["write8"] = pick(write, r"calib_write8_k")[0] / CAL
    rows = n ** 3
    z = 7 * rows - 6 * n * n
    res = {}
    for fmt, vi in (("csr-mp", "mp"), ("csr-rpp", "rpp"), ("csr-rp", "rp"), ("csr-dc", "dc"), ("csr-vi", "true"), ("csr", "false")):
        pat = {"mp": r"csr_mp_kernel<1, false, amgk::EpiGemv,",
               "rpp": r"csr_rpp_kernel<1, false, amgk::EpiGemv,",
               "rp": r"csr_rp_kernel<1, false, amgk::EpiGemv,",
               "dc": r"csr_dc_kernel<1, false, amgk::EpiGemv,"}.get(
                   vi, r"csr_tile_kernel<.*>, 1, false, amgk::EpiGemv, %s" % vi)
        F = pick(fetch, pat, rows)
        W = pick(write, pat, rows)
        if not F or not W:
            continue
        Fm, Wm = sum(F) / len(F), sum(W) / len(W)
        # the paired kernel reads f with 16-byte lanes and one pattern byte per row pair
        if vi == "mp":
            vi = "rpp"  # same streams: f in 16-byte lanes, one pattern byte per row pair
        s16 = {"rpp": 8 * rows, "rp": 0, "dc": 0, "true": 4 * z, "false": 12 * z}[vi]
        s4 = {"rpp": 0, "rp": 0, "dc": 0, "true": z, "false": 0}[vi] + (
            0 if vi in ("rp", "rpp") else 4 * (rows + 1))
        s8 = (0 if vi == "rpp" else 8 * rows) + (z if vi == "dc" else 0)  # dictionary: 8-byte lanes
        s1 = {"rp": rows, "rpp": (rows + 1) // 2}.get(vi, 0)  # row-pattern bytes: one per lane
        known_rep = s16 * fac["read16"] + s4 * fac["read4"] + s8 * fac["read8"] + s1 * fac["read1"]
        gather = (Fm - known_rep) / fac["read8"]
        writes = Wm / fac["write8"]
        traffic = s16 + s4 + s8 + s1 + gather + writes
        alg = (rows + 24 * rows if vi == "rp" else (rows + 1) // 2 + 24 * rows if vi == "rpp" else
               {"dc": 1, "true": 5, "false": 12}[vi] * z + 28 * rows + 4)
        res[fmt] = {"fine_residual_bytes_per_launch": traffic, "alg_bytes_per_launch": alg,
                    "traffic_over_alg": traffic / alg, "fetch_size_raw": Fm, "write_size_raw": Wm,
                    "gather_bytes_est": gather, "gather_alg_bytes": 8 * rows, "launches": len(F)}
    doc = {str(n): {"factors": fac, **res,
                    "note": "FETCH_SIZE/WRITE_SIZE from separate rocprofv3 --pmc passes, corrected per "
                            "access width by calibration streams of known size (tools/pmc_traffic.py)"}}
    try:  # keep formats profiled earlier (other storage forms) for this n
        old = json.load(open(out))
        for k, v in old.get(str(n), {}).items():
            doc[str(n)].setdefault(k, v)
        for k, v in old.items():
            doc.setdefault(k, v)
    except (OSError, ValueError):
        pass
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
