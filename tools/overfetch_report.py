"""Post-sweep read traffic per march variant (tools/gpu_overfetch.sh output):
FETCH_SIZE of csr_mz_kernel<1, true, EpiJacobi> over its algorithmic reads
(f, u, the pattern byte per row pair), corrected by the run's 2 GiB read
calibration, the L2 hit rate, and the kernel time of the FETCH pass."""
import csv
import glob
import re
import sys
from collections import defaultdict


def load(path):
    rows = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return rows


def ktime(path, pat):
    ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(path))
          if re.search(pat, r["Kernel_Name"])]
    return sum(ds) / len(ds) / 1e3 if ds else float("nan")


root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/overfetch"
n = 512
rows = n ** 3
read_alg = (rows + 1) // 2 + 16 * rows
pat = r"csr_mz_kernel<1, true, amgk::EpiJacobi,"
print(f"{'variant':10s} {'reads/alg':>9s} {'reads GB':>9s} {'L2 hit':>7s} {'us':>7s}")
for d in sorted(glob.glob(f"{root}/*/fetch")):
    v = d.split("/")[-2]
    f = load(glob.glob(f"{d}/*counter_collection.csv")[0])
    h = load(glob.glob(f"{root}/{v}/hit/*counter_collection.csv")[0])
    cal = [x for (k, c), vals in f.items() if "calib_read" in k for x in vals][0] * 1024 / (2 << 30)
    sw = [x for (k, c), vals in f.items() if re.search(pat, k) for x in vals]
    fetch = sum(sw) / len(sw) * 1024 / cal
    hit = sum(x for (k, c), vals in h.items() if re.search(pat, k) and c.startswith("TCC_HIT") for x in vals)
    miss = sum(x for (k, c), vals in h.items() if re.search(pat, k) and c.startswith("TCC_MISS") for x in vals)
    us = ktime(glob.glob(f"{d}/*kernel_trace.csv")[0], pat)
    print(f"{v:10s} {fetch / read_alg:9.3f} {fetch / 1e9:9.2f} {hit / (hit + miss):7.3f} {us:7.1f}")
