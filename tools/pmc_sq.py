"""SQ instruction and wait counters per fine-level kernel of the 512^3 step
(a rocprofv3 --pmc pass over tools/pmc_run.py with SQ_WAVES, SQ_INSTS_VALU,
SQ_INSTS_VMEM_RD, SQ_INSTS_VMEM_WR, SQ_INSTS_LDS, SQ_WAIT_INST_ANY,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES (+ GRBM_GUI_ACTIVE)), averaged over the
kernel's launches at its largest grid.  Derived:
  valu_per_wave, vmem_rd_per_wave, vmem_wr_per_wave, lds_per_wave  -- issue counts per wave;
  wait_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES -- the share of the waves' resident time
              spent waiting on any dependency (memory, barrier, export): near 1 = latency /
              memory bound, low = issue bound;
  valu_per_vmem = VALU instructions per vector-memory instruction.

usage: pmc_sq.py <counter_collection.csv> [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict

KERNELS = {
    "outer_residual_sweep": r"csr_mz_kernel<1, true, amgk::EpiResJacobi",
    "post_sweep": r"csr_mz_kernel<1, true, amgk::EpiJacobi,",
    "residual_restrict": r"mz_res_restrict_kernel",
    "prolong0": r"geo_prolong_(march_)?k",
    "level1_post_sweep": r"csr_mz27_kernel<1, true, amgk::EpiJacobi",
    "level1_residual": r"csr_mz27_kernel<1, false, amgk::EpiGemv",
}


def main():
    per = defaultdict(dict)  # dispatch -> counter -> value
    meta = {}
    with open(sys.argv[1]) as fh:
        for r in csv.DictReader(fh):
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[d] = (r["Kernel_Name"], int(r["Grid_Size"]))
    out = {}
    for name, pat in KERNELS.items():
        ds = [d for d, (k, g) in meta.items() if re.search(pat, k)]
        if not ds:
            continue
        gmax = max(meta[d][1] for d in ds)
        ds = [d for d in ds if meta[d][1] == gmax]
        avg = defaultdict(float)
        for d in ds:
            for c, v in per[d].items():
                avg[c] += v / len(ds)
        w = avg.get("SQ_WAVES", 0.0) or 1.0
        rec = {"launches": len(ds), "grid": gmax, "counters": dict(avg)}
        rec["valu_per_wave"] = avg.get("SQ_INSTS_VALU", 0.0) / w
        rec["vmem_rd_per_wave"] = avg.get("SQ_INSTS_VMEM_RD", 0.0) / w
        rec["vmem_wr_per_wave"] = avg.get("SQ_INSTS_VMEM_WR", 0.0) / w
        rec["lds_per_wave"] = avg.get("SQ_INSTS_LDS", 0.0) / w
        if avg.get("SQ_WAVE_CYCLES"):
            rec["wait_frac"] = avg.get("SQ_WAIT_INST_ANY", 0.0) / avg["SQ_WAVE_CYCLES"]
        vm = avg.get("SQ_INSTS_VMEM_RD", 0.0) + avg.get("SQ_INSTS_VMEM_WR", 0.0)
        if vm:
            rec["valu_per_vmem"] = avg.get("SQ_INSTS_VALU", 0.0) / vm
        out[name] = rec
    for name, rec in out.items():
        print(f"{name:22s} launches {rec['launches']:3d} grid {rec['grid']:>9}  VALU/wave {rec['valu_per_wave']:8.1f}  "
              f"VMEM rd/wave {rec['vmem_rd_per_wave']:6.1f} wr/wave {rec['vmem_wr_per_wave']:5.1f}  "
              f"LDS/wave {rec['lds_per_wave']:6.1f}  VALU/VMEM {rec.get('valu_per_vmem', 0):6.1f}  "
              f"wait {rec.get('wait_frac', float('nan')):.3f}")
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
