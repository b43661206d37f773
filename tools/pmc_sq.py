"""SQ / TCC counters per fine-level kernel of the 512^3 step (rocprofv3 --pmc
passes over tools/pmc_run.py), averaged over the kernel's launches at its
largest grid; several counter_collection.csv files (one per pass) merge by
kernel.  Derived, where the pass holds the counters:
  valu_per_wave, vmem_rd_per_wave, vmem_wr_per_wave, lds_per_wave  -- issue counts per wave;
  parked = SQ_WAIT_ANY / SQ_WAVE_CYCLES -- resident time parked on s_waitcnt / a barrier
           (memory latency not hidden);
  issue_stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES -- ready but not issued (pipe busy,
           dependency on an issued instruction);
  active = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES, active_valu = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
           (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES);
  valu_per_vmem = VALU instructions per vector-memory instruction;
  tcc_hit = TCC_HIT / (TCC_HIT + TCC_MISS); rdreq_32b = share of the L2's fabric read
           requests that are 32-byte; rdreq_dram = share that go to DRAM (the rest are
           served by the Infinity Cache).
(Round 5's first pass reported SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES as the wait share; that
counter is the issue stall, not the waitcnt wait -- see issue_stall / parked.)

usage: pmc_sq.py <counter_collection.csv>[,<more.csv>...] [out.json]
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
    out = {}
    for fi, path in enumerate(sys.argv[1].split(",")):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                d = (fi, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                meta[d] = (r["Kernel_Name"], int(r["Grid_Size"]))
    for name, pat in KERNELS.items():
        ds = [d for d, (k, g) in meta.items() if re.search(pat, k)]
        if not ds:
            continue
        gmax = max(meta[d][1] for d in ds)
        avg = defaultdict(float)
        for fi in sorted({d[0] for d in ds}):
            dd = [d for d in ds if d[0] == fi and meta[d][1] == gmax]
            for d in dd:
                for c, v in per[d].items():
                    avg[c] += v / len(dd)
        ds = [d for d in ds if meta[d][1] == gmax and d[0] == ds[0][0]]  # launches of one pass
        w = avg.get("SQ_WAVES", 0.0) or 1.0
        rec = {"launches": len(ds), "grid": gmax, "counters": dict(avg)}
        rec["valu_per_wave"] = avg.get("SQ_INSTS_VALU", 0.0) / w
        rec["vmem_rd_per_wave"] = avg.get("SQ_INSTS_VMEM_RD", 0.0) / w
        rec["vmem_wr_per_wave"] = avg.get("SQ_INSTS_VMEM_WR", 0.0) / w
        rec["lds_per_wave"] = avg.get("SQ_INSTS_LDS", 0.0) / w
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for key, c in (("parked", "SQ_WAIT_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"),
                           ("active", "SQ_ACTIVE_INST_ANY"), ("active_valu", "SQ_ACTIVE_INST_VALU")):
                if c in avg:
                    rec[key] = avg[c] / wc
        h, m = avg.get("TCC_HIT_sum"), avg.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m:
            rec["tcc_hit"] = h / (h + m)
        rq = avg.get("TCC_EA0_RDREQ_sum")
        if rq:
            if "TCC_EA0_RDREQ_32B_sum" in avg:
                rec["rdreq_32b"] = avg["TCC_EA0_RDREQ_32B_sum"] / rq
            if "TCC_EA0_RDREQ_DRAM_sum" in avg:
                rec["rdreq_dram"] = avg["TCC_EA0_RDREQ_DRAM_sum"] / rq
        vm = avg.get("SQ_INSTS_VMEM_RD", 0.0) + avg.get("SQ_INSTS_VMEM_WR", 0.0)
        if vm:
            rec["valu_per_vmem"] = avg.get("SQ_INSTS_VALU", 0.0) / vm
        out[name] = rec
    for name, rec in out.items():
        line = f"{name:22s} launches {rec['launches']:3d} grid {rec['grid']:>9}  VALU/wave {rec['valu_per_wave']:8.1f}"
        if rec["vmem_rd_per_wave"]:
            line += (f"  VMEM rd/wave {rec['vmem_rd_per_wave']:6.1f} wr/wave {rec['vmem_wr_per_wave']:5.1f}"
                     f"  LDS/wave {rec['lds_per_wave']:6.1f}  VALU/VMEM {rec.get('valu_per_vmem', 0):6.1f}")
        for key in ("parked", "issue_stall", "active", "active_valu", "tcc_hit", "rdreq_32b", "rdreq_dram"):
            if key in rec:
                line += f"  {key} {rec[key]:.3f}"
        print(line)
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
