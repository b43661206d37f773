"""HBM bytes per launch of the 512^3 fine-level kernels of a step (bench.py's
fine_kernels names) from the rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes
of tools/pmc_run.py, corrected by the calibration streams of the same run
(gfx950 FETCH_SIZE reports one half of the bytes read, WRITE_SIZE all of them:
tools/pmc_traffic.py).  Writes profiles/traffic.json[n]["kernels"][name].

usage: pmc_fine.py <fetch counter_collection.csv> <write counter_collection.csv> <n> <out.json>
"""
import json
import re
import sys

from pmc_traffic import CAL, load, pick

KERNELS = {
    # name in bench.fine_kernels: (kernel pattern, algorithmic bytes per launch as f(n))
    "outer_residual_sweep": (r"csr_mz_kernel<1, true, amgk::EpiResJacobi", lambda r: (r + 1) // 2 + 24 * r),
    "post_sweep": (r"csr_mz_kernel<1, true, amgk::EpiJacobi,", lambda r: (r + 1) // 2 + 24 * r),
    # + level 1's zero-guess sweep folded in: f_1, u_1 written, a_1 read (r / 8 rows each)
    "residual_restrict": (r"mz_res_restrict_kernel", lambda r: (r + 1) // 2 + 16 * r + 3 * r),
    "prolong_sweep": (r"mz_prolong_sweep", lambda r: (r + 1) // 2 + 24 * r + r),
    "prolong0": (r"geo_prolong_(march_)?k", lambda r: 16 * r + r),
}


def main():
    fetch, write, n, out = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    fr = pick(fetch, r"calib_read_k<16>")[0] / CAL
    fw = pick(write, r"calib_write8_k")[0] / CAL
    rows = n ** 3
    res = {}
    for name, (pat, alg) in KERNELS.items():
        # the fine-level launches: the largest grid of the pattern
        cand = [(g, v) for (k, g), v in fetch.items() if re.search(pat, k)]
        if not cand:
            continue
        g = max(c[0] for c in cand)
        F = [v for (k, gg), vals in fetch.items() if gg == g and re.search(pat, k) for v in vals]
        W = [v for (k, gg), vals in write.items() if gg == g and re.search(pat, k) for v in vals]
        if not F or not W:
            continue
        Fm, Wm = sum(F) / len(F), sum(W) / len(W)
        traffic = Fm / fr + Wm / fw
        a = alg(rows)
        res[name] = {"bytes_per_launch": traffic, "alg_bytes_per_launch": a, "traffic_over_alg": traffic / a,
                     "fetch_size_raw": Fm, "write_size_raw": Wm, "launches": len(F), "grid": g}
    try:
        doc = json.load(open(out))
    except (OSError, ValueError):
        doc = {}
    d = doc.setdefault(str(n), {})
    d.setdefault("kernels", {}).update(res)
    d["kernels_note"] = ("fine-level kernels of a 512^3 step: FETCH_SIZE / read factor + WRITE_SIZE / write "
                         f"factor (factors {fr:.4f} / {fw:.4f} from the run's calibration streams), "
                         "tools/pmc_fine.py")
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
