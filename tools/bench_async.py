"""Config 3 throughput: SMEM_Async_Add_AMG (ASYNC_MULTADD, hybrid JGS, FULL_ASYNC,
LOCAL residuals and convergence) on the 256^3 7-pt Laplacian, one MI355X.

Each level's correction loop runs on its own HIP stream (amg_async_solve).
Reports level corrections per second of the whole solve (every level performs
num_cycles corrections), the V-cycle-equivalent rate (num_cycles / wall), the
final relative residual, and -- beside it -- the synchronous MULTADD cycle
(sync_add_vcycle, one stream) with the same smoother and transfers, so the
overlap of the level streams shows as the ratio of the two.  The hierarchy
uses smoothed transfers P~ = (I - w D^-1 A) P (SMEM_Setup.cpp:244-261), built
here with the oracle's SpGEMM (setup, not timed).

usage: python tools/bench_async.py [--n 256] [--cycles 20] [--block 64] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--cycles", type=int, default=20)
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--smoother", default="hybrid")
    ap.add_argument("--transfers", default="explicit", choices=("explicit", "composed"),
                    help="smoothed transfers as explicit products (host SpGEMM) or composed on the device "
                         "(smooth_transfer = 1: R~ r = R (r - w A D^-1 r))")
    ap.add_argument("--graphs", type=int, default=0,
                    help="hipGraph replay of the level corrections / the sync cycle (amg_set_graphs)")
    a = ap.parse_args()
    amg = load_package()
    from oracle import pyoracle as po
    n, w = a.n, 0.8
    t0 = time.time()
    g = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    L = g.L
    A = [po.Csr(*g.host_csr(amg.AMG_GEN_A, l)) for l in range(L)]
    P = [po.Csr(*g.host_csr(amg.AMG_GEN_P, l)) for l in range(L - 1)]
    Ps, Rs = [], []
    if a.transfers == "composed":
        Ps = P
        Rs = [po.Csr(*g.host_csr(amg.AMG_GEN_R, l)) for l in range(L - 1)]
    else:
        for l in range(L - 1):
            p, r = po.smooth_transfer(A[l], P[l], w)
            Ps.append(p)
            Rs.append(r)
    print(f"[async] {L}-level smoothed hierarchy built in {time.time() - t0:.1f}s", file=sys.stderr)
    ctx = amg.Context(0, nstreams=16)
    ctx.set_graphs(a.graphs)
    dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v]
           for k, v in (("A", A), ("P", Ps), ("R", Rs))}
    sm = amg.AMG_HYBRID_JGS if a.smoother == "hybrid" else amg.AMG_JACOBI
    f = amg.rhs_rand(0, n ** 3)
    fv = ctx.vec(f)
    out = {"config": {"workload": f"{n}^3 7-pt Laplacian, ASYNC_MULTADD {a.smoother} "
                                  f"(blocks of {a.block} rows), FULL_ASYNC, LOCAL residual / convergence, "
                                  f"{a.cycles} corrections per level, smoothed linear transfers ({a.transfers})"
                                  f"{', hipGraph replay' if a.graphs else ''}",
                      "levels": L, "n": n}}
    for tag, solver in (("async", amg.AMG_ASYNC_MULTADD), ("sync", amg.AMG_MULTADD)):
        opts = amg.default_opts(solver=solver, smoother=sm, smooth_weight=w, num_cycles=a.cycles, tol=0.0,
                                num_threads=0, jgs_block_rows=a.block,
                                smooth_transfer=1 if a.transfers == "composed" else 0)
        H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
        times, rels = [], []
        for rep in range(a.reps + 1):
            ctx.sync()
            t1 = time.perf_counter()
            if tag == "async":
                _, rel, cnt = H.async_solve(fv)
            else:
                _, hist, k = H.solve(fv)
                rel = hist[k] / hist[0]
            ctx.sync()
            dt = time.perf_counter() - t1
            if rep:  # rep 0 warms up
                times.append(dt)
                rels.append(rel)
        H.free()
        best = min(times)
        corr = a.cycles * max(1, L - 1)
        out[tag] = {"seconds": best, "cycles_per_s": a.cycles / best, "level_corrections_per_s": corr / best,
                    "relres": rels, "times": times}
        print(f"[{tag}] {a.cycles} cycles in {best * 1e3:.1f} ms -> {a.cycles / best:.1f} cycles/s; "
              f"relres {rels}", file=sys.stderr)
    out["async_over_sync_speed"] = out["sync"]["seconds"] / out["async"]["seconds"]
    print(json.dumps(out))
    for v in dev.values():
        for M in v:
            M.free()
    ctx.close()


if __name__ == "__main__":
    main()
