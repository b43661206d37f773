"""Level-grouped asynchronous additive solve (DMEM_Add, csrc/amg_grid.cpp):
host transport against device-resident messages (amg_devhub), one MI355X.

One grid per level, one rank per grid, ranks as threads sharing the GPU; every
grid holds the whole n^3 problem.  Times amg_grid_add_solve (all ranks start
together behind a barrier; wall = the slowest rank's solve) for the host
transport (rendezvous mailboxes: each correction leaves the GPU by D2H and
comes back by H2D) and for the device hub (the receiver's kernel reads the
sender's slot in place).  Reports grid cycles per second (all grids' cycles
over the wall), the messages, and every grid's final relative residual.
The hierarchy uses smoothed transfers built on the host with the oracle's
SpGEMM, as tools/bench_async.py does (setup, not timed).

usage: python tools/bench_grid.py [--n 64] [--cycles 50] [--reps 3]
"""
import argparse
import json
import os
import sys
import threading
import time


ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--cycles", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    amg = load_package()
    from oracle import pyoracle as po
    from test_gpu_dist import run_ranks, split_host
    n, w = a.n, 0.8
    g = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    L = g.L
    A = [po.Csr(*g.host_csr(amg.AMG_GEN_A, l)) for l in range(L)]
    P = [po.Csr(*g.host_csr(amg.AMG_GEN_P, l)) for l in range(L - 1)]
    Ps, Rs = [], []
    for l in range(L - 1):
        p, r = po.smooth_transfer(A[l], P[l], w)
        Ps.append(p)
        Rs.append(r)
    host = {"A": A, "P": Ps, "R": Rs}
    f = amg.rhs_rand(0, n ** 3)
    ppg = (1,) * L
    rank_grid, rank_rows = amg.grid.layout(ppg, n ** 3)
    world = len(rank_grid)
    rs, parts = split_host(host, ())
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=w, tol=0.0, num_cycles=a.cycles,
                            max_inflight=2, converge_test_type=amg.AMG_LOCAL)
    out = {"config": {"workload": f"{n}^3 7-pt Laplacian, level-grouped ASYNC_MULTADD (DMEM_Add), "
                                  f"{L} grids x 1 rank (threads on one GPU), {a.cycles} cycles per grid, "
                                  "LOCAL convergence, max_inflight 2", "levels": L}}
    for transport in ("host", "device"):
        runs = []
        for rep in range(a.reps + 1):
            nb = amg.grid.ThreadNbHub(rank_grid) if transport == "host" else None
            dh = amg.grid.DevHub(rank_grid) if transport == "device" else None
            start = threading.Barrier(world)

            def rank(r):
                c = amg.Context(0, nstreams=2)
                # a one-rank grid: its intra-grid transport has no peers
                amg.dist.init_host(c, 1, 0, amg.dist.HostTransport(amg.dist.ThreadMailbox(1), 0))
                Ap, Pp, Rp = parts[0]
                D = amg.dist.DistHier.from_parts(c, rs, Ap, Pp, Rp, opts)
                G = amg.grid.GridAdd(dh if dh is not None else nb.transport(r), int(rank_grid[r]), world, r,
                                     rank_grid, rank_rows, dist_hier=D)
                c.sync()
                start.wait()
                t0 = time.perf_counter()
                x, cyc, rel, msgs = G.solve(f)
                dt = time.perf_counter() - t0
                G.free()
                D.free()
                amg.dist.finalize(c)
                c.close()
                return dt, cyc, rel, msgs
            res = run_ranks(world, rank)
            if dh is not None:
                dh.free()
            if rep:  # rep 0 warms up
                wall = max(r[0] for r in res)
                cyc = sum(r[1] for r in res)
                runs.append({"wall_ms": 1e3 * wall, "grid_cycles_per_s": cyc / wall,
                             "messages": int(sum(int(r[3][0]) for r in res)),
                             "rel": [float(r[2]) for r in res]})
            print(f"[grid] {transport} rep {rep}: {max(r[0] for r in res) * 1e3:.1f} ms", file=sys.stderr,
                  flush=True)
        best = max(runs, key=lambda r: r["grid_cycles_per_s"])
        out[transport] = {"best": best, "grid_cycles_per_s": [r["grid_cycles_per_s"] for r in runs]}
    out["device_over_host"] = out["device"]["best"]["grid_cycles_per_s"] / out["host"]["best"]["grid_cycles_per_s"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
