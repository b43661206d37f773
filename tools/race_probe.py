"""Probe of the device's asynchronous race against the oracle's replay of its
recorded update order (tests/async_band.py replay_check): the z-slab async
solve at one rank, repeated, printing per run the device relres, the replay's
and the level finish times.  Usage: python tools/race_probe.py [--n 48] [--runs 6]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--cycles", type=int, default=12)
    ap.add_argument("--form", choices=("slab", "single"), default="slab")
    a = ap.parse_args()
    from conftest import load_package
    from oracle import pyoracle as oracle
    from async_band import timed_band, replay_tables, sliced_replay
    from test_gpu_slab_async import host_hier, slab_async
    amg = load_package()
    gen = amg.Gen(a.n)
    f = amg.rhs_rand(0, a.n ** 3)
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=a.cycles, tol=0.0,
                            smooth_transfer=1)
    host = host_hier(amg, oracle, gen)
    L = gen.L
    if a.form == "single":
        ctx = amg.Context(0, nstreams=L + 2)
        dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
        H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
        runs = []
        for _ in range(a.runs):
            u, rel, cnt = H.async_solve(f)
            runs.append((rel, cnt, u, [H.async_correction_ms()], [0, a.n ** 3]))
        H.free()
    else:
        runs = slab_async(amg, gen, opts, f, a.ranks, rccl1=True, runs=a.runs)
    for i, (rel, cnt, u, ms, rs) in enumerate(runs):
        if a.ranks > 1:
            rep = sliced_replay(amg, oracle, host, f, opts, ms, rs, composed=True)
        else:
            rep = timed_band(amg, oracle, host, f, opts, replay_tables(ms, L), composed=True)[0]
        t = ms[0]
        ev = sorted((float(x), k) for k in range(L) for x in t[k])
        gaps = [ev[q + 1][0] - ev[q][0] for q in range(len(ev) - 1) if ev[q + 1][1] != ev[q][1]]
        close = sum(1 for g in gaps if g < 0.005)
        print(f"run {i}: device {rel:.4e} replay {rep:.4e} ratio {rel / rep:.2f}; level finish ms "
              f"{[round(float(x[-1]), 3) if len(x) else 0 for x in t]}; cross-level update gaps < 5 us: "
              f"{close}/{len(gaps)}, min gap {min(gaps) * 1e3:.1f} us", flush=True)
    gen.free()


if __name__ == "__main__":
    main()
