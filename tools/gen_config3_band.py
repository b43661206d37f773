"""Oracle band fixture for config 3 (tests/golden/config3_band.json): the
256^3 7-pt Laplacian, 8-level linear Galerkin hierarchy with the explicit
smoothed transfers (oracle.smooth_transfer, SMEM_Setup.cpp:244-261), ASYNC_MULTADD
with hybrid JGS (blocks of 64 rows), FULL_ASYNC, READ_SOL, LOCAL, N corrections
per level.  or_async_add (SMEM_Async_Add_AMG restated on OpenMP thread groups)
runs `reps` times with one thread per level and `reps` times with two; the
synchronous MULTADD cycle's relres is stored beside it.  The runs are races, so
the fixture records a sample of the oracle's outcomes on this container's cores
(8 CPUs); tests/test_gpu_configs.py checks the device's runs against
[0.5 min, 2 max] of it.  usage: python tools/gen_config3_band.py [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--n", type=int, default=256)
    a = ap.parse_args()
    from conftest import load_package
    from oracle import pyoracle as oracle
    amg = load_package()
    n, w, N, B = a.n, 0.8, 8, 64
    g = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    L = g.L
    A = [oracle.Csr(*g.host_csr(amg.AMG_GEN_A, l)) for l in range(L)]
    P = [oracle.Csr(*g.host_csr(amg.AMG_GEN_P, l)) for l in range(L - 1)]
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(A[lev], P[lev], w)
        Ps.append(ps)
        Rs.append(rs)
    f = amg.rhs_rand(0, n ** 3)
    opts = oracle.make_opts(solver=oracle.OR_MULTADD, smoother=oracle.OR_HYBRID_JGS, smooth_weight=w,
                            num_cycles=N, tol=0.0)
    OH = oracle.Hier(A, Ps, Rs, opts)
    for lev in range(L):
        nr = A[lev].nrows
        OH.set_blocks(lev, np.unique(np.minimum(np.arange(0, nr + B, B), nr)).astype(np.int32))
    _, h, _ = OH.solve(f)
    sync_rel = float(h[-1] / h[0])
    aopts = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smoother=oracle.OR_HYBRID_JGS, smooth_weight=w,
                             num_cycles=N, tol=0.0)
    OA = oracle.Hier(A, Ps, Rs, aopts)
    for lev in range(L):
        nr = A[lev].nrows
        OA.set_blocks(lev, np.unique(np.minimum(np.arange(0, nr + B, B), nr)).astype(np.int32))
    runs = {}
    for tpl in (1, 2):
        rels = []
        for r in range(a.reps):
            t0 = time.time()
            u, rel, cnt = OA.async_add(f, [tpl] * L)
            assert np.all(np.isfinite(u)) and list(cnt[:L - 1]) == [N] * (L - 1)
            rels.append(float(rel))
            print(f"threads/level {tpl} run {r}: relres {rel:.6e} ({time.time() - t0:.1f}s)", file=sys.stderr,
                  flush=True)
        runs[str(tpl)] = rels
    out = {"n": n, "levels": L, "num_cycles": N, "smooth_weight": w, "jgs_block_rows": B,
           "solver": "ASYNC_MULTADD", "smoother": "hybrid JGS", "async_type": "FULL_ASYNC",
           "read_type": "READ_SOL", "res_compute": "LOCAL", "converge": "LOCAL",
           "transfers": "explicit smoothed (oracle.smooth_transfer)", "rhs": "rhs_rand(0)",
           "threads_per_level_runs": runs, "sync_multadd_relres": sync_rel,
           "host": f"{os.cpu_count()} CPUs", "generator": "tools/gen_config3_band.py"}
    path = os.path.join(ROOT, "tests", "golden", "config3_band.json")
    json.dump(out, open(path, "w"), indent=1)
    allr = [x for v in runs.values() for x in v]
    print(f"band [{min(allr):.4e}, {max(allr):.4e}] width {max(allr) / min(allr):.2f}x, sync {sync_rel:.4e}",
          file=sys.stderr)


if __name__ == "__main__":
    main()
