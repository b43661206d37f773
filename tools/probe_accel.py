"""Probe: async additive AMG with DMEM_ChebyUpdate for a few eigenvalue bounds
(one rank, RCCL transport).  Prints relres per (alpha, beta, accel, cheby_grid)."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_package  # noqa: E402
from oracle import pyoracle as O  # noqa: E402
from test_gpu_solve import hierarchy  # noqa: E402
from test_gpu_dist import split_host  # noqa: E402

amg = load_package()
_, L, host = hierarchy(amg, O, 24, amg.AMG_INTERP_LINEAR)
w = 0.8
Ps, Rs = [], []
for lev in range(L - 1):
    ps, rs_ = O.smooth_transfer(host["A"][lev], host["P"][lev], w)
    Ps.append(ps)
    Rs.append(rs_)
host = {"A": host["A"], "P": Ps, "R": Rs}
f = amg.rhs_rand(0, 24 ** 3)
rs, parts = split_host(host, ())
c = amg.Context(0, nstreams=L)
amg.dist.init_rccl(c, 1, 0, lambda b: b)
A, P, R = parts[0]
for solver in (amg.AMG_ASYNC_MULTADD, amg.AMG_ASYNC_AFACX):
    for (a, b) in ((0.05, 1.1), (0.2, 2.0), (0.2, 4.0), (0.5, 4.0), (0.1, 8.0), (0.5, 8.0)):
        mu, de = (b + a) / (b - a), 2 / (b + a)
        row = []
        for acc, grid in ((0, 0), (1, 0), (2, 0), (1, 1), (2, 1)):
            opts = amg.default_opts(solver=solver, smooth_weight=w, num_cycles=15, tol=0.0,
                                    accel_type=acc, cheby_mu=mu, cheby_delta=de, cheby_grid=grid)
            D = amg.dist.DistHier.from_parts(c, rs, A, P, R, opts)
            rel, _ = D.async_solve(f)
            D.free()
            row.append(rel)
        print(solver, a, b, " ".join(f"{x:.3e}" for x in row), flush=True)
amg.dist.finalize(c)
c.close()
