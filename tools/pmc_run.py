"""Workload for the rocprofv3 --pmc passes (tools/rounds/gpu_r05_r.sh): PMC calibration
streams of known size per access width, then 512^3 V-cycles (default storage:
row-pattern-coded) and fine residuals of the same operator stored
dictionary-coded, value-indexed and as plain CSR.  tools/pmc_traffic.py reads
the counters."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402

amg = load_package()
lib = amg.lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
ctx = amg.Context(0, 4)
CAL = 2 << 30  # 2 GiB per calibration stream, far beyond the 256 MiB Infinity Cache
for mode in range(5):
    amg.check(lib.amg_pmc_calib(ctx.h, mode, CAL))
g = amg.Gen(n)
H = amg.build_hierarchy(ctx, g, amg.default_opts(smooth_weight=0.8, num_cycles=1 << 30, tol=0.0,
                                                  reuse_outer_residual=2))
f = ctx.vec(amg.rhs_rand(0, n ** 3))
H.solve_start(f, ctx.vec(n ** 3))
H.iterate(3)
ctx.sync()
H.free()
# dictionary-coded (row patterns off) fine residuals
ctx.set_row_pattern(0)
A0d = g.register(ctx, amg.AMG_GEN_A, 0)
xd = ctx.vec(np.random.default_rng(0).uniform(-1, 1, A0d.ncols))
yd = ctx.vec(A0d.nrows)
for _ in range(3):
    amg.smem.SMEM_Sync_SpGEMV(ctx, A0d, xd, f, -1.0, 1.0, yd)
ctx.sync()
A0d.free()
xd.free()
yd.free()
# value-indexed (dictionary off) fine residuals
ctx.set_dict_index(0)
A0v = g.register(ctx, amg.AMG_GEN_A, 0)
xv = ctx.vec(np.random.default_rng(0).uniform(-1, 1, A0v.ncols))
yv = ctx.vec(A0v.nrows)
for _ in range(3):
    amg.smem.SMEM_Sync_SpGEMV(ctx, A0v, xv, f, -1.0, 1.0, yv)
ctx.sync()
A0v.free()
ctx.set_value_index(0)
A0 = g.register(ctx, amg.AMG_GEN_A, 0)
x = ctx.vec(np.random.default_rng(0).uniform(-1, 1, A0.ncols))
y = ctx.vec(A0.nrows)
for _ in range(3):
    amg.smem.SMEM_Sync_SpGEMV(ctx, A0, x, f, -1.0, 1.0, y)
ctx.sync()
print(f"pmc workload done: n={n} nnz={A0.nnz}")
