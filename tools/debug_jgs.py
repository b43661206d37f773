import sys, os, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from conftest import load_package
amg = load_package()
from oracle import pyoracle as po
ctx = amg.Context(0, 4)
A = po.laplace_7pt(16)
dA = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
g = np.random.default_rng(0)
f = g.uniform(-1, 1, A.nrows); u = g.uniform(-1, 1, A.nrows)
for T in (1, 4):
    blk = po.partition_equal(A.nrows, T)
    for sweeps in (1, 2):
        for parfor in (False, True, False):
            ds = po.a_diag(A, 0.7)
            ru, rp = u.copy(), np.zeros(A.nrows)
            po.hybrid_jgs(A, f, ru, rp, blk, ds if parfor else None, 1.0, sweeps, 0, 0)
            du, dp = ctx.vec(u), ctx.vec(A.nrows)
            dds = ctx.vec(ds)
            if parfor:
                amg.smem.SMEM_Sync_Parfor_HybridJacobiGaussSeidel(ctx, dA, ctx.vec(f), du, dp, blk, dds, sweeps, 0, 0)
            else:
                amg.smem.SMEM_Sync_HybridJacobiGaussSeidel(ctx, dA, ctx.vec(f), du, dp, sweeps, 0, blk, 0)
            gu = du.download(); gp = dp.download()
            bad = np.nonzero(gu != ru)[0]
            print(f"T={T} sweeps={sweeps} parfor={parfor}: mismatches={bad.size} first={bad[:3]} uprev_ok={np.array_equal(gp, rp)}")
            if bad.size:
                i = bad[0]
                print("   gpu", gu[i:i+3], "ref", ru[i:i+3], "u0", u[i:i+3])
