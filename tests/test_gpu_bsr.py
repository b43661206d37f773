"""3x3 block form (bsr3_kernel) of the DMEM elasticity operator
(num_functions = 3, byVDIM; DMEM_BuildMatrix.cpp:442-719 restated in
csrc/amg_elasticity.cpp): which block rows block, and SpGEMV in every (alpha,
beta) branch, Jacobi / L1 Jacobi sweeps and row slices bit-identical to plain
CSR -- value-indexed blocks and fp64 blocks."""
import numpy as np
import pytest

from test_gpu_kernels import assert_bitwise, _vecs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def elast(amg):
    return {r: amg.classical.elasticity(r) for r in (2, 3)}


def reg(ctx, n, rp, cj, v, bsr=1, vi=1):
    ctx.set_bsr3(bsr)
    ctx.set_value_index(vi)
    try:
        return ctx.csr(n, n, rp, cj, v)
    finally:
        ctx.set_bsr3(2)
        ctx.set_value_index(1)


@pytest.mark.parametrize("form", [1, 2], ids=["lane-per-row", "lane-per-block-row"])
@pytest.mark.parametrize("r", [2, 3])
@pytest.mark.parametrize("vi", [1, 0])
def test_bsr3_bitwise(amg, oracle, ctx, elast, r, vi, form):
    """form 2 (amg_set_bsr3(ctx, 2)): value-indexed blocks walked one lane per
    block row (64-row slices); fp64 blocks keep form 1"""
    n, rp, cj, v, b = elast[r]
    Mb = reg(ctx, n, rp, cj, v, form, vi)
    Mp = reg(ctx, n, rp, cj, v, 0, 0)
    assert Mb.bsr3 == (1 if vi else 2) and Mp.bsr3 == 0
    assert amg.lib.amg_mat_bsr3_slice(Mb.h) == (64 if vi and form == 2 else 21)
    A = oracle.Csr(n, n, rp, cj, v)
    l1 = ctx.vec(oracle.l1_norms(A))
    x = ctx.vec(_vecs(n, 61))
    f = ctx.vec(_vecs(n, 62))
    outs = {}
    for tag, M in (("bsr", Mb), ("csr", Mp)):
        o = []
        for ab in ((1.0, 0.0), (-1.0, 1.0), (1.0, 1.0), (2.5, -0.5), (-1.0, 0.7)):
            y = ctx.vec(n)
            amg.smem.SMEM_SpGEMV(ctx, M, x, f, ab[0], ab[1], y, 0, n)
            o.append(y.download())
        # slice-aligned row ranges (63 / 192 rows: blocks) and others (CSR)
        for rb, re in ((63, 63 * (n // 63 - 1)), (126, n), (192, 192 * (n // 192 - 1)), (384, n), (3, n - 6),
                       (1, n - 2)):
            y = ctx.vec(_vecs(n, 63))
            amg.smem.SMEM_SpGEMV(ctx, M, x, f, -1.0, 1.0, y, rb, re)
            o.append(y.download())
        u = ctx.vec(_vecs(n, 64))
        amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, f, u, ctx.vec(n), 3, 0, 0.6)
        o.append(u.download())
        u = ctx.vec(_vecs(n, 65))
        amg.smem.SMEM_Sync_Parfor_L1Jacobi(ctx, M, f, u, ctx.vec(n), l1, 2, 1)
        o.append(u.download())
        outs[tag] = o
    for k, (g, ref) in enumerate(zip(outs["bsr"], outs["csr"])):
        assert_bitwise(g, ref, f"r={r} vi={vi} output {k}")
    Mb.free()
    Mp.free()


def test_bsr3_selection(amg, oracle, ctx, elast):
    """Scalar operators (7-pt) and row counts not divisible by 3 stay CSR."""
    A = oracle.laplace_7pt(12)  # 1728 rows, 7-entry rows
    M = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    assert M.bsr3 == 0
    M.free()
    n, rp, cj, v, b = elast[2]
    M = ctx.csr(n, n, rp, cj, v)
    assert M.bsr3 == 1
    M.free()
