"""The optional MI355X scheduling knobs, each bit-identical to the default
path: the plane marches' prefetch distance and occupancy-sized chunks
(amg_set_march_tuning; 7-pt and 27-pt) and the hipGraph replay of the
additive cycles' launch-bound loops (amg_set_graphs)."""
import numpy as np
import pytest

from async_band import blocks64
from test_gpu_kernels import _vecs, assert_bitwise
from test_gpu_march import boxes, boxes27, register  # noqa: F401  (fixtures)
from test_gpu_solve import gpu_hier, hierarchy, oracle_opts

pytestmark = pytest.mark.gpu

W = 0.8


@pytest.mark.parametrize("tune", [(2, 2, -1, -1), (1, 1, 0, 0), (2, 1, 3, 5), (3, 2, -1, -1)],
                         ids=["pf2-occ", "pf1-off", "mixed", "halo-pf"])
@pytest.mark.parametrize("name", ["lap64x8x5", "lap512x8x4", "neu32x16x7"])
def test_march_tuning_bitwise(ctx, amg, boxes, name, tune):
    """the 7-pt march's scheduling knobs (prefetch distance, halo operands two
    planes ahead, occupancy-sized chunks; amg_set_march_tuning) change only who
    computes which plane: SpGEMV
    and Jacobi outputs bit-identical to plain CSR"""
    A = boxes[name]
    ctx.set_plane_march(1, -1, 1)
    ctx.set_march_tuning(*tune)
    try:
        mz = register(ctx, A)
        pl = register(ctx, A, plain=True)
        n = A.nrows
        x = ctx.vec(_vecs(n, 61))
        b = ctx.vec(_vecs(n, 62))
        for lines in (1, 2):
            ctx.set_march_lines(lines)
            for ab in ((1.0, 0.0), (-1.0, 1.0)):
                ys = []
                for M in (pl, mz):
                    y = ctx.vec(n)
                    amg.smem.SMEM_SpGEMV(ctx, M, x, b, ab[0], ab[1], y, 0, n)
                    ys.append(y.download())
                assert_bitwise(ys[1], ys[0], f"{name} {tune} lines {lines} spgemv {ab}")
            us = []
            for M in (pl, mz):
                u = ctx.vec(_vecs(n, 63))
                amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(n), 3, 0, 0.7)
                us.append(u.download())
            assert_bitwise(us[1], us[0], f"{name} {tune} lines {lines} jacobi")
        mz.free()
        pl.free()
    finally:
        ctx.set_march_tuning(3, 2, 0, -1)  # the defaults
        ctx.set_march_lines(1, gemv=2)


@pytest.mark.parametrize("tune", [(1, 1, 0, 0), (1, 2, 0, 3), (1, 2, 0, -1)], ids=["pf1-off", "pf2-occ3", "pf2-auto"])
@pytest.mark.parametrize("name", ["galerkin32", "uni64x8x4"])
def test_march27_tuning_bitwise(ctx, amg, oracle, boxes27, name, tune):
    """the 27-pt march's prefetch distance and occupancy-sized chunks: SpGEMV
    and Jacobi bit-identical to plain CSR"""
    A = boxes27[name]
    ctx.set_plane_march(1, -1, 1)
    ctx.set_march_tuning(*tune)
    try:
        mz = register(ctx, A)
        pl = register(ctx, A, plain=True)
        assert mz.march_points == 27
        n = A.nrows
        x = ctx.vec(_vecs(n, 71))
        b = ctx.vec(_vecs(n, 72))
        for ab in ((1.0, 0.0), (-1.0, 1.0), (2.5, -0.5)):
            ys = []
            for M in (pl, mz):
                y = ctx.vec(n)
                amg.smem.SMEM_SpGEMV(ctx, M, x, b, ab[0], ab[1], y, 0, n)
                ys.append(y.download())
            assert_bitwise(ys[1], ys[0], f"{name} {tune} spgemv {ab}")
        us = []
        for M in (pl, mz):
            u = ctx.vec(_vecs(n, 73))
            amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(n), 3, 0, 0.7)
            us.append(u.download())
        assert_bitwise(us[1], us[0], f"{name} {tune} jacobi")
        mz.free()
        pl.free()
    finally:
        ctx.set_march_tuning(3, 2, 0, -1)  # the defaults


@pytest.mark.parametrize("mode", ["async-jacobi-s3", "async-hybrid-s1", "sync"])
def test_graphs_bitwise(amg, oracle, ctx, mode):
    """hipGraph replay of the additive cycles (amg_set_graphs): every level's
    correction captured after its first eager run and replayed (async), the
    whole synchronous additive cycle likewise -- the iterate is the oracle's
    bit for bit, over two solves (the second replays graphs made by the first)"""
    n = 64
    _, L, host = hierarchy(amg, oracle, n, amg.AMG_INTERP_LINEAR)
    f = amg.rhs_rand(0, n ** 3)
    sm = amg.AMG_HYBRID_JGS if "hybrid" in mode else amg.AMG_JACOBI
    sched = int(mode[-1]) if mode != "sync" else 0
    opts = amg.default_opts(solver=amg.AMG_MULTADD if mode == "sync" else amg.AMG_ASYNC_MULTADD, smoother=sm,
                            smooth_weight=W, num_cycles=6, tol=0.0, num_threads=0, jgs_block_rows=64,
                            async_schedule=sched, smooth_transfer=1)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    OH.set_composed_transfers()
    if sm == amg.AMG_HYBRID_JGS:
        for lev, blk in blocks64(host).items():
            OH.set_blocks(lev, blk)
    if mode == "sync":
        uo, ho, _ = OH.solve(f)
    else:
        oracle.lib().or_set_async_schedule(sched)
        try:
            uo, relo, _ = OH.async_add(f, [1] * L)
        finally:
            oracle.lib().or_set_async_schedule(0)
    ctx.set_graphs(1)
    try:
        H, _ = gpu_hier(amg, ctx, host, opts)
        for rep in range(2):
            if mode == "sync":
                u, hist, k = H.solve(f)
                np.testing.assert_allclose(hist, ho, rtol=1e-12, atol=0)
            else:
                u, rel, cnt = H.async_solve(f)
                assert abs(rel - relo) <= 1e-12 * relo
            nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
            print(f"graphs {mode} solve {rep}: differing entries {nd}")
            assert nd == 0
        H.free()
    finally:
        ctx.set_graphs(0)


@pytest.mark.parametrize("nranks,sched", [(2, 3), (1, 1)])
def test_slab_fused_prolong_bitwise(amg, oracle, ctx, monkeypatch, nranks, sched):
    """the slab async solve's level-0 composed prolongation and atomic
    correction as one fused march (AMG_FUSE_XFP_SLAB=1; level-1 ghost planes
    over the level channels): under a deterministic schedule the 64^3
    iterate is the oracle's bit for bit"""
    from test_gpu_slab_async import test_slab_async_schedule_bitwise
    monkeypatch.setenv("AMG_FUSE_XFP_SLAB", "1")
    test_slab_async_schedule_bitwise(amg, oracle, ctx, "multadd", True, nranks, sched, 64)


@pytest.mark.parametrize("name", ["galerkin32", "pat32x16x5", "uni64x8x4"])
def test_march27_lds_ring_bitwise(ctx, amg, oracle, boxes27, name):
    """the 27-pt march's LDS plane-ring form (csr_mz27l_kernel, march tuning
    mz27_pf = 3): SpGEMV in three branches, weighted and L1 Jacobi, bit-identical
    to plain CSR -- dominant, x-edge and masked (boundary-pattern) rows"""
    A = boxes27[name]
    ctx.set_plane_march(1, -1, 1)
    ctx.set_march_tuning(3, 3, 0, -1)
    try:
        mz = register(ctx, A)
        pl = register(ctx, A, plain=True)
        assert mz.march_points == 27
        n = A.nrows
        x = ctx.vec(_vecs(n, 81))
        b = ctx.vec(_vecs(n, 82))
        l1 = ctx.vec(oracle.l1_norms(A))
        for ab in ((1.0, 0.0), (-1.0, 1.0), (2.5, -0.5)):
            ys = []
            for M in (pl, mz):
                y = ctx.vec(n)
                amg.smem.SMEM_SpGEMV(ctx, M, x, b, ab[0], ab[1], y, 0, n)
                ys.append(y.download())
            assert_bitwise(ys[1], ys[0], f"{name} spgemv {ab}")
        for l1j in (False, True):
            us = []
            for M in (pl, mz):
                u = ctx.vec(_vecs(n, 83))
                if l1j:
                    amg.smem.SMEM_Sync_Parfor_L1Jacobi(ctx, M, b, u, ctx.vec(n), l1, 2, 0)
                else:
                    amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(n), 3, 0, 0.7)
                us.append(u.download())
            assert_bitwise(us[1], us[0], f"{name} {'l1 ' if l1j else ''}jacobi")
        mz.free()
        pl.free()
    finally:
        ctx.set_march_tuning(3, 2, 0, -1)  # the defaults


@pytest.mark.parametrize("zc", [-1, 3])
def test_march27_lds_ring_solve(ctx, amg, oracle, zc):
    """SMEM_Solve on a hierarchy whose fine operator is 27-pt (levels 1.. of the
    64^3 linear hierarchy): the outer residual + first sweep with its norm
    partials, the residuals and sweeps all through the LDS plane ring; iterate
    and norm history bit-identical to the register-march run, iterate to the
    oracle"""
    from oracle import pyoracle as po
    g = amg.Gen(64, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(lo, cnt)]
            for w, c, lo, cnt in (("A", amg.AMG_GEN_A, 1, g.L), ("P", amg.AMG_GEN_P, 1, g.L - 1),
                                  ("R", amg.AMG_GEN_R, 1, g.L - 1))}
    f = amg.rhs_rand(0, host["A"][0].nrows)
    res = {}
    ctx.set_plane_march(1, zc, 1)
    try:
        for pf in (3, 2):
            ctx.set_march_tuning(3, pf, 0, -1)
            dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
            assert dev["A"][0].march_points == 27
            opts = amg.default_opts(smooth_weight=0.8, num_cycles=8, tol=0.0, reuse_outer_residual=2)
            H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
            res[pf] = H.solve(f)
            H.free()
            for v in dev.values():
                for M in v:
                    M.free()
    finally:
        ctx.set_march_tuning(3, 2, 0, -1)
        ctx.set_plane_march(1, -1, 1)
    (u3, h3, k3), (u2, h2, k2) = res[3], res[2]
    assert_bitwise(u3, u2, "lds ring vs register march iterate")
    assert_bitwise(np.asarray(h3[:k3 + 1]), np.asarray(h2[:k2 + 1]), "norm history")
    OH = po.Hier(host["A"], host["P"], host["R"], po.make_opts(smooth_weight=0.8, num_cycles=8))
    u_cpu, _, _ = OH.solve(f)
    assert_bitwise(u3, u_cpu, "lds ring vs oracle iterate")
