"""Plane-marching kernel (csr_mz_kernel) for master-coded operators whose
master list is [0, -P, -S, -1, +1, +S, +P] (the reference's 7-pt Laplacian,
Laplacian_3D_7pt, on an nx*ny*nz box: S = nx, P = nx*ny): which operators take
it, and bit-identical results -- SpGEMV in every (alpha, beta) branch
(SMEM_MatVec.cpp:140-258), Jacobi / L1 Jacobi sweeps (SMEM_Smooth.cpp:35-45,
122-130), the fused outer residual + first sweep and its norm partials
(SMEM_Solve.cpp:192-197) -- against plain CSR, the non-marched master form and
the oracle, for every chunk length and workgroup order."""
import numpy as np
import pytest

from test_gpu_kernels import assert_bitwise, _vecs

pytestmark = pytest.mark.gpu


def neumann_7pt(oracle, nx, ny, nz):
    """7-pt operator with the diagonal = number of neighbours + 0.5 and
    anisotropic off-diagonals: the master list of the Laplacian, but per-pattern
    values (master-coded without uniform values)."""
    L = oracle.laplace_7pt(nx, ny, nz)
    val = L.val.copy()
    rows = np.repeat(np.arange(L.nrows), np.diff(L.rowptr))
    off = L.col.astype(np.int64) - rows
    val[off == 1] = val[off == -1] = -1.0
    val[np.abs(off) == nx] = -0.5
    val[np.abs(off) == nx * ny] = -0.25
    first = L.rowptr[:-1]
    cnt = np.diff(L.rowptr)
    s = np.add.reduceat(np.where(off == 0, 0.0, -val), first)
    val[first] = s + 0.5 * (cnt > 0)
    return oracle.Csr(L.nrows, L.ncols, L.rowptr, L.col, val)


def register(ctx, A, march=1, plain=False):
    ctx.set_plane_march(march)
    if plain:
        ctx.set_value_index(0)
    try:
        return ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    finally:
        ctx.set_plane_march(1)
        ctx.set_value_index(1)


@pytest.fixture(scope="module")
def boxes(oracle):
    return {
        "lap32": oracle.laplace_7pt(32),
        "lap64x8x5": oracle.laplace_7pt(64, 8, 5),
        "lap512x2x3": oracle.laplace_7pt(512, 2, 3),
        "lap512x6x5": oracle.laplace_7pt(512, 6, 5),
        "lap512x8x4": oracle.laplace_7pt(512, 8, 4),
        "neu32x16x7": neumann_7pt(oracle, 32, 16, 7),
    }


def test_plane_march_selection(ctx, oracle, boxes):
    want = {"lap32": 1024, "lap64x8x5": 512, "lap512x2x3": 1024, "lap512x6x5": 3072, "lap512x8x4": 4096,
            "neu32x16x7": 512}
    for name, A in boxes.items():
        M = register(ctx, A)
        assert M.plane_march == want[name], (name, M.plane_march)
        assert M.master_pattern == (-7 if name.startswith("lap") else 7), name
        M.free()
        M = register(ctx, A, march=0)
        assert M.plane_march == 0
        M.free()
    # planes of 256 rows (16^3), 13*7 rows (odd box): the master kernel
    for A in (oracle.laplace_7pt(16), oracle.laplace_7pt(13, 7, 5)):
        M = register(ctx, A)
        assert M.master_pattern == -7 and M.plane_march == 0
        M.free()


@pytest.mark.parametrize("lines", [1, 2, 4])
@pytest.mark.parametrize("zc,xcd", [(32, 1), (1, 0), (3, 1), (64, 0), (2, 1)])
@pytest.mark.parametrize("name", ["lap32", "lap64x8x5", "lap512x2x3", "lap512x6x5", "lap512x8x4", "neu32x16x7"])
def test_plane_march_bitwise(ctx, amg, boxes, name, zc, xcd, lines):
    A = boxes[name]
    ctx.set_plane_march(1, zc, xcd)
    ctx.set_march_lines(lines)
    try:
        mz = register(ctx, A)
        mp = register(ctx, A, march=0)
        pl = register(ctx, A, plain=True)
        assert mz.plane_march > 0 and mp.plane_march == 0 and pl.value_index == 0
        n = A.nrows
        x = ctx.vec(_vecs(n, 41))
        b = ctx.vec(_vecs(n, 42))
        outs = {}
        for tag, M in (("plain", pl), ("master", mp), ("march", mz)):
            o = []
            for ab in ((1.0, 0.0), (-1.0, 1.0), (1.0, 1.0), (2.5, -0.5), (-1.0, 0.7), (0.3, 0.0)):
                y = ctx.vec(n)
                amg.smem.SMEM_SpGEMV(ctx, M, x, b, ab[0], ab[1], y, 0, n)
                o.append(y.download())
            # a row slice runs the master kernel (the march needs whole planes)
            y = ctx.vec(_vecs(n, 43))
            amg.smem.SMEM_SpGEMV(ctx, M, x, b, -1.0, 1.0, y, 2, n - 4)
            o.append(y.download())
            u = ctx.vec(_vecs(n, 44))
            amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(n), 3, 0, 0.7)
            o.append(u.download())
            u = ctx.vec(_vecs(n, 45))
            amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(n), 2, 1, 0.8)
            o.append(u.download())
            outs[tag] = o
        for tag in ("master", "march"):
            for k, (g, r) in enumerate(zip(outs[tag], outs["plain"])):
                assert_bitwise(g, r, f"{name} zc={zc} {tag} output {k}")
        for M in (mz, mp, pl):
            M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)
        ctx.set_march_lines(1, gemv=2)


@pytest.mark.parametrize("zc", [32, 5])
@pytest.mark.parametrize("smoother", ["jacobi", "l1"])
def test_plane_march_solve(ctx, amg, oracle, smoother, zc):
    """SMEM_Solve on a 64^3 linear-interpolation hierarchy whose fine operator
    is marched: the fused outer residual + first sweep, the level-0 residual,
    the post-sweep; iterate bit-identical to the oracle after every cycle's
    worth (12 cycles), the residual-norm history bit-identical to the
    non-marched run (same per-tile partials) and to the oracle to 1e-12."""
    from oracle import pyoracle as po
    g = amg.Gen(64, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
            for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                              ("R", amg.AMG_GEN_R, g.L - 1))}
    sm = amg.AMG_JACOBI if smoother == "jacobi" else amg.AMG_L1_JACOBI
    f = amg.rhs_rand(0, 64 ** 3)
    res = {}
    ctx.set_plane_march(1, zc, 1)
    try:
        for march in (1, 0):
            ctx.set_plane_march(march)
            dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v]
                   for k, v in host.items()}
            assert (dev["A"][0].plane_march > 0) == bool(march)
            opts = amg.default_opts(smooth_weight=0.8, num_cycles=12, tol=0.0, reuse_outer_residual=2,
                                    smoother=sm)
            H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
            res[march] = H.solve(f)
            H.free()
            for v in dev.values():
                for M in v:
                    M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)
    OH = po.Hier(host["A"], host["P"], host["R"],
                 po.make_opts(smooth_weight=0.8, num_cycles=12, smoother=sm))
    u_cpu, hist_cpu, _ = OH.solve(f)
    u1, h1, k1 = res[1]
    u0, h0, k0 = res[0]
    assert k1 == k0 == 12
    assert_bitwise(u1, u_cpu, "iterate vs oracle")
    assert_bitwise(u1, u0, "iterate vs master kernel")
    assert_bitwise(h1[:k1 + 1], h0[:k0 + 1], "norm history vs master kernel")
    np.testing.assert_allclose(h1[:k1 + 1], hist_cpu[:k1 + 1], rtol=1e-12)


def _hier_solve(ctx, amg, host, f, cycles, march, fuse, sm=0, zc=16):
    ctx.set_plane_march(march, zc, 1)
    ctx.set_fuse_transfer(fuse)
    try:
        dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
        opts = amg.default_opts(smooth_weight=0.8, num_cycles=cycles, tol=0.0, reuse_outer_residual=2,
                                smoother=sm)
        H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
        fused = H.fused
        out = H.solve(f)
        H.free()
        for v in dev.values():
            for M in v:
                M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)
        ctx.set_fuse_transfer(1)
    return fused, out


@pytest.mark.parametrize("dims,zc", [((64, 64, 64), 16), ((512, 8, 6), 4), ((256, 12, 8), 2),
                                     ((128, 16, 10), 6), ((64, 32, 14), 64), ((64, 64, 64), 3)])
def test_fused_residual_restrict(ctx, amg, oracle, dims, zc):
    """Level-0 residual + restriction fused (mz_res_restrict_kernel) on the
    geometric linear-interpolation hierarchy of several boxes (lanes per coarse
    line 32..256, chunks of 1..32 coarse planes, a chunk length not dividing
    the plane count): the iterate bit-identical to the unfused run and to the
    oracle after 8 cycles, the norm history bit-identical to the unfused run."""
    from oracle import pyoracle as po
    g = amg.Gen(*dims, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
            for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                              ("R", amg.AMG_GEN_R, g.L - 1))}
    n = dims[0] * dims[1] * dims[2]
    f = amg.rhs_rand(0, n)
    fz, (u1, h1, k1) = _hier_solve(ctx, amg, host, f, 8, 1, 1, zc=zc)
    f0, (u0, h0, k0) = _hier_solve(ctx, amg, host, f, 8, 1, 0, zc=zc)
    assert fz & 3 == 3 and f0 == 0  # fused level 0, geometric R_0 / P_0
    OH = po.Hier(host["A"], host["P"], host["R"], po.make_opts(smooth_weight=0.8, num_cycles=8))
    u_cpu, hist_cpu, _ = OH.solve(f)
    assert_bitwise(u1, u0, "fused vs unfused iterate")
    assert_bitwise(u1, u_cpu, "fused vs oracle iterate")
    assert_bitwise(h1[:k1 + 1], h0[:k0 + 1], "norm history")
    np.testing.assert_allclose(h1[:k1 + 1], hist_cpu[:k1 + 1], rtol=1e-12)


@pytest.mark.parametrize("dims,zc", [((512, 8, 6), 4), ((512, 6, 10), 3), ((1024, 4, 6), 64)])
def test_march_two_lines_solve(ctx, amg, oracle, dims, zc):
    """Two lines per lane (csr_mz_kernel<..., 2>: +-S operands of the inner
    lines from registers) through whole solves: the fused outer residual + norm
    partials + first sweep and the post sweeps on 512- and 1024-wide boxes.
    Iterate and norm history bit-identical to one line per lane and to the
    oracle (iterate), 8 cycles."""
    from oracle import pyoracle as po
    g = amg.Gen(*dims, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
            for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                              ("R", amg.AMG_GEN_R, g.L - 1))}
    f = amg.rhs_rand(0, dims[0] * dims[1] * dims[2])
    out = {}
    for lines in (2, 1):
        ctx.set_march_lines(lines)
        try:
            _, out[lines] = _hier_solve(ctx, amg, host, f, 8, 1, 1, zc=zc)
        finally:
            ctx.set_march_lines(1, gemv=2)
    (u2, h2, k2), (u1, h1, k1) = out[2], out[1]
    OH = po.Hier(host["A"], host["P"], host["R"], po.make_opts(smooth_weight=0.8, num_cycles=8))
    u_cpu, hist_cpu, _ = OH.solve(f)
    assert k2 == k1 == 8
    assert_bitwise(u2, u1, "two lines vs one line iterate")
    assert_bitwise(h2[:k2 + 1], h1[:k1 + 1], "two lines vs one line norm history")
    assert_bitwise(u2, u_cpu, "two lines vs oracle iterate")


def test_fused_transfer_detection(ctx, amg, oracle):
    """Only the geometric form takes the geometric kernels (amg_hier_fused bit
    l + 1: level l's transfers, bit 0: level 0's fused residual + restriction):
    aggregation transfers, a perturbed R_0 value, a perturbed P_0 column and
    boxes whose planes are not marched (nx = 96) keep the CSR kernels."""
    from oracle import pyoracle as po

    def hier(g, tweak=None):
        host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
                for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                                  ("R", amg.AMG_GEN_R, g.L - 1))}
        if tweak:
            tweak(host)
        dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
        H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], amg.default_opts(num_cycles=1))
        fused = H.fused
        H.free()
        for v in dev.values():
            for M in v:
                M.free()
        return fused

    # 64^3: level 0 fused, geometric transfers on levels 0..3 (boxes 64..8;
    # the 4^3 level is below the check's interior row)
    assert hier(amg.Gen(64, interp=amg.AMG_INTERP_LINEAR)) == 0b11111
    # lines of 32: below the fused kernel's range, transfers still geometric
    assert hier(amg.Gen(32, interp=amg.AMG_INTERP_LINEAR)) == 0b1110
    assert hier(amg.Gen(64, interp=amg.AMG_INTERP_AGGREGATE)) == 0
    assert hier(amg.Gen(96, 8, 8, interp=amg.AMG_INTERP_LINEAR)) == 0

    def bump_r(host):
        R = host["R"][0]
        R.val[R.val.size // 2] *= 1.0000001

    def move_p(host):
        P = host["P"][0]
        r = (5 * 64 + 7) * 64 + 9  # fine (5, 7, 9): all odd, one entry
        i = P.rowptr[r]
        assert P.rowptr[r + 1] - i == 1
        P.col[i] = (P.col[i] + 1) % P.ncols

    assert hier(amg.Gen(64, interp=amg.AMG_INTERP_LINEAR), bump_r) == 0
    assert hier(amg.Gen(64, interp=amg.AMG_INTERP_LINEAR), move_p) == 0


def box_27pt(oracle, nx, ny, nz, per_pattern=True):
    """27-pt operator on an nx*ny*nz box, diagonal-first rows, the other entries
    ascending (the Galerkin coarse operators' CSR order).  per_pattern: the
    off-diagonal weights depend on (dz, dy, dx) and the row's boundary class
    (27 pair patterns, per-pattern values); else the uniform 26 / -1 stencil."""
    n = nx * ny * nz
    idx = np.arange(n)
    x, y, z = idx % nx, (idx // nx) % ny, idx // (nx * ny)
    cls = ((x == 0) | (x == nx - 1)).astype(int) + 2 * ((y == 0) | (y == ny - 1)) + 4 * ((z == 0) | (z == nz - 1))
    rows, cols, vals = [idx], [idx], [np.full(n, 26.0)]
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if dz == dy == dx == 0:
                    continue
                ok = (x + dx >= 0) & (x + dx < nx) & (y + dy >= 0) & (y + dy < ny) & (z + dz >= 0) & (z + dz < nz)
                w = -1.0 if not per_pattern else -(1.0 + 0.125 * abs(dz) + 0.25 * abs(dy) + 0.0625 * dx) * (1.0 + 0.5 * cls)
                w = np.broadcast_to(w, (n,))
                rows.append(idx[ok])
                cols.append((idx + dz * nx * ny + dy * nx + dx)[ok])
                vals.append(np.asarray(w)[ok])
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    v = np.concatenate(vals)
    # diagonal first, then ascending columns
    key = np.where(c == r, -1, c)
    order = np.lexsort((key, r))
    r, c, v = r[order], c[order], v[order]
    rowptr = np.zeros(n + 1, dtype=np.int32)
    np.add.at(rowptr, r + 1, 1)
    rowptr = np.cumsum(rowptr).astype(np.int32)
    return oracle.Csr(n, n, rowptr, c.astype(np.int32), v.astype(np.float64))


@pytest.fixture(scope="module")
def boxes27(oracle, amg):
    from oracle import pyoracle as po
    g = amg.Gen(64, interp=amg.AMG_INTERP_LINEAR)
    return {
        "galerkin32": po.Csr(*g.host_csr(amg.AMG_GEN_A, 1)),  # R A P of the 64^3 Laplacian
        "pat32x16x5": box_27pt(oracle, 32, 16, 5),
        "uni64x8x4": box_27pt(oracle, 64, 8, 4, per_pattern=False),
        "pat256x2x3": box_27pt(oracle, 256, 2, 3),
    }


def test_plane_march27_selection(ctx, oracle, boxes27):
    want = {"galerkin32": 1024, "pat32x16x5": 512, "uni64x8x4": 512, "pat256x2x3": 0}
    # below the pair-coding size (4M rows) a 27-pt operator keeps the pair /
    # master forms only when it marches; otherwise the row-pattern form
    for name, A in boxes27.items():
        M = register(ctx, A)
        assert abs(M.master_pattern) == (27 if want[name] else 0), (name, M.master_pattern)
        assert M.plane_march == want[name], (name, M.plane_march)
        assert M.march_points == (27 if want[name] else 0), name
        M.free()
    # planes of 256 rows: not marched
    M = register(ctx, box_27pt(oracle, 16, 16, 4))
    assert M.master_pattern == 0 and M.plane_march == 0 and M.row_pattern > 0
    M.free()
    # forced pair coding (pair_pattern 2): the master kernel
    ctx.set_pair_pattern(2)
    try:
        M = register(ctx, box_27pt(oracle, 16, 16, 4))
        assert abs(M.master_pattern) == 27 and M.plane_march == 0
        M.free()
    finally:
        ctx.set_pair_pattern(1)


@pytest.mark.parametrize("zc,xcd", [(16, 1), (1, 0), (3, 1), (64, 0)])
@pytest.mark.parametrize("name", ["galerkin32", "pat32x16x5", "uni64x8x4"])
def test_plane_march27_bitwise(ctx, amg, oracle, boxes27, name, zc, xcd):
    """csr_mz27_kernel: SpGEMV in every (alpha, beta) branch, Jacobi sweeps
    (zero-guess and not), bit-identical to plain CSR and the master kernel."""
    A = boxes27[name]
    ctx.set_plane_march(1, zc, xcd)
    try:
        mz = register(ctx, A)
        ctx.set_pair_pattern(2)
        try:
            mp = register(ctx, A, march=0)
        finally:
            ctx.set_pair_pattern(1)
        pl = register(ctx, A, plain=True)
        assert mz.march_points == 27 and mp.plane_march == 0 and abs(mp.master_pattern) == 27
        assert pl.value_index == 0
        n = A.nrows
        l1 = ctx.vec(oracle.l1_norms(A))
        x = ctx.vec(_vecs(n, 51))
        b = ctx.vec(_vecs(n, 52))
        outs = {}
        for tag, M in (("plain", pl), ("master", mp), ("march", mz)):
            o = []
            for ab in ((1.0, 0.0), (-1.0, 1.0), (1.0, 1.0), (2.5, -0.5), (-1.0, 0.7)):
                y = ctx.vec(n)
                amg.smem.SMEM_SpGEMV(ctx, M, x, b, ab[0], ab[1], y, 0, n)
                o.append(y.download())
            u = ctx.vec(_vecs(n, 54))
            amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(n), 3, 0, 0.7)
            o.append(u.download())
            u = ctx.vec(_vecs(n, 55))
            amg.smem.SMEM_Sync_Parfor_L1Jacobi(ctx, M, b, u, ctx.vec(n), l1, 2, 0)
            o.append(u.download())
            outs[tag] = o
        for tag in ("master", "march"):
            for k, (g, r) in enumerate(zip(outs[tag], outs["plain"])):
                assert_bitwise(g, r, f"{name} zc={zc} {tag} output {k}")
        for M in (mz, mp, pl):
            M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)


def test_plane_march27_hierarchy(ctx, amg):
    """The 64^3 linear-interpolation hierarchy marches its level-1 Galerkin
    operator with the 27-point kernel (test_plane_march_solve checks the solve
    bit for bit against the oracle with every level's kernels)."""
    g = amg.Gen(64, interp=amg.AMG_INTERP_LINEAR)
    A0 = g.register(ctx, amg.AMG_GEN_A, 0)
    A1 = g.register(ctx, amg.AMG_GEN_A, 1)
    assert A0.march_points == 7 and A1.march_points == 27
    A0.free()
    A1.free()


@pytest.mark.parametrize("dims,zc,sm,post,form", [((64, 64, 64), 16, "jacobi", 1, 2), ((512, 8, 6), 4, "l1", 1, 2),
                                                  ((128, 16, 10), 3, "jacobi", 2, 2), ((64, 32, 14), 64, "l1", 2, 2),
                                                  ((256, 12, 8), 2, "jacobi", 1, 2),
                                                  ((512, 8, 6), 4, "l1", 1, 1), ((512, 16, 12), 5, "jacobi", 1, 1),
                                                  ((512, 12, 10), 3, "l1", 2, 1), ((1024, 8, 6), 2, "jacobi", 1, 1),
                                                  ((512, 16, 12), 64, "jacobi", 2, 3), ((512, 6, 10), 3, "l1", 1, 3),
                                                  ((512, 8, 6), 4, "l1", 1, 4), ((512, 16, 12), 5, "jacobi", 1, 4),
                                                  ((512, 12, 10), 3, "jacobi", 2, 4), ((1024, 8, 6), 2, "jacobi", 1, 4),
                                                  ((512, 16, 12), 64, "l1", 2, 5), ((512, 8, 14), 3, "jacobi", 1, 5),
                                                  ((1024, 16, 6), 5, "l1", 1, 5), ((512, 16, 12), 5, "jacobi", 1, 6),
                                                  ((512, 8, 10), 3, "jacobi", 2, 7)])
def test_fused_prolong_sweep(ctx, amg, oracle, dims, zc, sm, post, form):
    """Prolongation + correction fused into the first post-smoothing sweep
    (SMEM_Sync_AMG.cpp:118-134): iterate and norm history bit-identical to the
    unfused run (geo_prolong_k + csr_mz_kernel) and the iterate to the oracle
    after 6 cycles; Jacobi and L1 Jacobi, one and two post sweeps, chunk
    lengths 2..64.  form 2: one line per lane (mz_prolong_sweep_kernel, lines
    of 64..512); 1 / 3: four / two lines per workgroup, each corrected value
    formed once (mz_prolong_sweep_nl_kernel, lines of 512 and 1024); 4 / 5: two /
    four lines per workgroup with the coarse correction from an LDS ring of
    coarse planes (mz_prolong_sweep_lds_kernel; odd chunk starts at zc 3 / 5);
    6 / 7: the two-line LDS form held to 5 / 6 waves per SIMD."""
    from oracle import pyoracle as po
    g = amg.Gen(*dims, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
            for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                              ("R", amg.AMG_GEN_R, g.L - 1))}
    n = dims[0] * dims[1] * dims[2]
    f = amg.rhs_rand(0, n)
    smoother = amg.AMG_JACOBI if sm == "jacobi" else amg.AMG_L1_JACOBI
    res = {}
    ctx.set_plane_march(1, zc, 1)
    try:
        for fp in (1, 0):
            ctx.set_fuse_prolong(form if fp else 0)
            dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
            opts = amg.default_opts(smooth_weight=0.8, num_cycles=6, tol=0.0, reuse_outer_residual=2,
                                    smoother=smoother, num_post_smooth_sweeps=post)
            H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
            res[fp] = (H.fused_prolong, H.solve(f))
            H.free()
            for v in dev.values():
                for M in v:
                    M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)
        ctx.set_fuse_prolong(0)
    (fp1, (u1, h1, k1)), (fp0, (u0, h0, k0)) = res[1], res[0]
    assert fp1 & 1 and fp0 == 0, (fp1, fp0)
    OH = po.Hier(host["A"], host["P"], host["R"],
                 po.make_opts(smooth_weight=0.8, num_cycles=6, smoother=smoother, num_post=post))
    u_cpu, hist_cpu, _ = OH.solve(f)
    assert_bitwise(u1, u0, "fused vs unfused iterate")
    assert_bitwise(u1, u_cpu, "fused vs oracle iterate")
    assert_bitwise(h1[:k1 + 1], h0[:k0 + 1], "norm history")
    np.testing.assert_allclose(h1[:k1 + 1], hist_cpu[:k1 + 1], rtol=1e-12)



@pytest.mark.parametrize("dims,zc,post,reuse,slab,sm", [((512, 8, 6), 4, 1, 2, 2, "jacobi"),
                                                         ((512, 16, 12), 3, 1, 2, 5, "jacobi"),
                                                         ((256, 8, 11), 64, 2, 2, 3, "l1"),
                                                         ((512, 2, 5), 1, 1, 1, 1, "jacobi"),
                                                         ((512, 6, 9), 5, 1, 1, 4, "l1"),
                                                         ((512, 4, 16), 16, 2, 2, 64, "jacobi")])
def test_slab_sweep_outer(ctx, amg, oracle, dims, zc, post, reuse, slab, sm):
    """fuse_outer 3: level 0's last post sweep and the outer residual + the next
    cycle's first sweep slab by slab over z (sweep 1 over a slab plus its z
    halo into a slab scratch, then the residual sweep of the slab; the
    Infinity-Cache form): iterate and norm history bit-identical to the
    unfused run and the iterate to the oracle, through amg_solve (u' stored)
    and iterate batches (u' only in a batch's last step); slabs of 1..64
    planes (one slab, ragged last slabs), Jacobi and L1 Jacobi, r stored or not."""
    from oracle import pyoracle as po
    g = amg.Gen(*dims, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
            for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                              ("R", amg.AMG_GEN_R, g.L - 1))}
    n = dims[0] * dims[1] * dims[2]
    f = amg.rhs_rand(0, n)
    smoother = amg.AMG_JACOBI if sm == "jacobi" else amg.AMG_L1_JACOBI
    res = {}
    ctx.set_plane_march(1, zc, 1)
    ctx.set_outer_slab(slab)
    try:
        for fo in (3, 0):
            ctx.set_fuse_outer(fo)
            dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
            opts = amg.default_opts(smooth_weight=0.8, num_cycles=6, tol=0.0, reuse_outer_residual=reuse,
                                    smoother=smoother, num_post_smooth_sweeps=post)
            H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
            sol = H.solve(f)
            fv, uv = ctx.vec(f), ctx.vec(np.zeros(n))
            r0 = H.solve_start(fv, uv)
            hist = [r0]
            for b in (2, 3, 1):
                H.iterate(b)
                hist.append(H.resnorm())
            H.get_u(uv)
            res[fo] = (H.fused_outer, sol, uv.download(), np.array(hist))
            H.free()
            for v in dev.values():
                for M in v:
                    M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)
        ctx.set_fuse_outer(0)
        ctx.set_outer_slab(32)
    (fo1, (u1, h1, k1), ui1, hi1), (fo0, (u0, h0, k0), ui0, hi0) = res[3], res[0]
    assert fo1 == 3 and fo0 == 0, (fo1, fo0)
    OH = po.Hier(host["A"], host["P"], host["R"],
                 po.make_opts(smooth_weight=0.8, num_cycles=6, smoother=smoother, num_post=post))
    u_cpu, hist_cpu, _ = OH.solve(f)
    assert_bitwise(u1, u0, "slab vs unfused iterate")
    assert_bitwise(u1, u_cpu, "slab vs oracle iterate")
    assert_bitwise(h1[:k1 + 1], h0[:k0 + 1], "norm history")
    np.testing.assert_allclose(h1[:k1 + 1], hist_cpu[:k1 + 1], rtol=1e-12)
    assert_bitwise(ui1, ui0, "slab vs unfused iterate (batches)")
    assert_bitwise(hi1, hi0, "slab vs unfused norm history (batches)")


@pytest.mark.parametrize("dims,zc,post,reuse,mode", [((512, 8, 6), 4, 1, 2, 1), ((512, 16, 12), 3, 1, 2, 2),
                                                      ((512, 6, 10), 64, 2, 2, 1), ((512, 2, 5), 1, 1, 1, 1),
                                                      ((512, 12, 9), 5, 1, 1, 2), ((512, 4, 16), 16, 2, 2, 2)])
def test_fused_sweep_outer(ctx, amg, oracle, dims, zc, post, reuse, mode):
    """Level 0's last post-smoothing sweep fused with the outer residual + the
    next cycle's first sweep (mz_sweep_outer_kernel: one march, u' never
    round-trips through HBM): iterate and norm history bit-identical to the
    unfused run (csr_mz_kernel<EpiJacobi> then csr_mz_kernel<EpiResJacobi>)
    and the iterate to the oracle, through amg_solve and through
    solve_start + iterate batches + get_u (mode 2 writes u' only in a batch's
    last step); chunks of 1..64 planes, one / two post sweeps, r stored or not."""
    from oracle import pyoracle as po
    g = amg.Gen(*dims, interp=amg.AMG_INTERP_LINEAR)
    host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
            for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                              ("R", amg.AMG_GEN_R, g.L - 1))}
    n = dims[0] * dims[1] * dims[2]
    f = amg.rhs_rand(0, n)
    res = {}
    ctx.set_plane_march(1, zc, 1)
    try:
        for fo in (mode, 0):
            ctx.set_fuse_outer(fo)
            dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
            opts = amg.default_opts(smooth_weight=0.8, num_cycles=6, tol=0.0, reuse_outer_residual=reuse,
                                    num_post_smooth_sweeps=post)
            H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
            sol = H.solve(f)
            # iterate batches of 2 + 3 + 1 (mode 2: u' materialised at each batch's end)
            fv, uv = ctx.vec(f), ctx.vec(np.zeros(n))
            r0 = H.solve_start(fv, uv)
            hist = [r0]
            for b in (2, 3, 1):
                H.iterate(b)
                hist.append(H.resnorm())
            H.get_u(uv)
            res[fo] = (H.fused_outer, sol, uv.download(), np.array(hist))
            H.free()
            for v in dev.values():
                for M in v:
                    M.free()
    finally:
        ctx.set_plane_march(1, -1, 1)
        ctx.set_fuse_outer(0)
    (fo1, (u1, h1, k1), ui1, hi1), (fo0, (u0, h0, k0), ui0, hi0) = res[mode], res[0]
    assert fo1 == mode and fo0 == 0, (fo1, fo0)
    OH = po.Hier(host["A"], host["P"], host["R"], po.make_opts(smooth_weight=0.8, num_cycles=6, num_post=post))
    u_cpu, hist_cpu, _ = OH.solve(f)
    assert_bitwise(u1, u0, "fused vs unfused iterate")
    assert_bitwise(u1, u_cpu, "fused vs oracle iterate")
    assert_bitwise(h1[:k1 + 1], h0[:k0 + 1], "norm history")
    assert_bitwise(ui1, ui0, "fused vs unfused iterate (iterate batches)")
    assert_bitwise(ui1, u_cpu, "fused iterate batches vs oracle")
    assert_bitwise(hi1, hi0, "norm history (iterate batches)")
    np.testing.assert_allclose(h1[:k1 + 1], hist_cpu[:k1 + 1], rtol=1e-12)
