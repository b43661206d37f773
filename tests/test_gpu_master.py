"""Master-pattern storage of square diagonal-first operators (csr_mp_kernel):
which operators qualify, and bit-identical results against the paired-row,
row-pattern and plain CSR forms of the same matrix and against the oracle.

A row qualifies when its column offsets (relative to the row) follow the
master order: 0 first, then ascending.  The master is the sorted set of all
offsets (diagonal first, at most 32); every row's entries are then an ordered
subsequence of it, so walking the master with per-row use bits adds exactly
the row's products in CSR order (the reference's SMEM_SpGEMV loop,
SMEM_MatVec.cpp:140-258, and the Jacobi sweep, SMEM_Smooth.cpp:35-45).
"""
import numpy as np
import pytest

from test_gpu_kernels import assert_bitwise, mats, matrices, _vecs, ALL, SQUARE  # noqa: F401

pytestmark = pytest.mark.gpu

MP_LDS = 48 * 1024  # AMG_MP_LDS: per-pattern value table budget


def expected_master(A, pair_pattern):
    """J (uniform values: -J) the library must report for A, or 0."""
    if not pair_pattern or A.nrows != A.ncols or A.nrows == 0:
        return 0
    lens = np.diff(A.rowptr)
    if np.any(lens == 0):
        return 0
    rows = np.repeat(np.arange(A.nrows), lens)
    off = A.col.astype(np.int64) - rows
    first = A.rowptr[:-1]
    if not np.all(off[first] == 0):
        return 0
    # strictly ascending after the diagonal within each row
    nxt = np.arange(1, off.size)
    same_row = rows[nxt] == rows[nxt - 1]
    after_first = ~np.isin(nxt - 1, first)
    chk = same_row & after_first
    if not np.all(off[nxt][chk] > off[nxt - 1][chk]):
        return 0
    offs = np.unique(off)
    if offs.size > 32:
        return 0
    uni = all(np.unique(A.val[off == o].view(np.int64)).size == 1 for o in offs)
    if not uni and pair_pattern * offs.size * 16 > MP_LDS:
        return 0
    return -offs.size if uni else offs.size


def test_master_pattern_selection(mats):
    host, dev = mats
    for name in ALL:
        want = expected_master(host[name], dev[name].pair_pattern)
        assert dev[name].master_pattern == want, (name, want, dev[name].master_pattern)
    assert dev["lap16"].master_pattern == -7  # the 7-pt stencil: one value per offset
    assert dev["lap_rect"].master_pattern == -7  # odd row count: a half pair at the end
    assert dev["A1"].master_pattern == 27  # 27-pt Galerkin: boundary rows carry other values
    for name in ("P0", "P1", "R0", "R1"):  # not square: no master
        assert dev[name].master_pattern == 0, name


@pytest.mark.parametrize("name", ["lap16", "lap_rect", "A1", "A2"])
def test_master_matches_pair_and_plain(mats, ctx, amg, name):
    """The same matrix as plain CSR, paired-row patterns without the master,
    and master-coded: bit-identical SpGEMV (every (alpha, beta) branch, row
    slices), Jacobi sweeps with and without the zero guess."""
    host, dev = mats
    A = host[name]
    dA = dev[name]
    if dA.master_pattern == 0:
        pytest.skip(f"{name} not master-coded")
    ctx.set_value_index(0)
    plain = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    ctx.set_value_index(1)
    ctx.set_pair_pattern(2)
    ctx.set_master_pattern(0)
    pp_only = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    ctx.set_master_pattern(1)
    ctx.set_pair_pattern(1)
    assert plain.value_index == 0 and pp_only.master_pattern == 0
    assert pp_only.pair_pattern == dA.pair_pattern
    x = ctx.vec(_vecs(A.ncols, 15))
    b = ctx.vec(_vecs(A.nrows, 16))
    variants = (plain, pp_only, dA)
    outs = [[] for _ in variants]
    for vi, M in enumerate(variants):
        for ab in ((1.0, 0.0), (-1.0, 1.0), (1.0, 1.0), (2.5, -0.5), (-1.0, 0.7), (0.3, 0.0)):
            y = ctx.vec(A.nrows)
            amg.smem.SMEM_SpGEMV(ctx, M, x, b, ab[0], ab[1], y, 0, A.nrows)
            outs[vi].append(y.download())
        # row slices: even starts run paired, odd ends leave half a pair
        for ns, ne in ((2, A.nrows - 3), (4, A.nrows - 1), (1, A.nrows - 2)):
            y = ctx.vec(_vecs(A.nrows, 17))
            amg.smem.SMEM_SpGEMV(ctx, M, x, b, -1.0, 1.0, y, ns, ne)
            outs[vi].append(y.download())
        u = ctx.vec(_vecs(A.nrows, 7))
        amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(A.nrows), 3, 0, 0.7)
        outs[vi].append(u.download())
        u = ctx.vec(_vecs(A.nrows, 8))
        amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(A.nrows), 2, 1, 0.8)
        outs[vi].append(u.download())
    for vi in (1, 2):
        for k, (g, r) in enumerate(zip(outs[vi], outs[0])):
            assert_bitwise(g, r, f"{name} variant {vi} output {k}")
    plain.free()
    pp_only.free()


@pytest.mark.parametrize("interp", ["linear", "aggregate"])
def test_master_solve_matches_oracle(amg, oracle, ctx, interp):
    """A whole SMEM_Solve (MULT V(1,1) Jacobi, fused outer residual + first
    pre-sweep, norms) on a hierarchy whose square operators are master-coded
    (pair coding forced on the 27-pt levels): iterate bit-identical to the
    oracle, residual history to 1e-12."""
    from oracle import pyoracle as po
    code = amg.AMG_INTERP_LINEAR if interp == "linear" else amg.AMG_INTERP_AGGREGATE
    g = amg.Gen(32, interp=code)
    ctx.set_pair_pattern(2)
    try:
        host = {w: [po.Csr(*g.host_csr(c, l)) for l in range(cnt)]
                for w, c, cnt in (("A", amg.AMG_GEN_A, g.L), ("P", amg.AMG_GEN_P, g.L - 1),
                                  ("R", amg.AMG_GEN_R, g.L - 1))}
        dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
    finally:
        ctx.set_pair_pattern(1)
    assert dev["A"][0].master_pattern == -7
    if interp == "linear":
        assert any(M.master_pattern > 0 for M in dev["A"][1:])
    opts = amg.default_opts(smooth_weight=0.8, num_cycles=12, tol=0.0, reuse_outer_residual=2)
    H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
    f = amg.rhs_rand(0, 32 ** 3)
    u_gpu, hist, k = H.solve(f)
    OH = po.Hier(host["A"], host["P"], host["R"], po.make_opts(smooth_weight=0.8, num_cycles=12))
    u_cpu, hist_cpu, _ = OH.solve(f)
    assert k == 12
    assert_bitwise(u_gpu, u_cpu, "iterate")
    np.testing.assert_allclose(hist[:k + 1], hist_cpu[:k + 1], rtol=1e-12)
    H.free()
    for v in dev.values():
        for M in v:
            M.free()


def test_master_long_range_edges(ctx, amg):
    """Rows coupling at +-1 and +-L (L = 1000, N = 5001): the 16-byte gather
    runs only in waves whose rows keep row + omin >= 0 and row + omax + 2 <= N;
    the waves at both ends (and the half pair at the odd end) take the exact
    per-entry form.  Bit-identical to plain CSR."""
    N, L = 5001, 1000
    rows, cols, vals = [], [], []
    rp = [0]
    for i in range(N):
        ent = [(i, 4.0)]
        for o in (-L, -1, 1, L):
            if 0 <= i + o < N:
                ent.append((i + o, -0.75 if abs(o) == 1 else -0.125))
        cols += [c for c, _ in ent]
        vals += [v for _, v in ent]
        rp.append(len(cols))
    rp = np.array(rp, np.int32)
    cols = np.array(cols, np.int32)
    vals = np.array(vals, np.float64)
    ctx.set_pair_pattern(2)
    try:
        M = ctx.csr(N, N, rp, cols, vals)
    finally:
        ctx.set_pair_pattern(1)
    ctx.set_value_index(0)
    ctx.set_dict_index(0)
    try:
        P = ctx.csr(N, N, rp, cols, vals)
    finally:
        ctx.set_value_index(1)
        ctx.set_dict_index(1)
    assert M.master_pattern == -5 and P.master_pattern == 0
    x = ctx.vec(_vecs(N, 21))
    b = ctx.vec(_vecs(N, 22))
    for ab in ((1.0, 0.0), (-1.0, 1.0), (2.5, -0.5)):
        ys = []
        for A in (P, M):
            y = ctx.vec(N)
            amg.smem.SMEM_SpGEMV(ctx, A, x, b, ab[0], ab[1], y, 0, N)
            ys.append(y.download())
        assert_bitwise(ys[1], ys[0], f"gemv {ab}")
    us = []
    for A in (P, M):
        u = ctx.vec(_vecs(N, 23))
        amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, A, b, u, ctx.vec(N), 3, 0, 0.7)
        us.append(u.download())
    assert_bitwise(us[1], us[0], "jacobi")
    M.free()
    P.free()


def test_pair_anchor_compression(ctx, amg):
    """With amg_set_pair_anchor16 (default off), pair-coded operators with
    per-row anchors (interpolation) read them slab-compressed (anchor(2t) = pbase[2t >> 9] + uint16 delta); a matrix whose
    512-row slabs span more than 65535 columns keeps the int32 anchors.  Both
    bit-identical to plain CSR, over full ranges and row slices."""
    g = amg.Gen(32)
    N, M, rp, cj, v = g.host_csr(amg.AMG_GEN_P, 0)
    # wide anchors: rows (2t, 2t+1) at a + {0, 1} and a + 1 + {0, 1}, a = (t % 2) * 100000
    nw, mw = 2048, 200004
    rpw = np.arange(0, 2 * nw + 1, 2, dtype=np.int32)
    cw = np.empty(2 * nw, np.int32)
    for i in range(nw):
        a = ((i // 2) % 2) * 100000 + (i & 1)
        cw[2 * i], cw[2 * i + 1] = a, a + 1
    vw = np.tile([0.5, 0.25], nw)
    for n, m, r, c, val, want in ((N, M, rp, cj, v, 1), (nw, mw, rpw, cw, vw, 0)):
        ctx.set_pair_pattern(2)
        ctx.set_pair_anchor16(1)
        try:
            Mp = ctx.csr(n, m, r, c, val)
        finally:
            ctx.set_pair_pattern(1)
            ctx.set_pair_anchor16(0)
        ctx.set_value_index(0)
        ctx.set_dict_index(0)
        try:
            Pl = ctx.csr(n, m, r, c, val)
        finally:
            ctx.set_value_index(1)
            ctx.set_dict_index(1)
        assert Mp.pair_pattern > 0 and Mp.pair_anchor16 == want, (n, Mp.pair_pattern, Mp.pair_anchor16)
        x = ctx.vec(_vecs(m, 31))
        b = ctx.vec(_vecs(n, 32))
        for ab, (ns, ne) in (((1.0, 0.0), (0, n)), ((1.0, 1.0), (0, n)), ((-1.0, 0.7), (0, n)),
                             ((1.0, 1.0), (2, n - 3)), ((1.0, 1.0), (514, n - 1))):
            ys = []
            for A in (Pl, Mp):
                y = ctx.vec(_vecs(n, 33))
                amg.smem.SMEM_SpGEMV(ctx, A, x, b, ab[0], ab[1], y, ns, ne)
                ys.append(y.download())
            assert_bitwise(ys[1], ys[0], f"n={n} {ab} rows {ns}:{ne}")
        Mp.free()
        Pl.free()
