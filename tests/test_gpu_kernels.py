"""Per-kernel parity: every HIP kernel against the CPU oracle, bit for bit.

Bar: the integer/index work and the fp64 per-row sums are reproduced exactly
(the library keeps the reference's summation order and rounds every product
before accumulating), so results must be bitwise identical to the oracle's
restatement of the reference loops.
"""
import numpy as np
import pytest

from conftest import random_csr, rng

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def assert_bitwise(gpu, ref, what=""):
    """Bitwise equality; a NaN must meet a NaN (x86 and gfx950 differ only in
    the default NaN's sign/payload bits, e.g. 0/0 on an empty row)."""
    gpu = np.asarray(gpu)
    ref = np.asarray(ref)
    assert gpu.shape == ref.shape, what
    both_nan = np.isnan(gpu) & np.isnan(ref)
    bad = np.nonzero((bits(gpu) != bits(ref)) & ~both_nan)[0]
    assert bad.size == 0, (f"{what}: {bad.size} mismatches, first at {bad[:5]}: "
                           f"gpu={gpu[bad[:5]]} ref={ref[bad[:5]]}")


def matrices(oracle, amg):
    """Test operators: 7-pt Laplacian, generated coarse operators, P, R,
    random CSR with empty rows / zero diagonals, and a long-row matrix that
    exercises the multi-chunk path of the tile kernel."""
    out = {}
    out["lap16"] = oracle.laplace_7pt(16)
    out["lap_rect"] = oracle.laplace_7pt(13, 7, 5)
    # 7-pt Laplacian with an empty row: dictionary-coded, but not row-pattern
    # coded (a_ii of an empty row is the next row's first value, as in CSR)
    L = oracle.laplace_7pt(12)
    keep = np.ones(L.col.size, bool)
    keep[L.rowptr[300]:L.rowptr[301]] = False
    cnt = np.diff(L.rowptr)
    cnt[300] = 0
    out["lap_hole"] = oracle.Csr(L.nrows, L.ncols, np.concatenate([[0], np.cumsum(cnt)]),
                                 L.col[keep], L.val[keep])
    g = amg.Gen(24, interp=amg.AMG_INTERP_LINEAR)
    for which, name in ((amg.AMG_GEN_A, "A"), (amg.AMG_GEN_P, "P"), (amg.AMG_GEN_R, "R")):
        for lev in (0, 1) if which != amg.AMG_GEN_A else (1, 2):
            nr, nc, rp, cj, cv = g.host_csr(which, lev)
            out[f"{name}{lev}"] = oracle.Csr(nr, nc, rp, cj, cv)
    # smoothed restriction (R (I - w D^-1 A), ~77 entries per row): the
    # long-row kernel on the async additive cycle's transfers
    A0 = oracle.Csr(*g.host_csr(amg.AMG_GEN_A, 0))
    _, out["Rs0"] = oracle.smooth_transfer(A0, out["P0"], 0.8)
    out["rand_sq"] = random_csr(oracle, 3000, 3000, 9, seed=1, with_zero_diag=True)
    out["rand_nz"] = random_csr(oracle, 2500, 2500, 9, seed=4)
    out["rand_rect"] = random_csr(oracle, 1777, 901, 5, seed=2, diag_first=False)
    # >= 64 entries per row on average: the long-row kernel (classical coarse levels)
    out["dense"] = random_csr(oracle, 2100, 2100, 90, seed=7, with_zero_diag=True)
    # long rows: > AMG_CHUNK (2048) entries in one row and in one tile
    g2 = rng(3)
    n = 600
    rows = []
    for i in range(n):
        k = 5000 if i in (7, 300) else int(g2.integers(1, 40))
        c = sorted(set(g2.integers(0, n, size=k).tolist()) - {i})
        rows.append([i] + c)
    rp = np.cumsum([0] + [len(r) for r in rows])
    cj = np.concatenate([np.array(r, dtype=np.int32) for r in rows])
    cv = g2.uniform(-1, 1, size=cj.size)
    cv[rp[:-1]] = 50.0
    out["longrows"] = oracle.Csr(n, n, rp, cj, cv)
    # value-indexed CSR: the same structures with values drawn from a small set
    # (256 distinct values: the largest table; 257: falls back to plain CSR)
    for name, src, nv in (("rand_q", "rand_sq", 256), ("longrows_q", "longrows", 37),
                          ("rand_q257", "rand_nz", 257), ("dense_q", "dense", 200)):
        A = out[src]
        levels = np.linspace(-1.0, 1.0, nv) * (1.0 + 1.0 / 3.0)
        q = levels[rng(nv).integers(0, nv, size=A.val.size)]
        d = A.rowptr[:-1][np.diff(A.rowptr) > 0]
        q[d] = levels[-1]  # diagonal entries: the largest level
        off = np.ones(q.size, bool)
        off[d] = False
        q[np.nonzero(off)[0][:nv]] = levels  # every level present
        out[name] = oracle.Csr(A.nrows, A.ncols, A.rowptr, A.col, q)
    return out


@pytest.fixture(scope="module")
def mats(oracle, amg, ctx):
    host = matrices(oracle, amg)
    ctx.set_pair_pattern(2)  # pair-code long rows at any size (the default gates them by size)
    dev = {k: ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val) for k, A in host.items()}
    ctx.set_pair_pattern(1)
    # the default builds no long-row pairs below 4M rows
    A1 = ctx.csr(host["A1"].nrows, host["A1"].ncols, host["A1"].rowptr, host["A1"].col, host["A1"].val)
    assert A1.row_pattern > 0 and A1.pair_pattern == 0
    A1.free()
    return host, dev


SQUARE = ["lap16", "A1", "A2", "rand_sq", "longrows", "rand_q", "longrows_q", "rand_q257", "lap_hole",
          "dense", "dense_q"]
ALL = SQUARE + ["lap_rect", "P0", "P1", "R0", "R1", "rand_rect", "Rs0"]


def _vecs(n, seed):
    g = rng(seed)
    return g.uniform(-1, 1, n)


def test_value_index_selection(mats):
    """Which registered matrices use the value-indexed form (table size) and
    which stay plain CSR (0): decided by the number of distinct values."""
    host, dev = mats
    for name in ALL:
        nd = np.unique(host[name].val.view(np.int64)).size
        want = nd if nd <= 256 else 0
        assert dev[name].value_index == want, (name, nd, dev[name].value_index)
    assert dev["lap16"].value_index == 2
    assert dev["rand_q"].value_index == 256 and dev["rand_q257"].value_index == 0
    # dictionary-coded: stencil / structured Galerkin operators and their
    # transfers (anchor = each row's first column); not random sparsity or long rows
    assert dev["lap16"].dict_index == 7 and dev["A1"].dict_index == 54
    assert dev["P0"].dict_index == 20 and dev["R0"].dict_index == 27
    for name in ("rand_sq", "rand_q", "rand_q257", "longrows_q", "rand_rect"):
        assert dev[name].dict_index == 0, name
    # row-pattern-coded: dictionary-coded, no empty row, <= 256 distinct rows
    # (a row = its sequence of (column - first column, value) pairs)
    for name in ALL:
        A = host[name]
        pats = set()
        for i in range(A.nrows):
            c = A.col[A.rowptr[i]:A.rowptr[i + 1]].astype(np.int64)
            v = A.val[A.rowptr[i]:A.rowptr[i + 1]].view(np.int64)
            pats.add(tuple((c - c[0]).tolist()) + tuple(v.tolist()) if c.size else ())
        ok = dev[name].dict_index > 0 and np.all(np.diff(A.rowptr) > 0) and len(pats) <= 256
        assert dev[name].row_pattern == (len(pats) if ok else 0), (name, len(pats), dev[name].row_pattern)
    assert dev["lap16"].row_pattern == 27  # interior, 6 faces, 12 edges, 8 corners
    assert dev["lap_hole"].dict_index == 7 and dev["lap_hole"].row_pattern == 0
    for name in ("A1", "P0", "R0"):
        assert dev[name].row_pattern > 0, name
    # paired rows: row-pattern-coded, rows of <= 32 entries, <= 256 distinct
    # (pattern of row 2t, pattern of row 2t+1, anchor delta in [-8, 8)) pairs
    # (anchor = a row's first column) whose table (17 words per pair for rows
    # of <= 8 entries, 65 for <= 32) fits 32 KiB of LDS
    for name in ALL:
        A = host[name]
        if not dev[name].row_pattern or A.nrows == 0:
            assert dev[name].pair_pattern == 0, name
            continue
        lens = np.diff(A.rowptr)
        anch = A.col[A.rowptr[:-1]].astype(np.int64)
        # every row starts at its own index: no anchor array (square, or a slab)
        anch_is_row = bool(np.all(anch == np.arange(A.nrows)))
        pat = []
        for i in range(A.nrows):
            c = A.col[A.rowptr[i]:A.rowptr[i + 1]].astype(np.int64)
            v = A.val[A.rowptr[i]:A.rowptr[i + 1]].view(np.int64)
            pat.append(tuple((c - c[0]).tolist()) + tuple(v.tolist()))
        pairs, da_ok = set(), True
        # a row's entries as (column relative to its anchor) for the merge test
        rel = [tuple((A.col[A.rowptr[i]:A.rowptr[i + 1]].astype(np.int64) - anch[i]).tolist())
               for i in range(A.nrows)]
        for t in range((A.nrows + 1) // 2):
            if 2 * t + 1 < A.nrows:
                da = int(anch[2 * t + 1] - anch[2 * t])
                da_ok &= -8 <= da < 8
                pairs.add((pat[2 * t], pat[2 * t + 1], da))
            else:
                pairs.add((pat[2 * t], None, 0))
        stride = 17 if lens.max() <= 8 else 65
        # merged list = shortest common supersequence: la + lb - LCS, entries
        # matched when row 2t+1's column is row 2t's + 1 (anchor delta da)
        merged = single = 0
        seen = {}
        for t in range(A.nrows // 2):
            key = (pat[2 * t], pat[2 * t + 1], int(anch[2 * t + 1] - anch[2 * t]))
            if key in seen:  # counted over all row pairs
                merged += seen[key][0]
                single += seen[key][1]
                continue
            ra, rb_ = rel[2 * t], rel[2 * t + 1]
            da = key[2] if not anch_is_row else 1
            L = np.zeros((len(ra) + 1, len(rb_) + 1), dtype=np.int64)
            for i in range(len(ra) - 1, -1, -1):
                for j in range(len(rb_) - 1, -1, -1):
                    L[i, j] = L[i + 1, j + 1] + 1 if rb_[j] + da == ra[i] + 1 else max(L[i + 1, j], L[i, j + 1])
            seen[key] = (len(ra) + len(rb_) - L[0, 0], max(len(ra), len(rb_)))
            merged += seen[key][0]
            single += seen[key][1]
        ok = (da_ok and lens.max() <= 32 and len(pairs) <= 256 and len(pairs) * stride * 4 <= 32768
              and merged <= 1.15 * single)
        assert dev[name].pair_pattern == (len(pairs) if ok else 0), (name, len(pairs), dev[name].pair_pattern)
    # 16^3 (x even): pairs (x=0,1), (2k,2k+1) interior, (14,15) times 9 (y,z) classes
    assert dev["lap16"].pair_pattern == 27
    assert dev["A1"].pair_pattern > 0  # the 27-pt Galerkin operator
    for name in ("P0", "P1"):  # anchored: interpolation
        assert dev[name].pair_pattern > 0, name
    for name in ("R0", "R1"):  # restriction: anchors 2 apart, merged lists 5/4 as long
        assert dev[name].pair_pattern == 0, name
    assert dev["lap_rect"].pair_pattern > 0 and dev["lap_rect"].nrows % 2 == 1


@pytest.mark.parametrize("name", ["lap16", "lap_rect", "A1", "rand_q", "longrows_q", "P0", "R1",
                                  "lap_hole"])
def test_value_index_matches_plain(mats, ctx, amg, name):
    """The same matrix registered as plain CSR, value-indexed, dictionary-coded
    and row-pattern-coded gives bit-identical SpGEMV and Jacobi results."""
    host, dev = mats
    A = host[name]
    ctx.set_value_index(0)
    plain = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    ctx.set_value_index(1)
    ctx.set_dict_index(0)
    vi_only = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    ctx.set_dict_index(1)
    ctx.set_row_pattern(0)
    dc_only = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    ctx.set_row_pattern(1)
    ctx.set_pair_pattern(0)
    rp_only = ctx.csr(A.nrows, A.ncols, A.rowptr, A.col, A.val)
    ctx.set_pair_pattern(1)
    assert plain.value_index == 0 and dev[name].value_index > 0 and vi_only.dict_index == 0
    assert dc_only.row_pattern == 0 and dc_only.dict_index == dev[name].dict_index
    assert rp_only.pair_pattern == 0 and rp_only.row_pattern == dev[name].row_pattern
    x = ctx.vec(_vecs(A.ncols, 5))
    b = ctx.vec(_vecs(A.nrows, 6))
    outs = []
    variants = (plain, vi_only, dc_only, rp_only, dev[name])
    for M in variants:
        y = ctx.vec(A.nrows)
        amg.smem.SMEM_SpGEMV(ctx, M, x, b, -1.0, 1.0, y, 0, A.nrows)
        outs.append(y.download())
        if A.nrows == A.ncols:
            u = ctx.vec(_vecs(A.nrows, 7))
            amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, M, b, u, ctx.vec(A.nrows), 2, 0, 0.7)
            outs.append(u.download())
    k = len(outs) // len(variants)
    for i in range(k):
        for v in range(1, len(variants)):
            assert_bitwise(outs[v * k + i], outs[i], f"{name} variant {v}")
    plain.free()
    vi_only.free()
    dc_only.free()
    rp_only.free()


@pytest.mark.parametrize("name", ["lap16", "lap_rect", "A1", "P0", "P1"])
@pytest.mark.parametrize("rng_", [(0, 0), (2, -5), (4, -4), (3, -6), (0, -1), (6, -2)])
def test_pair_pattern_row_ranges(mats, ctx, oracle, amg, name, rng_):
    """Paired-row kernel on row slices: even starts run paired (an odd end
    leaves a half pair), odd starts the single-row kernel; residual, SpGEMV,
    Jacobi and L1 Jacobi (square operators; interpolation and restriction run
    anchored pairs) bit-identical to the oracle, rows outside untouched."""
    host, dev = mats
    A, dA = host[name], dev[name]
    assert dA.pair_pattern > 0
    ns, ne = rng_[0], A.nrows + rng_[1]
    x, b = _vecs(A.ncols, 40), _vecs(A.nrows, 41)
    y0, r0 = _vecs(A.nrows, 42), _vecs(A.nrows, 43)
    ry, rr = y0.copy(), r0.copy()
    oracle.smem_residual(A, b, x, ry, rr, ns, ne)
    y, r = ctx.vec(y0), ctx.vec(r0)
    amg.smem.SMEM_Residual(ctx, dA, ctx.vec(b), ctx.vec(x), y, r, ns, ne)
    assert_bitwise(y.download(), ry, "y")
    assert_bitwise(r.download(), rr, "r")
    for ab in ((1.0, 0.0), (-1.0, 1.0), (2.5, -0.5), (-1.0, 0.7)):
        ref = y0.copy()
        oracle.smem_spgemv(A, x, b, ab[0], ab[1], ref, ns, ne)
        dy = ctx.vec(y0)
        amg.smem.SMEM_SpGEMV(ctx, dA, ctx.vec(x), ctx.vec(b), ab[0], ab[1], dy, ns, ne)
        assert_bitwise(dy.download(), ref, f"spgemv {ab}")
    if A.nrows != A.ncols:  # interpolation / restriction: no smoother
        return
    # amg_jacobi copies the whole u to u_prev (the team's slices together);
    # the oracle's single slice copies only [ns, ne): start u_prev = u
    for zero in (0, 1):
        ru, rp = y0.copy(), y0.copy()
        oracle.smem_jacobi(A, b, ru, rp, 0.8, 2, zero, ns, ne)
        du, dp = ctx.vec(y0), ctx.vec(A.nrows)
        amg.smem.SMEM_Sync_Jacobi(ctx, dA, ctx.vec(b), du, dp, 2, zero, 0.8, ns, ne)
        assert_bitwise(du.download(), ru, f"jacobi zero={zero}")
    l1 = oracle.l1_norms(A)
    ru, rp = y0.copy(), y0.copy()
    oracle.smem_l1jacobi(A, b, ru, rp, l1, 2, 0, ns, ne)
    du, dp = ctx.vec(y0), ctx.vec(A.nrows)
    check = amg.check
    check(amg.lib.amg_l1_jacobi(ctx.h, dA.h, ctx.vec(b).h, du.h, dp.h, ctx.vec(l1).h, 2, 0, ns, ne, 0))
    assert_bitwise(du.download(), ru, "l1 jacobi")


@pytest.mark.parametrize("name", ALL)
def test_matvec(mats, ctx, oracle, amg, name):
    host, dev = mats
    A, dA = host[name], dev[name]
    x = _vecs(A.ncols, 10)
    ref = oracle.smem_matvec(A, x, np.zeros(A.nrows))
    y = ctx.vec(A.nrows)
    amg.smem.SMEM_Sync_Parfor_MatVec(ctx, dA, ctx.vec(x), y)
    assert_bitwise(y.download(), ref, name)


@pytest.mark.parametrize("form,xcd", [(1, 1), (2, 1), (1, 0)])
@pytest.mark.parametrize("name", ["dense", "dense_q", "longrows", "longrows_q"])
def test_long_forms(mats, ctx, oracle, amg, name, form, xcd):
    """The wave-independent long-row kernel (csr_longw_kernel, ctx long_form 1 / 2,
    with and without XCD-contiguous row blocks) on rows of 90..> 2048 entries,
    plain and value-indexed: SpMV, two SpGEMV branches over a row range, the
    two-pass residual, weighted and L1 Jacobi, bit-identical to the oracle."""
    host, dev = mats
    A, dA = host[name], dev[name]
    x, b = _vecs(A.ncols, 40), _vecs(A.nrows, 41)
    ctx.set_long_form(form, xcd)
    try:
        y = ctx.vec(A.nrows)
        amg.smem.SMEM_Sync_Parfor_MatVec(ctx, dA, ctx.vec(x), y)
        assert_bitwise(y.download(), oracle.smem_matvec(A, x, np.zeros(A.nrows)), "matvec")
        for alpha, beta in ((-1, 1), (1.7, -0.4)):
            u = _vecs(A.nrows, 42)
            ref = u.copy()
            oracle.smem_spgemv(A, x, b, alpha, beta, ref, 5, A.nrows - 3)
            du = ctx.vec(u)
            amg.smem.SMEM_SpGEMV(ctx, dA, ctx.vec(x), ctx.vec(b), alpha, beta, du, 5, A.nrows - 3)
            assert_bitwise(du.download(), ref, f"spgemv {alpha} {beta}")
        y0, r0 = np.zeros(A.nrows), np.zeros(A.nrows)
        oracle.smem_residual(A, b, x, y0, r0, 3, A.nrows - 5)
        y, r = ctx.vec(A.nrows), ctx.vec(A.nrows)
        amg.smem.SMEM_Residual(ctx, dA, ctx.vec(b), ctx.vec(x), y, r, 3, A.nrows - 5)
        assert_bitwise(y.download(), y0, "residual y")
        assert_bitwise(r.download(), r0, "residual r")
        if A.nrows == A.ncols:
            f, u = _vecs(A.nrows, 43), _vecs(A.nrows, 44)
            ru, rp = u.copy(), np.zeros(A.nrows)
            oracle.smem_jacobi(A, f, ru, rp, 0.8, 3, 0)
            du, dp = ctx.vec(u), ctx.vec(A.nrows)
            amg.smem.SMEM_Sync_Parfor_Jacobi(ctx, dA, ctx.vec(f), du, dp, 3, 0, 0.8)
            assert_bitwise(du.download(), ru, "jacobi u")
    finally:
        ctx.set_long_form(0, 1)


@pytest.mark.parametrize("name", ["lap16", "rand_rect", "longrows", "P0", "Rs0"])
@pytest.mark.parametrize("ab", [(1, 0), (-1, 0), (2.5, 0), (1, -1), (-1, 1), (0.5, -0.5),
                                (1, 1), (-1, -1), (3, 3), (1, 0.3), (-1, 0.7), (1.7, -0.4)])
def test_spgemv_branches(mats, ctx, oracle, amg, name, ab):
    host, dev = mats
    A, dA = host[name], dev[name]
    alpha, beta = ab
    x = _vecs(A.ncols, 11)
    b = _vecs(A.nrows, 12)
    ref = oracle.smem_spgemv(A, x, b, alpha, beta, np.zeros(A.nrows))
    y = ctx.vec(A.nrows)
    amg.smem.SMEM_SpGEMV(ctx, dA, ctx.vec(x), ctx.vec(b), alpha, beta, y, 0, A.nrows)
    assert_bitwise(y.download(), ref, f"{name} {ab}")


def test_spgemv_row_range_and_inplace(mats, ctx, oracle, amg):
    """Row slices leave other rows untouched; b may alias y (prolong+correct)."""
    host, dev = mats
    A, dA = host["P0"], dev["P0"]
    x = _vecs(A.ncols, 13)
    u = _vecs(A.nrows, 14)
    ref = u.copy()
    oracle.smem_spgemv(A, x, ref.copy(), 1.0, 1.0, ref, 37, A.nrows - 101)
    du = ctx.vec(u)
    amg.smem.SMEM_SpGEMV(ctx, dA, ctx.vec(x), du, 1.0, 1.0, du, 37, A.nrows - 101)
    assert_bitwise(du.download(), ref)


@pytest.mark.parametrize("name", ["lap16", "A1", "rand_sq"])
def test_residual_two_pass(mats, ctx, oracle, amg, name):
    host, dev = mats
    A, dA = host[name], dev[name]
    x, b = _vecs(A.ncols, 15), _vecs(A.nrows, 16)
    y0, r0 = np.zeros(A.nrows), np.zeros(A.nrows)
    oracle.smem_residual(A, b, x, y0, r0, 3, A.nrows - 5)
    y, r = ctx.vec(A.nrows), ctx.vec(A.nrows)
    amg.smem.SMEM_Residual(ctx, dA, ctx.vec(b), ctx.vec(x), y, r, 3, A.nrows - 5)
    assert_bitwise(y.download(), y0, "y")
    assert_bitwise(r.download(), r0, "r")


@pytest.mark.parametrize("name", ["P0", "R1", "rand_rect", "lap16"])
@pytest.mark.parametrize("T", [1, 4, 7])
def test_matvec_t(mats, ctx, oracle, amg, name, T):
    host, dev = mats
    A, dA = host[name], dev[name]
    x = _vecs(A.nrows, 17)
    ref = oracle.seq_matvec_t(A, x) if T == 1 else oracle.smem_matvec_t_expand(A, x, T)
    y = ctx.vec(A.ncols)
    amg.smem.SMEM_Sync_Parfor_MatVecT(ctx, dA, ctx.vec(x), y, T)
    assert_bitwise(y.download(), ref, f"{name} T={T}")


@pytest.mark.parametrize("name", SQUARE)
@pytest.mark.parametrize("zero", [0, 1])
@pytest.mark.parametrize("variant", ["smem", "seq"])
def test_jacobi(mats, ctx, oracle, amg, name, zero, variant):
    host, dev = mats
    A, dA = host[name], dev[name]
    f, u = _vecs(A.nrows, 18), _vecs(A.nrows, 19)
    ru, rp = u.copy(), np.zeros(A.nrows)
    w = 0.8
    if variant == "smem":
        oracle.smem_jacobi(A, f, ru, rp, w, 3, zero)
    else:
        oracle.seq_jacobi(A, f, ru, rp, w, 3, zero)
    du, dp = ctx.vec(u), ctx.vec(A.nrows)
    fn = amg.smem.SMEM_Sync_Parfor_Jacobi if variant == "smem" else amg.smem.SEQ_Jacobi
    fn(ctx, dA, ctx.vec(f), du, dp, 3, zero, w)
    assert_bitwise(du.download(), ru, f"{name} u")
    assert_bitwise(dp.download(), rp, f"{name} u_prev")


@pytest.mark.parametrize("name", ["lap16", "A2", "rand_sq"])
@pytest.mark.parametrize("zero", [0, 1])
def test_l1_jacobi(mats, ctx, oracle, amg, name, zero):
    host, dev = mats
    A, dA = host[name], dev[name]
    f, u = _vecs(A.nrows, 20), _vecs(A.nrows, 21)
    l1 = oracle.l1_norms(A)
    dl1 = ctx.vec(A.nrows)
    amg.smem.L1_row_norm(ctx, dA, dl1)
    assert_bitwise(dl1.download(), l1, "l1 norms")
    for variant in ("smem", "seq"):
        ru, rp = u.copy(), np.zeros(A.nrows)
        if variant == "smem":
            oracle.smem_l1jacobi(A, f, ru, rp, l1, 2, zero)
        else:
            oracle.seq_l1jacobi(A, f, ru, rp, l1, 2, zero)
        du, dp = ctx.vec(u), ctx.vec(A.nrows)
        fn = amg.smem.SMEM_Sync_Parfor_L1Jacobi if variant == "smem" else amg.smem.SEQ_L1Jacobi
        fn(ctx, dA, ctx.vec(f), du, dp, dl1, 2, zero)
        assert_bitwise(du.download(), ru, f"{name} {variant}")


@pytest.mark.parametrize("name", ["lap16", "A1", "rand_sq", "lap_hole"])
@pytest.mark.parametrize("T", [1, 4, 8, "perf64", "ragged"])
@pytest.mark.parametrize("zero", [0, 1])
@pytest.mark.parametrize("wave", [1, 2, 0, 3, "1s0", "1s1"])
def test_hybrid_jgs(mats, ctx, oracle, amg, name, T, zero, wave):
    """Hybrid Jacobi/GS is partition dependent: the same blocks must give the
    same bits -- the reference's thread ranges (T) and the device partition --
    in every kernel form: 8 lanes per block and 8 blocks per wave (1), one
    wave per block (2; the chain carried lane to lane, blocks spanning many
    64-row chunks), one lane per block (0), the LDS tile of 64 blocks (3)."""
    host, dev = mats
    small = 2
    if isinstance(wave, str):  # form 1 with the small levels' form 0 / 1
        wave, small = 1, int(wave[2])
    ctx.set_jgs_wave(wave)
    ctx.set_jgs_small(small)
    A, dA = host[name], dev[name]
    if T == "perf64":
        blk = np.minimum(np.arange(0, A.nrows + 64, 64), A.nrows).astype(np.int32)
        blk = np.unique(blk)
    elif T == "ragged":  # blocks of 1 .. 200 rows, some empty
        cuts = np.cumsum(rng(5).integers(0, 200, size=A.nrows // 50))
        blk = np.concatenate([[0], cuts[cuts < A.nrows], [A.nrows]]).astype(np.int32)
    else:
        blk = oracle.partition_equal(A.nrows, T)
    f, u = _vecs(A.nrows, 22), _vecs(A.nrows, 23)
    w = 0.7
    ds = oracle.a_diag(A, w)
    dds = ctx.vec(A.nrows)
    amg.smem.A_diag(ctx, dA, w, dds)
    assert_bitwise(dds.download(), ds, "A_diag")
    for reverse in (0, 1):
        for parfor in (True, False):
            ru, rp = u.copy(), np.zeros(A.nrows)
            oracle.hybrid_jgs(A, f, ru, rp, blk, ds if parfor else None, 1.0, 2, zero, reverse)
            du, dp = ctx.vec(u), ctx.vec(A.nrows)
            if parfor:
                amg.smem.SMEM_Sync_Parfor_HybridJacobiGaussSeidel(ctx, dA, ctx.vec(f), du, dp, blk,
                                                                 dds, 2, zero, reverse)
            else:
                amg.smem.SMEM_Sync_HybridJacobiGaussSeidel(ctx, dA, ctx.vec(f), du, dp, 2, zero,
                                                          blk, reverse)
            assert_bitwise(du.download(), ru, f"{name} T={T} rev={reverse} parfor={parfor} wave={wave}")
    ctx.set_jgs_wave(1)
    ctx.set_jgs_small(2)


def test_gauss_seidel(mats, ctx, oracle, amg):
    host, dev = mats
    A, dA = host["lap16"], dev["lap16"]
    f, u = _vecs(A.nrows, 24), _vecs(A.nrows, 25)
    ru = u.copy()
    oracle.seq_gauss_seidel(A, f, ru, 2)
    du = ctx.vec(u)
    amg.smem.SEQ_GaussSeidel(ctx, dA, ctx.vec(f), du, 2)
    assert_bitwise(du.download(), ru)


@pytest.mark.parametrize("name", ["lap16", "rand_sq", "A1"])
@pytest.mark.parametrize("semi", [0, 1])
@pytest.mark.parametrize("reverse", [0, 1])
def test_async_gauss_seidel_single_block(mats, ctx, oracle, amg, name, semi, reverse):
    """One block (one thread): the asynchronous Gauss-Seidel is deterministic."""
    host, dev = mats
    A, dA = host[name], dev[name]
    f, u = _vecs(A.nrows, 40), _vecs(A.nrows, 41)
    ru = u.copy()
    oracle.async_gs(A, f, ru, [0, A.nrows], 3, reverse)
    du = ctx.vec(u)
    amg.smem.SMEM_Async_Parfor_GaussSeidel(ctx, dA, ctx.vec(f), du, 3, None, semi, reverse)
    assert_bitwise(du.download(), ru, name)


@pytest.mark.parametrize("semi", [0, 1])
def test_async_gauss_seidel_many_blocks(mats, ctx, oracle, amg, semi):
    """Many blocks: racy across blocks like the reference, so the residual after
    the sweeps must lie in [0.5 x min, 2 x max] of the oracle's band: the
    blocks one after another, 10 runs with one OpenMP thread per block on the
    live iterate (SMEM_Async_GaussSeidel's race) and all blocks in lockstep."""
    host, dev = mats
    A, dA = host["A1"], dev["A1"]
    f = _vecs(A.nrows, 42)
    blk = np.linspace(0, A.nrows, 65).astype(np.int32)
    res = lambda x: np.linalg.norm(f - oracle.smem_matvec(A, x, np.zeros(A.nrows)))
    band = []
    try:
        for mode, reps in ((0, 1), (1, 10), (2, 1)):
            oracle.lib().or_set_async_gs_threads(mode)
            for _ in range(reps):
                ru = np.zeros(A.nrows)
                oracle.async_gs(A, f, ru, blk, 4, 0)
                band.append(res(ru))
    finally:
        oracle.lib().or_set_async_gs_threads(0)
    du = ctx.vec(np.zeros(A.nrows))
    amg.smem.SMEM_Async_Parfor_GaussSeidel(ctx, dA, ctx.vec(f), du, 4, blk, semi, 0)
    rg = res(du.download())
    lo, hi = min(band), max(band)
    print(f"async GS {semi}: oracle band [{lo:.4e}, {hi:.4e}], device {rg:.4e}")
    assert rg < 0.5 * np.linalg.norm(f)
    assert 0.5 * lo <= rg <= 2.0 * hi, (rg, lo, hi)


@pytest.mark.parametrize("name", ["lap16", "A1", "rand_nz"])
@pytest.mark.parametrize("sweeps", [1, 2])
@pytest.mark.parametrize("zero", [0, 1])
def test_symmetric_jacobi(mats, ctx, oracle, amg, name, sweeps, zero):
    host, dev = mats
    A, dA = host[name], dev[name]
    f, u = _vecs(A.nrows, 26), _vecs(A.nrows, 27)
    w = 0.9
    n = A.nrows
    l1 = oracle.l1_norms(A)
    dl1 = ctx.vec(l1)
    cases = [
        ("smem", lambda ru, y, r: oracle.smem_sym_jacobi(A, f, ru, y, r, w, sweeps, zero),
         lambda du, dy, dr: amg.smem.SMEM_Sync_SymmetricJacobi(ctx, dA, ctx.vec(f), du, dy, dr,
                                                                sweeps, zero, w, 0, n)),
        ("smem_l1", lambda ru, y, r: oracle.smem_sym_l1jacobi(A, f, ru, y, r, l1, sweeps, zero),
         lambda du, dy, dr: amg.smem.SMEM_Sync_SymmetricL1Jacobi(ctx, dA, ctx.vec(f), du, dy, dr,
                                                                  dl1, sweeps, zero, 0, n)),
        ("seq", lambda ru, y, r: oracle.seq_sym_jacobi(A, f, ru, y, r, w, sweeps),
         lambda du, dy, dr: amg.smem.SEQ_SymmetricJacobi(ctx, dA, ctx.vec(f), du, dy, dr, sweeps, w)),
        ("seq_l1", lambda ru, y, r: oracle.seq_sym_l1jacobi(A, f, ru, y, r, l1, sweeps),
         lambda du, dy, dr: amg.smem.SEQ_SymmetricL1Jacobi(ctx, dA, ctx.vec(f), du, dy, dr, dl1,
                                                            sweeps)),
    ]
    for tag, ref_fn, gpu_fn in cases:
        if tag.startswith("seq") and zero == 1:
            continue
        ru, y, r = u.copy(), np.zeros(n), np.zeros(n)
        ref_fn(ru, y, r)
        du, dy, dr = ctx.vec(u), ctx.vec(n), ctx.vec(n)
        gpu_fn(du, dy, dr)
        assert_bitwise(du.download(), ru, f"{name} {tag} u")
        assert_bitwise(dr.download(), r, f"{name} {tag} r")


def test_vector_ops_and_norm(ctx, amg):
    g = rng(30)
    n = 100003
    x, y, s = g.uniform(-1, 1, n), g.uniform(-1, 1, n), g.uniform(1, 2, n)
    dx, dy, ds = ctx.vec(x), ctx.vec(y), ctx.vec(s)
    amg.smem.DMEM_HypreParVector_Ivaxpy(ctx, dy, dx, ds)
    assert_bitwise(dy.download(), y + x / s, "ivaxpy")
    amg.smem.DMEM_HypreRealArray_Axpy(ctx, dy, dx, 0.25)
    assert_bitwise(dy.download(), (y + x / s) + 0.25 * x, "axpy")
    nrm = dx.norm2()
    assert abs(nrm - np.sqrt(np.sum(x * x))) <= 1e-13 * nrm
    assert nrm == dx.norm2()  # deterministic


def test_error_reporting(ctx, amg, mats):
    host, dev = mats
    dA = dev["lap16"]
    small = ctx.vec(10)
    with pytest.raises(amg.AmgError, match="vector sizes"):
        amg.smem.SMEM_Sync_Parfor_MatVec(ctx, dA, small, small)
    with pytest.raises(amg.AmgError, match="row range"):
        amg.smem.SMEM_MatVec(ctx, dA, ctx.vec(dA.ncols), ctx.vec(dA.nrows), 5, dA.nrows + 1)
