"""CPU: the oracle restatement (parity unpinned: the reference has no fixtures)
against the survey's stand-in-build cross-check value and against independent
closed-form / numpy restatements."""
import json
import os

import numpy as np
import pytest

from conftest import random_csr, rng

HERE = os.path.dirname(os.path.abspath(__file__))


def aggregation_hierarchy(oracle, n):
    A = oracle.laplace_7pt(n)
    nc = n // 2
    rows = np.arange(n ** 3)
    x, y, z = rows % n, (rows // n) % n, rows // (n * n)
    c = (x // 2) + nc * ((y // 2) + nc * (z // 2))
    P = oracle.Csr(n ** 3, nc ** 3, np.arange(n ** 3 + 1), c, np.ones(n ** 3))
    R = oracle.transpose(P)
    A1 = oracle.spgemm(oracle.spgemm(R, A), P)
    return A, A1, P, R


def test_known_answer_crosscheck(oracle):
    """SMEM_Solve value the survey session recorded from a stand-in-header build
    of the reference: a cross-check of the restatement, not a parity pin (the
    oracle is parity unpinned)."""
    ka = json.load(open(os.path.join(HERE, "golden", "known_answer.json")))
    case = ka["smem_solve_16cube_aggregation"]
    A, A1, P, R = aggregation_hierarchy(oracle, 16)
    f = oracle.rhs_rand(16 ** 3)
    opts = oracle.make_opts(smooth_weight=0.8, num_cycles=20)
    H = oracle.Hier([A, A1], [P], [R], opts)
    u, hist, k = H.solve(f)
    assert k == 20
    rel = hist[-1] / hist[0]
    assert abs(rel - case["relres"]) <= 1e-12 * case["relres"]


def test_laplacian_closed_form(oracle):
    n = 9
    A = oracle.laplace_7pt(n)
    assert A.nnz == 7 * n ** 3 - 6 * n ** 2
    y = oracle.seq_matvec(A, np.ones(n ** 3))
    # row sum = number of missing neighbours (Dirichlet boundary)
    idx = np.arange(n ** 3)
    x, yy, z = idx % n, (idx // n) % n, idx // (n * n)
    missing = sum(((v == 0).astype(int) + (v == n - 1).astype(int)) for v in (x, yy, z))
    np.testing.assert_array_equal(y, missing.astype(float))
    assert np.all(A.val[A.rowptr[:-1]] == 6.0)


def test_matvec_against_numpy(oracle):
    A = random_csr(oracle, 500, 300, 6, seed=5, diag_first=False)
    x = rng(1).uniform(-1, 1, 300)
    y = oracle.seq_matvec(A, x)
    ref = np.array([sum(A.val[k] * x[A.col[k]] for k in range(A.rowptr[i], A.rowptr[i + 1]))
                    for i in range(A.nrows)])
    np.testing.assert_array_equal(y, ref)   # same sequential order -> same bits
    yt = oracle.seq_matvec_t(A, rng(2).uniform(-1, 1, 500))
    assert yt.shape == (300,)


@pytest.mark.parametrize("alpha,beta", [(1, 0), (-1, 1), (1, 1), (2, -3), (-1, -1), (0.5, 0.5)])
def test_spgemv_math(oracle, alpha, beta):
    A = random_csr(oracle, 400, 400, 7, seed=6)
    g = rng(3)
    x, b = g.uniform(-1, 1, 400), g.uniform(-1, 1, 400)
    y = oracle.smem_spgemv(A, x, b, alpha, beta, np.zeros(400))
    ref = alpha * A.to_scipy().dot(x) + beta * b
    np.testing.assert_allclose(y, ref, rtol=1e-12, atol=1e-12)


def test_jacobi_fixed_point_and_gs(oracle):
    A = oracle.laplace_7pt(6)
    n = A.nrows
    u_star = rng(4).uniform(-1, 1, n)
    f = oracle.seq_matvec(A, u_star)
    u, up = u_star.copy(), np.zeros(n)
    oracle.smem_jacobi(A, f, u, up, 0.8, 3, 0)
    np.testing.assert_allclose(u, u_star, atol=1e-14)
    u = np.zeros(n)
    oracle.seq_gauss_seidel(A, f, u, 200)
    np.testing.assert_allclose(u, u_star, atol=1e-9)
    # hybrid JGS with one block per row == Jacobi with weight 1
    blk = np.arange(n + 1, dtype=np.int32)
    u1, u2, p = np.zeros(n), np.zeros(n), np.zeros(n)
    oracle.hybrid_jgs(A, f, u1, p, blk, None, 1.0, 2, 0)
    oracle.smem_jacobi(A, f, u2, np.zeros(n), 1.0, 2, 0)
    np.testing.assert_array_equal(u1, u2)


def test_partitions(oracle):
    A = random_csr(oracle, 1001, 1001, 8, seed=7)
    for T in (1, 3, 8):
        blk = oracle.partition_nnz(A, T)
        per = (A.nnz + T - 1) // T
        ref = [0] + [int(np.searchsorted(A.rowptr[:-1], per * t, side="left")) for t in range(1, T)] + [1001]
        np.testing.assert_array_equal(blk, ref)
        eq = oracle.partition_equal(1001, T)
        assert eq[0] == 0 and eq[-1] == 1001 and np.all(np.diff(eq) >= 1001 // T)


def test_rhs_is_glibc_sequence(oracle):
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(0)
    ref = [-1 + 2 * (libc.rand() / 2147483647) for _ in range(10)]
    np.testing.assert_array_equal(oracle.rhs_rand(10), ref)


def test_dmem_cheby_update(oracle):
    """DMEM_Misc.cpp:612-666: first cycle copies u into d; later cycles use the
    Richardson omega (the only branch the reference CLI reaches, since
    CHEBY_ACCEL == RICHARD_ACCEL == 1) or the c_k recurrence, on the sync
    (d only), cheby_grid (d and u) or other-grid (u only) branch."""
    g = np.random.default_rng(3)
    n, mu, delta = 257, 1.7, 0.6
    u0, d0 = g.uniform(-1, 1, n), g.uniform(-1, 1, n)
    for accel in (oracle.OR_RICHARD_ACCEL, oracle.OR_CHEBY_RECUR_ACCEL):
        for branch in (oracle.OR_CHEBY_SYNC, oracle.OR_CHEBY_GRID, oracle.OR_CHEBY_OTHER):
            d, u, st = d0.copy(), u0.copy(), np.array([mu, 1.0])
            oracle.dmem_cheby_update(d, u, 0, accel, branch, mu, delta, st)
            assert np.array_equal(d, u0) and np.array_equal(u, u0)
            c, cp = mu, 1.0
            d, u = d0.copy(), u0.copy()
            for cyc in (1, 2, 3):
                if accel == oracle.OR_RICHARD_ACCEL:
                    w = 2.0 / (1.0 + np.sqrt(1.0 - mu ** -2.0))
                else:
                    c, cp = 2.0 * mu * c - cp, c
                    w = 2.0 * mu * cp / c
                dn = (w - 1.0) * d + w * delta * u
                un = {oracle.OR_CHEBY_SYNC: u, oracle.OR_CHEBY_GRID: (w - 1.0) * d + w * delta * u,
                      oracle.OR_CHEBY_OTHER: w * delta * u}[branch]
                if branch == oracle.OR_CHEBY_OTHER:
                    dn = d
                oracle.dmem_cheby_update(d, u, cyc, accel, branch, mu, delta, st)
                assert np.array_equal(d, dn) and np.array_equal(u, un)
                d, u = dn.copy(), un.copy()


def test_dmem_async_jacobi_one_rank(oracle):
    """DMEM_AsyncSmooth on one rank without acceleration is weighted Jacobi in
    residual form: same iterate as the SMEM sweep up to rounding."""
    A = oracle.laplace_7pt(9)
    b = oracle.rhs_rand(A.nrows)
    x, rn = oracle.dmem_async_jacobi(A, b, 12, 0.7)
    u = np.zeros(A.nrows)
    for _ in range(12):
        oracle.smem_jacobi(A, b, u, np.zeros(A.nrows), 0.7, 1, 0)
    np.testing.assert_allclose(x, u, rtol=1e-10, atol=1e-13)
    r = b - A.to_scipy() @ x
    np.testing.assert_allclose(rn, np.linalg.norm(r), rtol=1e-10)


def test_async_add_oracle(oracle, amg):
    """or_async_add (SMEM_Async_Add_AMG on OpenMP threads): every level group does
    num_cycles corrections (LOCAL) or at least that many (GLOBAL), the solve
    converges for MULTADD / AFACx with Jacobi, L1 and hybrid JGS, FULL / SEMI,
    READ_SOL / READ_RES; with two levels only the fine group changes u (the
    coarsest correction is zero: the reference's coarsest solve is commented
    out), so the run is deterministic and equals the synchronous additive
    cycle up to the residual's two-pass rounding."""
    g = amg.Gen(16, interp=amg.AMG_INTERP_LINEAR)
    L = g.L
    A = [oracle.Csr(*g.host_csr(amg.AMG_GEN_A, l)) for l in range(L)]
    P = [oracle.Csr(*g.host_csr(amg.AMG_GEN_P, l)) for l in range(L - 1)]
    Ps, Rs = [], []
    for l in range(L - 1):
        p, r = oracle.smooth_transfer(A[l], P[l], 0.8)
        Ps.append(p)
        Rs.append(r)
    f = amg.rhs_rand(0, 16 ** 3)
    N = 12
    for solver, host_p, host_r in ((oracle.OR_ASYNC_MULTADD, Ps, Rs), (oracle.OR_ASYNC_AFACX, P, [
            oracle.Csr(*g.host_csr(amg.AMG_GEN_R, l)) for l in range(L - 1)])):
        for sm in (oracle.OR_JACOBI, oracle.OR_L1_JACOBI, oracle.OR_HYBRID_JGS):
            H = oracle.Hier(A, host_p, host_r, oracle.make_opts(solver=solver, smoother=sm, smooth_weight=0.8,
                                                                num_cycles=N))
            for at in (oracle.OR_FULL_ASYNC, oracle.OR_SEMI_ASYNC):
                for rt in (oracle.OR_READ_SOL, oracle.OR_READ_RES):
                    for ct in (oracle.OR_CONVERGE_LOCAL, oracle.OR_CONVERGE_GLOBAL):
                        u, rel, cnt = H.async_add(f, [1] * L, async_type=at, read_type=rt, converge_type=ct)
                        assert np.all(np.isfinite(u))
                        # AFACx on the plain transfers contracts slowly; with GLOBAL
                        # convergence its fast coarse groups run many stale corrections
                        if solver == oracle.OR_ASYNC_MULTADD:
                            assert rel < 0.05, (solver, sm, at, rt, ct, rel)
                        elif ct == oracle.OR_CONVERGE_LOCAL:
                            assert rel < 1.0, (solver, sm, at, rt, ct, rel)
                        if ct == oracle.OR_CONVERGE_LOCAL:
                            assert list(cnt) == [N] * L, cnt
                        else:
                            assert min(cnt) >= N, cnt
    # two levels: deterministic, equal to the synchronous additive cycle
    A2, P2, R2 = A[:2], Ps[:1], Rs[:1]
    o = dict(smoother=oracle.OR_JACOBI, smooth_weight=0.8, num_cycles=N)
    _, h, _ = oracle.Hier(A2, P2, R2, oracle.make_opts(solver=oracle.OR_MULTADD, **o)).solve(f)
    Ha = oracle.Hier(A2, P2, R2, oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, **o))
    rels = [Ha.async_add(f, [2, 1])[1] for _ in range(3)]
    assert max(rels) == min(rels)
    assert abs(rels[0] - h[-1] / h[0]) <= 1e-9 * h[-1] / h[0], (rels, h[-1] / h[0])


def test_async_add_sequential_schedules(amg, oracle):
    """or_set_async_schedule: the groups one after another (finest / coarsest
    first) -- every level still runs num_cycles corrections and the iterate
    converges, slower than the free race."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=12, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    rels = {}
    for sched in (0, 1, 2):
        oracle.lib().or_set_async_schedule(sched)
        try:
            u, rel, cnt = OH.async_add(f, [1] * L, async_type=oracle.OR_FULL_ASYNC,
                                       converge_type=oracle.OR_CONVERGE_LOCAL)
        finally:
            oracle.lib().or_set_async_schedule(0)
        assert np.all(np.isfinite(u)) and list(cnt[:L]) == [12] * L
        rels[sched] = rel
    assert rels[0] < 1e-2 and rels[1] < 1.0 and rels[2] < 1.0
    assert rels[0] < rels[1] and rels[0] < rels[2], rels


def test_async_add_res_global(amg, oracle):
    """or_set_async_res_global (res_compute_type GLOBAL, SMEM_Async_AMG.cpp:35-77,
    356-414): no level-0 group; every level group runs num_cycles corrections,
    the free race converges, and with one thread per group run one after
    another the result is deterministic."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=12, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    nt = [0] + [1] * (L - 1)
    for at in (oracle.OR_FULL_ASYNC, oracle.OR_SEMI_ASYNC):
        u, rel, cnt = OH.async_add(f, nt, async_type=at, res_global=True)
        assert np.all(np.isfinite(u)) and list(cnt[:L]) == [0] + [12] * (L - 1)
        assert rel < 0.5, rel
        seq = []
        for _ in range(2):
            oracle.lib().or_set_async_schedule(1)
            try:
                seq.append(OH.async_add(f, nt, async_type=at, res_global=True))
            finally:
                oracle.lib().or_set_async_schedule(0)
        assert np.array_equal(seq[0][0].view(np.uint64), seq[1][0].view(np.uint64))
        assert rel < seq[0][1] < 1.0, (rel, seq[0][1])
    # a level-0 group is refused with GLOBAL residuals
    with pytest.raises(AssertionError):
        OH.async_add(f, [1] * L, res_global=True)
