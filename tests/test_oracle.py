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
    rels, us = {}, {}
    for sched in (0, 1, 2, 1, 2):
        oracle.lib().or_set_async_schedule(sched)
        try:
            u, rel, cnt = OH.async_add(f, [1] * L, async_type=oracle.OR_FULL_ASYNC,
                                       converge_type=oracle.OR_CONVERGE_LOCAL)
        finally:
            oracle.lib().or_set_async_schedule(0)
        assert np.all(np.isfinite(u)) and list(cnt[:L]) == [12] * L
        if sched in us:  # a sequential schedule is deterministic
            assert np.array_equal(u.view(np.uint64), us[sched].view(np.uint64))
        rels[sched], us[sched] = rel, u
    assert rels[0] < 1e-2 and rels[1] < 1.0 and rels[2] < 1.0, rels
    # the finest-first order is the slowest: the coarse corrections all
    # come last, from the initial residual's restriction
    assert rels[1] > rels[0] and rels[1] > rels[2], rels


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
        assert seq[0][1] < 1.0, (rel, seq[0][1])
    # a level-0 group is refused with GLOBAL residuals
    with pytest.raises(AssertionError):
        OH.async_add(f, [1] * L, res_global=True)


@pytest.mark.parametrize("ct", ["local", "global"])
def test_async_add_round_robin_schedule(amg, oracle, ct):
    """or_set_async_schedule(3): the groups take turns, one whole correction
    each -- deterministic (repeated runs are the same bits, also with two
    threads per group), every group runs num_cycles corrections under
    converge LOCAL and num_cycles + 1 under GLOBAL (the finest group raises
    the flag in the round after every group has num_cycles), and it converges."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    N = 10
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    conv = oracle.OR_CONVERGE_GLOBAL if ct == "global" else oracle.OR_CONVERGE_LOCAL
    out = []
    for nt in ([1] * L, [1] * L, [2] * L):
        oracle.lib().or_set_async_schedule(3)
        try:
            out.append(OH.async_add(f, nt, async_type=oracle.OR_FULL_ASYNC, converge_type=conv))
        finally:
            oracle.lib().or_set_async_schedule(0)
    for u, rel, cnt in out:
        assert np.array_equal(u.view(np.uint64), out[0][0].view(np.uint64))
        assert list(cnt[:L]) == [N + (ct == "global")] * L, cnt
        assert rel < 0.1, rel
    # the sequential schedules refuse converge GLOBAL (they would never end)
    oracle.lib().or_set_async_schedule(1)
    try:
        with pytest.raises(AssertionError):
            OH.async_add(f, [1] * L, converge_type=oracle.OR_CONVERGE_GLOBAL)
    finally:
        oracle.lib().or_set_async_schedule(0)


@pytest.mark.parametrize("ct", ["local", "global"])
def test_async_add_timed_schedule(amg, oracle, ct):
    """or_set_async_schedule(4), the race at fixed level speeds: with equal
    durations it is the round robin (end times tie, the finer group first);
    under converge LOCAL, durations growing 1000x per level give the groups
    finest first and durations falling 1000x per level coarsest first (every
    group's corrections end before the next group's first); uneven durations
    are deterministic and converge."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    N = 10
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    conv = oracle.OR_CONVERGE_GLOBAL if ct == "global" else oracle.OR_CONVERGE_LOCAL

    def run(sched, d=None):
        if d is not None:
            oracle.set_async_durations(d)
        oracle.lib().or_set_async_schedule(sched)
        try:
            return OH.async_add(f, [1] * L, async_type=oracle.OR_FULL_ASYNC, converge_type=conv)
        finally:
            oracle.lib().or_set_async_schedule(0)

    def same(a, b):
        return np.array_equal(a[0].view(np.uint64), b[0].view(np.uint64)) and list(a[2]) == list(b[2])

    assert same(run(4, np.ones(L)), run(3))
    if ct == "local":
        assert same(run(4, 1000.0 ** np.arange(L)), run(1))
        assert same(run(4, 1000.0 ** -np.arange(L)), run(2))
    d = np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)])
    a, b = run(4, d), run(4, d)
    assert same(a, b)
    # the recorded-times form (or_set_async_times) of the same end times, also
    # through the repeated last interval past a short table
    for m in (N + 2, 3):
        oracle.set_async_times([d[k] * np.arange(1, m + 1) for k in range(L)])
        oracle.lib().or_set_async_schedule(4)
        try:
            c = OH.async_add(f, [1] * L, async_type=oracle.OR_FULL_ASYNC, converge_type=conv)
        finally:
            oracle.lib().or_set_async_schedule(0)
        assert same(a, c)
    assert a[1] < 0.1, a[1]
    if ct == "local":
        assert list(a[2][:L]) == [N] * L


def test_async_add_replay(amg, oracle):
    """or_async_add_replay (the row-sliced replay of a distributed free race):
    with one slice it is the timed schedule with the same end times, bit for
    bit; with two slices updated at the same times it is the one-slice replay;
    with slices updated in different orders it differs from both single-order
    replays and still converges."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    N = 10
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    n0 = 16 ** 3
    d = np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)])
    times = [d[k] * np.arange(1, N + 1) for k in range(L - 1)] + [np.zeros(0)]
    oracle.set_async_times(times[:-1] + [times[-2]])
    oracle.lib().or_set_async_schedule(4)
    try:
        ut, relt, _ = OH.async_add(f, [1] * L)
    finally:
        oracle.lib().or_set_async_schedule(0)
    u1, rel1, c1 = OH.async_add_replay(f, [0, n0], [t[:, None] for t in times])
    assert np.array_equal(u1.view(np.uint64), ut.view(np.uint64)) and rel1 == relt
    assert list(c1[:L - 1]) == [N] * (L - 1)
    half = [0, n0 // 2, n0]
    u2, rel2, _ = OH.async_add_replay(f, half, [np.stack([t, t], axis=1) for t in times])
    assert np.array_equal(u2.view(np.uint64), u1.view(np.uint64))
    # slice 1 runs the fine level late: a blend of two orders
    skew = [np.stack([t, t + (1.7 if k == 0 else 0.0)], axis=1) for k, t in enumerate(times)]
    u3, rel3, _ = OH.async_add_replay(f, half, skew)
    assert not np.array_equal(u3.view(np.uint64), u1.view(np.uint64))
    assert rel3 < 0.1, rel3


def test_torn_replay_model(amg, oracle):
    """async_band.torn_replay (the row-time model of overlapping update windows):
    zero-length windows give the plain replay of the end order, bit for bit;
    windows of two levels that overlap interleave their updates by rows (a
    different iterate, still converging).  Under converge GLOBAL a replay runs
    exactly the recorded corrections per level (the race's stopping point)."""
    from async_band import torn_replay
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    N = 6
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    f = amg.rhs_rand(0, 16 ** 3)
    n0 = 16 ** 3
    d = np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)])
    ends = [list(d[k] * np.arange(1, N + 1)) for k in range(L - 1)] + [[]]
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle.make_opts(
        solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0))
    _, rel1, _ = OH.async_add_replay(f, [0, n0], [np.asarray(t)[:, None] for t in ends])
    rel0 = torn_replay(amg, oracle, host, f, opts, ends, ends, slices=8)
    assert rel0 == rel1
    # level 0's windows span the previous half interval: they overlap level 1's
    starts = [list(np.asarray(e) - (0.5 * d[0] if k == 0 else 0.0)) for k, e in enumerate(ends)]
    relt = torn_replay(amg, oracle, host, f, opts, ends, starts, slices=8)
    assert relt != rel1 and relt < 0.5, (relt, rel1)
    # converge GLOBAL replay: exactly the table's counts
    cnt = [N + 3] + [N] * (L - 2) + [N]
    oracle.set_async_times([d[k] * np.arange(1, cnt[k] + 1) for k in range(L)], exact=True)
    oracle.lib().or_set_async_schedule(4)
    try:
        _, _, c = OH.async_add(f, [1] * L, converge_type=oracle.OR_CONVERGE_GLOBAL)
    finally:
        oracle.lib().or_set_async_schedule(0)
    assert list(c[:L - 1]) == cnt[:L - 1], c


def test_row_replay_model(amg, oracle):
    """async_band.row_replay (the exact replay of a row-stamped free race): rows
    that saw the same update order are merged into one slice, which changes
    nothing -- the merged replay is bit-identical to the replay with one slice
    per row; untorn tables (every row updated at its correction's time) give one
    slice and the whole-correction replay; torn tables (two levels' update
    kernels overlapping, their 64-row waves interleaved in random order) give
    a different iterate that still converges."""
    from async_band import row_order_slices, row_replay, _replay_slices
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 12, amg.AMG_INTERP_LINEAR)
    N = 6
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    n0 = 12 ** 3
    f = amg.rhs_rand(0, n0)
    d = np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)])
    ends = [d[k] * np.arange(1, N + 1) for k in range(L - 1)] + [np.zeros(0)]
    flat = [[np.repeat(e[:, None], n0, axis=1) for e in ends]]
    cuts, tabs, _ = row_order_slices(flat, L)
    assert cuts == [0, n0] and len(tabs) == 1
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle.make_opts(
        solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0))
    _, rel1, _ = OH.async_add_replay(f, [0, n0], [e[:, None] for e in ends])
    relf, nsl, _ = row_replay(amg, oracle, host, f, opts, flat)
    assert nsl == 1 and relf == rel1
    # torn: level 0's update j = 2 (9.15) overlaps level 1's update j = 5
    # (9.78); waves of 64 rows of each run at random times inside the overlap
    g = np.random.default_rng(5)
    torn = [[t.copy() for t in flat[0]]]
    mid = 0.5 * (ends[0][2] + ends[1][5])
    assert ends[0][1] < mid - 0.01 and ends[0][3] > mid + 0.01 and ends[1][4] < mid - 0.01
    for w in range(0, n0, 64):
        torn[0][0][2, w:w + 64] = mid + g.uniform(-0.01, 0.01)
        torn[0][1][5, w:w + 64] = mid + g.uniform(-0.01, 0.01)
    cuts, tabs, _ = row_order_slices(torn, L)
    assert 2 < len(tabs) <= n0 // 64
    relm, _, _ = row_replay(amg, oracle, host, f, opts, torn)
    per_row = [[torn[0][k][:, i] for k in range(L)] for i in range(n0)]
    relr = _replay_slices(amg, oracle, host, f, opts, list(range(n0 + 1)), per_row)
    assert relm == relr
    assert relm != rel1 and relm < 0.5, (relm, rel1)


def test_chain_order():
    """async_band.chain_order: a row whose adds the clock put in the wrong order
    is put back in the order its adds' values chain in (each add's old value the
    previous add's new value); rows that already chain are left alone."""
    from async_band import chain_order
    e = np.array([1.0, 2.0, 0.5])
    # true order 2, 0, 1 from u0 = 0
    old = np.zeros(3)
    new = np.zeros(3)
    cur = 0.0
    for x in (2, 0, 1):
        old[x], new[x] = cur, cur + e[x]
        cur = new[x]
    vo = np.stack([old, np.array([0.0, 1.0, 3.0])])
    vn = np.stack([new, np.array([1.0, 3.0, 3.5])])
    order = np.array([[0, 1, 2], [0, 1, 2]])
    got, nrep, nleft = chain_order(order, vo, vn)
    assert got[0].tolist() == [2, 0, 1] and got[1].tolist() == [0, 1, 2]
    assert (nrep, nleft) == (1, 0)


def test_composed_transfers_match_explicit(amg, oracle):
    """or_hier_set_composed_transfers: the smoothed transfers applied composed
    from the plain P / R (R~ r = R (r - w A D^-1 r), P~ e = P e - w D^-1 A P e)
    are the explicit SmoothTransfer products (or_smooth_transfer) up to
    rounding: the synchronous MULTADD iterates agree to 1e-12 relative, and the
    round-robin asynchronous runs likewise."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    f = amg.rhs_rand(0, 16 ** 3)
    for solver in (oracle.OR_MULTADD, oracle.OR_ASYNC_MULTADD):
        o = oracle.make_opts(solver=solver, smooth_weight=0.8, num_cycles=10, tol=0.0)
        EX = oracle.Hier(host["A"], Ps, Rs, o)
        CO = oracle.Hier(host["A"], host["P"], host["R"], o)
        CO.set_composed_transfers()
        if solver == oracle.OR_MULTADD:
            ue, he, _ = EX.solve(f)
            uc, hc, _ = CO.solve(f)
        else:
            oracle.lib().or_set_async_schedule(3)
            try:
                ue, re_, _ = EX.async_add(f, [1] * L)
                uc, rc_, _ = CO.async_add(f, [1] * L)
            finally:
                oracle.lib().or_set_async_schedule(0)
            assert abs(re_ - rc_) <= 1e-10 * re_, (re_, rc_)
        assert np.max(np.abs(ue - uc)) <= 1e-12 * np.max(np.abs(ue))
        # composed without smoothing weight effect is not the plain cycle
        PL = oracle.Hier(host["A"], host["P"], host["R"], o)
        if solver == oracle.OR_MULTADD:
            up, _, _ = PL.solve(f)
            assert np.max(np.abs(up - uc)) > 1e-6 * np.max(np.abs(uc))


@pytest.mark.parametrize("conv,at,inflight,save", [("local", 0, 1, 1), ("global", 0, 2, 1), ("local", 1, 1, 1),
                                                    ("local", 0, 3, 2)])
def test_dmem_add_oracle(amg, oracle, conv, at, inflight, save):
    """or_dmem_add (DMEM_Add restated, threads for ranks, one rank per grid):
    the round-robin schedule is deterministic (two runs, the same bits), both
    it and the free race converge on the smoothed-transfer 16^3 hierarchy,
    every message sent is received, converge LOCAL runs exactly num_cycles per
    grid and GLOBAL at least that many"""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    N = 12
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    ct = oracle.OR_CONVERGE_GLOBAL if conv == "global" else oracle.OR_CONVERGE_LOCAL
    kw = dict(converge_type=ct, async_type=at, max_inflight=inflight, save_divisor=save)
    runs = [OH.dmem_add(f, sched=1, **kw) for _ in range(2)] + [OH.dmem_add(f, sched=0, **kw) for _ in range(3)]
    x1 = runs[0][0]
    assert np.array_equal(runs[1][0].view(np.uint64), x1.view(np.uint64))
    assert np.array_equal(runs[1][1], runs[0][1])
    for q, (x, cyc, rel, msg) in enumerate(runs):
        assert np.all(np.isfinite(x))
        assert msg[:, 0].sum() == msg[:, 1].sum(), msg
        if conv == "local":
            assert np.all(cyc == N), cyc
        else:
            assert np.all(cyc >= N), cyc
        # round robin: every correction reaches every grid a turn later (the
        # synchronous MULTADD reaches 1.9e-5 in 12 cycles here); the free race
        # can run a grid's cycles before the others' corrections arrive
        assert np.all(rel < ((1e-3 if save == 1 else 1e-2) if q < 2 else 1.0)), (q, rel)
    print(f"dmem_add {conv} async_type {at} inflight {inflight} save {save}: round robin relres {runs[0][2]}, "
          f"cycles {runs[0][1]}; free {[r[2].max() for r in runs[2:]]}")


@pytest.mark.parametrize("sched", [2, 3])
def test_dmem_add_sequential_schedules(amg, oracle, sched):
    """or_dmem_add's sequential schedules (converge LOCAL): the finest / coarsest
    grid keeps the token through its main loop and hands it on only where a
    reference rank would block -- the race's extreme speed ratios, members of
    the grid tests' band.  Deterministic (two runs, the same bits), every grid
    runs num_cycles, every message sent is received; GLOBAL is refused."""
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    N = 12
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    OH = oracle.Hier(host["A"], Ps, Rs, o)
    f = amg.rhs_rand(0, 16 ** 3)
    runs = [OH.dmem_add(f, sched=sched, max_inflight=2) for _ in range(2)]
    assert np.array_equal(runs[0][0].view(np.uint64), runs[1][0].view(np.uint64))
    x, cyc, rel, msg = runs[0]
    assert np.all(np.isfinite(x)) and np.all(cyc == N), cyc
    assert msg[:, 0].sum() == msg[:, 1].sum(), msg
    rr = OH.dmem_add(f, sched=1, max_inflight=2)
    print(f"dmem_add sequential {sched}: relres {rel}; round robin {rr[2]}")
    with pytest.raises(Exception):
        OH.dmem_add(f, sched=sched, converge_type=oracle.OR_CONVERGE_GLOBAL)
