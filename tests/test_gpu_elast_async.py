"""Config 5's solver on its own problem: the asynchronous additive cycle on
the DMEM elasticity hierarchy (DMEM_BuildMfemMatrix, DMEM_BuildMatrix.cpp:
442-719: Q1 vector H1, 3 unknowns per node, 81-entry rows; classical setup
with the DMEM parameters -- PMIS (coarsen 9), extended+i, theta 0.5, three
functions) driven through DMEM_Add's asynchronous additive cycle
(DMEM_Add.cpp:20-178; SMEM_Async_AMG.cpp:7-437), pinned at r = 3:

* one GPU (amg_async_solve) and the row-partitioned distributed solve
  (amg_dist_async_solve, 1-3 ranks) under the deterministic schedules
  (finest / coarsest first, round robin, timed) -- the iterate bit-identical
  to the oracle's or_async_add under the same schedule, with the reference's
  smoothed transfers explicit (SmoothTransfer, SMEM_Setup.cpp:1173-1254) and
  composed on the fly (smooth_transfer = 1);
* the level-grouped DMEM_Add solve (one grid per level, the device hub)
  under round robin -- every grid's iterate bit-identical to or_dmem_add's,
  with equal cycle and message counts;
* the free races (one GPU, 2 ranks) against the oracle's replays of their
  recorded update orders."""
import numpy as np
import pytest

from async_band import race_tables

from test_gpu_dist import run_ranks, split_host
from test_gpu_kernels import assert_bitwise
from test_gpu_solve import gpu_hier, oracle_opts

pytestmark = pytest.mark.gpu

W = 0.6   # weighted Jacobi on the elasticity operator (test_gpu_classical.py)
N = 10


@pytest.fixture(scope="module")
def elast(amg, oracle):
    from test_gpu_classical import host_levels
    n, rp, cj, v, b = amg.classical.elasticity(3)
    H = amg.classical.ClassicalAMG(n, rp, cj, v, coarsen_type=9, strong_threshold=0.5, num_functions=3)
    lv = host_levels(amg, H)
    plain = {k: [oracle.Csr(*m) for m in lv_] for k, lv_ in lv.items()}
    L = len(plain["A"])
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(plain["A"][lev], plain["P"][lev], W)
        Ps.append(ps)
        Rs.append(rs)
    smoothed = {"A": plain["A"], "P": Ps, "R": Rs}
    return L, plain, smoothed, np.ascontiguousarray(b, dtype=np.float64)


def timed_durations(L):
    return np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)])


def oracle_sched(oracle, OH, f, L, sched):
    if sched == 4:
        oracle.set_async_durations(timed_durations(L))
    oracle.lib().or_set_async_schedule(sched)
    try:
        return OH.async_add(f, [1] * L)
    finally:
        oracle.lib().or_set_async_schedule(0)


CASES = [(s, c) for s in (1, 2, 3, 4) for c in ("explicit", "composed")]


@pytest.mark.parametrize("sched,xfer", CASES, ids=[f"s{s}-{c}" for s, c in CASES])
def test_elast_async_schedule_bitwise(amg, oracle, ctx, elast, sched, xfer):
    """one GPU: ASYNC_MULTADD on the r = 3 elasticity hierarchy (81-entry fine
    rows, value-indexed / long-row kernels) under a deterministic schedule,
    bit-identical to or_async_add"""
    L, plain, smoothed, f = elast
    comp = xfer == "composed"
    host = plain if comp else smoothed
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=W, num_cycles=N, tol=0.0,
                            async_schedule=sched, smooth_transfer=1 if comp else 0)
    H, _ = gpu_hier(amg, ctx, host, opts)
    if sched == 4:
        H.set_async_durations(timed_durations(L))
    u, rel, cnt = H.async_solve(f)
    H.free()
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if comp:
        OH.set_composed_transfers()
    uo, relo, cnto = oracle_sched(oracle, OH, f, L, sched)
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"elasticity r=3 ({host['A'][0].nrows} dofs, {L} levels) async {xfer} s{sched}: device {rel:.13e} "
          f"oracle {relo:.13e}, differing entries {nd}")
    assert list(cnt[:L - 1]) == list(cnto[:L - 1]) == [N] * (L - 1)
    assert nd == 0
    assert abs(rel - relo) <= 1e-12 * relo
    # (the finest-first schedule -- every fine correction before any coarse one --
    # need not contract in N corrections on this operator)
    assert np.isfinite(rel)


def dist_async(amg, host, f, opts, cuts, L, dur=None, runs=1):
    rs, parts = split_host(host, cuts)
    nranks = len(cuts) + 1
    hub = amg.dist.ThreadMailbox(nranks)

    def rank(r):
        c = amg.Context(0, nstreams=L)
        if nranks == 1:
            amg.dist.init_rccl(c, 1, 0, lambda b: b)
        else:
            amg.dist.init_host(c, nranks, r, amg.dist.HostTransport(hub, r))
        A, P, R = parts[r]
        D = amg.dist.DistHier.from_parts(c, rs, A, P, R, opts)
        if dur is not None:
            D.set_async_durations(dur)
        out = []
        for _ in range(runs):
            rel, cnt = D.async_solve(f[D.row0:D.row0 + D.n0])
            e_, s_ = race_tables(D)
            out.append((rel, cnt.copy(), D.get_u(), e_, s_))
        row0 = D.row0
        D.free()
        amg.dist.finalize(c)
        c.close()
        return row0, out

    res = sorted(run_ranks(nranks, rank), key=lambda t: t[0])
    out = []
    for q in range(runs):
        rel = res[0][1][q][0]
        assert all(t[1][q][0] == rel for t in res)
        out.append((rel, res[0][1][q][1], np.concatenate([t[1][q][2] for t in res]), [t[1][q][3] for t in res],
                    [int(x) for x in rs[0]], [t[1][q][4] for t in res]))
    return out


DCASES = [((0.5,), 3, "explicit"), ((0.3, 0.7), 1, "explicit"), ((0.45,), 2, "composed"), ((), 4, "composed"),
          ((0.5,), 4, "explicit")]


@pytest.mark.parametrize("cuts,sched,xfer", DCASES, ids=[f"{len(c) + 1}r-s{s}-{x}" for c, s, x in DCASES])
def test_elast_dist_async_schedule_bitwise(amg, oracle, elast, cuts, sched, xfer):
    """the row-partitioned distributed solve (DMEM_Add's ranks; halos of every
    level over the per-level channels) on the elasticity hierarchy under a
    deterministic schedule: the assembled iterate bit-identical to or_async_add"""
    L, plain, smoothed, f = elast
    comp = xfer == "composed"
    host = plain if comp else smoothed
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=W, num_cycles=N, tol=0.0,
                            async_schedule=sched, smooth_transfer=1 if comp else 0)
    ((rel, cnt, u, _, _, _),) = dist_async(amg, host, f, opts, cuts, L, dur=timed_durations(L) if sched == 4 else None)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if comp:
        OH.set_composed_transfers()
    uo, relo, cnto = oracle_sched(oracle, OH, f, L, sched)
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"elasticity dist async {len(cuts) + 1} ranks {xfer} s{sched}: device {rel:.13e} oracle {relo:.13e}, "
          f"differing entries {nd}")
    assert list(cnt[:L - 1]) == list(cnto[:L - 1]) == [N] * (L - 1)
    assert_bitwise(u, uo, "elasticity distributed async iterate vs oracle")
    assert abs(rel - relo) <= 1e-12 * relo


@pytest.mark.parametrize("conv", ["local", "global"])
def test_elast_grid_round_robin_bitwise(amg, oracle, elast, conv):
    """DMEM_Add's level-grouped solve (one grid per level; every grid holds
    the whole elasticity problem; AddCycle with the coarsest grid's exact
    solve; correction messages with done flags over the device hub) under
    round robin: every grid's iterate bit-identical to or_dmem_add's, with the
    same cycle and message counts"""
    from test_gpu_grid import grid_solve
    L, plain, smoothed, f = elast
    res, opts = grid_solve(amg, L, smoothed, f, (1,) * L, transport="device", num_cycles=N, max_inflight=2,
                           converge_test_type=amg.AMG_GLOBAL if conv == "global" else amg.AMG_LOCAL,
                           async_schedule=amg.AMG_SCHED_ROUND_ROBIN, smooth_weight=W)
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=W, num_cycles=N, tol=0.0)
    OH = oracle.Hier(smoothed["A"], smoothed["P"], smoothed["R"], o)
    xo, co, ro, mo = OH.dmem_add(f, sched=1, converge_type=oracle.OR_CONVERGE_GLOBAL if conv == "global"
                                 else oracle.OR_CONVERGE_LOCAL, max_inflight=2)
    for g, row0, x, cyc, rel, msgs in res:
        nd = int(np.count_nonzero(x.view(np.uint64) != xo[g].view(np.uint64)))
        print(f"elasticity grid {g}: device relres {rel:.6e} oracle {ro[g]:.6e}, cycles {cyc}/{co[g]}, "
              f"messages {list(msgs)}/{list(mo[g])}, differing entries {nd}")
        assert cyc == co[g]
        assert list(msgs) == list(mo[g])
        assert nd == 0, g
        assert abs(rel - ro[g]) <= 1e-10 * ro[g]


def test_elast_async_free_race_replay(amg, oracle, ctx, elast):
    """the free races on the elasticity hierarchy -- one GPU (a stream per
    level) and 2 ranks (a host thread and stream per level group on each) --
    within [0.5x, 2x] of the oracle's replay of each run's recorded update
    order (timed schedule / sliced replay), every level N corrections"""
    from async_band import replay_check
    L, plain, smoothed, f = elast
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=W, num_cycles=N, tol=0.0)
    H, _ = gpu_hier(amg, ctx, smoothed, opts)
    runs = []
    for _ in range(2):
        u, rel, cnt = H.async_solve(f)
        assert np.all(np.isfinite(u)) and list(cnt[:L - 1]) == [N] * (L - 1)
        e_, s_ = race_tables(H)
        runs.append((rel, e_, None, s_))
    H.free()
    replay_check(amg, oracle, smoothed, f, opts, runs, what="elasticity one GPU")
    druns = dist_async(amg, smoothed, f, opts, (0.5,), L, runs=3)
    for rel, cnt, u, _, _, _ in druns:
        assert np.all(np.isfinite(u)) and list(cnt[:L - 1]) == [N] * (L - 1)
    replay_check(amg, oracle, smoothed, f, opts, [(r[0], r[3], r[4], r[5]) for r in druns],
                 what="elasticity 2 ranks")
