"""Asynchronous additive AMG options on one GPU (SMEM_Async_Add_AMG,
SMEM_Async_AMG.cpp:7-437): async_type FULL_ASYNC / SEMI_ASYNC (the lock of
:238-283 as one serialised update stream), read_type READ_SOL / READ_RES
(:227-236, 288-295, 416-426), res_compute_type LOCAL / GLOBAL (:35-77,
356-414; ASYNC_MULTADD only, SMEM_Main.cpp:650-660) and converge_test_type
LOCAL / GLOBAL (:317-337, Misc.cpp:418-441).

Every asynchronous run is nondeterministic, as in the reference, so each
combination is checked against the oracle's ASYNCHRONOUS band: the reference's
SMEM_Async_Add_AMG restated on OpenMP threads (oracle or_async_add, groups of
one and two threads per level, 10 runs each) with the same smoother, blocks,
corrections, async / read / converge types; the device's final relative
residual must lie in [0.5 x min, 2 x max] of the band.
res_compute GLOBAL (no level-0 group; every group smooths its slice of the
fine grid and writes its slice of the shared residual) is restated in the
oracle too (or_set_async_res_global); its band adds the two sequential group
schedules (the race's extreme speed ratios) in place of a lockstep member.
converge GLOBAL also checks the per-level correction counts."""
import numpy as np
import pytest

from async_band import blocks64, in_band, oracle_async_band, race_tables, replay_check, times_of
from test_gpu_kernels import assert_bitwise
from test_gpu_solve import hierarchy, gpu_hier, oracle_opts

pytestmark = pytest.mark.gpu

N = 15
W = 0.8


@pytest.fixture(scope="module")
def setup(amg, oracle):
    _, L, host = hierarchy(amg, oracle, 24, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], W)
        Ps.append(ps)
        Rs.append(rs)
    mult = {"A": host["A"], "P": Ps, "R": Rs}  # MULTADD: smoothed transfers
    afacx = host
    f = amg.rhs_rand(0, 24 ** 3)
    return L, mult, afacx, f


def sync_band(amg, oracle, host, f, solver, smoother):
    o = amg.default_opts(solver=solver, smoother=smoother, smooth_weight=W, num_cycles=N, tol=0.0,
                         num_threads=0, jgs_block_rows=64)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, o))
    if smoother == amg.AMG_HYBRID_JGS:
        for lev in range(len(host["A"])):
            n = host["A"][lev].nrows
            OH.set_blocks(lev, np.unique(np.minimum(np.arange(0, n + 64, 64), n)).astype(np.int32))
    _, h, _ = OH.solve(f)
    return h[-1] / h[0]


CASES = [
    # (solver, smoother, async_type, read_type, res_compute_type, converge_test_type)
    ("multadd", "jacobi", "semi", "sol", "local", "local"),
    ("multadd", "jacobi", "full", "res", "local", "local"),
    ("multadd", "jacobi", "semi", "res", "local", "local"),
    ("multadd", "jacobi", "full", "sol", "global", "local"),
    ("multadd", "jacobi", "semi", "sol", "global", "local"),
    ("multadd", "hybrid", "semi", "sol", "local", "local"),
    ("multadd", "hybrid", "full", "sol", "global", "local"),
    ("multadd", "jacobi", "full", "sol", "local", "global"),
    ("multadd", "jacobi", "semi", "res", "local", "global"),
    # res_compute GLOBAL with converge GLOBAL: the correction that sees the
    # converge flag leaves before the GLOBAL residual update (:353-356)
    ("multadd", "jacobi", "full", "sol", "global", "global"),
    ("afacx", "jacobi", "semi", "sol", "local", "local"),
    ("afacx", "jacobi", "full", "res", "local", "local"),
]


@pytest.mark.parametrize("case", CASES, ids=["-".join(c) for c in CASES])
def test_async_options_band(amg, oracle, ctx, setup, case):
    solver, smoother, at, rt, rc, ct = case
    L, mult, afacx, f = setup
    host = mult if solver == "multadd" else afacx
    sv_sync = amg.AMG_MULTADD if solver == "multadd" else amg.AMG_AFACX
    sv = amg.AMG_ASYNC_MULTADD if solver == "multadd" else amg.AMG_ASYNC_AFACX
    sm = amg.AMG_JACOBI if smoother == "jacobi" else amg.AMG_HYBRID_JGS
    sync_rel = sync_band(amg, oracle, host, f, sv_sync, sm)
    opts = amg.default_opts(
        solver=sv, smoother=sm, smooth_weight=W, num_cycles=N, tol=0.0, num_threads=0, jgs_block_rows=64,
        async_type=amg.AMG_SEMI_ASYNC if at == "semi" else amg.AMG_FULL_ASYNC,
        read_type=amg.AMG_READ_RES if rt == "res" else amg.AMG_READ_SOL,
        res_compute_type=amg.AMG_GLOBAL if rc == "global" else amg.AMG_LOCAL,
        converge_test_type=amg.AMG_GLOBAL if ct == "global" else amg.AMG_LOCAL)
    H, _ = gpu_hier(amg, ctx, host, opts)
    rels, cmax, durs = [], 0, []
    for _ in range(2):
        u, rel, cnt = H.async_solve(f)
        assert np.all(np.isfinite(u))
        rels.append(rel)
        e_, s_ = race_tables(H)
        durs.append((rel, e_, None, s_))
        # correcting levels: [k_lo, k_hi); GLOBAL residuals replace level 0's
        # group by the sliced fine smoothing (SMEM_Setup.cpp:609-615)
        # (and the coarsest level's group runs: it smooths its slice)
        gres = rc == "global" and solver == "multadd"
        k_lo = 1 if gres else 0
        k_hi = L if gres else max(k_lo + 1, L - 1)
        assert np.all(cnt[:k_lo] == 0) and np.all(cnt[k_hi:] == 0), cnt
        if ct == "global":
            # every level ran at least num_cycles corrections; faster ones more
            assert np.all(cnt[k_lo:k_hi] >= N), cnt
            assert np.all(cnt[k_lo:k_hi] <= 1000 * N), cnt
            cmax = max(cmax, int(np.max(cnt[k_lo:k_hi])))
        else:
            assert np.all(cnt[k_lo:k_hi] == N), cnt
    H.free()
    blocks = blocks64(host) if sm == amg.AMG_HYBRID_JGS else None
    # the oracle's model of each device run: the replay of the order in which
    # its corrections ended (or_async_add under the timed schedule with the
    # recorded end times)
    widest = replay_check(amg, oracle, host, f, opts, durs, blocks=blocks, what="-".join(case))
    # for the record: the oracle's own free races on this container's threads
    # (every speed ratio the OS happens to give; not the acceptance window)
    flo, fhi, orels, _ = oracle_async_band(amg, oracle, host, f, opts, reps=4, blocks=blocks)
    print(f"{'-'.join(case)}: device relres {rels}, max corrections {cmax}; "
          f"oracle free races [{flo:.3e}, {fhi:.3e}] ({fhi / flo:.1f}x)")
    from async_band import free_band_check
    free_band_check(amg, opts, rels, flo, fhi, what="-".join(case))
    assert sync_rel < 1.0
    assert widest <= 20.0
    for rel in rels:
        assert rel < 1.0, (case, rels)


SCHED_CASES = [(c, s) for c in CASES for s in ((3, 4) if c[5] == "global" else (1, 2, 3, 4))]


def timed_durations(L):
    """fixed per-level correction times for the timed schedule's bitwise tests
    (fine levels slower; every ratio non-integer so the order interleaves)"""
    return np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)])


@pytest.mark.parametrize("case,sched", SCHED_CASES, ids=["-".join(c) + f"-s{s}" for c, s in SCHED_CASES])
def test_async_schedule_bitwise(amg, oracle, ctx, setup, case, sched):
    """The asynchronous arithmetic pinned bit for bit: the device's
    deterministic-schedule mode (amg_opts.async_schedule: the level groups one
    after another, finest / coarsest first, or taking turns one whole
    correction each) against the oracle's restatement of SMEM_Async_Add_AMG
    (SMEM_Async_AMG.cpp:7-437) run with the same schedule
    (or_set_async_schedule), one thread per level group.  Every update of the
    shared iterate / residual (atomic adds and the private copies they return,
    SEMI_ASYNC's exclusive updates, READ_RES sums, the GLOBAL residual slices,
    converge GLOBAL's stopping rule) then happens in one order on both sides:
    the iterate must be the same bits and the correction counts equal."""
    solver, smoother, at, rt, rc, ct = case
    L, mult, afacx, f = setup
    host = mult if solver == "multadd" else afacx
    sv = amg.AMG_ASYNC_MULTADD if solver == "multadd" else amg.AMG_ASYNC_AFACX
    sm = amg.AMG_JACOBI if smoother == "jacobi" else amg.AMG_HYBRID_JGS
    opts = amg.default_opts(
        solver=sv, smoother=sm, smooth_weight=W, num_cycles=N, tol=0.0, num_threads=0, jgs_block_rows=64,
        async_type=amg.AMG_SEMI_ASYNC if at == "semi" else amg.AMG_FULL_ASYNC,
        read_type=amg.AMG_READ_RES if rt == "res" else amg.AMG_READ_SOL,
        res_compute_type=amg.AMG_GLOBAL if rc == "global" else amg.AMG_LOCAL,
        converge_test_type=amg.AMG_GLOBAL if ct == "global" else amg.AMG_LOCAL,
        async_schedule=sched)
    H, _ = gpu_hier(amg, ctx, host, opts)
    if sched == 4:
        H.set_async_durations(timed_durations(L))
        oracle.set_async_durations(timed_durations(L))
    u, rel, cnt = H.async_solve(f)
    H.free()
    gres = rc == "global" and solver == "multadd"
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if sm == amg.AMG_HYBRID_JGS:
        for lev, blk in blocks64(host).items():
            OH.set_blocks(lev, blk)
    oracle.lib().or_set_async_schedule(sched)
    try:
        uo, relo, cnto = OH.async_add(
            f, [0 if gres else 1] + [1] * (L - 1),
            async_type=oracle.OR_SEMI_ASYNC if at == "semi" else oracle.OR_FULL_ASYNC,
            converge_type=oracle.OR_CONVERGE_GLOBAL if ct == "global" else oracle.OR_CONVERGE_LOCAL,
            read_type=oracle.OR_READ_RES if rt == "res" else oracle.OR_READ_SOL, res_global=gres)
    finally:
        oracle.lib().or_set_async_schedule(0)
    # correcting levels: [k_lo, k_hi) (GLOBAL residuals: the coarsest group too)
    k_lo = 1 if gres else 0
    k_hi = L if gres else max(k_lo + 1, L - 1)
    assert list(cnt[k_lo:k_hi]) == list(cnto[k_lo:k_hi]), (cnt, cnto)
    if ct == "local":
        assert np.all(cnt[k_lo:k_hi] == N), cnt
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"{'-'.join(case)} schedule {sched}: device relres {rel:.13e}, oracle {relo:.13e}, "
          f"counts {list(cnt[k_lo:k_hi])}, differing entries {nd}")
    assert nd == 0
    assert abs(rel - relo) <= 1e-12 * relo


def test_semi_async_single_level_matches_local_residual_order(amg, oracle, ctx):
    """With one active level (2-level hierarchy) SEMI_ASYNC and FULL_ASYNC
    READ_SOL do the same arithmetic: their iterates agree bit for bit."""
    _, L, host = hierarchy(amg, oracle, 16, amg.AMG_INTERP_AGGREGATE, levels=2)
    f = amg.rhs_rand(0, 16 ** 3)
    outs = []
    for at in (amg.AMG_FULL_ASYNC, amg.AMG_SEMI_ASYNC):
        opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=W, num_cycles=10, tol=0.0,
                                async_type=at)
        H, _ = gpu_hier(amg, ctx, host, opts)
        u, rel, cnt = H.async_solve(f)
        H.free()
        outs.append((u, rel))
    assert np.array_equal(outs[0][0].view(np.uint64), outs[1][0].view(np.uint64))
    assert outs[0][1] == outs[1][1]


@pytest.mark.parametrize("case,sched", [(CASES[0], 3), (CASES[1], 1), (CASES[5], 2), (CASES[6], 3), (CASES[7], 3)],
                         ids=["jacobi-semi-sol-s3", "jacobi-full-res-s1", "hybrid-semi-s2", "hybrid-gres-s3",
                              "jacobi-convglobal-s3"])
def test_composed_transfers_async_bitwise(amg, oracle, ctx, setup, case, sched):
    """smooth_transfer = 1: the MULTADD transfers are the reference's smoothed
    P~ = (I - w D^-1 A) P, R~ = P~^T (SmoothTransfer, SMEM_Setup.cpp:1173-1254)
    applied composed on the device from the plain P / R / A; under a
    deterministic schedule the iterate is bit-identical to the oracle's
    composed restatement (or_hier_set_composed_transfers) and, to rounding,
    to the explicit smoothed operators."""
    solver, smoother, at, rt, rc, ct = case
    L, mult, afacx, f = setup
    host = afacx  # plain transfers: the device composes the smoothing
    sm = amg.AMG_JACOBI if smoother == "jacobi" else amg.AMG_HYBRID_JGS
    gres = rc == "global"
    opts = amg.default_opts(
        solver=amg.AMG_ASYNC_MULTADD, smoother=sm, smooth_weight=W, num_cycles=N, tol=0.0, num_threads=0,
        jgs_block_rows=64, async_type=amg.AMG_SEMI_ASYNC if at == "semi" else amg.AMG_FULL_ASYNC,
        read_type=amg.AMG_READ_RES if rt == "res" else amg.AMG_READ_SOL,
        res_compute_type=amg.AMG_GLOBAL if gres else amg.AMG_LOCAL,
        converge_test_type=amg.AMG_GLOBAL if ct == "global" else amg.AMG_LOCAL,
        async_schedule=sched, smooth_transfer=1)
    H, _ = gpu_hier(amg, ctx, host, opts)
    u, rel, cnt = H.async_solve(f)
    H.free()
    res = {}
    for name, hh, comp in (("composed", host, True), ("explicit", mult, False)):
        OH = oracle.Hier(hh["A"], hh["P"], hh["R"], oracle_opts(oracle, opts))
        if comp:
            OH.set_composed_transfers()
        if sm == amg.AMG_HYBRID_JGS:
            for lev, blk in blocks64(hh).items():
                OH.set_blocks(lev, blk)
        oracle.lib().or_set_async_schedule(sched)
        try:
            res[name] = OH.async_add(
                f, [0 if gres else 1] + [1] * (L - 1),
                async_type=oracle.OR_SEMI_ASYNC if at == "semi" else oracle.OR_FULL_ASYNC,
                converge_type=oracle.OR_CONVERGE_GLOBAL if ct == "global" else oracle.OR_CONVERGE_LOCAL,
                read_type=oracle.OR_READ_RES if rt == "res" else oracle.OR_READ_SOL, res_global=gres)
        finally:
            oracle.lib().or_set_async_schedule(0)
    uo, relo, cnto = res["composed"]
    ue, rele, _ = res["explicit"]
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"composed {'-'.join(case)} s{sched}: device {rel:.13e} oracle {relo:.13e} explicit {rele:.13e}, "
          f"differing entries {nd}")
    assert nd == 0
    assert np.max(np.abs(ue - u)) <= 1e-10 * np.max(np.abs(ue))


def test_composed_transfers_sync_bitwise(amg, oracle, ctx, setup):
    """the synchronous MULTADD cycle (SMEM_Sync_Add_Vcycle) with composed
    smoothed transfers: iterate bit-identical to the oracle's after every
    cycle, relres history within 1e-12"""
    L, mult, afacx, f = setup
    opts = amg.default_opts(solver=amg.AMG_MULTADD, smooth_weight=W, num_cycles=10, tol=0.0, smooth_transfer=1)
    H, _ = gpu_hier(amg, ctx, afacx, opts)
    u, hist, k = H.solve(f)
    H.free()
    OH = oracle.Hier(afacx["A"], afacx["P"], afacx["R"], oracle_opts(oracle, opts))
    OH.set_composed_transfers()
    uo, ho, _ = OH.solve(f)
    assert k == 10
    assert np.array_equal(u.view(np.uint64), uo.view(np.uint64))
    np.testing.assert_allclose(hist, ho, rtol=1e-12, atol=0)
    assert hist[-1] / hist[0] < 0.05


@pytest.mark.parametrize("mode", ["sync", "async-jacobi-s3", "async-hybrid-s1"])
def test_composed_transfers_geometric_bitwise(amg, oracle, ctx, mode):
    """composed smoothed transfers on a plane-marched 64^3 hierarchy whose plain
    P / R are the checked geometric transfers (amg_hier_fused bit l + 1): the
    transfers run as the geometric restriction / prolongation kernels (and the
    fused level-0 forms), and the iterate is bit-identical to the oracle's
    composed restatement -- synchronous MULTADD after every cycle, the
    asynchronous cycle under a deterministic schedule"""
    n = 64
    _, L, host = hierarchy(amg, oracle, n, amg.AMG_INTERP_LINEAR)
    f = amg.rhs_rand(0, n ** 3)
    hybrid = "hybrid" in mode
    sm = amg.AMG_HYBRID_JGS if hybrid else amg.AMG_JACOBI
    sched = int(mode[-1]) if mode != "sync" else 0
    opts = amg.default_opts(solver=amg.AMG_MULTADD if mode == "sync" else amg.AMG_ASYNC_MULTADD, smoother=sm,
                            smooth_weight=W, num_cycles=8, tol=0.0, num_threads=0, jgs_block_rows=64,
                            async_schedule=sched, smooth_transfer=1)
    H, _ = gpu_hier(amg, ctx, host, opts)
    assert H.fused & 2, "level 0's transfers not detected as geometric"
    if mode == "sync":
        u, hist, k = H.solve(f)
    else:
        u, rel, cnt = H.async_solve(f)
    H.free()
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    OH.set_composed_transfers()
    if hybrid:
        for lev, blk in blocks64(host).items():
            OH.set_blocks(lev, blk)
    if mode == "sync":
        uo, ho, _ = OH.solve(f)
        assert k == 8
        np.testing.assert_allclose(hist, ho, rtol=1e-12, atol=0)
    else:
        oracle.lib().or_set_async_schedule(sched)
        try:
            uo, relo, cnto = OH.async_add(f, [1] * L)
        finally:
            oracle.lib().or_set_async_schedule(0)
        assert list(cnt[:L - 1]) == list(cnto[:L - 1])
        assert abs(rel - relo) <= 1e-12 * relo
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"composed geometric {mode}: differing entries {nd}")
    assert nd == 0



ZERO_SWEEPS = [(0, 1), (1, 0), (0, 0)]


@pytest.mark.parametrize("pre,post", ZERO_SWEEPS, ids=[f"pre{a}-post{b}" for a, b in ZERO_SWEEPS])
@pytest.mark.parametrize("mode", ["sync", "async-s3", "geo-sync", "geo-async-s1"])
def test_composed_transfers_zero_sweeps_bitwise(amg, oracle, ctx, setup, pre, post, mode):
    """SmoothTransfer (SMEM_Setup.cpp:1173-1254) forms P~ only when
    num_post_smooth_sweeps > 0 and R~ only when num_pre_smooth_sweeps > 0:
    with a zero sweep count the corresponding transfer stays the plain one.
    The device (the generic composed chain on 24^3 and the fused geometric
    forms on a marched 64^3 hierarchy) is bit-identical to the oracle's
    composed restatement with the same gating, synchronous MULTADD after every
    cycle and the asynchronous cycle under a deterministic schedule."""
    geo = mode.startswith("geo")
    if geo:
        n = 64
        _, L, host = hierarchy(amg, oracle, n, amg.AMG_INTERP_LINEAR)
        f = amg.rhs_rand(0, n ** 3)
    else:
        L, _, host, f = setup
    sched = int(mode[-1]) if "async" in mode else 0
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD if sched else amg.AMG_MULTADD, smooth_weight=W,
                            num_cycles=6, tol=0.0, async_schedule=sched, smooth_transfer=1,
                            num_pre_smooth_sweeps=pre, num_post_smooth_sweeps=post)
    H, _ = gpu_hier(amg, ctx, host, opts)
    if geo:
        assert H.fused & 2, "level 0's transfers not detected as geometric"
    if sched:
        u, rel, cnt = H.async_solve(f)
    else:
        u, hist, k = H.solve(f)
    H.free()
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    OH.set_composed_transfers()
    if sched:
        oracle.lib().or_set_async_schedule(sched)
        try:
            uo, relo, cnto = OH.async_add(f, [1] * L)
        finally:
            oracle.lib().or_set_async_schedule(0)
        assert list(cnt[:L - 1]) == list(cnto[:L - 1])
    else:
        uo, ho, _ = OH.solve(f)
        np.testing.assert_allclose(hist, ho, rtol=1e-12, atol=0)
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"composed pre {pre} post {post} {mode}: differing entries {nd}")
    assert nd == 0


@pytest.mark.parametrize("hybrid", [0, 1], ids=["jacobi", "hybrid-fold"])
def test_update_windows(amg, oracle, ctx, setup, hybrid):
    """the device-clock execution windows of a free race's update kernels
    (amg_async_update_windows; the hybrid case's level 0 folds its correction
    into the last JGS sweep, which stamps it): one per correction, start <
    end, a level's windows in order without overlap (its stream runs them one
    after another), every window inside the solve; replayed in their end order
    (AMG_SCHED_TIMED with the ends) the device's iterate is the oracle's
    replay's bit for bit"""
    L, mult, afacx, f = setup
    host = mult
    kw = dict(solver=amg.AMG_ASYNC_MULTADD, smoother=amg.AMG_HYBRID_JGS if hybrid else amg.AMG_JACOBI,
              smooth_weight=W, num_cycles=N, tol=0.0, num_threads=0, jgs_block_rows=64)
    opts = amg.default_opts(**kw)
    blocks = blocks64(host) if hybrid else None
    ctx.set_jgs_fold(hybrid)
    H, _ = gpu_hier(amg, ctx, host, opts)
    _, rel, cnt = H.async_solve(f)
    w0, w1 = H.async_update_windows()
    H.free()
    lo = min(float(x[0]) for x in w0 if len(x))
    for k in range(L - 1):
        s_, e_ = np.asarray(w0[k]), np.asarray(w1[k])
        assert len(s_) == len(e_) == cnt[k] == N, (k, len(s_), len(e_), cnt[k])
        assert np.all(np.isfinite(s_)) and np.all(np.isfinite(e_)), k
        assert np.all(s_ < e_), k
        assert np.all(s_[1:] >= e_[:-1]), k
        print(f"level {k}: windows {1e3 * np.mean(e_ - s_):.1f} us on average, first at {1e3 * (s_[0] - lo):.1f} us")
    times = [np.asarray(w1[k]) - lo for k in range(L - 1)]
    times.append(times[-1].copy())  # the reference's idle coarsest group
    opts = amg.default_opts(async_schedule=4, **kw)
    H, _ = gpu_hier(amg, ctx, host, opts)
    H.set_async_times(times)
    u, rel, cnt = H.async_solve(f)
    H.free()
    ctx.set_jgs_fold(0)
    oracle.set_async_times(times)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if blocks is not None:
        for lev, blk in blocks.items():
            OH.set_blocks(lev, blk)
    oracle.lib().or_set_async_schedule(4)
    try:
        uo, relo, cnto = OH.async_add(f, [1] * L)
    finally:
        oracle.lib().or_set_async_schedule(0)
    assert_bitwise(u, uo, "windows replay")


@pytest.mark.parametrize("case", [CASES[1], CASES[4], CASES[7]], ids=["jacobi-full-res", "jacobi-semi-gres",
                                                                      "jacobi-convglobal"])
def test_async_replay_bitwise(amg, oracle, ctx, setup, case):
    """the replay of a free race: the device records the end of every
    correction (async_correction_ms); AMG_SCHED_TIMED with those end times
    (amg_hier_set_async_times) re-runs the corrections in that order on one
    stream, bit-identical to the oracle's or_async_add under schedule 4 with
    the same times (or_set_async_times) -- the model the free-race checks
    compare against"""
    solver, smoother, at, rt, rc, ct = case
    L, mult, afacx, f = setup
    host = mult
    kw = dict(solver=amg.AMG_ASYNC_MULTADD, smoother=amg.AMG_JACOBI, smooth_weight=W, num_cycles=N, tol=0.0,
              async_type=amg.AMG_SEMI_ASYNC if at == "semi" else amg.AMG_FULL_ASYNC,
              read_type=amg.AMG_READ_RES if rt == "res" else amg.AMG_READ_SOL,
              res_compute_type=amg.AMG_GLOBAL if rc == "global" else amg.AMG_LOCAL,
              converge_test_type=amg.AMG_GLOBAL if ct == "global" else amg.AMG_LOCAL)
    opts_free = amg.default_opts(**kw)
    H, _ = gpu_hier(amg, ctx, host, opts_free)
    _, rel_free, cnt_free = H.async_solve(f)
    times = times_of(H.async_correction_ms(), L)
    race = race_tables(H)
    H.free()
    opts = amg.default_opts(async_schedule=4, **kw)
    H, _ = gpu_hier(amg, ctx, host, opts)
    H.set_async_times(times)
    u, rel, cnt = H.async_solve(f)
    H.free()
    gres = rc == "global"
    oracle.set_async_times(times)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    oracle.lib().or_set_async_schedule(4)
    try:
        uo, relo, cnto = OH.async_add(
            f, [0 if gres else 1] + [1] * (L - 1),
            async_type=oracle.OR_SEMI_ASYNC if at == "semi" else oracle.OR_FULL_ASYNC,
            converge_type=oracle.OR_CONVERGE_GLOBAL if ct == "global" else oracle.OR_CONVERGE_LOCAL,
            read_type=oracle.OR_READ_RES if rt == "res" else oracle.OR_READ_SOL, res_global=gres)
    finally:
        oracle.lib().or_set_async_schedule(0)
    k_lo = 1 if gres else 0
    k_hi = L if gres else L - 1
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"replay {'-'.join(case)}: free race {rel_free:.6e} (counts {list(cnt_free)}), device replay {rel:.13e}, "
          f"oracle {relo:.13e}, counts {list(cnt[k_lo:k_hi])} / {list(cnto[k_lo:k_hi])}, differing {nd}")
    assert list(cnt[k_lo:k_hi]) == list(cnto[k_lo:k_hi])
    assert nd == 0
    # the free race itself against the replay of its own update order (the
    # update kernels' row stamps where the options allow the exact replay)
    replay_check(amg, oracle, host, f, opts_free, [(rel_free, race[0], None, race[1])],
                 what=f"free race {'-'.join(case)}")
