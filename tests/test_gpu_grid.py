"""Level-grouped asynchronous additive solve (DMEM_Add, csrc/amg_grid.cpp) on the
GPU: ranks as threads sharing one GPU, split into one grid per level; every
grid holds the whole 24^3 problem row-partitioned among its ranks (intra-grid
halo over the host transport), computes its level's AddCycle correction
(restriction, DMEM_AddSmooth or the coarsest grid's exact solve, prolongation)
and exchanges corrections with the overlapping ranks of the other grids
through the message protocol: over the host transport (rendezvous mailboxes:
the in-flight pools fill) or the device hub (amg_devhub: payloads read device
to device, never staged through host memory).  The arithmetic and protocol are
pinned bit for bit against the oracle's DMEM_Add restatement (or_dmem_add)
under the round-robin schedule; the free race is checked as a band of that
restatement: every grid's final relative residual lies in [0.5 x min, 2 x max]
of or_dmem_add's free races and round robin, every message sent is received,
and the grids' iterates agree (they all add every correction)."""
import threading

import numpy as np
import pytest

from test_gpu_dist import run_ranks, split_host

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mult24(amg, oracle):
    from test_gpu_solve import hierarchy
    _, L, host = hierarchy(amg, oracle, 24, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    return L, {"A": host["A"], "P": Ps, "R": Rs}, amg.rhs_rand(0, 24 ** 3)


def grid_solve(amg, L, host, f, ppg, transport="host", **kw):
    n = host["A"][0].nrows
    rank_grid, rank_rows = amg.grid.layout(ppg, n)
    world = len(rank_grid)
    nb = amg.grid.ThreadNbHub(rank_grid) if transport == "host" else None
    # per grid: its ranks' row cuts of every level (the fine cuts of layout)
    parts, hubs, first = {}, {}, {}
    for g in range(len(ppg)):
        ranks = [r for r in range(world) if rank_grid[r] == g]
        first[g] = ranks[0]
        cuts = tuple(i / len(ranks) for i in range(1, len(ranks)))
        parts[g] = split_host(host, cuts)
        hubs[g] = amg.dist.ThreadMailbox(len(ranks))
    w = kw.pop("smooth_weight", 0.8)
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=w, tol=0.0, **kw)
    dh = amg.grid.DevHub(rank_grid) if transport == "device" else None
    # every rank starts its solve once all hierarchies are built (the
    # reference's ranks start DMEM_Add together): otherwise a fast grid runs
    # its cycles before slower ones post anything
    start = threading.Barrier(world)

    def rank(r):
        g = int(rank_grid[r])
        gr = r - first[g]
        rs, pr = parts[g]
        c = amg.Context(0, nstreams=2)
        tr = amg.dist.HostTransport(hubs[g], gr)
        amg.dist.init_host(c, int(np.sum(rank_grid == g)), gr, tr)
        A, P, R = pr[gr]
        D = amg.dist.DistHier.from_parts(c, rs, A, P, R, opts)
        assert D.row0 == rank_rows[2 * r] and D.row0 + D.n0 == rank_rows[2 * r + 1]
        G = amg.grid.GridAdd(dh if dh is not None else nb.transport(r), g, world, r, rank_grid, rank_rows,
                             dist_hier=D)
        start.wait()
        x, cyc, rel, msgs = G.solve(f[D.row0:D.row0 + D.n0])
        row0 = D.row0
        G.free()
        D.free()
        amg.dist.finalize(c)
        c.close()
        if tr.error is not None:
            raise tr.error
        return g, row0, x, cyc, rel, msgs

    try:
        return run_ranks(world, rank), opts
    finally:
        if dh is not None:
            dh.free()


_bands = {}


def dmem_cycle_members(oracle, host, f, opts, cycles):
    """further band members for grids that ran other cycle counts than the band's
    runs (converge GLOBAL: every grid keeps correcting until the slowest is done):
    the DMEM_Add restatement under round robin with converge LOCAL and
    num_cycles = c for every device cycle count c -- each grid's relres after
    exactly c cycles of the same protocol"""
    out = []
    for c in sorted(set(int(x) for x in cycles)):
        o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=opts.smooth_weight, num_cycles=c,
                             tol=opts.tol)
        OH = oracle.Hier(host["A"], host["P"], host["R"], o)
        _, _, rel, _ = OH.dmem_add(f, sched=1, converge_type=oracle.OR_CONVERGE_LOCAL, async_type=opts.async_type,
                                   max_inflight=opts.max_inflight, save_divisor=opts.async_comm_save_divisor,
                                   tol=opts.tol)
        out += rel.tolist()
    return out


def dmem_band(oracle, host, f, opts, reps=10, sequential=False):
    """the band of the DMEM_Add restatement (oracle or_dmem_add: grids as
    threads, one rank per grid, the same AddCycle / message protocol /
    termination): `reps` free races and the round-robin schedule; every grid's
    final relative residual of every run.  sequential (converge LOCAL): also
    the finest- / coarsest-first sequential schedules, the race's extreme speed
    ratios -- for runs whose grids are known to run at very uneven speeds"""
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=opts.smooth_weight,
                         num_cycles=opts.num_cycles, tol=opts.tol)
    OH = oracle.Hier(host["A"], host["P"], host["R"], o)
    kw = dict(converge_type=oracle.OR_CONVERGE_GLOBAL if opts.converge_test_type == 1 else oracle.OR_CONVERGE_LOCAL,
              async_type=opts.async_type, max_inflight=opts.max_inflight,
              save_divisor=opts.async_comm_save_divisor, tol=opts.tol)
    rels, cycs = [], []
    extra = [2, 3] if sequential and kw["converge_type"] == oracle.OR_CONVERGE_LOCAL else []
    for sched in [0] * reps + [1] + extra:
        _, cyc, rel, _ = OH.dmem_add(f, sched=sched, **kw)
        rels += rel.tolist()
        cycs += [int(c) for c in cyc]
    return min(rels), max(rels), rels, cycs


@pytest.mark.parametrize("conv,at,inflight,save", [("local", 0, 1, 1), ("global", 0, 2, 1), ("local", 1, 1, 1),
                                                    ("local", 0, 2, 2)])
def test_grid_add_round_robin_bitwise(amg, oracle, mult24, conv, at, inflight, save):
    """The level-grouped solve's arithmetic and protocol pinned bit for bit:
    one rank per grid over the device hub with async_schedule = ROUND_ROBIN
    (a token passes between the grids at the oracle's yield points) against
    the oracle's DMEM_Add restatement (or_dmem_add, DMEM_Add.cpp:20-944,
    DMEM_Comm.cpp:11-382) under the same schedule: every grid's iterate is the
    same bits, with the same cycle and message counts -- AddCycle with the
    coarsest grid's exact solve, AddCorrect / AddCheckComm including the
    dropped final payload, CheckInFlight with max_inflight, the save divisor,
    CheckConverge LOCAL / GLOBAL and AsyncRecvCleanup."""
    L, host, f = mult24
    N = 12
    res, opts = grid_solve(amg, L, host, f, (1,) * L, transport="device", num_cycles=N, max_inflight=inflight,
                           async_comm_save_divisor=save, async_type=at,
                           converge_test_type=amg.AMG_GLOBAL if conv == "global" else amg.AMG_LOCAL,
                           async_schedule=amg.AMG_SCHED_ROUND_ROBIN)
    o = oracle.make_opts(solver=oracle.OR_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0)
    OH = oracle.Hier(host["A"], host["P"], host["R"], o)
    xo, co, ro, mo = OH.dmem_add(f, sched=1, converge_type=oracle.OR_CONVERGE_GLOBAL if conv == "global"
                                 else oracle.OR_CONVERGE_LOCAL, async_type=at, max_inflight=inflight,
                                 save_divisor=save)
    for g, row0, x, cyc, rel, msgs in res:
        nd = int(np.count_nonzero(x.view(np.uint64) != xo[g].view(np.uint64)))
        print(f"grid {g}: device relres {rel:.6e} oracle {ro[g]:.6e}, cycles {cyc}/{co[g]}, "
              f"messages {list(msgs)}/{list(mo[g])}, differing entries {nd}")
        assert cyc == co[g]
        assert list(msgs) == list(mo[g])
        assert nd == 0, g
        assert abs(rel - ro[g]) <= 1e-10 * ro[g]


@pytest.mark.parametrize("transport", ["host", "device"])
@pytest.mark.parametrize("ppg,conv,inflight", [((1, 1, 1, 1), "local", 1), ((2, 1, 1, 1), "global", 2),
                                               ((2, 2, 1, 1), "local", 3)])
def test_grid_add_converges(amg, oracle, mult24, ppg, conv, inflight, transport):
    from async_band import in_band
    L, host, f = mult24
    ppg = ppg[:L] if len(ppg) >= L else ppg + (1,) * (L - len(ppg))
    N = 20
    res, opts = grid_solve(amg, L, host, f, ppg, transport=transport, num_cycles=N, max_inflight=inflight,
                           converge_test_type=amg.AMG_GLOBAL if conv == "global" else amg.AMG_LOCAL)
    # the band of the DMEM_Add restatement itself (or_dmem_add free races and
    # its round robin; one rank per grid there -- multi-rank device grids
    # exchange the same corrections in row pieces)
    # converge LOCAL: also the sequential schedules (the race's extreme speed
    # ratios) -- the device grids' fine grid can trail the coarse ones by far
    # more than any host-thread run (the arithmetic is pinned by
    # test_grid_add_round_robin_bitwise)
    key = (conv, inflight)
    if key not in _bands:
        _bands[key] = dmem_band(oracle, host, f, opts, sequential=True)
    lo, hi, brels, bcycs = _bands[key]
    # grids that ran other cycle counts than the band's runs: the restatement's
    # relres after exactly that many cycles joins the band
    extra = dmem_cycle_members(oracle, host, f, opts, [cyc for _, _, _, cyc, _, _ in res if cyc not in bcycs])
    if extra:
        lo, hi = min([lo] + extra), max([hi] + extra)
    n = host["A"][0].nrows
    xs = {}
    sent = recv = 0
    rels = sorted({(g, rel, int(m[0]), int(m[1])) for g, _, _, _, rel, m in res})
    print(f"grid add {transport} {ppg} {conv}: oracle band [{lo:.4e}, {hi:.4e}] (cycles {[r[3] for r in res]}), "
          f"grids (grid, rel, sent, received) {rels}")
    for g, row0, x, cyc, rel, msgs in res:
        assert np.all(np.isfinite(x))
        assert cyc >= N
        assert in_band(rel, lo, hi), (g, rel, cyc, lo, hi)
        sent += int(msgs[0])
        recv += int(msgs[1])
        xs.setdefault(g, np.zeros(n))[row0:row0 + x.size] = x
    assert sent == recv
    # every grid ends with (nearly) the same iterate: all corrections reach all
    # grids, up to the reference's dropped final payloads (test_grid_add.py)
    x0 = xs[0]
    for g, x in xs.items():
        assert np.linalg.norm(x - x0) <= 0.2 * np.linalg.norm(x0), g
