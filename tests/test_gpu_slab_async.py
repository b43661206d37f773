"""The asynchronous additive solve on z-slab hierarchies (config 4's path):
amg_dist_async_solve with per-level device-resident channels between ranks
(csrc/amg_link.cpp) and the reference's smoothed transfers composed on the fly
(smooth_transfer = 1: P~ = (I - w D^-1 A) P, R~ = P~^T, SmoothTransfer,
SMEM_Setup.cpp:1173-1254; DMEM_Add.cpp:20-178 / SMEM_Async_AMG.cpp:7-437).

* Deterministic schedules (async_schedule 1 / 2 / 3) pin the arithmetic: the
  assembled iterate of 1-3 ranks is bit-identical to the oracle's
  or_async_add under the same schedule with composed transfers
  (or_hier_set_composed_transfers), one thread per level group.
* The free race converges and lands in the oracle's asynchronous band.
* At 512^3 the free race converges (relres < 0.5 after N corrections per
  level) at 1 rank (RCCL) and 2 / 8 ranks (the host transport for setup, the
  device-resident channels for every exchange).

Ranks run as threads of this process on cuda:0 (RCCL refuses two ranks per
device); each rank's level groups run on their own host threads."""
import numpy as np
import pytest

from async_band import race_tables, replay_check
from test_gpu_dist import run_ranks
from test_gpu_kernels import assert_bitwise

pytestmark = pytest.mark.gpu

W = 0.8


def slab_async(amg, gen, opts, f, nranks, rep=1 << 12, rccl1=True, runs=1, dur=None):
    hub = amg.dist.ThreadMailbox(nranks, timeout=900.0)

    def rank(r):
        c = amg.Context(0, nstreams=gen.L + 2)
        tr = None
        if nranks == 1 and rccl1:
            amg.dist.init_rccl(c, 1, 0, lambda b: b)
        else:
            tr = amg.dist.HostTransport(hub, r)
            amg.dist.init_host(c, nranks, r, tr)
        amg.dist.set_replicate_rows(c, rep)
        D = amg.dist.DistHier(c, gen, opts, slab=True)
        if dur is not None:
            D.set_async_durations(dur)
        out = []
        for _ in range(runs):
            rel, cnt = D.async_solve(f[D.row0:D.row0 + D.n0])
            e_, s_ = race_tables(D)
            out.append((rel, cnt.copy(), D.get_u(), e_, s_))
        row0, n0 = D.row0, D.n0
        D.free()
        amg.dist.finalize(c)
        c.close()
        if tr is not None and tr.error is not None:
            raise tr.error
        return row0, out, n0

    res = run_ranks(nranks, rank)
    res.sort(key=lambda t: t[0])
    runs_out = []
    for q in range(runs):
        rel = res[0][1][q][0]
        assert all(t[1][q][0] == rel for t in res)  # one allreduced norm
        u = np.concatenate([t[1][q][2] for t in res])
        rs = [t[0] for t in res] + [res[-1][0] + res[-1][2]]  # the fine-row partition
        runs_out.append((rel, res[0][1][q][1], u, [t[1][q][3] for t in res], rs, [t[1][q][4] for t in res]))
    return runs_out


def host_hier(amg, oracle, gen):
    L = gen.L
    host = {}
    for which, tag, cnt in ((amg.AMG_GEN_A, "A", L), (amg.AMG_GEN_P, "P", L - 1), (amg.AMG_GEN_R, "R", L - 1)):
        host[tag] = [oracle.Csr(*gen.host_csr(which, l)) for l in range(cnt)]
    return host


def oracle_opts_of(oracle, o):
    return oracle.make_opts(solver=o.solver, smoother=o.smoother, num_pre=o.num_pre_smooth_sweeps,
                            num_post=o.num_post_smooth_sweeps, num_fine=o.num_fine_smooth_sweeps,
                            num_coarse=o.num_coarse_smooth_sweeps, smooth_weight=o.smooth_weight,
                            num_cycles=o.num_cycles, tol=o.tol)


SCHED = [
    # (solver, composed transfers, nranks, schedule, n)
    ("multadd", True, 1, 3, 32),
    ("multadd", True, 2, 3, 32),
    ("multadd", True, 3, 1, 32),
    ("multadd", True, 2, 2, 32),
    ("afacx", False, 2, 3, 32),
    ("afacx", False, 3, 2, 32),
    # 64^3: level 0 runs the fused residual + restriction form, so the composed
    # restriction of level 0 is the one-pass kernel (ghost planes over the channels)
    ("multadd", True, 2, 3, 64),
    ("multadd", True, 1, 1, 64),
    # AMG_SCHED_TIMED (the race at fixed level speeds)
    ("multadd", True, 2, 4, 32),
    ("multadd", True, 3, 4, 64),
]


@pytest.mark.parametrize("solver,comp,nranks,sched,n", SCHED,
                         ids=[f"{s}-{n}r-s{q}-{m}" for s, _, n, q, m in SCHED])
def test_slab_async_schedule_bitwise(amg, oracle, ctx, solver, comp, nranks, sched, n):
    """deterministic schedules of the slab-distributed asynchronous additive
    solve against the oracle's or_async_add (SMEM_Async_Add_AMG restated) under
    the same schedule: the assembled iterate is the same bits"""
    N = 8
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    sv = amg.AMG_ASYNC_MULTADD if solver == "multadd" else amg.AMG_ASYNC_AFACX
    opts = amg.default_opts(solver=sv, smooth_weight=W, num_cycles=N, tol=0.0, async_schedule=sched,
                            smooth_transfer=1 if comp else 0)
    L = gen.L
    dur = np.array([3.0 / (1.9 ** k) + 0.05 for k in range(L)]) if sched == 4 else None
    ((rel, cnt, u, _, _, _),) = slab_async(amg, gen, opts, f, nranks, rep=1 << 10, rccl1=False, dur=dur)
    host = host_hier(amg, oracle, gen)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts_of(oracle, opts))
    if comp:
        OH.set_composed_transfers()
    if dur is not None:
        oracle.set_async_durations(dur)
    oracle.lib().or_set_async_schedule(sched)
    try:
        uo, relo, cnto = OH.async_add(f, [1] * L)
    finally:
        oracle.lib().or_set_async_schedule(0)
    assert list(cnt[:L - 1]) == list(cnto[:L - 1]) == [N] * (L - 1)
    nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
    print(f"slab async {solver} composed={comp} {nranks} ranks schedule {sched}: device {rel:.13e} "
          f"oracle {relo:.13e}, differing entries {nd}")
    assert_bitwise(u, uo, "slab async iterate vs oracle")
    assert abs(rel - relo) <= 1e-12 * relo
    gen.free()


def test_slab_async_band(amg, oracle, ctx):
    """the free race (a host thread and a stream per level group, per-level
    channels) of ASYNC_MULTADD with composed smoothed transfers at 48^3 on 1-3
    ranks: every level runs num_cycles corrections and the relative residual
    lies within [0.5x, 2x] of the oracle's replay of that very race -- or_async_add
    under the timed schedule with the end times of every correction the device
    recorded (slowest rank), composed transfers"""
    n, N = 48, 12
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=W, num_cycles=N, tol=0.0, smooth_transfer=1)
    host = host_hier(amg, oracle, gen)
    L = gen.L
    for nranks in (1, 2, 3):
        runs = slab_async(amg, gen, opts, f, nranks, rccl1=True, runs=4)
        for rel, cnt, u, ms, _, _ in runs:
            assert list(cnt[:L - 1]) == [N] * (L - 1)
            assert np.all(np.isfinite(u))
            assert rel < 1.0
        widest = replay_check(amg, oracle, host, f, opts, [(r[0], r[3], r[4], r[5]) for r in runs], composed=True,
                              what=f"slab async {nranks} rank(s)")
        assert widest <= 20.0
    gen.free()


@pytest.mark.slow
def test_slab_512_async(amg, ctx):
    """config 4 at size: ASYNC_MULTADD with the smoothed transfers on the 512^3
    slab hierarchy, the free race, at 1 rank (RCCL), 2 and 8 ranks (the
    device-resident per-level channels): every level does N corrections and
    the relative residual falls below 0.5 (it contracts; the plain-transfer
    AFACx run of round 3 sat at 1.41)"""
    n, N = 512, 8
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=W, num_cycles=N, tol=0.0, smooth_transfer=1)
    rels = {}
    for nranks in (1, 2, 8):
        ((rel, cnt, u, ms, _, _),) = slab_async(amg, gen, opts, f, nranks, rep=1 << 18)
        assert list(cnt[:gen.L - 1]) == [N] * (gen.L - 1)
        assert np.all(np.isfinite(u))
        rels[nranks] = rel
        print(f"512^3 async MULTADD (smoothed transfers) {nranks} rank(s): relres {rel:.4e}, "
              f"level finish ms (rank 0) {[round(float(t[-1]), 1) if len(t) else 0.0 for t in ms[0][:gen.L - 1]]}")
        del u
    assert all(r < 0.5 for r in rels.values()), rels
    gen.free()
