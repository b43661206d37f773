"""The asynchronous additive solve on z-slab hierarchies with its ranks as
PROCESSES -- the production layout of config 4 (one process per GPU under
torchrun, DMEM_Add's MPI ranks, DMEM_Comm.cpp:81-348) -- here 2-3 processes
sharing cuda:0.

Across processes the per-level channels of csrc/amg_link.cpp take their
cross-process branch: each rank's receive slots are hipMalloc'ed and exported
with hipIpcGetMemHandle, every peer maps them with hipIpcOpenMemHandle, and the
`arrived` / `acked` sequence words live in POSIX shared-memory control blocks.
Setup exchanges (plans, handles, the final norm) go over gloo (TorchGroupHub).

* Deterministic schedules (async_schedule 1 / 2 / 3): the assembled iterate is
  bit-identical to the oracle's or_async_add under the same schedule (and so
  to the thread-rank run of tests/test_gpu_slab_async.py), for two solves in a
  row on the same channels (the slots are reused: a stale read would show).
* The free race lands within [0.5x, 2x] of the oracle's replay of its recorded
  update order.
"""
import os
import socket

import numpy as np
import pytest

from test_gpu_kernels import assert_bitwise

pytestmark = pytest.mark.gpu

W = 0.8


def _rank(rank, world, port, n, optd, rep, runs, q):
    try:
        import sys
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        from conftest import load_package
        amg = load_package()
        gen = amg.Gen(n)
        f = amg.rhs_rand(0, n ** 3)
        opts = amg.default_opts(**optd)
        c = amg.Context(0, nstreams=gen.L + 2)
        tr = amg.dist.HostTransport(amg.dist.TorchGroupHub(), rank)
        amg.dist.init_host(c, world, rank, tr)
        amg.dist.set_replicate_rows(c, rep)
        D = amg.dist.DistHier(c, gen, opts, slab=True)
        out = []
        for _ in range(runs):
            dist.barrier()  # the ranks enter the solve together
            rel, cnt = D.async_solve(f[D.row0:D.row0 + D.n0])
            from async_band import race_tables
            e_, s_ = race_tables(D)
            # the per-row update times / values travel too: the replay of a
            # process run is then the exact row replay, as for thread ranks
            out.append((float(rel), [int(x) for x in cnt], D.get_u(), [list(map(float, t)) for t in e_],
                        [list(map(float, t)) for t in s_], getattr(e_, "rows", None), getattr(e_, "vals", None)))
        row0 = D.row0
        D.free()
        amg.dist.finalize(c)
        c.close()
        gen.free()
        if tr.error is not None:
            raise tr.error
        dist.destroy_process_group()
        q.put((rank, row0, out))
    except BaseException as ex:  # noqa: BLE001
        import traceback
        q.put((rank, None, repr(ex) + "\n" + traceback.format_exc()))


def slab_async_procs(n, optd, world, rep=1 << 10, runs=1):
    """run the slab async solve as `world` processes; [(rel, counts, u)] per run"""
    import multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, n, optd, rep, runs, q), daemon=True)
          for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    try:
        for _ in range(world):
            item = q.get(timeout=240)
            got[item[0]] = item
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert got[r][1] is not None, got[r][2]
    order = sorted(range(world), key=lambda r: got[r][1])
    from async_band import Ends

    def ends_of(t):
        e = Ends(t[3])
        e.rows, e.vals = t[5], t[6]
        return e

    out = []
    for k in range(runs):
        rel = got[0][2][k][0]
        assert all(got[r][2][k][0] == rel for r in range(world))  # one allreduced norm
        u = np.concatenate([got[r][2][k][2] for r in order])
        rs = [got[r][1] for r in order] + [got[order[-1]][1] + got[order[-1]][2][k][2].size]
        out.append((rel, got[0][2][k][1], u, [ends_of(got[r][2][k]) for r in order], rs,
                    [got[r][2][k][4] for r in order]))  # per rank
    return out


def _optd(amg, solver, comp, N, sched):
    return dict(solver=amg.AMG_ASYNC_MULTADD if solver == "multadd" else amg.AMG_ASYNC_AFACX,
                smooth_weight=W, num_cycles=N, tol=0.0, async_schedule=sched, smooth_transfer=1 if comp else 0)


SCHED = [
    # (solver, composed transfers, processes, schedule, n)
    ("multadd", True, 2, 3, 32),
    ("multadd", True, 3, 1, 32),
    ("afacx", False, 3, 2, 32),
    # 64^3: level 0's composed restriction is the fused one-pass kernel, its
    # ghost planes over the cross-process channels
    ("multadd", True, 2, 3, 64),
]


@pytest.mark.parametrize("solver,comp,world,sched,n", SCHED,
                         ids=[f"{s}-{w}p-s{q}-{m}" for s, _, w, q, m in SCHED])
def test_slab_async_processes_schedule_bitwise(amg, oracle, solver, comp, world, sched, n):
    """one process per rank, deterministic schedule: the assembled iterate of
    two consecutive solves is bit-identical to the oracle's or_async_add under
    the same schedule (SMEM_Async_Add_AMG restated, composed transfers)"""
    from test_gpu_slab_async import host_hier, oracle_opts_of
    N = 8
    optd = _optd(amg, solver, comp, N, sched)
    runs = slab_async_procs(n, optd, world, runs=2)
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    host = host_hier(amg, oracle, gen)
    L = gen.L
    opts = amg.default_opts(**optd)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts_of(oracle, opts))
    if comp:
        OH.set_composed_transfers()
    oracle.lib().or_set_async_schedule(sched)
    try:
        uo, relo, cnto = OH.async_add(f, [1] * L)
    finally:
        oracle.lib().or_set_async_schedule(0)
    gen.free()
    for k, (rel, cnt, u, _, _, _) in enumerate(runs):
        nd = int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))
        print(f"slab async processes {solver} composed={comp} {world} processes schedule {sched} n={n} "
              f"solve {k}: device {rel:.13e} oracle {relo:.13e}, differing entries {nd}")
        assert list(cnt[:L - 1]) == list(cnto[:L - 1]) == [N] * (L - 1)
        assert_bitwise(u, uo, "process-rank slab async iterate vs oracle")
        assert abs(rel - relo) <= 1e-12 * relo


def test_slab_async_processes_free_race(amg, oracle):
    """the free race with one process per rank (2 and 3 processes, 48^3,
    composed MULTADD): every level runs num_cycles corrections, the iterate is
    finite and the relative residual lies within [0.5x, 2x] of the oracle's
    replay of the update order the processes recorded (or_async_add under the
    timed schedule with every correction's end time, slowest rank)"""
    from async_band import replay_check
    from test_gpu_slab_async import host_hier
    n, N = 48, 12
    optd = _optd(amg, "multadd", True, N, 0)
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    host = host_hier(amg, oracle, gen)
    L = gen.L
    gen.free()
    opts = amg.default_opts(**optd)
    for world in (2, 3):
        runs = slab_async_procs(n, optd, world, rep=1 << 12, runs=3)
        for rel, cnt, u, ms, _, _ in runs:
            assert list(cnt[:L - 1]) == [N] * (L - 1)
            assert np.all(np.isfinite(u))
            assert rel < 1.0
        widest = replay_check(amg, oracle, host, f, opts, [(r[0], r[3], r[4], r[5]) for r in runs], composed=True,
                              what=f"slab async {world} processes")
        assert widest <= 20.0
