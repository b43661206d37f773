"""Level-grouped asynchronous additive solve (DMEM_Add, csrc/amg_grid.cpp) on the
host: the grid assignment (DMEM_Setup.cpp:1638-1735) against a restatement,
and the message protocol -- outside classes between overlapping ranks, done
flags 0/1/2, max_inflight pools, async_comm_save_divisor, LOCAL / GLOBAL
termination, AsyncRecvCleanup -- over the host model grid (A = diag(a); grid k
corrects the rows i with i % grids == k by u = w r ./ a: complementary
subspaces, like the levels of an additive cycle) with ranks as threads
(rendezvous mailboxes) and as gloo processes (world sizes 2-3,
torch.distributed isend / irecv)."""
import math
import os
import socket
import threading

import numpy as np
import pytest


def ref_partition(num_procs, frac):
    """DMEM_Setup.cpp:1676-1735 (assign_procs_type default)."""
    out, count, L = [], num_procs, len(frac)
    for level in range(L):
        if level == L - 1 or count == 1:
            cur = count
        elif count == L - level:
            cur = 1
        else:
            cur = max(int(math.ceil(frac[level] * num_procs)), 1)
            while True:
                nxt = cur - 1
                dc = abs(frac[level] - cur / num_procs)
                dn = abs(frac[level] - nxt / num_procs)
                if count - cur <= L - level:
                    cur = count - (L - level) + 1
                    break
                if dc <= dn or cur == 1:
                    break
                cur -= 1
        out.append(cur)
        count -= cur
    return out


@pytest.mark.parametrize("procs,frac", [(8, [0.6, 0.3, 0.1]), (4, [0.5, 0.3, 0.2]), (3, [0.9, 0.05, 0.05]),
                                        (16, [0.55, 0.25, 0.12, 0.05, 0.03]), (9, [0.2, 0.2, 0.2, 0.2, 0.2]),
                                        (64, [0.875, 0.11, 0.014, 0.001])])
def test_partition(amg, procs, frac):
    got = list(amg.grid.partition(procs, frac))
    assert got == ref_partition(procs, frac)
    assert sum(got) == procs and min(got) >= 1


def run_threads(n, fn):
    out, errs = [None] * n, []

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(180)
    assert not any(t.is_alive() for t in th), "rank threads hung"
    if errs:
        raise errs[0]
    return out


def host_problem(n, seed=0):
    rng = np.random.default_rng(seed)
    return rng.uniform(1.0, 3.0, n), rng.uniform(-1.0, 1.0, n)


def solve_threads(amg, procs_per_grid, n, weights, eager=False, **kw):
    rank_grid, rank_rows = amg.grid.layout(procs_per_grid, n)
    world = len(rank_grid)
    a, b = host_problem(n)
    hub = amg.grid.ThreadNbHub(rank_grid, eager=eager)
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, tol=0.0, **kw)

    def rank(r):
        s, e = rank_rows[2 * r], rank_rows[2 * r + 1]
        G = amg.grid.GridAdd(hub.transport(r), int(rank_grid[r]), world, r, rank_grid, rank_rows,
                             diag=a[s:e], weight=weights[rank_grid[r]], opts=opts)
        peers = G.peers()
        x, cyc, rel, msgs = G.solve(b[s:e])
        G.free()
        return x, cyc, rel, msgs, peers

    return rank_grid, rank_rows, a, b, run_threads(world, rank)


@pytest.mark.parametrize("ppg,conv,inflight,save", [
    ((1, 1, 1), "local", 1, 1), ((2, 2, 1), "local", 2, 1), ((1, 3, 2), "global", 1, 1),
    ((2, 1, 1, 2), "global", 3, 2), ((3, 2), "local", 1, 3), ((1, 1), "global", 2, 1)])
def test_protocol_threads(amg, ppg, conv, inflight, save):
    """Every grid runs its cycles, every message class drains (every message
    sent is received: the totals match), and every grid's iterate converges
    to b ./ a on the rows it corrects itself.  The other rows arrive as
    messages; the reference drops the payload of a final (done-flag) message
    that comes in alone (SendRecv breaks before setting the receive flag,
    DMEM_Comm.cpp:297-312, and AddCheckComm adds e only under that flag,
    DMEM_Add.cpp:496-507) -- restated, so those rows are only checked not
    to diverge."""
    n = 97
    G = len(ppg)
    weights = [0.7] * G
    N = 30
    ct = amg.AMG_GLOBAL if conv == "global" else amg.AMG_LOCAL
    rank_grid, rank_rows, a, b, res = solve_threads(amg, ppg, n, weights, num_cycles=N, converge_test_type=ct,
                                                    max_inflight=inflight, async_comm_save_divisor=save)
    xstar = b / a
    sent = recv = 0
    for r, (x, cyc, rel, msgs, peers) in enumerate(res):
        g = int(rank_grid[r])
        assert np.all(np.isfinite(x))
        if conv == "local":
            assert cyc == N  # cycles 0..N-1 (CheckConverge: cycle >= num_cycles - 1)
        else:
            assert cyc >= N
        # peers: the ranks of the other grids whose rows overlap mine
        s, e = rank_rows[2 * r], rank_rows[2 * r + 1]
        ov = sum(1 for p in range(len(rank_grid)) if rank_grid[p] != g and
                 min(e, rank_rows[2 * p + 1]) > max(s, rank_rows[2 * p]))
        assert peers == (ov, ov)
        assert msgs[0] >= ov and msgs[1] >= ov  # at least the done-flag message each way
        sent += int(msgs[0])
        recv += int(msgs[1])
        own = (np.arange(s, e) % G) == g
        np.testing.assert_allclose(x[own], xstar[s:e][own], rtol=0, atol=1e-6)
        assert rel < 1.0, (r, rel)
    assert sent == recv


def test_save_divisor_cuts_messages(amg):
    """async_comm_save_divisor: corrections accumulate in y and travel every
    few cycles (eager sends: a slot is always free) -- one message per
    cycle, or one every 4 cycles plus the final one."""
    n = 64
    for save, want in ((1, 24), (4, 7)):
        _, _, _, _, res = solve_threads(amg, (1, 1), n, [0.7, 0.7], eager=True, num_cycles=24, max_inflight=1,
                                        async_comm_save_divisor=save)
        for r in res:
            assert r[3][0] == want, (save, r[3])
            assert r[2] < 1.0


def test_semi_async_global_refused(amg):
    rank_grid, rank_rows = amg.grid.layout((1, 1), 10)
    hub = amg.grid.ThreadNbHub(rank_grid)
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, async_type=amg.AMG_SEMI_ASYNC,
                            converge_test_type=amg.AMG_GLOBAL)
    with pytest.raises(amg.AmgError):
        amg.grid.GridAdd(hub.transport(0), 0, 2, 0, rank_grid, rank_rows, diag=np.ones(10), opts=opts)


# ---- gloo processes ---------------------------------------------------------------
def _gloo_rank(rank, world, port, ppg, conv, q):
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        from conftest import load_package
        amg = load_package()
        rank_grid, rank_rows = amg.grid.layout(ppg, 80)
        groups = {}
        for g in range(len(ppg)):
            groups[g] = dist.new_group([r for r in range(world) if rank_grid[r] == g])
        my = int(rank_grid[rank])
        a, b = host_problem(80, 1)
        s, e = rank_rows[2 * rank], rank_rows[2 * rank + 1]
        opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, tol=0.0, num_cycles=20, max_inflight=2,
                                converge_test_type=amg.AMG_GLOBAL if conv == "global" else amg.AMG_LOCAL)
        T = amg.grid.TorchNbTransport(groups[my])
        G = amg.grid.GridAdd(T, my, world, rank, rank_grid, rank_rows, diag=a[s:e], weight=0.7,
                             opts=opts)
        x, cyc, rel, msgs = G.solve(b[s:e])
        G.free()
        dist.barrier()
        dist.destroy_process_group()
        own = (np.arange(s, e) % len(ppg)) == my
        q.put((rank, float(np.max(np.abs(x - b[s:e] / a[s:e])[own])), cyc, rel, int(msgs[0]), int(msgs[1])))
    except BaseException as ex:  # noqa: BLE001
        q.put((rank, repr(ex)))


@pytest.mark.parametrize("ppg,conv", [((1, 1), "local"), ((2, 1), "global"), ((1, 1, 1), "global")])
def test_protocol_gloo(ppg, conv):
    import multiprocessing as mp
    world = sum(ppg)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_rank, args=(r, world, port, ppg, conv, q), daemon=True) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            item = q.get(timeout=120)
            out[item[0]] = item
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        item = out[r]
        assert len(item) == 6, item
        _, err, cyc, rel, sent, recv = item
        assert cyc >= 20 and rel < 1.0 and err < 1e-6, item
        assert sent >= 1 and recv >= 1
    assert sum(out[r][4] for r in range(world)) == sum(out[r][5] for r in range(world))
