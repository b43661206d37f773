"""CPU, world size 2 and 3 over gloo: the distributed plan and the host transport.

Runs without a GPU.  Each rank is a process of a gloo group (127.0.0.1):

* the structured slab partition (amg_dist_structured_row_starts) is the same
  on every rank, covers every level, and keeps restriction / prolongation
  neighbour-local (peers are only the adjacent slabs);
* the ghost-exchange protocol of amg_dist.cpp (request lists of global ids
  to the owner, values back, columns remapped to [owned | ghost] in row
  order) run through ``dist.TorchGroupHub`` reproduces every row of the
  global operator product exactly;
* ``dist.HostTransport``'s three operations (p2p, allreduce, allgather), the
  callback the library invokes, give the right bytes over gloo.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_package


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn_name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        globals()[fn_name](rank, world)
        q.put((rank, None))
    except BaseException as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def spawn(world, fn_name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    errs = [e for _, e in out if e]
    assert not errs, "\n".join(errs)


def _plan_body(rank, world):
    amg = load_package()
    hub = amg.dist.TorchGroupHub()
    gen = amg.Gen(16, 12, 21)
    rs = amg.dist.structured_row_starts(gen, world)
    every = hub.collective(rank, rs)
    for other in every:
        np.testing.assert_array_equal(other, rs)
    L = gen.L
    for l in range(L):
        assert rs[l, 0] == 0 and rs[l, -1] == gen.rows(amg.AMG_GEN_A, l)
        assert np.all(np.diff(rs[l]) >= 0)
    rng = np.random.default_rng(7)
    for l in range(L):
        for which, rl, cl in ((amg.AMG_GEN_A, l, l), (amg.AMG_GEN_P, l, l + 1),
                              (amg.AMG_GEN_R, l + 1, l)):
            if which != amg.AMG_GEN_A and l == L - 1:
                continue
            nx, ny, _ = gen.dims(rl)
            z0, z1 = rs[rl, rank] // (nx * ny), rs[rl, rank + 1] // (nx * ny)
            lev = l
            nr, nc, rp, cj, cv = gen.host_csr(which, lev, z0, z1)
            ncols = int(rs[cl, -1])
            x = rng.standard_normal(ncols)  # same seed order on every rank
            c0, c1 = rs[cl, rank], rs[cl, rank + 1]
            ghosts = np.unique(cj[(cj < c0) | (cj >= c1)])
            owner = np.searchsorted(rs[cl], ghosts, side="right") - 1
            peers = sorted(set(owner.tolist()))
            # neighbour-local: only the nearest non-empty slab on either side
            nonempty = [q for q in range(world) if rs[cl, q + 1] > rs[cl, q] and q != rank]
            below = [q for q in nonempty if q < rank][-1:]
            above = [q for q in nonempty if q > rank][:1]
            assert set(peers) <= set(below + above), (which, l, peers)
            # request lists -> owners, values back (the amg_dist.cpp protocol)
            all_peers = [q for q in range(world) if q != rank]
            reqs = {q: ghosts[owner == q].astype(np.int64).tobytes() for q in all_peers}
            got = hub.p2p(rank, all_peers, [reqs[q] for q in all_peers])
            replies = []
            for q in all_peers:
                ids = np.frombuffer(got[q], dtype=np.int64)
                assert np.all((ids >= c0) & (ids < c1))
                replies.append(x[ids].tobytes())
            vals = hub.p2p(rank, all_peers, replies)
            xg = np.concatenate([np.frombuffer(vals[q], dtype=np.float64) for q in all_peers]
                                + [np.zeros(0)])
            xl = np.concatenate([x[c0:c1], xg])
            local = np.where((cj >= c0) & (cj < c1), cj - c0,
                             (c1 - c0) + np.searchsorted(ghosts, cj))
            y_loc = sp.csr_matrix((cv, local, rp), shape=(nr, len(xl))) @ xl
            y_glob = sp.csr_matrix((cv, cj, rp), shape=(nr, ncols)) @ x
            np.testing.assert_array_equal(y_loc, y_glob)


def _transport_body(rank, world):
    amg = load_package()
    tr = amg.dist.HostTransport(amg.dist.TorchGroupHub(), rank)
    # op 0: ring p2p with payloads of different sizes
    peers = sorted({(rank + 1) % world, (rank - 1) % world} - {rank})
    send = [np.full(3 + rank, 100 * rank + q, dtype=np.float64) for q in peers]
    recv = [np.zeros(3 + q) for q in peers]
    P = (C.c_int * len(peers))(*peers)
    SP = (C.c_void_p * len(peers))(*[a.ctypes.data for a in send])
    SB = (C.c_longlong * len(peers))(*[a.nbytes for a in send])
    RP = (C.c_void_p * len(peers))(*[a.ctypes.data for a in recv])
    RB = (C.c_longlong * len(peers))(*[a.nbytes for a in recv])
    assert tr.cfn(None, 0, len(peers), P, SP, SB, RP, RB) == 0, tr.error
    for q, a in zip(peers, recv):
        np.testing.assert_array_equal(a, np.full(3 + q, 100 * q + rank))
    # op 1: allreduce
    v = np.array([rank + 1.0, 0.5 * rank])
    RP1 = (C.c_void_p * 1)(v.ctypes.data)
    RB1 = (C.c_longlong * 1)(v.nbytes)
    assert tr.cfn(None, 1, 0, None, None, None, RP1, RB1) == 0, tr.error
    np.testing.assert_array_equal(v, [sum(r + 1.0 for r in range(world)),
                                      sum(0.5 * r for r in range(world))])
    # op 2: allgather
    mine = np.array([rank, rank * rank], dtype=np.int64)
    out = np.zeros(2 * world, dtype=np.int64)
    SP2 = (C.c_void_p * 1)(mine.ctypes.data)
    SB2 = (C.c_longlong * 1)(mine.nbytes)
    RP2 = (C.c_void_p * 1)(out.ctypes.data)
    RB2 = (C.c_longlong * 1)(out.nbytes)
    assert tr.cfn(None, 2, 0, None, SP2, SB2, RP2, RB2) == 0, tr.error
    np.testing.assert_array_equal(out.reshape(world, 2)[:, 1], np.arange(world) ** 2)


@pytest.mark.parametrize("world", [2, 3])
def test_plan_gloo(world):
    spawn(world, "_plan_body")


@pytest.mark.parametrize("world", [2, 3])
def test_host_transport_gloo(world):
    spawn(world, "_transport_body")


def test_thread_mailbox_matching():
    """p2p messages are matched per ordered pair in posting order."""
    amg = load_package()
    import threading
    hub = amg.dist.ThreadMailbox(2, timeout=20)
    out = [None, None]

    def body(r):
        a = hub.p2p(r, [1 - r], [b"first%d" % r])
        b = hub.p2p(r, [1 - r], [b"second%d" % r])
        c = hub.collective(r, r * 10)
        out[r] = (a[1 - r], b[1 - r], c)

    th = [threading.Thread(target=body, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert out[0] == (b"first1", b"second1", [0, 10])
    assert out[1] == (b"first0", b"second0", [0, 10])
