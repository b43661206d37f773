"""Level-grouped asynchronous additive solve (DMEM_Add, DMEM_Add.cpp:20-944)
through the C-ABI (amg_grid_*, csrc/amg_grid.cpp).

The protocol needs a non-blocking transport with MPI point-to-point semantics
(amg_nb_transport).  Two are provided here:
  * ThreadNbHub  -- ranks as threads of one process (one GPU, tests): a send
    completes when the matching receive has taken it (rendezvous, so the
    in-flight pools of DMEM_Comm.cpp really fill up);
  * TorchNbTransport -- ranks as processes over torch.distributed (gloo on the
    host: isend / irecv / Work.is_completed, all_reduce over the grid's group).
DevHub (amg_devhub) replaces the transport for ranks as threads of one
process, and GridAdd(..., ipc=True) keeps the payloads on the device across
processes (IPC-mapped slots; the transport carries control words only): the
correction payloads stay in device memory end to end.
"""
import ctypes as C
import threading
import time

import numpy as np

from . import check, lib
from .abi import AmgOpts

from .abi import AmgNbTransport, _ISEND, _IRECV, _TEST, _WAIT, _ALLRED  # noqa: E402


def partition(num_procs, frac_work):
    """Ranks per grid (DMEM_Setup.cpp:1638-1735)."""
    fw = np.ascontiguousarray(frac_work, dtype=np.float64)
    out = np.zeros(fw.size, dtype=np.int32)
    check(lib.amg_grid_partition(int(num_procs), int(fw.size), fw.ctypes.data_as(C.POINTER(C.c_double)),
                                 out.ctypes.data_as(C.POINTER(C.c_int))))
    return out


def layout(procs_per_grid, n):
    """(rank_grid, rank_rows): grids in rank order, each grid's n rows split
    evenly among its ranks."""
    rank_grid, rank_rows = [], []
    for g, p in enumerate(procs_per_grid):
        cuts = [n * i // p for i in range(p + 1)]
        for i in range(p):
            rank_grid.append(g)
            rank_rows += [cuts[i], cuts[i + 1]]
    return np.array(rank_grid, dtype=np.int32), np.array(rank_rows, dtype=np.int64)


class _Transport:
    """ctypes callbacks around an implementation with isend / irecv / test /
    wait / grid_allreduce methods (requests are integer ids)."""

    def __init__(self):
        self.error = None
        self._reqs = {}
        self._next = 1

        def guard(fn):
            def w(*a):
                try:
                    return fn(*a)
                except Exception as e:  # surfaced after the C call returns
                    self.error = e
                    return -1
            return w

        def isend(user, peer, tag, buf, n, req):
            arr = np.ctypeslib.as_array(buf, (n,)) if n else np.zeros(0)
            req[0] = self._add(self.post_send(peer, tag, arr))
            return 0

        def irecv(user, peer, tag, buf, n, req):
            arr = np.ctypeslib.as_array(buf, (n,)) if n else np.zeros(0)
            req[0] = self._add(self.post_recv(peer, tag, arr))
            return 0

        def test(user, req, done):
            r = self._reqs[req]
            ok = self.done(r)
            if ok:
                del self._reqs[req]
            done[0] = 1 if ok else 0
            return 0

        def wait(user, req):
            r = self._reqs.pop(req, None)
            while r is not None and not self.done(r):
                time.sleep(0)
            return 0

        def allred(user, vals, n):
            arr = np.ctypeslib.as_array(vals, (n,))
            arr[:] = self.grid_sum(arr.copy())
            return 0

        self.c = AmgNbTransport(None, _ISEND(guard(isend)), _IRECV(guard(irecv)), _TEST(guard(test)),
                                _WAIT(guard(wait)), _ALLRED(guard(allred)))

    def _add(self, r):
        k = self._next
        self._next += 1
        self._reqs[k] = r
        return k


class ThreadNbHub:
    """Mailboxes of ranks running as threads of one process."""

    def __init__(self, rank_grid, eager=False):
        self.eager = eager  # eager: a send completes at once (its payload copied)
        self.rank_grid = list(rank_grid)
        self.lock = threading.Lock()
        self.box = {}  # (dst, src, tag) -> list of [payload view, done flag list]
        self.grids = {}
        for g in set(self.rank_grid):
            ranks = [r for r, gg in enumerate(self.rank_grid) if gg == g]
            self.grids[g] = {"n": len(ranks), "bar": threading.Barrier(len(ranks)), "acc": None,
                             "out": None, "lock": threading.Lock()}

    def transport(self, rank):
        return ThreadNbTransport(self, rank)


class ThreadNbTransport(_Transport):
    def __init__(self, hub, rank):
        self.hub = hub
        self.rank = rank
        super().__init__()

    def post_send(self, peer, tag, arr):
        rec = {"data": arr.copy() if self.hub.eager else arr, "done": self.hub.eager}
        with self.hub.lock:
            self.hub.box.setdefault((peer, self.rank, tag), []).append(rec)
        return ("s", rec)

    def post_recv(self, peer, tag, arr):
        return ("r", {"key": (self.rank, peer, tag), "buf": arr, "done": False})

    def done(self, r):
        kind, rec = r
        if kind == "s":
            return rec["done"]
        if rec["done"]:
            return True
        with self.hub.lock:
            q = self.hub.box.get(rec["key"])
            if not q:
                return False
            msg = q.pop(0)
            rec["buf"][:] = msg["data"]  # the sender's slot is untouched until done
            msg["done"] = True
        rec["done"] = True
        return True

    def grid_sum(self, vals):
        g = self.hub.grids[self.hub.rank_grid[self.rank]]
        with g["lock"]:
            g["acc"] = vals.copy() if g["acc"] is None else g["acc"] + vals
        g["bar"].wait()  # every rank of the grid has added
        out = g["acc"].copy()
        if g["bar"].wait() == 0:  # every rank has read: one resets
            g["acc"] = None
        g["bar"].wait()
        return out


class TorchNbTransport(_Transport):
    """torch.distributed point-to-point (gloo: CPU tensors) for the messages and
    all_reduce over the grid's process group for InnerProdFlag."""

    def __init__(self, grid_group):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, grid_group
        super().__init__()

    # gloo's send / recv Work completes only inside wait(): a helper thread per
    # request waits and raises a flag, which test() reads (MPI_Test semantics)
    def _watch(self, work):
        ev = threading.Event()

        def run():
            try:
                work.wait()
            finally:
                ev.set()
        threading.Thread(target=run, daemon=True).start()
        return ev

    def post_send(self, peer, tag, arr):
        return self._watch(self.dist.isend(self.torch.from_numpy(arr), dst=int(peer), tag=int(tag)))

    def post_recv(self, peer, tag, arr):
        return self._watch(self.dist.irecv(self.torch.from_numpy(arr), src=int(peer), tag=int(tag)))

    def done(self, ev):
        return ev.is_set()

    def grid_sum(self, vals):
        t = self.torch.from_numpy(np.ascontiguousarray(vals))
        self.dist.all_reduce(t, group=self.group)
        return t.numpy()


class DevHub:
    """Device-resident correction messages between ranks running as threads of
    one process (amg_devhub, csrc/amg_grid.cpp): payloads move device to
    device, done flags and InnerProdFlag sums on the hub."""

    def __init__(self, rank_grid):
        self.rank_grid = np.ascontiguousarray(rank_grid, dtype=np.int32)
        h = C.c_void_p()
        check(lib.amg_devhub_create(int(self.rank_grid.size), self.rank_grid.ctypes.data_as(C.POINTER(C.c_int)),
                                    C.byref(h)))
        self.h = h
        self.error = None  # the GridAdd transport interface

    def free(self):
        if getattr(self, "h", None):
            lib.amg_devhub_free(self.h)
            self.h = None


class GridAdd:
    """One rank of the level-grouped solve: over its grid's distributed
    hierarchy (`dist_hier`) or, with `diag` / `weight`, over the host model."""

    def __init__(self, transport, my_grid, world, rank, rank_grid, rank_rows, dist_hier=None, diag=None,
                 weight=1.0, opts=None, ipc=False):
        self.t = transport
        self.rank_grid = np.ascontiguousarray(rank_grid, dtype=np.int32)
        self.rank_rows = np.ascontiguousarray(rank_rows, dtype=np.int64)
        h = C.c_void_p()
        rg = self.rank_grid.ctypes.data_as(C.POINTER(C.c_int))
        rr = self.rank_rows.ctypes.data_as(C.POINTER(C.c_longlong))
        if dist_hier is not None and isinstance(transport, DevHub):
            st = lib.amg_grid_add_create_devhub(dist_hier.h, my_grid, world, rank, rg, rr, transport.h, C.byref(h))
            self.n = dist_hier.n0
        elif dist_hier is not None and ipc:
            # device-resident payloads across processes: the transport carries
            # the IPC handles (here, collectively), control words and acks
            st = lib.amg_grid_add_create_ipc(dist_hier.h, my_grid, world, rank, rg, rr, C.byref(transport.c),
                                             C.byref(h))
            self.n = dist_hier.n0
        elif dist_hier is not None:
            st = lib.amg_grid_add_create(dist_hier.h, my_grid, world, rank, rg, rr, C.byref(transport.c), C.byref(h))
            self.n = dist_hier.n0
        else:
            self.diag = np.ascontiguousarray(diag, dtype=np.float64)
            self.opts = opts
            st = lib.amg_grid_add_create_host(self.diag.size, self.diag.ctypes.data_as(C.POINTER(C.c_double)),
                                              float(weight), C.byref(opts), my_grid, world, rank, rg, rr,
                                              C.byref(transport.c), C.byref(h))
            self.n = self.diag.size
        self._raise(st)
        self.h = h

    def _raise(self, st):
        if self.t.error is not None:
            e, self.t.error = self.t.error, None
            raise e
        check(st)

    def peers(self):
        a, b = C.c_int(), C.c_int()
        check(lib.amg_grid_add_peers(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def solve(self, b_local, x0=None):
        b = np.ascontiguousarray(b_local, dtype=np.float64)
        x = np.zeros(self.n) if x0 is None else np.array(x0, dtype=np.float64)
        cyc, rel = C.c_int(), C.c_double()
        msgs = np.zeros(2, dtype=np.int64)
        st = lib.amg_grid_add_solve(self.h, b.ctypes.data_as(C.POINTER(C.c_double)),
                                    x.ctypes.data_as(C.POINTER(C.c_double)), C.byref(cyc), C.byref(rel),
                                    msgs.ctypes.data_as(C.POINTER(C.c_longlong)))
        self._raise(st)
        return x, cyc.value, rel.value, msgs

    def free(self):
        if getattr(self, "h", None):
            lib.amg_grid_add_free(self.h)
            self.h = None
