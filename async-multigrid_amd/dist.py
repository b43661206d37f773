"""Multi-GPU solve phase (amg_dist_* in include/amg_mi355x.h).

One process per GPU: ``init_rccl`` builds the RCCL communicator (the unique
id travels over an already-initialised torch.distributed group, normally the
gloo/TCP store group torchrun gives every rank).  ``HostTransport`` routes the
same exchanges through host memory instead -- it lets several ranks share one
GPU in tests (RCCL refuses two ranks per device) and is how the CPU tests
drive the communication plan.

Reference counterparts: DMEM_Comm.cpp (ghost exchange), DMEM_Setup.cpp:666
(comm-plan construction), DMEM_Misc.cpp:414 (InnerProdFlag allreduce).
"""
import ctypes as C
import threading

import numpy as np

from . import abi, check, lib, _dp, _ip, AmgError  # noqa: F401

OP_P2P, OP_ALLREDUCE, OP_ALLGATHER = 0, 1, 2


def _buf(ptr, nbytes):
    return (C.c_char * int(nbytes)).from_address(ptr) if nbytes > 0 else None


class ThreadMailbox:
    """Exchange hub for ranks running as threads of one process.

    Every rank calls the same sequence of collectives; point-to-point
    messages are matched per (src, dst) pair in posting order."""

    def __init__(self, nranks, timeout=120.0):
        self.n = nranks
        self.timeout = timeout
        self.cv = threading.Condition()
        self.msgs = {}
        self.seq = {}
        self.coll = {}
        self.coll_seq = [0] * nranks

    def p2p(self, me, peers, payloads):
        out = {}
        with self.cv:
            for q, data in zip(peers, payloads):
                k = (me, q)
                s = self.seq.get(k, 0)
                self.seq[k] = s + 1
                self.msgs[(me, q, s)] = data
            self.cv.notify_all()
        for q in peers:
            k = (q, me, "r")
            with self.cv:
                s = self.seq.get(k, 0)
                self.seq[k] = s + 1
                key = (q, me, s)
                if not self.cv.wait_for(lambda: key in self.msgs, timeout=self.timeout):
                    raise AmgError(f"rank {me}: no message from rank {q}")
                out[q] = self.msgs.pop(key)
        return out

    def collective(self, me, data):
        with self.cv:
            s = self.coll_seq[me]
            self.coll_seq[me] += 1
            slot = self.coll.setdefault(s, {})
            slot[me] = data
            self.cv.notify_all()
            if not self.cv.wait_for(lambda: len(self.coll[s]) == self.n, timeout=self.timeout):
                raise AmgError(f"rank {me}: collective {s} incomplete")
            res = [self.coll[s][r] for r in range(self.n)]
            done = self.coll.setdefault(("done", s), set())
            done.add(me)
            if len(done) == self.n:
                del self.coll[s]
                del self.coll[("done", s)]
        return res


class TorchGroupHub:
    """Exchange hub over an initialised torch.distributed (gloo) group."""

    def __init__(self):
        import torch.distributed as dist
        self.dist = dist
        self.n = dist.get_world_size()

    def p2p(self, me, peers, payloads):
        import torch
        d = self.dist
        # sizes first (receivers need them), then payloads
        reqs, sizes = [], {}
        for q, data in zip(peers, payloads):
            reqs.append(d.isend(torch.tensor([len(data)], dtype=torch.int64), q))
        for q in peers:
            t = torch.zeros(1, dtype=torch.int64)
            d.recv(t, q)
            sizes[q] = int(t.item())
        for r in reqs:
            r.wait()
        reqs, out = [], {}
        for q, data in zip(peers, payloads):
            if len(data):
                reqs.append(d.isend(torch.frombuffer(bytearray(data), dtype=torch.uint8), q))
        for q in peers:
            t = torch.empty(sizes[q], dtype=torch.uint8)
            if sizes[q]:
                d.recv(t, q)
            out[q] = t.numpy().tobytes()
        for r in reqs:
            r.wait()
        return out

    def collective(self, me, data):
        objs = [None] * self.n
        self.dist.all_gather_object(objs, data)
        return objs


class HostTransport:
    """amg_host_xchg_fn implementation over a hub (ThreadMailbox or gloo)."""

    def __init__(self, hub, rank):
        self.hub, self.rank = hub, rank
        self.error = None
        self.cfn = abi.HOST_XCHG_FN(self._call)

    def _call(self, user, op, npeers, peers, send, sbytes, recv, rbytes):
        try:
            me = self.rank
            if op == OP_P2P:
                pl = [int(peers[i]) for i in range(npeers)]
                data = [bytes(_buf(send[i], sbytes[i]) or b"") for i in range(npeers)]
                got = self.hub.p2p(me, pl, data)
                for i, q in enumerate(pl):
                    want = int(rbytes[i])
                    if len(got[q]) != want:
                        raise AmgError(f"rank {me}: {len(got[q])} bytes from {q}, expected {want}")
                    if want:
                        C.memmove(recv[i], got[q], want)
            elif op == OP_ALLREDUCE:
                n = int(rbytes[0]) // 8
                mine = np.frombuffer(bytes(_buf(recv[0], n * 8)), dtype=np.float64).copy()
                parts = self.hub.collective(me, mine)
                tot = np.zeros(n)
                for p in parts:  # rank order: the same sum on every rank
                    tot = tot + p
                C.memmove(recv[0], tot.tobytes(), n * 8)
            elif op == OP_ALLGATHER:
                nb = int(sbytes[0])
                mine = bytes(_buf(send[0], nb) or b"")
                parts = self.hub.collective(me, mine)
                blob = b"".join(parts)
                if len(blob) != int(rbytes[0]):
                    raise AmgError("allgather size mismatch")
                if blob:
                    C.memmove(recv[0], blob, len(blob))
            else:
                raise AmgError(f"unknown op {op}")
            return 0
        except Exception as e:  # reported as a status code to the library
            self.error = e
            return 1


def init_host(ctx, nranks, rank, transport):
    ctx._xport = transport  # keep the callback alive
    check(lib.amg_dist_init_host(ctx.h, nranks, rank, C.cast(transport.cfn, C.c_void_p), None))


def init_rccl(ctx, nranks, rank, group_broadcast):
    """group_broadcast(bytes or None) -> bytes: rank 0's unique id on every rank."""
    n = lib.amg_dist_unique_id_size()
    buf = C.create_string_buffer(n)
    if rank == 0:
        check(lib.amg_dist_get_unique_id(buf))
        uid = group_broadcast(buf.raw)
    else:
        uid = group_broadcast(None)
    buf = C.create_string_buffer(bytes(uid), n)
    check(lib.amg_dist_init(ctx.h, nranks, rank, buf))


def finalize(ctx):
    check(lib.amg_dist_finalize(ctx.h))


def set_replicate_rows(ctx, rows):
    check(lib.amg_dist_hier_set_replicate_rows(ctx.h, int(rows)))


def structured_row_starts(gen, nranks):
    """The z-slab row partition amg_dist_hier_create_structured uses: (L, nranks+1)."""
    rs = np.zeros((gen.L, nranks + 1), dtype=np.int64)
    check(lib.amg_dist_structured_row_starts(gen.h, nranks, rs.ctypes.data_as(C.POINTER(C.c_longlong))))
    return rs


def barrier(ctx):
    check(lib.amg_dist_barrier(ctx.h))


def allreduce_sum(ctx, vals):
    a = np.ascontiguousarray(vals, dtype=np.float64).copy()
    check(lib.amg_dist_allreduce_sum(ctx.h, _dp(a), a.size))
    return a


def _part(nrows, rowptr, col, val):
    rp = np.ascontiguousarray(rowptr, dtype=np.int32)
    cj = np.ascontiguousarray(col, dtype=np.int32)
    cv = np.ascontiguousarray(val, dtype=np.float64)
    p = abi.AmgCsrPart(int(nrows), int(rp[-1]), _ip(rp), _ip(cj), _dp(cv))
    return p, (rp, cj, cv)


class DistHier:
    """Row-distributed hierarchy + SMEM_Solve loop.

    ``DistHier(ctx, gen, opts)`` builds the structured problem slab by slab;
    ``DistHier.from_parts`` takes this rank's rows of every operator with
    global column ids and the per-level row partition (ParCSR row_starts)."""

    def __init__(self, ctx, gen, opts, _handle=None, slab=False):
        """slab=True: the z-slab form (amg_dist_hier_create_slab: extended slab
        operators, plane exchange, the single-GPU march / geometric / fused
        kernels); False: the row-partitioned form with [owned | ghost] columns."""
        self.ctx, self.gen, self.opts = ctx, gen, opts
        self.slab = bool(slab)
        if _handle is None:
            h = C.c_void_p()
            create = lib.amg_dist_hier_create_slab if slab else lib.amg_dist_hier_create_structured
            check(create(ctx.h, gen.h, C.byref(opts), C.byref(h)))
            _handle = h
        self.h = _handle
        self.L = gen.L if gen is not None else None
        self.row0, self.n0 = self.local_rows(0)

    def slab_info(self):
        """(distributed levels, bitmask of geometric-transfer levels, fused level-0
        residual + restriction) of a slab hierarchy ((0, 0, 0) otherwise)"""
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        check(lib.amg_dist_hier_slab_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    @classmethod
    def from_parts(cls, ctx, row_starts, A, P, R, opts):
        """row_starts: (L, nranks+1) ints; A/P/R: lists of (nrows, rowptr, col, val)."""
        rs = np.ascontiguousarray(row_starts, dtype=np.int64)
        L = rs.shape[0]
        keep = []

        def arr(parts, n):
            out = (abi.AmgCsrPart * max(n, 1))()
            for i, t in enumerate(parts):
                out[i], k = _part(*t)
                keep.append(k)
            return out
        a, p, r = arr(A, L), arr(P, L - 1), arr(R, L - 1)
        h = C.c_void_p()
        check(lib.amg_dist_hier_create(ctx.h, L, rs.ctypes.data_as(C.POINTER(C.c_longlong)),
                                       C.cast(a, C.c_void_p), C.cast(p, C.c_void_p),
                                       C.cast(r, C.c_void_p), C.byref(opts), C.byref(h)))
        D = cls(ctx, None, opts, _handle=h)
        D.L = L
        return D

    def matrix_info(self, level):
        """(local nnz, value-index table size, dictionary size, row patterns) of
        this rank's A_level (0 = that form is not used)."""
        nnz, vi, dc, rp = C.c_longlong(), C.c_int(), C.c_int(), C.c_int()
        check(lib.amg_dist_hier_matrix_info(self.h, level, C.byref(nnz), C.byref(vi), C.byref(dc),
                                            C.byref(rp)))
        return nnz.value, vi.value, dc.value, rp.value

    def pair_pattern(self, level):
        """distinct row-pair patterns of this rank's A_level (0 = not pair-coded)"""
        pp = C.c_int()
        check(lib.amg_dist_hier_pair_pattern(self.h, level, C.byref(pp)))
        return pp.value

    def local_rows(self, level):
        r0, n = C.c_int(), C.c_int()
        check(lib.amg_dist_hier_local_rows(self.h, level, C.byref(r0), C.byref(n)))
        return r0.value, n.value

    def solve_start(self, f_local):
        f = np.ascontiguousarray(f_local, dtype=np.float64)
        assert f.size == self.n0
        r0 = C.c_double()
        check(lib.amg_dist_solve_start(self.h, _dp(f), C.byref(r0)))
        return r0.value

    def iterate(self, k):
        check(lib.amg_dist_solve_iterate(self.h, int(k)))

    def resnorm(self):
        r = C.c_double()
        check(lib.amg_dist_solve_resnorm(self.h, C.byref(r)))
        return r.value

    def async_solve(self, f_local):
        """Asynchronous additive solve (ASYNC_MULTADD / ASYNC_AFACX opts):
        returns (relres, per-level correction counts); u via get_u()."""
        f = np.ascontiguousarray(f_local, dtype=np.float64)
        assert f.size == self.n0
        L = self.gen.L if self.gen is not None else 64
        cnt = np.zeros(max(L, 64), dtype=np.int32)
        rel = C.c_double()
        check(lib.amg_dist_async_solve(self.h, _dp(f), _ip(cnt), C.byref(rel)))
        return rel.value, cnt

    def set_async_durations(self, ms):
        """AMG_SCHED_TIMED: level k's time per correction (the same on every rank)"""
        d = np.ascontiguousarray(ms, dtype=np.float64)
        check(lib.amg_dist_hier_set_async_durations(self.h, _dp(d), int(d.size)))

    def set_async_times(self, times):
        """AMG_SCHED_TIMED replaying recorded end times (the same on every rank)"""
        from . import _times_flat
        flat, n = _times_flat(times)
        check(lib.amg_dist_hier_set_async_times(self.h, _dp(flat), _ip(n), int(n.size)))

    def async_correction_ms(self, start=False):
        """per level: end (start=True: start) times (ms) of this rank's update windows in the last
        free-race async_solve"""
        from . import _corr_ms
        return _corr_ms(lib.amg_dist_async_correction_ms, self.h, self.L, start)

    def async_update_windows(self):
        """(starts, ends) per level: device-clock execution windows (ms) of this rank's update
        kernels in the last free race (amg_dist_async_update_windows)"""
        from . import _corr_ms
        return (_corr_ms(lib.amg_dist_async_update_windows, self.h, self.L, True),
                _corr_ms(lib.amg_dist_async_update_windows, self.h, self.L, False))

    def async_update_rows(self):
        """per level: (corrections, n0) per-row update times (ms, the windows' clock) of
        this rank's rows in the last free race, or None where not recorded
        (amg_dist_async_update_rows)"""
        from . import _update_rows
        counts = [len(w) for w in self.async_update_windows()[1]]
        return _update_rows(lib.amg_dist_async_update_rows, self.h, counts, self.n0)

    def async_update_vals(self):
        """per level: (corrections, n0, 2) -- every row's (old, new) value of each add in
        the last free race on this rank (NaN: not recorded), or None"""
        from . import _update_rows
        counts = [len(w) for w in self.async_update_windows()[1]]
        return _update_rows(lib.amg_dist_async_update_rows, self.h, counts, self.n0, vals=True)

    def async_level_ms(self):
        """per level: ms from the last async_solve's start to the level's last correction"""
        L = self.gen.L if self.gen is not None else 64
        ms = np.zeros(max(L, 64), dtype=np.float64)
        check(lib.amg_dist_async_level_ms(self.h, _dp(ms)))
        return ms[:L]

    def async_jacobi(self, f_local, sweeps, l1=False):
        """DMEM_AsyncSmooth (ASYNC_JACOBI / ASYNC_L1_JACOBI) on the fine level: relres."""
        f = np.ascontiguousarray(f_local, dtype=np.float64)
        assert f.size == self.n0
        rel = C.c_double()
        check(lib.amg_dist_async_jacobi(self.h, _dp(f), int(sweeps), int(l1), C.byref(rel)))
        return rel.value

    def async_jacobi_stats(self):
        """the last async_jacobi run: dict of the exchange overlap and delta accounting"""
        st = np.zeros(9)
        check(lib.amg_dist_async_jacobi_stats(self.h, _dp(st), 9))
        keys = ("hidden_fraction", "exchange_ms_per_sweep", "interior_ms_per_sweep", "on_time_fraction",
                "late_deltas", "incremental_resnorm", "true_resnorm", "device_links", "send_wait_ms_per_sweep")
        return dict(zip(keys, st.tolist()))

    def async_jacobi_log(self):
        """the last async_jacobi run's schedule on this rank: (events, 5) array --
        [1, sweep, accel mode, om1, omd] update, [2, sweep] interior product,
        [3, peer, j] peer's delta j applied, [4, sweep] all peers' deltas of a sweep"""
        cnt = np.zeros(1, dtype=np.int32)
        check(lib.amg_dist_async_jacobi_log(self.h, None, 0, _ip(cnt)))
        ev = np.zeros(max(1, 5 * int(cnt[0])))
        check(lib.amg_dist_async_jacobi_log(self.h, _dp(ev), int(cnt[0]), _ip(cnt)))
        return ev[:5 * int(cnt[0])].reshape(int(cnt[0]), 5)

    def async_sps(self, f_local, sweeps):
        """-smoother async_sps (stochastic parallel Southwell gating of the
        asynchronous Jacobi, opts.sps_*): (relres, sweeps this rank relaxed in)."""
        f = np.ascontiguousarray(f_local, dtype=np.float64)
        assert f.size == self.n0
        rel, nrel = C.c_double(), C.c_longlong()
        check(lib.amg_dist_async_sps(self.h, _dp(f), int(sweeps), C.byref(rel), C.byref(nrel)))
        return rel.value, nrel.value

    def get_u(self):
        u = np.empty(self.n0)
        check(lib.amg_dist_get_u(self.h, _dp(u)))
        return u

    def profile(self, reset=True):
        ms = np.zeros(5)
        n = np.zeros(5, dtype=np.int64)
        check(lib.amg_dist_profile_read(self.h, _dp(ms), n.ctypes.data_as(C.POINTER(C.c_longlong)),
                                        int(reset)))
        return ms, n

    def fine_spmv_ms(self, reps=20):
        ms = C.c_double()
        check(lib.amg_dist_fine_spmv(self.h, int(reps), C.byref(ms)))
        return ms.value

    def free(self):
        if self.h:
            lib.amg_dist_hier_free(self.h)
            self.h = None
