"""The oracle's asynchronous additive band (test infrastructure).

oracle/amg_oracle.c or_async_add restates SMEM_Async_Add_AMG
(SMEM_Async_AMG.cpp:7-437) on real OpenMP threads: thread groups own levels and
race on the shared iterate exactly as the reference does, so repeated runs
give the reference's own spread of final relative residuals.  The GPU's
asynchronous solves must land in [0.5 x min, 2 x max] of that band
(SURVEY.md Sec.8(d)).  Thread sets: one and two threads per level (T = L and
2L; every level needs a group); the band is taken over all runs of both and
the equal-speed schedule: every level correcting from the same state each
cycle, which is the synchronous additive cycle (MULTADD / AFACX).  With
sequential=True (converge LOCAL) also the two extreme speed ratios: the groups
one after another, finest first and coarsest first.  How fast
the groups run relative to one another sets where a run lands, and that
differs between this container's 8 cores, the GPU box's host share and the
device's level streams; equal speed is the schedule the device's concurrent
streams tend to and one admissible schedule of the reference's race."""
import ctypes

import numpy as np

from test_gpu_solve import oracle_opts


def oracle_async_band(amg, oracle, host, f, opts, reps=10, thread_sets=None, blocks=None, lockstep=True,
                      sequential=False, lockstep_cycles=()):
    """res_compute_type GLOBAL (ASYNC_MULTADD): no level-0 group (thread sets
    [0, 1, ..] / [0, 2, ..]) and no synchronous equivalent, so no lockstep
    member; the sequential schedules are added instead.  accel_type (the
    distributed solve's ChebyUpdate per level, DMEM_Add.cpp:319-324) likewise
    has no synchronous equivalent: sequential schedules, no lockstep.
    lockstep_cycles: further equal-speed members with these cycle counts
    (converge GLOBAL: the device's grids keep correcting until the slowest is
    done, so the fastest may run many more than num_cycles corrections)."""
    """(lo, hi, rels, counts) of `reps` runs per thread set (rels[-1]: the
    synchronous schedule when lockstep); opts: the GPU run's
    amg_opts (solver ASYNC_MULTADD / ASYNC_AFACX, smoother, sweeps, num_cycles,
    async_type, read_type, converge_test_type)."""
    L = len(host["A"])
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if blocks is not None:
        for lev, blk in blocks.items():
            OH.set_blocks(lev, blk)
    at = oracle.OR_SEMI_ASYNC if opts.async_type == amg.AMG_SEMI_ASYNC else oracle.OR_FULL_ASYNC
    rt = oracle.OR_READ_RES if opts.read_type == amg.AMG_READ_RES else oracle.OR_READ_SOL
    ct = oracle.OR_CONVERGE_GLOBAL if opts.converge_test_type == amg.AMG_GLOBAL else oracle.OR_CONVERGE_LOCAL
    gres = opts.res_compute_type == amg.AMG_GLOBAL and opts.solver == amg.AMG_ASYNC_MULTADD
    if gres:
        thread_sets = thread_sets or ([0] + [1] * (L - 1), [0] + [2] * (L - 1))
        lockstep, sequential = False, True
    accel = None
    if opts.accel_type != amg.AMG_NO_ACCEL:
        # the device's cheby_grid is clamped to its last correcting level, L - 2
        accel = (opts.accel_type, min(opts.cheby_grid, L - 2), opts.cheby_mu, opts.cheby_delta)
        lockstep, sequential = False, True
    rels, counts = [], []
    for nt in thread_sets or ([1] * L, [2] * L):
        for _ in range(reps):
            u, rel, cnt = OH.async_add(f, nt, async_type=at, converge_type=ct, read_type=rt, res_global=gres,
                                       accel=accel)
            assert np.all(np.isfinite(u))
            rels.append(rel)
            counts.append(cnt)
    if sequential and ct == oracle.OR_CONVERGE_LOCAL:
        # the extreme speed ratios: the groups one after another, finest /
        # coarsest first (admissible schedules of the same race)
        for sched in (1, 2):
            oracle.lib().or_set_async_schedule(sched)
            try:
                u, rel, cnt = OH.async_add(f, [0 if gres else 1] + [1] * (L - 1), async_type=at, converge_type=ct,
                                           read_type=rt, res_global=gres, accel=accel)
            finally:
                oracle.lib().or_set_async_schedule(0)
            rels.append(rel)
            counts.append(cnt)
    if lockstep:
        so = amg.default_opts()
        ctypes.memmove(ctypes.byref(so), ctypes.byref(opts), ctypes.sizeof(so))
        so.solver = amg.AMG_AFACX if opts.solver == amg.AMG_ASYNC_AFACX else amg.AMG_MULTADD
        SH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, so))
        if blocks is not None:
            for lev, blk in blocks.items():
                SH.set_blocks(lev, blk)
        _, h, _ = SH.solve(f)
        rels.append(h[-1] / h[0])
        for nc in lockstep_cycles:
            so.num_cycles = int(nc)
            XH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, so))
            if blocks is not None:
                for lev, blk in blocks.items():
                    XH.set_blocks(lev, blk)
            _, h, _ = XH.solve(f)
            rels.append(h[-1] / h[0])
    return min(rels), max(rels), rels, counts


def blocks64(host):
    """the device's default hybrid JGS blocks (jgs_block_rows = 64) per level"""
    out = {}
    for lev, A in enumerate(host["A"]):
        n = A.nrows
        out[lev] = np.unique(np.minimum(np.arange(0, n + 64, 64), n)).astype(np.int32)
    return out


class Ends(list):
    """per-level window ends of one hierarchy's free race; .rows: the per-row
    update times (async_update_rows: per level a (corrections, rows) array, or
    None where the update kernels did not stamp every row)"""
    rows = None
    vals = None


def race_tables(h):
    """(ends, starts) per level of a hierarchy's last free race: the device-clock
    execution windows of its update kernels (async_update_windows) where every
    correction was stamped, else the HIP events around them
    (async_correction_ms; SEMI_ASYNC's serialised updates carry no stamp).
    ends.rows: every row's update time of every correction, where stamped"""
    w0, w1 = h.async_update_windows()
    if sum(len(x) for x in w1) and all(np.all(np.isfinite(x)) for x in list(w0) + list(w1)):
        e = Ends(w1)
        e.rows = h.async_update_rows()
        e.vals = h.async_update_vals()
        return e, w0
    return h.async_correction_ms(), h.async_correction_ms(start=True)


def _rows_of(ends, L):
    """the per-rank per-row tables of a run's ends (Ends per rank), or None unless
    every rank stamped every row of every correction"""
    per = _per_rank(ends)
    out = []
    for e in per:
        rows = getattr(e, "rows", None)
        if rows is None or len(rows) < L or any(r is None for r in rows[:L]):
            return None
        if any(len(r) != len(e[k]) for k, r in enumerate(rows[:L]) if k < len(e)):
            return None
        out.append(rows)
    return out


def _vals_of(ends, L):
    """the per-rank per-row (old, new) value tables of a run's ends, or None"""
    per = _per_rank(ends)
    out = []
    for e in per:
        v = getattr(e, "vals", None)
        if v is None or len(v) < L or any(x is None for x in v[:L]):
            return None
        out.append(v)
    return out


def chain_order(order, vold, vnew, u0=0.0, window=16):
    """repair per-row update orders with the values the adds returned: in the
    true order of a row's adds each add's old value is the previous add's new
    value (the first's: the initial u0), bit for bit -- the clock orders two
    levels' adds of one row only to within the adds' latency.  order: (n, E)
    event indices by time; vold / vnew: (n, E) values by event index.  Rows whose
    time order already chains are kept; in the others the next add is the one,
    among the next `window` by time, whose old value is the running value.
    Returns (order, repaired rows, rows left unchained)"""
    n, E = order.shape
    if E == 0:
        return order, 0, 0
    so = np.take_along_axis(vold, order, axis=1)
    sn = np.take_along_axis(vnew, order, axis=1)
    ok = np.all(so[:, 1:].view(np.uint64) == sn[:, :-1].view(np.uint64), axis=1)
    ok &= so[:, 0] == u0
    bad = np.nonzero(~ok)[0]
    left = 0
    order = order.copy()
    for i in bad:
        rem = list(order[i])
        cur = np.float64(u0)
        out = []
        broken = False
        while rem:
            pick = 0
            for q in range(min(window, len(rem))):
                if vold[i, rem[q]] == cur and np.float64(vold[i, rem[q]]).tobytes() == cur.tobytes():
                    pick = q
                    break
            else:
                broken = True
            x = rem.pop(pick)
            out.append(x)
            cur = np.float64(vnew[i, x])
        order[i] = out
        left += broken
    return order, len(bad), left


def row_order_slices(rows, L, vals=None, u0=0.0):
    """cut the fine rows into the fewest slices inside which every row received
    the corrections of all levels in the same order (rows: per rank, per level a
    (corrections, rank rows) array of update times; ranks' rows in order; vals:
    the same layout of (old, new) values, which repair the time order where the
    clock cannot tell two adds apart, chain_order).  Returns (cuts, per-slice
    per-level time arrays, (repaired rows, unchained rows)): a slice's times are
    its first row's, reassigned so that sorting them gives that row's order --
    or_async_add_replay applies every slice's updates in exactly the order its
    rows saw them"""
    nc = [min(r[k].shape[0] for r in rows) for k in range(L)]
    T, VO, VN = [], [], []
    for k in range(L):
        T.append(np.concatenate([np.asarray(r[k], dtype=np.float64)[:nc[k]] for r in rows], axis=1)
                 if nc[k] else None)
        if vals is not None and nc[k]:
            v = np.concatenate([np.asarray(r[k], dtype=np.float64)[:nc[k]] for r in vals], axis=1)
            VO.append(v[:, :, 0])
            VN.append(v[:, :, 1])
    n = sum(np.asarray(r[0]).shape[1] for r in rows)
    cols = [T[k].T for k in range(L) if T[k] is not None]
    M = np.concatenate(cols, axis=1) if cols else np.zeros((n, 0))
    order = np.argsort(M, axis=1, kind="stable")
    stats = (0, 0)
    if vals is not None and VO:
        vo = np.concatenate([x.T for x in VO], axis=1)
        vn = np.concatenate([x.T for x in VN], axis=1)
        if np.all(np.isfinite(vo)) and np.all(np.isfinite(vn)):
            order, nrep, nleft = chain_order(order, vo, vn, u0)
            stats = (nrep, nleft)
    change = np.any(order[1:] != order[:-1], axis=1) if len(order) > 1 else np.zeros(0, dtype=bool)
    starts = [0] + [int(i) + 1 for i in np.nonzero(change)[0]]
    cuts = starts + [n]
    # event index -> (level, correction)
    ev = [(k, j) for k in range(L) if T[k] is not None for j in range(nc[k])]
    tabs = []
    for a in starts:
        ts = np.sort(M[a])
        tab = [np.zeros(nc[k]) if T[k] is not None else np.zeros(0) for k in range(L)]
        for m, x in enumerate(order[a]):
            k, j = ev[x]
            tab[k][j] = ts[m]
        tabs.append(tab)
    return cuts, tabs, stats


def row_replay(amg, oracle, host, f, opts, rows, composed=False, blocks=None, vals=None):
    """the oracle's exact replay of a free race whose update kernels stamped every
    row: or_async_add_replay with one slice per run of rows that saw the same
    update order (row_order_slices; vals: the adds' values, which fix the order
    of adds the clock cannot separate).  Returns (relres, slices, (repaired rows,
    unchained rows))"""
    L = len(host["A"])
    cuts, tabs, stats = row_order_slices(rows, L, vals=vals)
    rel = _replay_slices(amg, oracle, host, f, opts, cuts, tabs, composed=composed, blocks=blocks)
    return rel, len(tabs), stats


def _per_rank(x):
    """per-rank lists of per-level time arrays: one hierarchy's tables (a list
    of per-level arrays) or a list of them, one per rank"""
    for lev in x:
        if len(lev):
            return list(x) if hasattr(lev[0], "__len__") else [x]
    return [x]


def in_band(rel, lo, hi):
    return 0.5 * lo <= rel <= 2.0 * hi


def free_band_check(amg, opts, rels, flo, fhi, what=""):
    """the device's free races against the oracle's own free races (the
    reference's spread of results on host threads, oracle_async_band): converge
    LOCAL -- every run in [0.5 min, 2 max]; converge GLOBAL (every level runs
    until all are done, so the device's fastest levels may run far more
    corrections than any host run) -- every run at most 2 max"""
    for r in rels:
        if opts.converge_test_type == amg.AMG_GLOBAL:
            assert r <= 2.0 * fhi, (what, r, flo, fhi)
        else:
            assert in_band(r, flo, fhi), (what, r, flo, fhi)


def durations_of(level_ms, counts, L):
    """per-level correction times of a device free race: finish time / corrections
    for the levels that corrected; the reference's idle coarsest group (no
    device group under LOCAL residuals) runs at the coarsest correcting level's
    speed; levels without a group take 1 (unused)"""
    d = np.ones(L)
    last = None
    for k in range(L):
        if counts[k] > 0 and level_ms[k] > 0:
            d[k] = level_ms[k] / counts[k]
            last = d[k]
    if counts[L - 1] == 0 and last is not None:
        d[L - 1] = last
    return d


def times_of(corr_ms, L, ranks=None):
    """the recorded end times of a device free race's corrections, per level
    (corr_ms: async_correction_ms() of one hierarchy, or a list of them, one
    per rank -- a distributed correction ends on its slowest rank); the
    reference's idle coarsest group (no device group under LOCAL residuals)
    takes the coarsest correcting level's times"""
    per = _per_rank(corr_ms)
    out = []
    for k in range(L):
        rows = [np.asarray(r[k], dtype=np.float64) for r in per]
        n = min(len(x) for x in rows)
        out.append(np.max(np.array([x[:n] for x in rows]), axis=0) if n else np.zeros(0))
    if len(out[L - 1]) == 0:
        for k in range(L - 2, -1, -1):
            if len(out[k]):
                out[L - 1] = out[k].copy()
                break
    return out


def replay_tables(corr_ms, L):
    """the replay tables of one device free race: the update order of the
    slowest rank (times_of over every rank) and, with several ranks, each
    rank's own order -- every rank's rows receive the corrections in that
    rank's order, so a distributed race lies between these replays"""
    per = _per_rank(corr_ms)
    out = [times_of(per, L)]
    if len(per) > 1:
        out += [times_of([r], L) for r in per]
    return out


def _replay_slices(amg, oracle, host, f, opts, rs, per_slice, composed=False, blocks=None):
    """or_async_add_replay: slice s = [rs[s], rs[s+1]) of the fine rows receives
    every level's corrections at the times per_slice[s][k] (a correction's
    update is formed once, at its first slice's time)"""
    L = len(host["A"])
    S = len(rs) - 1
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if composed:
        OH.set_composed_transfers()
    if blocks is not None:
        for lev, blk in blocks.items():
            OH.set_blocks(lev, blk)
    accel = None
    if opts.accel_type != amg.AMG_NO_ACCEL:
        accel = (opts.accel_type, min(opts.cheby_grid, L - 2), opts.cheby_mu, opts.cheby_delta)
    times = []
    for k in range(L):
        n = min(len(per_slice[q][k]) for q in range(S))
        times.append(np.stack([np.asarray(per_slice[q][k][:n], dtype=np.float64) for q in range(S)], axis=1)
                     if n else np.zeros((0, S)))
    u, rel, _ = OH.async_add_replay(f, rs, times, accel=accel)
    assert np.all(np.isfinite(u))
    return rel


def sliced_replay(amg, oracle, host, f, opts, corr_ms, rs, composed=False, blocks=None):
    """the oracle's replay of a DISTRIBUTED free race (or_async_add_replay):
    rank r's slice [rs[r], rs[r+1]) of the fine rows receives every level's
    corrections at that rank's recorded update times"""
    return _replay_slices(amg, oracle, host, f, opts, rs, corr_ms, composed=composed, blocks=blocks)


def torn_replay(amg, oracle, host, f, opts, ends, starts, rs=None, slices=16, composed=False, blocks=None):
    """the row-time model of a torn race: a correction's update pass, recorded
    as the window [start, end] on its rank, reaches the rank's rows in order --
    row position x in [0, 1) of the rank's rows at start + (end - start) x --
    so inside overlapping windows the levels' updates interleave by rows.  The
    rank's rows are cut into `slices` pieces, each receiving every correction
    at its interpolated time (or_async_add_replay)"""
    per_e = _per_rank(ends)
    per_s = _per_rank(starts)
    L = len(host["A"])
    n0 = host["A"][0].nrows
    rs = list(rs) if rs is not None else [0, n0]
    cuts, tabs = [0], []
    for r in range(len(per_e)):
        a, b = rs[r], rs[r + 1]
        for q in range(slices):
            lo_, hi_ = a + (b - a) * q // slices, a + (b - a) * (q + 1) // slices
            if hi_ <= lo_:
                continue
            x = (q + 0.5) / slices
            tab = []
            for k in range(L):
                e = np.asarray(per_e[r][k], dtype=np.float64)
                st = np.asarray(per_s[r][k], dtype=np.float64) if k < len(per_s[r]) else e
                n = len(e)
                st = st[:n] if len(st) >= n else np.concatenate([st, e[len(st):]])
                tab.append(st + (e - st) * x)
            tabs.append(tab)
            cuts.append(hi_)
    return _replay_slices(amg, oracle, host, f, opts, cuts, tabs, composed=composed, blocks=blocks)


def torn_updates(ends, starts):
    """how many pairs of update windows of DIFFERENT levels overlap in time on
    one rank (ends / starts: per rank, per level, the recorded window ends /
    starts).  Inside an overlap the two atomic updates interleave row by row,
    so each level's captured iterate holds the other's correction on some
    rows only: a torn update, which the FULL_ASYNC race allows (the
    reference's omp atomic loops of two groups can interleave the same way)
    and no order of whole corrections reproduces."""
    per_e = _per_rank(ends)
    per_s = _per_rank(starts)
    torn = 0
    for e_r, s_r in zip(per_e, per_s):
        win = []
        for k, (e, s) in enumerate(zip(e_r, s_r)):
            n = min(len(e), len(s))
            win += [(float(s[j]), float(e[j]), k) for j in range(n)]
        win.sort()
        for a in range(len(win)):
            for b in range(a + 1, len(win)):
                if win[b][0] >= win[a][1]:
                    break
                if win[b][2] != win[a][2]:
                    torn += 1
    return torn


def replay_check(amg, oracle, host, f, opts, runs, blocks=None, composed=False, what=""):
    """Every free run (rel, ends[, rs[, starts]]) against the oracle's replay of
    its own recorded update order; every run must lie in [0.5 lo, 2 hi] of its
    replay band.
    * Row-stamped runs (ends.rows: the update kernels stamped every row with
      the time its add + read-back completed) are replayed EXACTLY: the rows
      are cut into slices inside which every row saw the same order of
      updates, and or_async_add_replay applies each slice's updates in that
      order (row_replay).  A torn update -- update kernels of different levels
      overlapping, their atomics interleaved row by row in whatever order the
      workgroups ran -- is reproduced row for row.
    * Otherwise: whole corrections in the order of their update points (rows of
      rank r in rank r's order; race_tables: the update kernels' device-clock
      windows), and for a torn run also the row-time model (torn_replay), the
      band spanning both."""
    L = len(host["A"])
    widest = 1.0
    # (or_async_add_replay restates FULL_ASYNC / READ_SOL / LOCAL residuals only)
    sliceable = (opts.async_type != amg.AMG_SEMI_ASYNC and opts.read_type != amg.AMG_READ_RES and
                 not (opts.res_compute_type == amg.AMG_GLOBAL and opts.solver == amg.AMG_ASYNC_MULTADD))
    for i, run in enumerate(runs):
        rel, corr_ms = run[0], run[1]
        rs = run[2] if len(run) > 2 else None
        starts = run[3] if len(run) > 3 else None
        torn = torn_updates(corr_ms, starts) if starts is not None else 0
        rows = _rows_of(corr_ms, L) if sliceable else None
        tm = None
        if rows is not None:
            lo, nsl, (nrep, nleft) = row_replay(amg, oracle, host, f, opts, rows, composed=composed, blocks=blocks,
                                                vals=_vals_of(corr_ms, L))
            hi, rr = lo, [lo]
            model = f"row replay, {nsl} slice(s), {nrep} row(s) reordered by value, {nleft} unchained"
        else:
            if rs is not None and len(rs) > 2:
                lo = hi = sliced_replay(amg, oracle, host, f, opts, corr_ms, rs, composed=composed, blocks=blocks)
                rr = [lo]
            else:
                lo, hi, rr = timed_band(amg, oracle, host, f, opts, replay_tables(corr_ms, L), blocks=blocks,
                                        composed=composed)
            if torn and sliceable:
                tm = torn_replay(amg, oracle, host, f, opts, corr_ms, starts, rs=rs, composed=composed,
                                 blocks=blocks)
                lo, hi = min(lo, tm), max(hi, tm)
                rr = list(rr) + [tm]
            model = f"{len(rr)} order(s)"
        widest = max(widest, hi / lo)
        ok = in_band(rel, lo, hi)
        print(f"  {what} run {i}: device {rel:.4e}, replay [{lo:.4e}, {hi:.4e}] ({model}, width "
              f"{hi / lo:.2f}x), device / replay {rel / lo:.2f}-{rel / hi:.2f}, torn updates {torn}"
              + (f", row-time model {tm:.4e}" if tm is not None else "") + ("" if ok else "  OUTSIDE"))
        _dump(what, i, host, f, opts, run, composed, blocks)
        assert np.isfinite(rel), (what, i, rel)
        assert ok, (what, i, rel, lo, hi, torn)
    return widest


def _dump(what, i, host, f, opts, run, composed, blocks):
    """AMG_REPLAY_DUMP=dir: the run's recorded tables (JSON) and, once per
    case, the hierarchy and right-hand side (npz) -- for studying the replay
    models off the GPU"""
    import json
    import os
    d = os.environ.get("AMG_REPLAY_DUMP")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    tag = "".join(c if c.isalnum() else "_" for c in what)
    arr = os.path.join(d, f"{tag}.npz")
    if not os.path.exists(arr):
        mats = {}
        for key in ("A", "P", "R"):
            for lev, M in enumerate(host[key]):
                mats[f"{key}{lev}_shape"] = np.array([M.nrows, M.ncols])
                mats[f"{key}{lev}_rowptr"] = np.asarray(M.rowptr)
                mats[f"{key}{lev}_col"] = np.asarray(M.col)
                mats[f"{key}{lev}_val"] = np.asarray(M.val)
        import ctypes
        mats["opts"] = np.frombuffer(ctypes.string_at(ctypes.addressof(opts), ctypes.sizeof(opts)), dtype=np.uint8)
        mats["f"] = np.asarray(f)
        if blocks is not None:
            for lev, blk in blocks.items():
                mats[f"blk{lev}"] = np.asarray(blk)
        np.savez_compressed(arr, **mats)
    def lst(x):
        if x is None:
            return None
        if hasattr(x, "tolist"):
            return x.tolist()
        if isinstance(x, (list, tuple)):
            return [lst(v) for v in x]
        return float(x)

    rec = {"what": what, "run": i, "rel": float(run[0]), "composed": bool(composed),
           "ends": lst(run[1]), "rs": None if len(run) < 3 or run[2] is None else [int(x) for x in run[2]],
           "starts": lst(run[3]) if len(run) > 3 else None}
    with open(os.path.join(d, f"{tag}_run{i}.json"), "w") as fh:
        json.dump(rec, fh)
    rows = _rows_of(run[1], len(host["A"]))
    if rows is not None:
        np.savez_compressed(os.path.join(d, f"{tag}_run{i}_rows.npz"),
                            **{f"r{r}_l{k}": np.asarray(t) for r, rr in enumerate(rows) for k, t in enumerate(rr)})


def timed_band(amg, oracle, host, f, opts, durations, blocks=None, composed=False, nt=None):
    """The oracle's model of a device free race: or_async_add under the timed
    schedule (or_set_async_schedule 4: whole corrections in the order of their
    end times) -- the replay of the update order each device run recorded
    (times_of: every correction's end event), or the race at the fixed
    per-level speeds it measured (durations_of).  Returns (lo, hi, rels): the device's
    free race must lie in [0.5 lo, 2 hi] (in_band) -- the window of the race's
    jitter around its model, instead of the band of every speed ratio."""
    L = len(host["A"])
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    if composed:
        OH.set_composed_transfers()
    if blocks is not None:
        for lev, blk in blocks.items():
            OH.set_blocks(lev, blk)
    at = oracle.OR_SEMI_ASYNC if opts.async_type == amg.AMG_SEMI_ASYNC else oracle.OR_FULL_ASYNC
    rt = oracle.OR_READ_RES if opts.read_type == amg.AMG_READ_RES else oracle.OR_READ_SOL
    ct = oracle.OR_CONVERGE_GLOBAL if opts.converge_test_type == amg.AMG_GLOBAL else oracle.OR_CONVERGE_LOCAL
    gres = opts.res_compute_type == amg.AMG_GLOBAL and opts.solver == amg.AMG_ASYNC_MULTADD
    accel = None
    if opts.accel_type != amg.AMG_NO_ACCEL:
        accel = (opts.accel_type, min(opts.cheby_grid, L - 2), opts.cheby_mu, opts.cheby_delta)
    rels = []
    for d in durations:
        if isinstance(d, list):  # recorded end times per level (times_of): the replay
            oracle.set_async_times(d, exact=True)
        else:  # per-level correction times (durations_of)
            oracle.set_async_durations(d)
        oracle.lib().or_set_async_schedule(4)
        try:
            u, rel, cnt = OH.async_add(f, nt or ([0 if gres else 1] + [1] * (L - 1)), async_type=at,
                                       converge_type=ct, read_type=rt, res_global=gres, accel=accel)
        finally:
            oracle.lib().or_set_async_schedule(0)
        assert np.all(np.isfinite(u))
        rels.append(rel)
    return min(rels), max(rels), rels
