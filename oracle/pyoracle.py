"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  The product library never does.  See amg_oracle.h for the parity status.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

OR_JACOBI, OR_GAUSS_SEIDEL, OR_HYBRID_JGS, OR_SYMM_JACOBI = 0, 1, 2, 3
OR_L1_JACOBI, OR_L1_HYBRID_JGS = 6, 12
OR_MULT, OR_AFACX, OR_MULTADD = 0, 1, 2
OR_ASYNC_AFACX, OR_ASYNC_MULTADD = 5, 6
OR_FULL_ASYNC, OR_SEMI_ASYNC = 0, 1
OR_CONVERGE_LOCAL, OR_CONVERGE_GLOBAL = 0, 1
OR_READ_SOL, OR_READ_RES = 0, 1

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class OrCsr(C.Structure):
    _fields_ = [("nrows", C.c_int), ("ncols", C.c_int), ("nnz", C.c_longlong),
                ("i", _ip), ("j", _ip), ("data", _dp)]


class OrCsrOwned(C.Structure):
    _fields_ = [("nrows", C.c_int), ("ncols", C.c_int), ("nnz", C.c_longlong),
                ("i", _ip), ("j", _ip), ("data", _dp)]


class OrOpts(C.Structure):
    _fields_ = [("solver", C.c_int), ("smoother", C.c_int),
                ("num_pre", C.c_int), ("num_post", C.c_int),
                ("num_fine", C.c_int), ("num_coarse", C.c_int),
                ("smooth_weight", C.c_double), ("num_cycles", C.c_int),
                ("tol", C.c_double), ("check_resnorm", C.c_int),
                ("cheby_flag", C.c_int), ("cheby_mu", C.c_double),
                ("cheby_delta", C.c_double), ("num_threads", C.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.or_rand_double.restype = C.c_double
        L.or_rand_double.argtypes = [C.c_double, C.c_double]
        L.or_norm2.restype = C.c_double
        L.or_hier_create.restype = C.c_void_p
        L.or_hier_create.argtypes = [C.c_int, C.POINTER(OrCsr), C.POINTER(OrCsr),
                                     C.POINTER(OrCsr), C.POINTER(OrOpts)]
        L.or_hier_free.argtypes = [C.c_void_p]
        L.or_hier_set_blocks.argtypes = [C.c_void_p, C.c_int, _ip, C.c_int]
        L.or_hier_set_composed_transfers.argtypes = [C.c_void_p, C.c_int]
        L.or_solve.argtypes = [C.c_void_p, _dp, _dp, _dp]
        L.or_solve.restype = C.c_int
        L.or_vcycle.argtypes = [C.c_void_p]
        L.or_sync_add_vcycle.argtypes = [C.c_void_p]
        L.or_hier_vec.restype = _dp
        L.or_hier_vec.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.or_eigs_power.argtypes = [C.c_void_p, C.c_int, _dp, _dp]
        L.or_num_threads.restype = C.c_int
        L.or_set_threads.argtypes = [C.c_int]
        L.or_last_loop_seconds.restype = C.c_double
        L.or_dmem_cheby_update.argtypes = [_dp, _dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                           C.c_double, _dp]
        L.or_dmem_mult_solve.restype = C.c_int
        L.or_dmem_mult_solve.argtypes = [C.c_void_p, _dp, _dp, _dp, C.c_int, C.c_double, C.c_double]
        L.or_set_async_gs_threads.argtypes = [C.c_int]
        L.or_set_async_schedule.argtypes = [C.c_int]
        L.or_set_async_durations.argtypes = [_dp, C.c_int]
        L.or_set_async_times.argtypes = [_dp, _ip, C.c_int]
        L.or_set_async_res_global.argtypes = [C.c_int]
        L.or_set_async_accel.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double]
        L.or_dmem_add.restype = C.c_int
        L.or_dmem_add.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                  C.c_int, C.c_int, C.c_double, C.c_double, _ip, _dp, C.POINTER(C.c_longlong)]
        L.or_async_add.restype = C.c_int
        L.or_async_add_replay.restype = C.c_int
        L.or_async_add_replay.argtypes = [C.c_void_p, _dp, _dp, C.c_int, _ip, _dp, _ip, _ip, C.POINTER(C.c_double)]
        L.or_async_add.argtypes = [C.c_void_p, _dp, _dp, _ip, C.c_int, C.c_int, C.c_int, _ip,
                                   C.POINTER(C.c_double)]
        L.or_dmem_async_jacobi.restype = C.c_double
        L.or_dmem_async_jacobi.argtypes = [C.POINTER(OrCsr), _dp, _dp, C.c_int, C.c_double, _dp,
                                           C.c_int, C.c_double, C.c_double]
        _LIB = L
    return _LIB


def dptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def iptr(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_ip)


class Csr:
    """Host CSR held as numpy arrays (int32 rowptr/col, float64 values)."""

    def __init__(self, nrows, ncols, rowptr, col, val):
        self.nrows, self.ncols = int(nrows), int(ncols)
        self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int32)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        self.val = np.ascontiguousarray(val, dtype=np.float64)
        self.nnz = int(self.rowptr[-1])

    def c(self):
        return OrCsr(self.nrows, self.ncols, self.nnz, iptr(self.rowptr), iptr(self.col),
                     dptr(self.val))

    def to_scipy(self):
        import scipy.sparse as sp
        return sp.csr_matrix((self.val, self.col, self.rowptr), shape=(self.nrows, self.ncols))


def _owned_to_csr(o):
    n, nnz = o.nrows, o.nnz
    rp = np.ctypeslib.as_array(o.i, shape=(n + 1,)).copy()
    cj = np.ctypeslib.as_array(o.j, shape=(max(nnz, 1),))[:nnz].copy()
    cv = np.ctypeslib.as_array(o.data, shape=(max(nnz, 1),))[:nnz].copy()
    lib().or_csr_free_owned(C.byref(o))
    return Csr(n, o.ncols, rp, cj, cv)


def laplace_7pt(nx, ny=None, nz=None):
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    o = OrCsrOwned()
    lib().or_laplace_7pt(nx, ny, nz, C.byref(o))
    return _owned_to_csr(o)


def transpose(A):
    o = OrCsrOwned()
    ac = A.c()
    lib().or_csr_transpose(C.byref(ac), C.byref(o))
    return _owned_to_csr(o)


def spgemm(A, B):
    o = OrCsrOwned()
    ac, bc = A.c(), B.c()
    lib().or_csr_spgemm(C.byref(ac), C.byref(bc), C.byref(o))
    return _owned_to_csr(o)


def smooth_transfer(A, P, omega):
    ps, rs = OrCsrOwned(), OrCsrOwned()
    ac, pc = A.c(), P.c()
    lib().or_smooth_transfer(C.byref(ac), C.byref(pc), C.c_double(omega), C.byref(ps), C.byref(rs))
    return _owned_to_csr(ps), _owned_to_csr(rs)


def rhs_rand(n, lo=-1.0, hi=1.0):
    f = np.empty(n, dtype=np.float64)
    lib().or_rhs_rand(C.c_int(n), C.c_double(lo), C.c_double(hi), dptr(f))
    return f


# ---- kernels ---------------------------------------------------------------
def seq_matvec(A, x):
    y = np.zeros(A.nrows)
    ac = A.c()
    lib().or_seq_matvec(C.byref(ac), dptr(x), dptr(y))
    return y


def seq_matvec_t(A, x):
    y = np.zeros(A.ncols)
    ac = A.c()
    lib().or_seq_matvec_t(C.byref(ac), dptr(x), dptr(y))
    return y


def smem_matvec_t_expand(A, x, T):
    y = np.zeros(A.ncols)
    ac = A.c()
    lib().or_smem_matvec_t_expand(C.byref(ac), dptr(x), dptr(y), C.c_int(T))
    return y


def smem_matvec(A, x, y, ns=0, ne=None):
    ne = A.nrows if ne is None else ne
    ac = A.c()
    lib().or_smem_matvec(C.byref(ac), dptr(x), dptr(y), C.c_int(ns), C.c_int(ne))
    return y


def smem_spgemv(A, x, b, alpha, beta, y, ib=0, ie=None):
    ie = A.nrows if ie is None else ie
    ac = A.c()
    bp = dptr(b) if b is not None else None
    lib().or_smem_spgemv(C.byref(ac), dptr(x), bp, C.c_double(alpha), C.c_double(beta),
                         dptr(y), C.c_int(ib), C.c_int(ie))
    return y


def smem_residual(A, b, x, y, r, ns=0, ne=None):
    ne = A.nrows if ne is None else ne
    ac = A.c()
    lib().or_smem_residual(C.byref(ac), dptr(b), dptr(x), dptr(y), dptr(r), C.c_int(ns), C.c_int(ne))
    return r


def seq_residual(A, b, x, y, r):
    ac = A.c()
    lib().or_seq_residual(C.byref(ac), dptr(b), dptr(x), dptr(y), dptr(r))
    return r


def smem_jacobi(A, f, u, u_prev, omega, sweeps, zero_flag, ns=0, ne=None):
    ne = A.nrows if ne is None else ne
    ac = A.c()
    lib().or_smem_jacobi(C.byref(ac), dptr(f), dptr(u), dptr(u_prev), C.c_double(omega),
                         C.c_int(sweeps), C.c_int(zero_flag), C.c_int(ns), C.c_int(ne))


def smem_l1jacobi(A, f, u, u_prev, l1, sweeps, zero_flag, ns=0, ne=None):
    ne = A.nrows if ne is None else ne
    ac = A.c()
    lib().or_smem_l1jacobi(C.byref(ac), dptr(f), dptr(u), dptr(u_prev), dptr(l1),
                           C.c_int(sweeps), C.c_int(zero_flag), C.c_int(ns), C.c_int(ne))


def seq_jacobi(A, f, u, u_prev, omega, sweeps, zero_flag):
    ac = A.c()
    lib().or_seq_jacobi(C.byref(ac), dptr(f), dptr(u), dptr(u_prev), C.c_double(omega),
                        C.c_int(sweeps), C.c_int(zero_flag))


def seq_l1jacobi(A, f, u, u_prev, l1, sweeps, zero_flag):
    ac = A.c()
    lib().or_seq_l1jacobi(C.byref(ac), dptr(f), dptr(u), dptr(u_prev), dptr(l1),
                          C.c_int(sweeps), C.c_int(zero_flag))


def seq_gauss_seidel(A, f, u, sweeps):
    ac = A.c()
    lib().or_seq_gauss_seidel(C.byref(ac), dptr(f), dptr(u), C.c_int(sweeps))


def async_gs(A, f, u, blk, sweeps, reverse=0):
    """or_async_gs: blocks run one after another (the single-block result is exact)."""
    ac = A.c()
    blk = np.ascontiguousarray(blk, dtype=np.int32)
    lib().or_async_gs(C.byref(ac), dptr(f), dptr(u), iptr(blk), C.c_int(len(blk) - 1),
                      C.c_int(sweeps), C.c_int(reverse))


def hybrid_jgs(A, f, u, u_prev, blk, diag_scale, weight, sweeps, zero_flag, reverse=0):
    ac = A.c()
    blk = np.ascontiguousarray(blk, dtype=np.int32)
    ds = dptr(diag_scale) if diag_scale is not None else None
    lib().or_hybrid_jgs(C.byref(ac), dptr(f), dptr(u), dptr(u_prev), iptr(blk),
                        C.c_int(len(blk) - 1), ds, C.c_double(weight), C.c_int(sweeps),
                        C.c_int(zero_flag), C.c_int(reverse))


def seq_sym_jacobi(A, f, u, y, r, omega, sweeps):
    ac = A.c()
    lib().or_seq_sym_jacobi(C.byref(ac), dptr(f), dptr(u), dptr(y), dptr(r), C.c_double(omega),
                            C.c_int(sweeps))


def seq_sym_l1jacobi(A, f, u, y, r, l1, sweeps):
    ac = A.c()
    lib().or_seq_sym_l1jacobi(C.byref(ac), dptr(f), dptr(u), dptr(y), dptr(r), dptr(l1),
                              C.c_int(sweeps))


def smem_sym_jacobi(A, f, u, y, r, omega, sweeps, zero_flag, ns=0, ne=None):
    ne = A.nrows if ne is None else ne
    ac = A.c()
    lib().or_smem_sym_jacobi(C.byref(ac), dptr(f), dptr(u), dptr(y), dptr(r), C.c_double(omega),
                             C.c_int(sweeps), C.c_int(zero_flag), C.c_int(ns), C.c_int(ne))


def smem_sym_l1jacobi(A, f, u, y, r, l1, sweeps, zero_flag, ns=0, ne=None):
    ne = A.nrows if ne is None else ne
    ac = A.c()
    lib().or_smem_sym_l1jacobi(C.byref(ac), dptr(f), dptr(u), dptr(y), dptr(r), dptr(l1),
                               C.c_int(sweeps), C.c_int(zero_flag), C.c_int(ns), C.c_int(ne))


def a_diag(A, omega):
    out = np.zeros(A.nrows)
    ac = A.c()
    lib().or_a_diag(C.byref(ac), C.c_double(omega), dptr(out))
    return out


def l1_norms(A):
    out = np.zeros(A.nrows)
    ac = A.c()
    lib().or_l1_norms(C.byref(ac), dptr(out))
    return out


def partition_equal(n, T):
    blk = np.zeros(T + 1, dtype=np.int32)
    lib().or_partition_equal(C.c_int(n), C.c_int(T), iptr(blk))
    return blk


def partition_nnz(A, T):
    blk = np.zeros(T + 1, dtype=np.int32)
    ac = A.c()
    lib().or_partition_nnz(C.byref(ac), C.c_int(T), iptr(blk))
    return blk


def norm2(x):
    return lib().or_norm2(dptr(x), C.c_int(len(x)))


# ---- DMEM outer acceleration (DMEM_Misc.cpp:612-666) ---------------------------
OR_NO_ACCEL, OR_RICHARD_ACCEL, OR_CHEBY_RECUR_ACCEL = 0, 1, 2
OR_CHEBY_SYNC, OR_CHEBY_GRID, OR_CHEBY_OTHER = 0, 1, 2


def dmem_cheby_update(d, u, cycle, accel, branch, mu, delta, state):
    """In place on d, u; state = [c, c_prev] (float64 array of 2)."""
    lib().or_dmem_cheby_update(dptr(d), dptr(u), len(u), cycle, accel, branch, mu, delta, dptr(state))


def dmem_async_jacobi(A, b, sweeps, omega, l1=None, accel=0, mu=0.0, delta=0.0):
    """DMEM_AsyncSmooth on one rank (DMEM_Smooth.cpp:16-313): returns (x, ||b - A x||)."""
    x = np.zeros(A.nrows)
    Ac = A.c()
    l1p = dptr(np.ascontiguousarray(l1, dtype=np.float64)) if l1 is not None else None
    rn = lib().or_dmem_async_jacobi(C.byref(Ac), dptr(np.ascontiguousarray(b, dtype=np.float64)), dptr(x),
                                    sweeps, omega, l1p, accel, mu, delta)
    return x, rn


# ---- hierarchy / solve -------------------------------------------------------
def set_async_durations(d):
    """or_set_async_durations: per-level correction times of schedule 4 (timed)"""
    d = np.ascontiguousarray(d, dtype=np.float64)
    lib().or_set_async_durations(dptr(d), int(d.size))
    lib().or_set_async_exact(0)


def set_async_times(times, exact=False):
    """or_set_async_times: times[k] = end times of level k's corrections (schedule 4 replay);
    exact: every level runs exactly len(times[k]) corrections (or_set_async_exact)"""
    n = np.array([len(t) for t in times], dtype=np.int32)
    flat = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.float64) for t in times] + [np.zeros(1)]))
    lib().or_set_async_times(dptr(flat), iptr(n), int(n.size))
    lib().or_set_async_exact(1 if exact else 0)


def make_opts(solver=OR_MULT, smoother=OR_JACOBI, num_pre=1, num_post=1, num_fine=1,
              num_coarse=1, smooth_weight=1.0, num_cycles=20, tol=0.0, check_resnorm=1,
              cheby_flag=0, cheby_mu=0.0, cheby_delta=0.0, num_threads=1):
    return OrOpts(solver, smoother, num_pre, num_post, num_fine, num_coarse, smooth_weight,
                  num_cycles, tol, check_resnorm, cheby_flag, cheby_mu, cheby_delta, num_threads)


class Hier:
    """Oracle hierarchy over host CSR levels A[0..L-1], P/R[0..L-2]."""

    def __init__(self, As, Ps, Rs, opts):
        self.L = len(As)
        self._keep = (As, Ps, Rs)
        self.Ac = (OrCsr * self.L)(*[a.c() for a in As])
        pr = Ps + [Ps[0]] if Ps else [As[0]]
        rr = Rs + [Rs[0]] if Rs else [As[0]]
        self.Pc = (OrCsr * self.L)(*[p.c() for p in pr[:self.L]])
        self.Rc = (OrCsr * self.L)(*[r.c() for r in rr[:self.L]])
        self.opts = opts
        self.h = lib().or_hier_create(self.L, self.Ac, self.Pc, self.Rc, C.byref(self.opts))

    def set_composed_transfers(self, on=True):
        """MULTADD transfers = the smoothed P~ = (I - w D^-1 A) P, R~ = P~^T
        (SmoothTransfer, SMEM_Setup.cpp:1173-1254) applied composed from the
        plain P / R (or_hier_set_composed_transfers)"""
        lib().or_hier_set_composed_transfers(self.h, 1 if on else 0)

    def set_blocks(self, level, blk):
        blk = np.ascontiguousarray(blk, dtype=np.int32)
        lib().or_hier_set_blocks(self.h, level, iptr(blk), len(blk) - 1)

    def solve(self, f, u0=None):
        n0 = self._keep[0][0].nrows
        u = np.zeros(n0) if u0 is None else np.array(u0, dtype=np.float64)
        hist = np.zeros(self.opts.num_cycles + 1)
        k = lib().or_solve(self.h, dptr(np.ascontiguousarray(f)), dptr(u), dptr(hist))
        return u, hist[:k + 1], k

    def dmem_mult_solve(self, b, accel, mu=0.0, delta=0.0, x0=None):
        """DMEM_Mult (DMEM_Mult.cpp:13-93) with DMEM_ChebyUpdate acceleration."""
        n0 = self._keep[0][0].nrows
        x = np.zeros(n0) if x0 is None else np.array(x0, dtype=np.float64)
        hist = np.zeros(self.opts.num_cycles + 1)
        k = lib().or_dmem_mult_solve(self.h, dptr(np.ascontiguousarray(b, dtype=np.float64)), dptr(x),
                                     dptr(hist), accel, mu, delta)
        return x, hist[:k + 1], k

    def dmem_add(self, b, sched=0, converge_type=0, async_type=0, max_inflight=1, save_divisor=1, tol=0.0,
                 accel=None):
        """DMEM_Add (DMEM_Add.cpp:20-944) on L threads, one rank per grid:
        (x per grid [L, n0], cycles[L], relres[L], messages[L, 2] (sent, received)).
        sched 0: the free race (nondeterministic); 1: round robin; 2 / 3 (converge LOCAL):
        finest- / coarsest-first sequential (the race's extreme speed ratios)."""
        n0 = self._keep[0][0].nrows
        x = np.zeros(self.L * n0)
        cyc = np.zeros(self.L, dtype=np.int32)
        rel = np.zeros(self.L)
        msg = np.zeros(2 * self.L, dtype=np.int64)
        acc = accel if accel is not None else (0, 0, 0.0, 0.0)
        st = lib().or_dmem_add(self.h, dptr(np.ascontiguousarray(b, dtype=np.float64)), dptr(x), int(sched),
                               int(converge_type), int(async_type), int(max_inflight), int(save_divisor),
                               float(tol), int(acc[0]), int(acc[1]), float(acc[2]), float(acc[3]), iptr(cyc),
                               dptr(rel), msg.ctypes.data_as(C.POINTER(C.c_longlong)))
        assert st == 0, st
        return x.reshape(self.L, n0), cyc, rel, msg.reshape(self.L, 2)

    def async_add(self, f, nt, async_type=0, converge_type=0, u0=None, read_type=0, res_global=False,
                  accel=None):
        """SMEM_Async_Add_AMG on sum(nt) OpenMP threads (nt[k] threads own level k):
        (u, relres, per-level correction counts).  Nondeterministic.
        res_global: res_compute_type GLOBAL (nt[0] must be 0: no level-0 group).
        accel: (accel_type, cheby level, mu, delta) -- DMEM ChebyUpdate per level."""
        n0 = self._keep[0][0].nrows
        u = np.zeros(n0) if u0 is None else np.array(u0, dtype=np.float64)
        ntv = np.ascontiguousarray(nt, dtype=np.int32)
        assert ntv.size == self.L
        assert (ntv[0] == 0 and np.all(ntv[1:] >= 1)) if res_global else np.all(ntv >= 1)
        cnt = np.zeros(self.L, dtype=np.int32)
        rel = C.c_double()
        lib().or_set_async_res_global(1 if res_global else 0)
        if accel is not None:
            lib().or_set_async_accel(int(accel[0]), int(accel[1]), float(accel[2]), float(accel[3]))
        try:
            st = lib().or_async_add(self.h, dptr(np.ascontiguousarray(f, dtype=np.float64)), dptr(u), iptr(ntv),
                                    int(async_type), int(read_type), int(converge_type), iptr(cnt), C.byref(rel))
        finally:
            lib().or_set_async_res_global(0)
            lib().or_set_async_accel(0, 0, 0.0, 0.0)
        assert st == 0, st
        return u, rel.value, cnt

    def async_add_replay(self, f, rs, times, accel=None):
        """or_async_add_replay: times[k] = (corrections, R) update times of level k's
        slices (rank r: fine rows [rs[r], rs[r+1])); (u, relres, corrections)"""
        n0 = self._keep[0][0].nrows
        R = len(rs) - 1
        u = np.zeros(n0)
        nc = np.array([np.asarray(t).reshape(-1, R).shape[0] if np.size(t) else 0 for t in times], dtype=np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.float64).reshape(-1) for t in times]
                                                   + [np.zeros(1)]))
        rsv = np.ascontiguousarray(rs, dtype=np.int32)
        cnt = np.zeros(self.L, dtype=np.int32)
        rel = C.c_double()
        if accel is not None:
            lib().or_set_async_accel(int(accel[0]), int(accel[1]), float(accel[2]), float(accel[3]))
        try:
            st = lib().or_async_add_replay(self.h, dptr(np.ascontiguousarray(f, dtype=np.float64)), dptr(u), R,
                                           iptr(rsv), dptr(flat), iptr(nc), iptr(cnt), C.byref(rel))
        finally:
            lib().or_set_async_accel(0, 0, 0.0, 0.0)
        assert st == 0, st
        return u, rel.value, cnt

    def eigs_power(self, iters):
        emax, emin = C.c_double(), C.c_double()
        lib().or_eigs_power(self.h, iters, C.byref(emax), C.byref(emin))
        return emax.value, emin.value

    def __del__(self):
        try:
            lib().or_hier_free(self.h)
        except Exception:
            pass
