"""async-multigrid for AMD Instinct MI355X (gfx950): Python host binding.

Thin object layer over the C-ABI of libamg_mi355x.so (include/amg_mi355x.h).
All compute runs in the HIP library; this module only moves handles, host
arrays and status codes.  There is no CPU fallback: importing the package
without the built library raises ImportError, and every failed call raises
AmgError with the library's message.

Load it with ``_load_package()`` helpers (the directory name contains a dash):
    import importlib.util, sys
    spec = importlib.util.spec_from_file_location(
        "async_multigrid_amd", "async-multigrid_amd/__init__.py",
        submodule_search_locations=["async-multigrid_amd"])
"""
import ctypes as C

import numpy as np

from . import abi
from .abi import AmgError, AmgOpts  # noqa: F401
from .abi import (AMG_JACOBI, AMG_GAUSS_SEIDEL, AMG_HYBRID_JGS, AMG_SYMM_JACOBI,  # noqa: F401
                  AMG_L1_JACOBI, AMG_L1_HYBRID_JGS, AMG_MULT, AMG_AFACX, AMG_MULTADD,
                  AMG_ASYNC_AFACX, AMG_ASYNC_MULTADD, AMG_INTERP_LINEAR, AMG_INTERP_AGGREGATE,
                  AMG_GEN_A, AMG_GEN_P, AMG_GEN_R, AMG_VEC_F, AMG_VEC_U, AMG_VEC_R,
                  AMG_ASYNC_GS, AMG_SEMI_ASYNC_GS, AMG_BPX, AMG_NO_ACCEL, AMG_RICHARD_ACCEL,
                  AMG_CHEBY_RECUR_ACCEL, AMG_FULL_ASYNC, AMG_SEMI_ASYNC, AMG_LOCAL, AMG_GLOBAL,
                  AMG_READ_SOL, AMG_READ_RES, AMG_DELAY_NONE, AMG_DELAY_ONE, AMG_DELAY_SOME,
                  AMG_DELAY_ALL, AMG_FAIL_ONE, AMG_SPS_EXPONENTIAL, AMG_SPS_INVERSE, AMG_SPS_RANDOM,
                  AMG_SCHED_FREE, AMG_SCHED_FINEST_FIRST, AMG_SCHED_COARSEST_FIRST, AMG_SCHED_ROUND_ROBIN,
                  AMG_SCHED_TIMED)

lib = abi.load()


def check(status):
    if status != 0:
        msg = lib.amg_last_error()
        raise AmgError(f"status {status}: {msg.decode() if msg else ''}")
    return status


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def default_opts(**kw):
    o = AmgOpts()
    lib.amg_opts_default(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(k)
        setattr(o, k, v)
    return o



def _times_flat(times):
    n = np.array([len(t) for t in times], dtype=np.int32)
    flat = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.float64) for t in times] + [np.zeros(1)]))
    return flat, n


def _corr_ms(fn, h, L, start=False):
    """per level: the end (start=False) or start times of its update windows"""
    out = []
    for k in range(L):
        cnt = np.zeros(1, dtype=np.int32)
        check(fn(h, k, None, -1 if start else 0, _ip(cnt)))
        ms = np.zeros(max(1, int(cnt[0])))
        check(fn(h, k, _dp(ms), -max(1, int(cnt[0])) if start else int(cnt[0]), _ip(cnt)))
        out.append(ms[:int(cnt[0])])
    return out

def _update_rows(fn, h, counts, n, vals=False):
    """per level: (corrections, n) per-row update times (ms) of its first recorded
    corrections in the last free race (rows stamped by the update kernels), or None
    for a level whose corrections were not all row-stamped; vals: (corrections, n, 2)
    -- every row's (old, new) value of each add"""
    out = []
    w = 2 * n if vals else n
    buf = np.zeros(max(1, w))
    cnt = np.zeros(1, dtype=np.int32)
    for k, m in enumerate(counts):
        rows = []
        for j in range(int(m)):
            check(fn(h, k, j, _dp(buf), -w if vals else w, _ip(cnt)))
            if int(cnt[0]) != w:
                break
            rows.append(buf[:w].copy())
        shape = (len(rows), n, 2) if vals else (len(rows), n)
        out.append(np.array(rows).reshape(shape) if len(rows) == int(m) else None)
    return out


class Context:
    """Device, compute stream and level streams (amg_init)."""

    def __init__(self, device=0, nstreams=16):
        h = C.c_void_p()
        check(lib.amg_init(C.byref(h), device, nstreams))
        self.h = h
        self.device = device

    def sync(self):
        check(lib.amg_sync(self.h))

    def device_errors(self):
        """Device-side range-check flags raised since the last call (bit 0: a
        zero-guess fold write outside the coarse level's rows, dropped)."""
        v = C.c_int(0)
        check(lib.amg_device_errors(self.h, C.byref(v)))
        return v.value

    def set_value_index(self, enable):
        """Value-indexed CSR for matrices registered from now on (default on)."""
        check(lib.amg_set_value_index(self.h, int(enable)))

    def set_dict_index(self, enable):
        """Dictionary-coded CSR for square operators registered from now on (default on)."""
        check(lib.amg_set_dict_index(self.h, int(enable)))

    def set_row_pattern(self, enable):
        """Row-pattern-coded CSR on top of the dictionary (default on)."""
        check(lib.amg_set_row_pattern(self.h, int(enable)))

    def set_pair_pattern(self, enable):
        """Paired-row-pattern CSR on top of the row patterns (default on)."""
        check(lib.amg_set_pair_pattern(self.h, int(enable)))

    def set_pair_anchor16(self, enable):
        """Slab-compressed anchors of pair-coded P/R registered from now on (default off)."""
        check(lib.amg_set_pair_anchor16(self.h, int(enable)))

    def set_master_pattern(self, enable):
        """Master-pattern form of square pair-coded operators (default on)."""
        check(lib.amg_set_master_pattern(self.h, int(enable)))

    def set_plane_march(self, enable, zc=0, xcd=-1):
        """Plane-marching kernel for 7-pt box-grid masters (default on); zc planes
        per chunk (0 keeps), xcd workgroup order (-1 keeps)."""
        check(lib.amg_set_plane_march(self.h, int(enable), int(zc), int(xcd)))

    def set_fuse_transfer(self, enable):
        """Fused level-0 residual + restriction on geometric hierarchies (default on)."""
        check(lib.amg_set_fuse_transfer(self.h, int(enable)))

    def set_bsr3(self, enable):
        """3x3 block form of num_functions = 3 operators for matrices registered from now on (default on)."""
        check(lib.amg_set_bsr3(self.h, int(enable)))

    def set_jgs_small(self, form):
        """Small-level hybrid JGS form (bit-identical): 2 one batch per row (default), 1 wave per block, 0 as large."""
        check(lib.amg_set_jgs_small(self.h, int(form)))

    def set_jgs_fold(self, enable):
        """FULL_ASYNC: level 0's correction folded into the last hybrid-JGS sweep (bit-identical; off)."""
        check(lib.amg_set_jgs_fold(self.h, int(enable)))

    def set_jgs_wave(self, enable):
        """Hybrid JGS kernel form, all bit-identical: 1 (default) 8 lanes per block,
        8 blocks per wave; 2 one wave per block; 0 one lane per block; 3 an LDS tile of 64
        blocks (rows staged coalesced, the chains walked one lane per block)."""
        check(lib.amg_set_jgs_wave(self.h, int(enable)))

    def set_fuse_prolong(self, enable):
        """Prolongation fused into the first post-smoothing sweep of marched geometric levels (default off: VALU-bound, slower)."""
        check(lib.amg_set_fuse_prolong(self.h, int(enable)))

    def set_fuse_outer(self, mode):
        """level 0's last post sweep + the outer residual as one march (0 off, 1 on, 2 on with u'
        stored only at the end of an iterate batch, 3 the two sweeps slab by slab over z through the
        Infinity Cache, u' stored as in 2; bit-identical)"""
        check(lib.amg_set_fuse_outer(self.h, int(mode)))

    def set_outer_slab(self, planes):
        """planes per z-slab of fuse_outer mode 3"""
        check(lib.amg_set_outer_slab(self.h, int(planes)))

    def set_long_form(self, form, xcd=1):
        """long-row CSR kernel: 0 workgroup chunks, 1 / 2 wave-independent chunks of 8 / 16
        entries per lane, xcd: XCD-contiguous row blocks (bit-identical)"""
        check(lib.amg_set_long_form(self.h, int(form), int(xcd)))

    def set_graphs(self, enable):
        """hipGraphs of the additive cycles' launch-bound loops (bit-identical)."""
        check(lib.amg_set_graphs(self.h, int(bool(enable))))

    def set_march_tuning(self, mz_pf=None, mz27_pf=None, mz_occ=None, mz27_occ=None):
        """Plane-march scheduling (bit-identical): prefetch distance (1 / 2) of the
        7-pt / 27-pt march, occupancy-sized chunks (-1 the kernel's own, 0 off,
        > 0 workgroups per CU); None keeps a value."""
        k = lambda v: -2 if v is None else int(v)  # noqa: E731
        check(lib.amg_set_march_tuning(self.h, k(mz_pf), k(mz27_pf), k(mz_occ), k(mz27_occ)))

    def set_march_lines(self, lines, gemv=None):
        """Lines per lane of the 7-pt plane march (1, 2 or 4; bit-identical);
        gemv: a different count for SpMV / SpGEMV (default: the same)."""
        check(lib.amg_set_march_lines(self.h, int(lines)))
        if gemv is not None:
            check(lib.amg_set_march_lines_gemv(self.h, int(gemv)))

    def csr(self, nrows, ncols, rowptr, col, val, diag_first=1):
        return Mat.register(self, nrows, ncols, rowptr, col, val, diag_first)

    def vec(self, n_or_array):
        if isinstance(n_or_array, (int, np.integer)):
            return Vec(self, int(n_or_array))
        a = np.ascontiguousarray(n_or_array, dtype=np.float64)
        v = Vec(self, a.size)
        v.upload(a)
        return v

    def close(self):
        if self.h:
            lib.amg_finalize(self.h)
            self.h = None


class Mat:
    """Device CSR registered once (amg_csr_register)."""

    def __init__(self, ctx, handle):
        self.ctx, self.h = ctx, handle
        nr, nc, nz = C.c_int(), C.c_int(), C.c_longlong()
        check(lib.amg_mat_info(handle, C.byref(nr), C.byref(nc), C.byref(nz)))
        self.nrows, self.ncols, self.nnz = nr.value, nc.value, nz.value
        self.value_index = lib.amg_mat_value_index(handle)  # table size, 0 = plain CSR
        self.dict_index = lib.amg_mat_dict_index(handle)    # dictionary size, 0 = not coded
        self.row_pattern = lib.amg_mat_row_pattern(handle)  # distinct row patterns, 0 = not coded
        self.pair_pattern = lib.amg_mat_pair_pattern(handle)  # distinct row-pair patterns, 0 = not coded
        self.pair_anchor16 = lib.amg_mat_pair_anchor16(handle)  # slab-compressed anchors
        self.master_pattern = lib.amg_mat_master_pattern(handle)  # master length J (-J: uniform values), 0 = not coded
        self.plane_march = lib.amg_mat_plane_march(handle)  # plane size P of the marching kernel, 0 = not marched
        self.march_points = lib.amg_mat_march_points(handle)  # 7 / 27-point marching kernel, 0 = not marched
        self.bsr3 = lib.amg_mat_bsr3(handle)  # 3x3 blocks: 1 value-indexed, 2 fp64, 0 not blocked

    @classmethod
    def register(cls, ctx, nrows, ncols, rowptr, col, val, diag_first=1):
        rp = np.ascontiguousarray(rowptr, dtype=np.int32)
        cj = np.ascontiguousarray(col, dtype=np.int32)
        cv = np.ascontiguousarray(val, dtype=np.float64)
        h = C.c_void_p()
        check(lib.amg_csr_register(ctx.h, int(nrows), int(ncols), int(rp[-1]), _ip(rp), _ip(cj),
                                   _dp(cv), diag_first, C.byref(h)))
        return cls(ctx, h)

    def download(self):
        rp = np.empty(self.nrows + 1, dtype=np.int32)
        cj = np.empty(max(self.nnz, 1), dtype=np.int32)
        cv = np.empty(max(self.nnz, 1), dtype=np.float64)
        check(lib.amg_mat_download(self.ctx.h, self.h, _ip(rp), _ip(cj), _dp(cv)))
        return rp, cj[:self.nnz], cv[:self.nnz]

    def free(self):
        if self.h:
            lib.amg_mat_free(self.h)
            self.h = None


class Vec:
    """Device fp64 vector (amg_vec_create)."""

    def __init__(self, ctx, n, handle=None, owns=True):
        self.ctx, self.n = ctx, n
        if handle is None:
            h = C.c_void_p()
            check(lib.amg_vec_create(ctx.h, n, C.byref(h)))
            handle = h
        self.h = handle
        self._owns = owns

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        assert a.size == self.n
        check(lib.amg_vec_upload(self.ctx.h, self.h, _dp(a)))
        return self

    def download(self):
        out = np.empty(self.n, dtype=np.float64)
        check(lib.amg_vec_download(self.ctx.h, self.h, _dp(out)))
        return out

    def set(self, a):
        check(lib.amg_vec_set(self.ctx.h, self.h, float(a)))

    def norm2(self):
        r = C.c_double()
        check(lib.amg_vec_norm2(self.ctx.h, self.h, C.byref(r)))
        return r.value

    def free(self):
        if self.h and self._owns:
            lib.amg_vec_free(self.h)
        self.h = None


class Hier:
    """Level hierarchy + SMEM_Solve driver state (amg_hier_create)."""

    def __init__(self, ctx, As, Ps, Rs, opts):
        L = len(As)
        self.ctx, self.L, self.opts = ctx, L, opts
        self._keep = (As, Ps, Rs)
        arrA = (C.c_void_p * L)(*[a.h for a in As])
        arrP = (C.c_void_p * max(L, 1))(*([p.h for p in Ps] + [None] * (max(L, 1) - len(Ps))))
        arrR = (C.c_void_p * max(L, 1))(*([r.h for r in Rs] + [None] * (max(L, 1) - len(Rs))))
        h = C.c_void_p()
        check(lib.amg_hier_create(ctx.h, L, arrA, arrP, arrR, C.byref(opts), C.byref(h)))
        self.h = h
        self.n0 = As[0].nrows
        self.fused = lib.amg_hier_fused(h)  # bit 0: level-0 residual + restriction fused; bit l+1: level l geometric transfers
        self.fused_prolong = lib.amg_hier_fused_prolong(h)  # bit l: level l's prolongation fused into its post sweep
        self.fused_outer = lib.amg_hier_fused_outer(h)  # level 0's last post sweep fused with the outer residual

    def set_opts(self, opts):
        check(lib.amg_hier_set_opts(self.h, C.byref(opts)))
        self.opts = opts

    def set_blocks(self, level, blk):
        blk = np.ascontiguousarray(blk, dtype=np.int32)
        check(lib.amg_hier_set_blocks(self.h, level, _ip(blk), blk.size - 1))

    def vec(self, which, level):
        h = C.c_void_p()
        check(lib.amg_hier_vec(self.h, which, level, C.byref(h)))
        n = lib.amg_vec_size(h)
        return Vec(self.ctx, n, h)

    def solve(self, f, u0=None):
        """SMEM_Solve: returns (u, residual-norm history, cycles)."""
        fv = f if isinstance(f, Vec) else self.ctx.vec(f)
        uv = self.ctx.vec(np.zeros(self.n0) if u0 is None else u0)
        hist = np.zeros(self.opts.num_cycles + 1)
        k = C.c_int()
        check(lib.amg_solve(self.h, fv.h, uv.h, _dp(hist), C.byref(k)))
        u = uv.download()
        return u, hist[:k.value + 1], k.value

    def solve_start(self, f, u0):
        r0 = C.c_double()
        check(lib.amg_solve_start(self.h, f.h, u0.h, C.byref(r0)))
        return r0.value

    def iterate(self, k):
        check(lib.amg_solve_iterate(self.h, k))

    def resnorm(self):
        r = C.c_double()
        check(lib.amg_solve_resnorm(self.h, C.byref(r)))
        return r.value

    def get_u(self, out):
        check(lib.amg_solve_get_u(self.h, out.h))

    def vcycle(self):
        check(lib.amg_vcycle(self.h))

    def async_solve(self, f, u0=None):
        fv = f if isinstance(f, Vec) else self.ctx.vec(f)
        uv = self.ctx.vec(np.zeros(self.n0) if u0 is None else u0)
        cnt = np.zeros(self.L, dtype=np.int32)
        rel = C.c_double()
        check(lib.amg_async_solve(self.h, fv.h, uv.h, _ip(cnt), C.byref(rel)))
        return uv.download(), rel.value, cnt

    def async_level_ms(self):
        """per level: ms from the last async_solve's start to the level's last correction (free race)"""
        ms = np.zeros(self.L, dtype=np.float64)
        check(lib.amg_async_level_ms(self.h, _dp(ms)))
        return ms

    def set_async_durations(self, ms):
        """AMG_SCHED_TIMED: level k's time per correction"""
        d = np.ascontiguousarray(ms, dtype=np.float64)
        check(lib.amg_hier_set_async_durations(self.h, _dp(d), int(d.size)))

    def set_async_times(self, times):
        """AMG_SCHED_TIMED replaying recorded end times: times[k] = level k's correction end times"""
        flat, n = _times_flat(times)
        check(lib.amg_hier_set_async_times(self.h, _dp(flat), _ip(n), int(n.size)))

    def async_correction_ms(self, start=False):
        """per level: end times (ms) of its corrections' update windows in the last free-race
        async_solve (start=True: the windows' start times, where recorded)"""
        return _corr_ms(lib.amg_async_correction_ms, self.h, self.L, start)

    def async_update_windows(self):
        """per level: (starts, ends) in ms of the device wall clock of its corrections' update
        kernels in the last free-race async_solve (their actual execution windows)"""
        return (_corr_ms(lib.amg_async_update_windows, self.h, self.L, True),
                _corr_ms(lib.amg_async_update_windows, self.h, self.L, False))

    def async_update_rows(self):
        """per level: (corrections, n0) per-row update times (ms, the windows' clock) of
        the last free race, or None where not recorded (amg_async_update_rows)"""
        counts = [len(w) for w in self.async_update_windows()[1]]
        return _update_rows(lib.amg_async_update_rows, self.h, counts, self.n0)

    def async_update_vals(self):
        """per level: (corrections, n0, 2) -- every row's (old, new) value of each add in
        the last free race (NaN: not recorded), or None (amg_async_update_rows, cap < 0)"""
        counts = [len(w) for w in self.async_update_windows()[1]]
        return _update_rows(lib.amg_async_update_rows, self.h, counts, self.n0, vals=True)

    def eigs_power(self, iters):
        emax, emin = C.c_double(), C.c_double()
        check(lib.amg_eigs_power(self.h, iters, C.byref(emax), C.byref(emin)))
        return emax.value, emin.value

    def profile(self, reset=True):
        ms = np.zeros(5)
        n = np.zeros(5, dtype=np.int64)
        check(lib.amg_hier_profile_read(self.h, _dp(ms),
                                        n.ctypes.data_as(C.POINTER(C.c_longlong)), int(reset)))
        return ms, n

    def free(self):
        if self.h:
            lib.amg_hier_free(self.h)
            self.h = None


class Gen:
    """Structured 7-pt problem + geometric Galerkin hierarchy (amg_gen_create)."""

    def __init__(self, nx, ny=None, nz=None, interp=AMG_INTERP_LINEAR, max_levels=25, max_coarse=9):
        ny = nx if ny is None else ny
        nz = nx if nz is None else nz
        h = C.c_void_p()
        check(lib.amg_gen_create(nx, ny, nz, interp, max_levels, max_coarse, C.byref(h)))
        self.h = h
        self.L = lib.amg_gen_num_levels(h)

    def dims(self, level):
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        check(lib.amg_gen_dims(self.h, level, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def rows(self, which, level):
        d = self.dims(level + 1 if which == AMG_GEN_R else level)
        return d[0] * d[1] * d[2]

    def host_csr(self, which, level, z0=0, z1=None, nthreads=0):
        """(nrows, ncols, rowptr, col, val) of operator rows in planes [z0,z1)."""
        d = self.dims(level + 1 if which == AMG_GEN_R else level)
        z1 = d[2] if z1 is None else z1
        nnz = lib.amg_gen_nnz(self.h, which, level, z0, z1)
        if nnz < 0:
            raise AmgError(lib.amg_last_error().decode())
        nrows = d[0] * d[1] * (z1 - z0)
        rp = np.empty(nrows + 1, dtype=np.int32)
        cj = np.empty(max(nnz, 1), dtype=np.int32)
        cv = np.empty(max(nnz, 1), dtype=np.float64)
        check(lib.amg_gen_fill(self.h, which, level, z0, z1, _ip(rp), _ip(cj), _dp(cv), nthreads))
        cd = self.dims(level) if which == AMG_GEN_R else (
            self.dims(level + 1) if which == AMG_GEN_P else self.dims(level))
        return nrows, cd[0] * cd[1] * cd[2], rp, cj[:nnz], cv[:nnz]

    def register(self, ctx, which, level, z0=0, z1=None):
        d = self.dims(level + 1 if which == AMG_GEN_R else level)
        z1 = d[2] if z1 is None else z1
        h = C.c_void_p()
        check(lib.amg_gen_register(ctx.h, self.h, which, level, z0, z1, C.byref(h)))
        return Mat(ctx, h)

    def free(self):
        if self.h:
            lib.amg_gen_free(self.h)
            self.h = None


def rhs_rand(r0, r1, lo=-1.0, hi=1.0):
    out = np.empty(r1 - r0, dtype=np.float64)
    check(lib.amg_rhs_rand(r0, r1, lo, hi, _dp(out)))
    return out


def rand_double_stream(seed, n, lo=0.0, hi=1.0):
    """n RandDouble(lo, hi) draws after srand(seed) (glibc rand(), Misc.cpp:282-285)."""
    out = np.empty(n, dtype=np.float64)
    check(lib.amg_rand_double_stream(int(seed), int(n), float(lo), float(hi), _dp(out)))
    return out


def build_hierarchy(ctx, gen, opts, levels=None):
    """Register every level operator of a generator on the device and build a Hier."""
    L = gen.L if levels is None else levels
    As = [gen.register(ctx, AMG_GEN_A, l) for l in range(L)]
    Ps = [gen.register(ctx, AMG_GEN_P, l) for l in range(L - 1)]
    Rs = [gen.register(ctx, AMG_GEN_R, l) for l in range(L - 1)]
    return Hier(ctx, As, Ps, Rs, opts)


from . import smem  # noqa: E402,F401  (reference-named kernel mirror)
from . import dist  # noqa: E402,F401  (multi-GPU solve phase)
from . import classical  # noqa: E402,F401  (in-house BoomerAMG-style setup)
from . import io  # noqa: E402,F401  (binary triplet matrix files)
from . import grid  # noqa: E402,F401  (level-grouped async additive solve)
