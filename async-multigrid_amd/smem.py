"""Reference-named host mirror of the SEQ_* / SMEM_* hot-path kernels.

Each function keeps the reference's name and argument meaning (minus the
AllData* first argument, replaced by the device Context; scalars that the
reference reads from AllData -- smooth_weight, zero_flags[level], the thread
ranges -- become explicit arguments).  Every call runs on the MI355X through
the C-ABI; none has a CPU path.  Like the reference the kernels return
nothing; a failing status raises AmgError.
"""
import ctypes as C

import numpy as np

from . import check, lib

_ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))  # noqa: E731


# ---- SEQ_MatVec.cpp ----------------------------------------------------------
def SEQ_MatVec(ctx, A, x, y):
    """SEQ_MatVec.cpp:3-24"""
    check(lib.amg_matvec(ctx.h, A.h, x.h, y.h, 0, A.nrows))


def SEQ_MatVecT(ctx, A, x, y):
    """SEQ_MatVec.cpp:26-46"""
    check(lib.amg_matvec_t(ctx.h, A.h, x.h, y.h, 1))


def SEQ_Residual(ctx, A, b, x, y, r):
    """SEQ_MatVec.cpp:48-63"""
    check(lib.amg_residual(ctx.h, A.h, b.h, x.h, y.h, r.h, 0, A.nrows))


# ---- SMEM_MatVec.cpp ---------------------------------------------------------
def SMEM_Sync_Parfor_MatVec(ctx, A, x, y):
    """SMEM_MatVec.cpp:5-25"""
    check(lib.amg_matvec(ctx.h, A.h, x.h, y.h, 0, A.nrows))


def SMEM_Sync_Parfor_MatVecT(ctx, A, x, y, num_threads):
    """SMEM_MatVec.cpp:27-58 (expansion-buffer summation order of num_threads)"""
    check(lib.amg_matvec_t(ctx.h, A.h, x.h, y.h, num_threads))


def SMEM_Sync_Parfor_SpGEMV(ctx, A, x, b, alpha, beta, y):
    """SMEM_MatVec.cpp:70-93"""
    check(lib.amg_spgemv(ctx.h, A.h, x.h, b.h if b is not None else None, alpha, beta, y.h, 0,
                         A.nrows))


def SMEM_Sync_Parfor_Residual(ctx, A, b, x, y, r):
    """SMEM_MatVec.cpp:60-68"""
    SMEM_Sync_Parfor_SpGEMV(ctx, A, x, b, -1.0, 1.0, r)


def SMEM_SpGEMV(ctx, A, x, b, alpha, beta, y, iBegin, iEnd):
    """SMEM_MatVec.cpp:123-259"""
    check(lib.amg_spgemv(ctx.h, A.h, x.h, b.h if b is not None else None, alpha, beta, y.h,
                         iBegin, iEnd))


def SMEM_Sync_SpGEMV(ctx, A, x, b, alpha, beta, y):
    """SMEM_MatVec.cpp:106-120"""
    SMEM_SpGEMV(ctx, A, x, b, alpha, beta, y, 0, A.nrows)


def SMEM_Sync_Residual(ctx, A, b, x, y, r):
    """SMEM_MatVec.cpp:95-103"""
    SMEM_Sync_SpGEMV(ctx, A, x, b, -1.0, 1.0, r)


def SMEM_MatVec(ctx, A, x, y, ns, ne):
    """SMEM_MatVec.cpp:302-323"""
    check(lib.amg_matvec(ctx.h, A.h, x.h, y.h, ns, ne))


def SMEM_Residual(ctx, A, b, x, y, r, ns, ne):
    """SMEM_MatVec.cpp:362-378"""
    check(lib.amg_residual(ctx.h, A.h, b.h, x.h, y.h, r.h, ns, ne))


def SMEM_Sync_Parfor_Restrict(ctx, R, v_fine, v_coarse):
    """SMEM_MatVec.cpp:380-392 (construct_R_flag = 1)"""
    SMEM_Sync_Parfor_MatVec(ctx, R, v_fine, v_coarse)


# ---- SMEM_Smooth.cpp ---------------------------------------------------------
def SMEM_Sync_Parfor_Jacobi(ctx, A, f, u, u_prev, num_sweeps, zero_flag, smooth_weight):
    """SMEM_Smooth.cpp:6-49"""
    check(lib.amg_jacobi(ctx.h, A.h, f.h, u.h, u_prev.h, smooth_weight, num_sweeps, zero_flag, 0,
                         A.nrows, 0))


def SMEM_Sync_Jacobi(ctx, A, f, u, u_prev, num_sweeps, zero_flag, smooth_weight, ns, ne):
    """SMEM_Smooth.cpp:365-407"""
    check(lib.amg_jacobi(ctx.h, A.h, f.h, u.h, u_prev.h, smooth_weight, num_sweeps, zero_flag, ns,
                         ne, 0))


def SMEM_Sync_Parfor_L1Jacobi(ctx, A, f, u, u_prev, l1, num_sweeps, zero_flag):
    """SMEM_Smooth.cpp:96-133"""
    check(lib.amg_l1_jacobi(ctx.h, A.h, f.h, u.h, u_prev.h, l1.h, num_sweeps, zero_flag, 0,
                            A.nrows, 0))


def SMEM_Sync_Parfor_HybridJacobiGaussSeidel(ctx, A, f, u, u_prev, blocks, diag_scale,
                                            num_sweeps, zero_flag, reverse=0):
    """SMEM_Smooth.cpp:222-363 (blocks = thread.A_ns/A_ne, diag_scale = A_diag)"""
    blk = np.ascontiguousarray(blocks, dtype=np.int32)
    check(lib.amg_hybrid_jgs(ctx.h, A.h, f.h, u.h, u_prev.h, _ip(blk), blk.size - 1,
                             diag_scale.h if diag_scale is not None else None, 1.0, num_sweeps,
                             zero_flag, reverse))


def SMEM_Sync_HybridJacobiGaussSeidel(ctx, A, f, u, u_prev, num_sweeps, zero_flag, blocks,
                                      reverse=0):
    """SMEM_Smooth.cpp:533-641 (divisor a_ii, weight 1; blocks = the level's thread ranges)"""
    blk = np.ascontiguousarray(blocks, dtype=np.int32)
    check(lib.amg_hybrid_jgs(ctx.h, A.h, f.h, u.h, u_prev.h, _ip(blk), blk.size - 1, None, 1.0,
                             num_sweeps, zero_flag, reverse))


def SMEM_Sync_SymmetricJacobi(ctx, A, f, u, y, r, num_sweeps, zero_flag, smooth_weight, ns, ne):
    """SMEM_Smooth.cpp:643-702"""
    check(lib.amg_sym_jacobi(ctx.h, A.h, f.h, u.h, y.h, r.h, smooth_weight, None, num_sweeps,
                             zero_flag, ns, ne, 0))


def SMEM_Sync_SymmetricL1Jacobi(ctx, A, f, u, y, r, l1, num_sweeps, zero_flag, ns, ne):
    """SMEM_Smooth.cpp:704-762"""
    check(lib.amg_sym_jacobi(ctx.h, A.h, f.h, u.h, y.h, r.h, 1.0, l1.h, num_sweeps, zero_flag, ns,
                             ne, 0))


# ---- SEQ_Smooth.cpp ----------------------------------------------------------
def SEQ_Jacobi(ctx, A, f, u, u_prev, num_sweeps, zero_flag, smooth_weight):
    """SEQ_Smooth.cpp:4-46"""
    check(lib.amg_jacobi(ctx.h, A.h, f.h, u.h, u_prev.h, smooth_weight, num_sweeps, zero_flag, 0,
                         A.nrows, 1))


def SEQ_L1Jacobi(ctx, A, f, u, u_prev, l1, num_sweeps, zero_flag):
    """SEQ_Smooth.cpp:48-87"""
    check(lib.amg_l1_jacobi(ctx.h, A.h, f.h, u.h, u_prev.h, l1.h, num_sweeps, zero_flag, 0,
                            A.nrows, 1))


def SEQ_GaussSeidel(ctx, A, f, u, num_sweeps):
    """SEQ_Smooth.cpp:89-117"""
    check(lib.amg_gauss_seidel(ctx.h, A.h, f.h, u.h, num_sweeps))


def SEQ_SymmetricJacobi(ctx, A, f, u, y, r, num_sweeps, smooth_weight):
    """SEQ_Smooth.cpp:119-155"""
    check(lib.amg_sym_jacobi(ctx.h, A.h, f.h, u.h, y.h, r.h, smooth_weight, None, num_sweeps, 0, 0,
                             A.nrows, 1))


def SEQ_SymmetricL1Jacobi(ctx, A, f, u, y, r, l1, num_sweeps):
    """SEQ_Smooth.cpp:157-189"""
    check(lib.amg_sym_jacobi(ctx.h, A.h, f.h, u.h, y.h, r.h, 1.0, l1.h, num_sweeps, 0, 0, A.nrows,
                             1))


# ---- setup arrays (SMEM_Setup.cpp) ---------------------------------------------
def L1_row_norm(ctx, A, out):
    """SMEM_Setup.cpp:222-232"""
    check(lib.amg_l1_norms(ctx.h, A.h, out.h))


def A_diag(ctx, A, smooth_weight, out):
    """SMEM_Setup.cpp:234-237"""
    check(lib.amg_a_diag(ctx.h, A.h, smooth_weight, out.h))


# ---- DMEM_Misc.cpp vector ops ----------------------------------------------------
def DMEM_HypreParVector_Ivaxpy(ctx, y, x, s):
    """DMEM_Misc.cpp:462-478: y += x ./ s"""
    check(lib.amg_vec_ivaxpy(ctx.h, x.h, s.h, y.h))


def DMEM_HypreRealArray_Axpy(ctx, y, x, alpha):
    """DMEM_Misc.cpp:527-548: y += alpha x"""
    check(lib.amg_vec_axpy(ctx.h, alpha, x.h, y.h))


def SMEM_Async_Parfor_GaussSeidel(ctx, A, f, u, num_sweeps, blk=None, semi=0, reverse=0):
    """SMEM_Smooth.cpp:164-220 (semi=1: SMEM_SemiAsync_Parfor_GaussSeidel :135-162,
    reverse=1: the T form :193-220); blk = the threads' row blocks (default one)."""
    import numpy as np
    blk = np.array([0, A.nrows] if blk is None else blk, dtype=np.int32)
    check(lib.amg_async_gauss_seidel(ctx.h, A.h, f.h, u.h, _ip(blk), blk.size - 1, num_sweeps,
                                     semi, reverse))
