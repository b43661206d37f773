/*
 * amg_oracle.c -- TEST INFRASTRUCTURE ONLY (see amg_oracle.h header comment).
 *
 * CPU restatement of the jwp3/async-multigrid solve-phase hot path.  Each
 * function names the reference file:line it restates (paths relative to
 * /root/reference/src).  Loop bodies keep the reference's floating-point
 * expression order so results are bit-comparable; OpenMP is used only on
 * row-independent loops (the reference's `omp for` loops), which does not
 * change any per-row result.
 *
 * PARITY UNPINNED: the reference ships no fixtures or tests for this path
 * and cannot be built here without stand-in headers, so this restatement is
 * checked against the cited reference loops, not against reference outputs
 * (DESIGN.md Sec.2).
 */
#include "amg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#include <sched.h>
#endif

#define OMP_MIN_ROWS 32768

/* OpenMP threads of the parallel loops (omp_set_num_threads; the CPU
 * baseline's SEQ leg runs the same loops on one thread) */
void or_set_threads(int t)
{
#ifdef _OPENMP
   if (t > 0) omp_set_num_threads(t);
#else
   (void)t;
#endif
}

int or_num_threads(void)
{
#ifdef _OPENMP
   return omp_get_max_threads();
#else
   return 1;
#endif
}

/* ------------------------------------------------------------------------- */
/* RNG: Misc.cpp:282-285 RandDouble; RHS SMEM_Setup.cpp:1729-1745            */
/* ------------------------------------------------------------------------- */
void or_srand(unsigned seed) { srand(seed); }

double or_rand_double(double low, double high)
{
   return low + (high - low) * ((double)rand() / RAND_MAX);
}

void or_rhs_rand(int n, double low, double high, double *f)
{
   srand(0);
   for (int i = 0; i < n; i++) f[i] = or_rand_double(low, high);
}

/* ------------------------------------------------------------------------- */
/* SpMV family                                                                */
/* ------------------------------------------------------------------------- */

/* SEQ_MatVec.cpp:3-24 (and SMEM_Sync_Parfor_MatVec SMEM_MatVec.cpp:5-25) */
void or_seq_matvec(const or_csr *A, const double *x, double *y)
{
   or_smem_matvec(A, x, y, 0, A->nrows);
}

/* SEQ_MatVec.cpp:26-46 */
void or_seq_matvec_t(const or_csr *A, const double *x, double *y)
{
   for (int i = 0; i < A->ncols; i++) y[i] = 0;
   for (int i = 0; i < A->nrows; i++) {
      for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) {
         int j = A->j[jj];
         y[j] += A->data[jj] * x[i];
      }
   }
}

/* SEQ_MatVec.cpp:48-63 */
void or_seq_residual(const or_csr *A, const double *b, const double *x, double *y, double *r)
{
   or_seq_matvec(A, x, y);
   for (int i = 0; i < A->nrows; i++) r[i] = b[i] - y[i];
}

/* SMEM_MatVec.cpp:302-323 */
void or_smem_matvec(const or_csr *A, const double *x, double *y, int ns, int ne)
{
   const int *A_i = A->i, *A_j = A->j;
   const double *A_data = A->data;
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
   for (int i = ns; i < ne; i++) {
      double Axi = 0.0;
      for (int jj = A_i[i]; jj < A_i[i + 1]; jj++) Axi += A_data[jj] * x[A_j[jj]];
      y[i] = Axi;
   }
}

/* SMEM_MatVec.cpp:27-58: per-thread expansion buffer, libgomp static chunks */
void or_smem_matvec_t_expand(const or_csr *A, const double *x, double *y, int T)
{
   int n = A->nrows, nc = A->ncols;
   double *y_expand = (double *)calloc((size_t)nc * (size_t)T, sizeof(double));
   int q = n / T, rem = n % T;
   for (int t = 0; t < T; t++) {
      int s = t < rem ? t * (q + 1) : t * q + rem;
      int e = s + (t < rem ? q + 1 : q);
      double *ye = y_expand + (size_t)nc * t;
      for (int i = s; i < e; i++)
         for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) ye[A->j[jj]] += A->data[jj] * x[i];
   }
   for (int i = 0; i < nc; i++) {
      y[i] = 0;
      for (int t = 0; t < T; t++) y[i] += y_expand[(size_t)t * nc + i];
   }
   free(y_expand);
}

/* SMEM_MatVec.cpp:123-259 SMEM_SpGEMV: y = alpha*A*x + beta*b, specialised on
 * temp = beta/alpha in {0,-1,1,other} x alpha in {1,-1,other}.  Each branch's
 * initial value and accumulate sign are restated verbatim. */
void or_smem_spgemv(const or_csr *A, const double *x, const double *b, double alpha, double beta,
                    double *y, int ib, int ie)
{
   const int *A_i = A->i, *A_j = A->j;
   const double *A_data = A->data;
   double temp = beta / alpha;
   int tcase = (temp == 0) ? 0 : (temp == -1) ? 1 : (temp == 1) ? 2 : 3;
   int acase = (alpha == 1) ? 0 : (alpha == -1) ? 1 : 2;
#pragma omp parallel for schedule(static) if (ie - ib > OMP_MIN_ROWS)
   for (int i = ib; i < ie; i++) {
      double tempx;
      switch (tcase) {
      case 0: tempx = 0.0; break;
      case 1: tempx = (acase == 1) ? b[i] : -b[i]; break;
      case 2: tempx = (acase == 1) ? -b[i] : b[i]; break;
      default: tempx = (acase == 1) ? -b[i] * temp : b[i] * temp; break;
      }
      if (acase == 1) {
         for (int jj = A_i[i]; jj < A_i[i + 1]; jj++) tempx -= A_data[jj] * x[A_j[jj]];
      } else {
         for (int jj = A_i[i]; jj < A_i[i + 1]; jj++) tempx += A_data[jj] * x[A_j[jj]];
      }
      y[i] = (acase == 2) ? alpha * tempx : tempx;
   }
}

/* SMEM_MatVec.cpp:362-378 SMEM_Residual: two passes, y = A x then r = b - y */
void or_smem_residual(const or_csr *A, const double *b, const double *x, double *y, double *r,
                      int ns, int ne)
{
   or_smem_matvec(A, x, y, ns, ne);
   for (int i = ns; i < ne; i++) {
      double ri = b[i] - y[i];
      r[i] = ri;
   }
}

/* ------------------------------------------------------------------------- */
/* Smoothers                                                                  */
/* ------------------------------------------------------------------------- */

/* SMEM_Smooth.cpp:6-49 (Parfor, ns=0 ne=n) and :365-407 (row range) */
void or_smem_jacobi(const or_csr *A, const double *f, double *u, double *u_prev, double omega,
                    int sweeps, int zero_flag, int ns, int ne)
{
   const int *A_i = A->i, *A_j = A->j;
   const double *A_data = A->data;
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zero_flag == 1) {
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
         for (int i = ns; i < ne; i++)
            if (A_data[A_i[i]] != 0.0) u[i] = omega * f[i] / A_data[A_i[i]];
      } else {
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
         for (int i = ns; i < ne; i++) u_prev[i] = u[i];
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
         for (int i = ns; i < ne; i++) {
            if (A_data[A_i[i]] != 0.0) {
               double res = f[i];
               for (int jj = A_i[i]; jj < A_i[i + 1]; jj++) res -= A_data[jj] * u_prev[A_j[jj]];
               u[i] += omega * res / A_data[A_i[i]];
            }
         }
      }
   }
}

/* SMEM_Smooth.cpp:96-133 (Parfor) and :409-443 (row range) */
void or_smem_l1jacobi(const or_csr *A, const double *f, double *u, double *u_prev, const double *l1,
                      int sweeps, int zero_flag, int ns, int ne)
{
   const int *A_i = A->i, *A_j = A->j;
   const double *A_data = A->data;
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zero_flag == 1) {
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
         for (int i = ns; i < ne; i++) u[i] = f[i] / l1[i];
      } else {
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
         for (int i = ns; i < ne; i++) u_prev[i] = u[i];
#pragma omp parallel for schedule(static) if (ne - ns > OMP_MIN_ROWS)
         for (int i = ns; i < ne; i++) {
            double res = f[i];
            for (int jj = A_i[i]; jj < A_i[i + 1]; jj++) res -= A_data[jj] * u_prev[A_j[jj]];
            u[i] += res / l1[i];
         }
      }
   }
}

/* SEQ_Smooth.cpp:4-46: the zero-guess sweep ADDS omega*f/a_ii */
void or_seq_jacobi(const or_csr *A, const double *f, double *u, double *u_prev, double omega,
                   int sweeps, int zero_flag)
{
   int n = A->nrows;
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zero_flag == 1) {
         for (int i = 0; i < n; i++)
            if (A->data[A->i[i]] != 0.0) {
               double res = f[i];
               u[i] += omega * res / A->data[A->i[i]];
            }
      } else {
         for (int i = 0; i < n; i++) u_prev[i] = u[i];
         for (int i = 0; i < n; i++) {
            if (A->data[A->i[i]] != 0.0) {
               double res = f[i];
               for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) res -= A->data[jj] * u_prev[A->j[jj]];
               u[i] += omega * res / A->data[A->i[i]];
            }
         }
      }
   }
}

/* SEQ_Smooth.cpp:48-87 */
void or_seq_l1jacobi(const or_csr *A, const double *f, double *u, double *u_prev, const double *l1,
                     int sweeps, int zero_flag)
{
   int n = A->nrows;
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zero_flag == 1) {
         for (int i = 0; i < n; i++)
            if (A->data[A->i[i]] != 0.0) {
               double res = f[i];
               u[i] += res / l1[i];
            }
      } else {
         for (int i = 0; i < n; i++) u_prev[i] = u[i];
         for (int i = 0; i < n; i++) {
            double res = f[i];
            for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) res -= A->data[jj] * u_prev[A->j[jj]];
            u[i] += res / l1[i];
         }
      }
   }
}

/* SEQ_Smooth.cpp:89-117 */
void or_seq_gauss_seidel(const or_csr *A, const double *f, double *u, int sweeps)
{
   for (int k = 0; k < sweeps; k++)
      for (int i = 0; i < A->nrows; i++)
         if (A->data[A->i[i]] != 0.0) {
            double res = f[i];
            for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) res -= A->data[jj] * u[A->j[jj]];
            u[i] += res / A->data[A->i[i]];
         }
}

/* Asynchronous / semi-asynchronous Gauss-Seidel over blocks blk[0..nblk]
 * (SMEM_Async_Parfor_GaussSeidel[T] SMEM_Smooth.cpp:164-220, SMEM_Async_GaussSeidel[T]
 * :475-531, SMEM_SemiAsync_* :135-162 / :445-473): each thread sweeps its block
 * in place reading the live u of every row.  The restatement runs the blocks
 * one after another -- one admissible interleaving of the racy reference, and
 * THE result for a single block.  No zero-guess case, no weight. */
static int g_async_gs_threads = 0;
void or_set_async_gs_threads(int mode) { g_async_gs_threads = mode; }

/* the same on one OpenMP thread per block, every u access a relaxed atomic:
 * the reference's race itself (or_set_async_gs_threads(1)), so repeated
 * solves give its spread of results */
static inline double ld_relaxed(const double *p)
{
   double v;
   __atomic_load(p, &v, __ATOMIC_RELAXED);
   return v;
}
static inline void st_relaxed(double *p, double v) { __atomic_store(p, &v, __ATOMIC_RELAXED); }

static void async_gs_threaded(const or_csr *A, const double *f, double *u, const int *blk, int nblk, int sweeps,
                              int reverse)
{
#pragma omp parallel num_threads(nblk)
   {
      const int b = omp_get_thread_num();
      for (int k = 0; k < sweeps; k++)
         for (int c = 0; c < blk[b + 1] - blk[b]; c++) {
            const int i = reverse ? blk[b + 1] - 1 - c : blk[b] + c;
            if (A->data[A->i[i]] == 0.0) continue;
            double res = f[i];
            for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) res -= A->data[jj] * ld_relaxed(&u[A->j[jj]]);
            st_relaxed(&u[i], ld_relaxed(&u[i]) + res / A->data[A->i[i]]);
         }
   }
}

/* the equal-speed interleaving (or_set_async_gs_threads(2)): every block at
 * the same row step c, all reading u before any stores of step c -- the
 * schedule of threads running in lockstep, which an 8-core host cannot
 * produce with 32 OS threads; also one admissible interleaving of the race */
static void async_gs_lockstep(const or_csr *A, const double *f, double *u, const int *blk, int nblk, int sweeps,
                              int reverse)
{
   int lmax = 0;
   for (int b = 0; b < nblk; b++) lmax = blk[b + 1] - blk[b] > lmax ? blk[b + 1] - blk[b] : lmax;
   double *nv = (double *)malloc(sizeof(double) * (size_t)(nblk > 0 ? nblk : 1));
   for (int k = 0; k < sweeps; k++)
      for (int c = 0; c < lmax; c++) {
         for (int b = 0; b < nblk; b++) {
            if (c >= blk[b + 1] - blk[b]) continue;
            const int i = reverse ? blk[b + 1] - 1 - c : blk[b] + c;
            if (A->data[A->i[i]] == 0.0) continue;
            double res = f[i];
            for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) res -= A->data[jj] * u[A->j[jj]];
            nv[b] = u[i] + res / A->data[A->i[i]];
         }
         for (int b = 0; b < nblk; b++) {
            if (c >= blk[b + 1] - blk[b]) continue;
            const int i = reverse ? blk[b + 1] - 1 - c : blk[b] + c;
            if (A->data[A->i[i]] != 0.0) u[i] = nv[b];
         }
      }
   free(nv);
}

void or_async_gs(const or_csr *A, const double *f, double *u, const int *blk, int nblk, int sweeps,
                 int reverse)
{
   if (g_async_gs_threads == 2 && nblk > 1) {
      async_gs_lockstep(A, f, u, blk, nblk, sweeps, reverse);
      return;
   }
   if (g_async_gs_threads && nblk > 1) {
      async_gs_threaded(A, f, u, blk, nblk, sweeps, reverse);
      return;
   }
   for (int k = 0; k < sweeps; k++)
      for (int b = 0; b < nblk; b++)
         for (int c = 0; c < blk[b + 1] - blk[b]; c++) {
            const int i = reverse ? blk[b + 1] - 1 - c : blk[b] + c;
            if (A->data[A->i[i]] == 0.0) continue;
            double res = f[i];
            for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) res -= A->data[jj] * u[A->j[jj]];
            u[i] += res / A->data[A->i[i]];
         }
}

/* Hybrid Jacobi/Gauss-Seidel over a block partition blk[0..nblk]:
 *   SMEM_Smooth.cpp:222-305 Parfor (diag_scale = A_diag = a_ii/omega, weight 1),
 *   SMEM_Smooth.cpp:533-586 row range (diag_scale = a_ii, weight 1),
 *   reverse != 0: the "T" variants :307-363 / :588-641 (rows visited ne-1..ns).
 * diag_scale == NULL means divide by a_ii.  Blocks are independent within a
 * sweep (in-block terms read u, out-of-block terms read u_prev copied before
 * the barrier), so visiting them in order is the reference's result. */
void or_hybrid_jgs(const or_csr *A, const double *f, double *u, double *u_prev, const int *blk,
                   int nblk, const double *diag_scale, double weight, int sweeps, int zero_flag,
                   int reverse)
{
   const int *A_i = A->i, *A_j = A->j;
   const double *A_data = A->data;
   for (int k = 0; k < sweeps; k++) {
      int zero = (k == 0 && zero_flag == 1);
      if (!zero) {
         for (int b = 0; b < nblk; b++)
            for (int i = blk[b]; i < blk[b + 1]; i++) u_prev[i] = u[i];
      }
#pragma omp parallel for schedule(dynamic, 1) if (nblk > 64)
      for (int b = 0; b < nblk; b++) {
         int ns = blk[b], ne = blk[b + 1];
         if (zero)
            for (int i = ns; i < ne; i++) u[i] = 0.0;
         for (int c = 0; c < ne - ns; c++) {
            int i = reverse ? ne - 1 - c : ns + c;
            if (A_data[A_i[i]] == 0.0) continue;
            double ds = diag_scale ? diag_scale[i] : A_data[A_i[i]];
            double res = f[i];
            for (int jj = A_i[i]; jj < A_i[i + 1]; jj++) {
               int ii = A_j[jj];
               if (ii >= ns && ii < ne)
                  res -= A_data[jj] * u[ii];
               else if (!zero)
                  res -= A_data[jj] * u_prev[ii];
            }
            if (zero)
               u[i] = weight * res / ds;
            else
               u[i] += weight * res / ds;
         }
      }
   }
}

/* SEQ_Smooth.cpp:119-155 */
void or_seq_sym_jacobi(const or_csr *A, const double *f, double *u, double *y, double *r,
                       double omega, int sweeps)
{
   int n = A->nrows, k = 0;
   for (int i = 0; i < n; i++) r[i] = f[i];
   while (1) {
      for (int i = 0; i < n; i++)
         if (A->data[A->i[i]] != 0.0) r[i] *= omega / A->data[A->i[i]];
      or_seq_matvec(A, r, y);
      for (int i = 0; i < n; i++) {
         if (A->data[A->i[i]] != 0.0) {
            r[i] = (2.0 * A->data[A->i[i]] * r[i] / omega) - y[i];
            r[i] *= omega / A->data[A->i[i]];
         }
         u[i] += r[i];
      }
      k++;
      if (k == sweeps) break;
      or_seq_residual(A, f, u, y, r);
   }
}

/* SEQ_Smooth.cpp:157-189 */
void or_seq_sym_l1jacobi(const or_csr *A, const double *f, double *u, double *y, double *r,
                         const double *l1, int sweeps)
{
   int n = A->nrows, k = 0;
   for (int i = 0; i < n; i++) r[i] = f[i];
   while (1) {
      for (int i = 0; i < n; i++) r[i] /= l1[i];
      or_seq_matvec(A, r, y);
      for (int i = 0; i < n; i++) {
         r[i] = (2.0 * l1[i] * r[i]) - y[i];
         r[i] /= l1[i];
         u[i] += r[i];
      }
      k++;
      if (k == sweeps) break;
      or_seq_residual(A, f, u, y, r);
   }
}

/* SMEM_Smooth.cpp:643-702 (one level group, res_compute_type LOCAL: ms=ns, me=ne).
 * zero_flag is level state that the function does not reset, so with
 * sweeps > 1 every sweep overwrites u (reference quirk, kept). */
void or_smem_sym_jacobi(const or_csr *A, const double *f, double *u, double *y, double *r,
                        double omega, int sweeps, int zero_flag, int ns, int ne)
{
   const int *A_i = A->i;
   const double *A_data = A->data;
   int k = 0;
   if (zero_flag == 1) {
      for (int i = ns; i < ne; i++) r[i] = f[i];
   } else {
      or_smem_residual(A, f, u, y, r, ns, ne);
   }
   while (1) {
      for (int i = ns; i < ne; i++) r[i] *= omega / A_data[A_i[i]];
      or_smem_matvec(A, r, y, ns, ne);
      for (int i = ns; i < ne; i++) {
         r[i] = (2.0 * A_data[A_i[i]] * r[i] / omega) - y[i];
         r[i] *= omega / A_data[A_i[i]];
      }
      if (zero_flag == 1) {
         for (int i = ns; i < ne; i++) u[i] = r[i];
      } else {
         for (int i = ns; i < ne; i++) u[i] += r[i];
      }
      k++;
      if (k == sweeps) break;
      or_smem_residual(A, f, u, y, r, ns, ne);
   }
}

/* SMEM_Smooth.cpp:704-762 */
void or_smem_sym_l1jacobi(const or_csr *A, const double *f, double *u, double *y, double *r,
                          const double *l1, int sweeps, int zero_flag, int ns, int ne)
{
   int k = 0;
   if (zero_flag == 1) {
      for (int i = ns; i < ne; i++) r[i] = f[i];
   } else {
      or_smem_residual(A, f, u, y, r, ns, ne);
   }
   while (1) {
      for (int i = ns; i < ne; i++) r[i] /= l1[i];
      or_smem_matvec(A, r, y, ns, ne);
      for (int i = ns; i < ne; i++) {
         r[i] = (2.0 * l1[i] * r[i]) - y[i];
         r[i] /= l1[i];
      }
      if (zero_flag == 1) {
         for (int i = ns; i < ne; i++) u[i] = r[i];
      } else {
         for (int i = ns; i < ne; i++) u[i] += r[i];
      }
      k++;
      if (k == sweeps) break;
      or_smem_residual(A, f, u, y, r, ns, ne);
   }
}

/* ------------------------------------------------------------------------- */
/* Setup helpers                                                              */
/* ------------------------------------------------------------------------- */

/* SMEM_Setup.cpp:234-237 A_diag[l][i] = a_ii / smooth_weight */
void or_a_diag(const or_csr *A, double omega, double *out)
{
   for (int i = 0; i < A->nrows; i++) out[i] = A->data[A->i[i]] / omega;
}

/* SMEM_Setup.cpp:222-232 L1_row_norm[l][i] = sum_j |a_ij| */
void or_l1_norms(const or_csr *A, double *out)
{
   for (int i = 0; i < A->nrows; i++) {
      out[i] = 0;
      for (int jj = A->i[i]; jj < A->i[i + 1]; jj++) out[i] += fabs(A->data[jj]);
   }
}

/* SMEM_Setup.cpp:1018-1030 (ONE_LEVEL thread ranges) */
void or_partition_equal(int n, int T, int *blk)
{
   int size = n / T, rest = n - size * T;
   for (int t = 0; t < T; t++) blk[t] = (t < rest) ? t * size + t : t * size + rest;
   blk[T] = n;
}

static int lower_bound_int(const int *a, int n, long long v)
{
   int lo = 0, hi = n;
   while (lo < hi) {
      int mid = lo + (hi - lo) / 2;
      if ((long long)a[mid] < v) lo = mid + 1; else hi = mid;
   }
   return lo;
}

/* SMEM_Setup.cpp:870-893 with nnz_per_thread = ceil(nnz/T) (:940-946) */
void or_partition_nnz(const or_csr *A, int T, int *blk)
{
   int n = A->nrows;
   long long nnz = A->i[n];
   long long per = (nnz + T - 1) / T;
   blk[0] = 0;
   for (int t = 1; t < T; t++) blk[t] = lower_bound_int(A->i, n, per * t);
   blk[T] = n;
}

/* SMEM_Solve.cpp:199-203: sqrt(sum r_i*r_i) */
double or_norm2(const double *x, int n)
{
   double s = 0;
#pragma omp parallel for schedule(static) reduction(+ : s) if (n > OMP_MIN_ROWS)
   for (int i = 0; i < n; i++) s += x[i] * x[i];
   return sqrt(s);
}

void or_csr_free_owned(or_csr_owned *M)
{
   free(M->i); free(M->j); free(M->data);
   M->i = NULL; M->j = NULL; M->data = NULL;
}

/* move the diagonal entry of each row of a square matrix to the front
 * (SMEM_Setup.cpp:1405-1419 StdVector_to_CSR convention) */
static void diag_first(or_csr_owned *M)
{
   if (M->nrows != M->ncols) return;
   for (int r = 0; r < M->nrows; r++) {
      int s = M->i[r], e = M->i[r + 1];
      for (int k = s; k < e; k++) {
         if (M->j[k] == r) {
            int cj = M->j[k]; double cv = M->data[k];
            for (int q = k; q > s; q--) { M->j[q] = M->j[q - 1]; M->data[q] = M->data[q - 1]; }
            M->j[s] = cj; M->data[s] = cv;
            break;
         }
      }
   }
}

/* counting-sort transpose; rows of the result hold ascending source rows */
void or_csr_transpose(const or_csr *A, or_csr_owned *T)
{
   int n = A->nrows, m = A->ncols;
   long long nnz = A->i[n];
   T->nrows = m; T->ncols = n; T->nnz = nnz;
   T->i = (int *)calloc((size_t)m + 1, sizeof(int));
   T->j = (int *)malloc((size_t)(nnz ? nnz : 1) * sizeof(int));
   T->data = (double *)malloc((size_t)(nnz ? nnz : 1) * sizeof(double));
   for (long long k = 0; k < nnz; k++) T->i[A->j[k] + 1]++;
   for (int c = 0; c < m; c++) T->i[c + 1] += T->i[c];
   int *pos = (int *)malloc(((size_t)m + 1) * sizeof(int));
   memcpy(pos, T->i, ((size_t)m + 1) * sizeof(int));
   for (int r = 0; r < n; r++)
      for (int k = A->i[r]; k < A->i[r + 1]; k++) {
         int c = A->j[k];
         T->j[pos[c]] = r; T->data[pos[c]] = A->data[k]; pos[c]++;
      }
   free(pos);
}

/* Gustavson SpGEMM, sorted columns, diag first when square.  Accumulation is
 * in the order (A row entry, B row entry), like a row-by-row product. */
void or_csr_spgemm(const or_csr *A, const or_csr *B, or_csr_owned *C)
{
   int n = A->nrows, m = B->ncols;
   int *mark = (int *)malloc((size_t)m * sizeof(int));
   double *acc = (double *)calloc((size_t)m, sizeof(double));
   int *cols = (int *)malloc((size_t)m * sizeof(int));
   for (int c = 0; c < m; c++) mark[c] = -1;
   C->nrows = n; C->ncols = m;
   C->i = (int *)malloc(((size_t)n + 1) * sizeof(int));
   long long cap = 16 + (long long)A->i[n] * 4, nnz = 0;
   C->j = (int *)malloc((size_t)cap * sizeof(int));
   C->data = (double *)malloc((size_t)cap * sizeof(double));
   C->i[0] = 0;
   for (int r = 0; r < n; r++) {
      int nc = 0;
      for (int ka = A->i[r]; ka < A->i[r + 1]; ka++) {
         int k = A->j[ka]; double av = A->data[ka];
         for (int kb = B->i[k]; kb < B->i[k + 1]; kb++) {
            int c = B->j[kb];
            if (mark[c] != r) { mark[c] = r; acc[c] = 0.0; cols[nc++] = c; }
            acc[c] += av * B->data[kb];
         }
      }
      /* insertion sort of the (small) column list */
      for (int a = 1; a < nc; a++) {
         int v = cols[a], b = a - 1;
         while (b >= 0 && cols[b] > v) { cols[b + 1] = cols[b]; b--; }
         cols[b + 1] = v;
      }
      if (nnz + nc > cap) {
         while (nnz + nc > cap) cap *= 2;
         C->j = (int *)realloc(C->j, (size_t)cap * sizeof(int));
         C->data = (double *)realloc(C->data, (size_t)cap * sizeof(double));
      }
      for (int a = 0; a < nc; a++) { C->j[nnz] = cols[a]; C->data[nnz] = acc[cols[a]]; nnz++; }
      C->i[r + 1] = (int)nnz;
   }
   C->nnz = nnz;
   free(mark); free(acc); free(cols);
   diag_first(C);
}

/* 7-point Laplacian, diag 6 / off -1, lexicographic x fastest, row entries in
 * the hypre GenerateLaplacian order: diag, -z, -y, -x, +x, +y, +z
 * (BuildHypreMatrix.cpp:250-275 with ax=ay=az=0 calls it; hypre itself is
 * not in the reference tree, so the entry order is restated, unpinned). */
void or_laplace_7pt(int nx, int ny, int nz, or_csr_owned *A)
{
   long long n = (long long)nx * ny * nz;
   A->nrows = A->ncols = (int)n;
   A->i = (int *)malloc((size_t)(n + 1) * sizeof(int));
   A->j = (int *)malloc((size_t)(7 * n) * sizeof(int));
   A->data = (double *)malloc((size_t)(7 * n) * sizeof(double));
   long long nnz = 0;
   A->i[0] = 0;
   for (int z = 0; z < nz; z++)
      for (int y = 0; y < ny; y++)
         for (int x = 0; x < nx; x++) {
            long long r = x + (long long)nx * (y + (long long)ny * z);
            A->j[nnz] = (int)r; A->data[nnz++] = 6.0;
            if (z > 0) { A->j[nnz] = (int)(r - (long long)nx * ny); A->data[nnz++] = -1.0; }
            if (y > 0) { A->j[nnz] = (int)(r - nx); A->data[nnz++] = -1.0; }
            if (x > 0) { A->j[nnz] = (int)(r - 1); A->data[nnz++] = -1.0; }
            if (x < nx - 1) { A->j[nnz] = (int)(r + 1); A->data[nnz++] = -1.0; }
            if (y < ny - 1) { A->j[nnz] = (int)(r + nx); A->data[nnz++] = -1.0; }
            if (z < nz - 1) { A->j[nnz] = (int)(r + (long long)nx * ny); A->data[nnz++] = -1.0; }
            A->i[r + 1] = (int)nnz;
         }
   A->nnz = nnz;
}

/* SMEM_Setup.cpp:1173-1254 SmoothTransfer (JACOBI smooth_interp_type):
 * G = I - omega D^-1 A with G_ii = 1-omega, Ps = G P, Rs = P^T G^T. */
void or_smooth_transfer(const or_csr *A, const or_csr *P, double omega, or_csr_owned *Ps,
                        or_csr_owned *Rs)
{
   int n = A->nrows;
   long long nnz = A->i[n];
   double *G = (double *)malloc((size_t)nnz * sizeof(double));
   double *GT = (double *)malloc((size_t)nnz * sizeof(double));
   for (int i = 0; i < n; i++) {
      G[A->i[i]] = GT[A->i[i]] = 1.0 - omega;
      for (int jj = A->i[i] + 1; jj < A->i[i + 1]; jj++) {
         G[jj] = -omega * A->data[jj] / A->data[A->i[i]];
         GT[jj] = -omega * A->data[jj] / A->data[A->i[A->j[jj]]];
      }
   }
   or_csr Gm = {n, A->ncols, nnz, A->i, A->j, G};
   or_csr GTm = {n, A->ncols, nnz, A->i, A->j, GT};
   or_csr_spgemm(&Gm, P, Ps);
   or_csr_owned PT;
   or_csr_transpose(P, &PT);
   or_csr PTm = {PT.nrows, PT.ncols, PT.nnz, PT.i, PT.j, PT.data};
   or_csr_spgemm(&PTm, &GTm, Rs);
   or_csr_free_owned(&PT);
   free(G); free(GT);
}

/* ------------------------------------------------------------------------- */
/* Hierarchy, cycles, solve driver                                            */
/* ------------------------------------------------------------------------- */
struct or_hier {
   int L;
   or_opts o;
   int precond_flag;
   or_csr *A, *P, *R;
   int *n;
   double **A_diag, **L1;
   /* vector (ONE_LEVEL) */
   double **f, **u, **u_prev, **y, **r, **r_fine, **e;
   /* level_vector (ALL_LEVELS): lv[k][l] for l < min(k+2, L) */
   double ***lv_r, ***lv_e, ***lv_u_prev, ***lv_y, ***lv_rr, ***lv_u_fine, ***lv_u_coarse,
      ***lv_u_fine_prev, ***lv_u_coarse_prev, ***lv_r_fine;
   int *zero_flags;
   int **blk; int *nblk;
   double *u_outer, *y_outer;
   int composed;        /* or_hier_set_composed_transfers */
   double **xt, **xy;   /* composed transfers: scratch per level group (n[0] each) */
};

static double *dvec(int n) { return (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }

or_hier *or_hier_create(int L, const or_csr *A, const or_csr *P, const or_csr *R,
                        const or_opts *opts)
{
   or_hier *H = (or_hier *)calloc(1, sizeof(or_hier));
   H->L = L;
   H->o = *opts;
   H->precond_flag = opts->cheby_flag ? 1 : 0;
   H->A = (or_csr *)malloc(L * sizeof(or_csr));
   H->P = (or_csr *)malloc(L * sizeof(or_csr));
   H->R = (or_csr *)malloc(L * sizeof(or_csr));
   H->n = (int *)malloc(L * sizeof(int));
   H->A_diag = (double **)malloc(L * sizeof(double *));
   H->L1 = (double **)malloc(L * sizeof(double *));
   double ***vs[] = {&H->f, &H->u, &H->u_prev, &H->y, &H->r, &H->r_fine, &H->e};
   for (unsigned q = 0; q < sizeof(vs) / sizeof(vs[0]); q++) *vs[q] = (double **)malloc(L * sizeof(double *));
   H->zero_flags = (int *)calloc(L, sizeof(int));
   H->blk = (int **)malloc(L * sizeof(int *));
   H->nblk = (int *)malloc(L * sizeof(int));
   int T = opts->num_threads > 0 ? opts->num_threads : 1;
   for (int l = 0; l < L; l++) {
      H->A[l] = A[l];
      if (l < L - 1) { H->P[l] = P[l]; H->R[l] = R[l]; }
      int n = A[l].nrows;
      H->n[l] = n;
      H->A_diag[l] = dvec(n); or_a_diag(&A[l], opts->smooth_weight, H->A_diag[l]);
      H->L1[l] = dvec(n); or_l1_norms(&A[l], H->L1[l]);
      for (unsigned q = 0; q < sizeof(vs) / sizeof(vs[0]); q++) (*vs[q])[l] = dvec(n);
      H->blk[l] = (int *)malloc((T + 1) * sizeof(int));
      H->nblk[l] = T;
      or_partition_equal(n, T, H->blk[l]);
   }
   double ****lvs[] = {&H->lv_r, &H->lv_e, &H->lv_u_prev, &H->lv_y, &H->lv_rr, &H->lv_u_fine,
                       &H->lv_u_coarse, &H->lv_u_fine_prev, &H->lv_u_coarse_prev, &H->lv_r_fine};
   /* level_vector sets exist only for the ALL_LEVELS (additive) solvers
    * (SMEM_Setup.cpp:292-341) */
   int all_levels = !(opts->solver == OR_MULT || opts->solver == OR_BPX);
   for (unsigned q = 0; q < sizeof(lvs) / sizeof(lvs[0]); q++) {
      *lvs[q] = (double ***)malloc(L * sizeof(double **));
      for (int k = 0; k < L; k++) {
         (*lvs[q])[k] = (double **)malloc(L * sizeof(double *));
         for (int l = 0; l < L; l++)
            (*lvs[q])[k][l] = (all_levels && l < k + 2) ? dvec(H->n[l]) : NULL;
      }
   }
   H->u_outer = dvec(H->n[0]);
   H->y_outer = dvec(H->n[0]);
   return H;
}

void or_hier_free(or_hier *H)
{
   if (!H) return;
   int L = H->L;
   double ***vs[] = {&H->f, &H->u, &H->u_prev, &H->y, &H->r, &H->r_fine, &H->e};
   for (int l = 0; l < L; l++) {
      free(H->A_diag[l]); free(H->L1[l]); free(H->blk[l]);
      for (unsigned q = 0; q < sizeof(vs) / sizeof(vs[0]); q++) free((*vs[q])[l]);
   }
   for (unsigned q = 0; q < sizeof(vs) / sizeof(vs[0]); q++) free(*vs[q]);
   double ****lvs[] = {&H->lv_r, &H->lv_e, &H->lv_u_prev, &H->lv_y, &H->lv_rr, &H->lv_u_fine,
                       &H->lv_u_coarse, &H->lv_u_fine_prev, &H->lv_u_coarse_prev, &H->lv_r_fine};
   for (unsigned q = 0; q < sizeof(lvs) / sizeof(lvs[0]); q++) {
      for (int k = 0; k < L; k++) {
         for (int l = 0; l < L; l++) free((*lvs[q])[k][l]);
         free((*lvs[q])[k]);
      }
      free(*lvs[q]);
   }
   free(H->A); free(H->P); free(H->R); free(H->n); free(H->A_diag); free(H->L1);
   free(H->zero_flags); free(H->blk); free(H->nblk); free(H->u_outer); free(H->y_outer);
   if (H->xt) {
      for (int k = 0; k < L; k++) {
         free(H->xt[k]);
         free(H->xy[k]);
      }
      free(H->xt);
      free(H->xy);
   }
   free(H);
}

void or_hier_set_composed_transfers(or_hier *H, int on)
{
   H->composed = on;
   if (on && !H->xt) {
      H->xt = (double **)malloc(H->L * sizeof(double *));
      H->xy = (double **)malloc(H->L * sizeof(double *));
      for (int k = 0; k < H->L; k++) {
         H->xt[k] = dvec(H->n[0]);
         H->xy[k] = dvec(H->n[0]);
      }
   }
}

/* does level transfer use the composed smoothed operators? (MULTADD only,
 * SMEM_Setup.cpp:244-261) */
static int composed_of(const or_hier *H)
{
   return H->composed && (H->o.solver == OR_MULTADD || H->o.solver == OR_ASYNC_MULTADD);
}

/* SmoothTransfer forms P~ only when num_post_smooth_sweeps > 0 and R~ only when
 * num_pre_smooth_sweeps > 0 (SMEM_Setup.cpp:1176-1180, 1245-1250) */
static int composed_r(const or_hier *H) { return composed_of(H) && H->o.num_pre > 0; }
static int composed_p(const or_hier *H) { return composed_of(H) && H->o.num_post > 0; }

/* rc = R~_l r (composed, see or_hier_set_composed_transfers) or R_l r; t / y:
 * scratch of level l's size */
static void xfer_restrict(or_hier *H, int l, const double *r, double *rc, double *t, double *y)
{
   if (!composed_r(H)) {
      or_smem_matvec(&H->R[l], r, rc, 0, H->n[l + 1]);
      return;
   }
   const or_csr *A = &H->A[l];
   const int n = H->n[l];
   const double w = H->o.smooth_weight;
   for (int i = 0; i < n; i++) t[i] = r[i] / A->data[A->i[i]];
   or_smem_matvec(A, t, y, 0, n);
   for (int i = 0; i < n; i++) t[i] = r[i] + (-w) * y[i];
   or_smem_matvec(&H->R[l], t, rc, 0, H->n[l + 1]);
}

/* ef = P~_l ec (composed) or P_l ec; y: scratch of level l's size */
static void xfer_prolong(or_hier *H, int l, const double *ec, double *ef, double *y)
{
   or_smem_matvec(&H->P[l], ec, ef, 0, H->n[l]);
   if (!composed_p(H)) return;
   const or_csr *A = &H->A[l];
   const int n = H->n[l];
   const double w = H->o.smooth_weight;
   or_smem_matvec(A, ef, y, 0, n);
   for (int i = 0; i < n; i++) y[i] = y[i] / A->data[A->i[i]];
   for (int i = 0; i < n; i++) ef[i] = ef[i] + (-w) * y[i];
}

void or_hier_set_blocks(or_hier *H, int level, const int *blk, int nblk)
{
   free(H->blk[level]);
   H->blk[level] = (int *)malloc((nblk + 1) * sizeof(int));
   memcpy(H->blk[level], blk, (nblk + 1) * sizeof(int));
   H->nblk[level] = nblk;
}

int or_hier_levels(or_hier *H) { return H->L; }

double *or_hier_vec(or_hier *H, const char *name, int level)
{
   if (!strcmp(name, "u")) return H->u[level];
   if (!strcmp(name, "f")) return H->f[level];
   if (!strcmp(name, "r")) return H->r[level];
   if (!strcmp(name, "u_prev")) return H->u_prev[level];
   if (!strcmp(name, "y")) return H->y[level];
   if (!strcmp(name, "e")) return H->e[level];
   if (!strcmp(name, "r_fine")) return H->r_fine[level];
   return NULL;
}

/* SMEM_Solve.cpp:264-377 SMEM_Smooth dispatcher.  Parameter names follow the
 * reference: (u, y, r) receive the caller's (u, u_prev, y). */
static void smooth(or_hier *H, int Alevel, const double *f, double *u, double *y, double *r,
                   int sweeps, int level, int all_levels, int ns, int ne)
{
   const or_csr *A = &H->A[Alevel];
   const or_opts *o = &H->o;
   int zf = H->zero_flags[level];
   int multadd = (o->solver == OR_MULTADD || o->solver == OR_ASYNC_MULTADD);
   int sym = multadd && o->num_post > 0 && o->num_pre > 0;
   if (o->smoother == OR_ASYNC_GAUSS_SEIDEL || o->smoother == OR_SEMI_ASYNC_GAUSS_SEIDEL) {
      /* SMEM_Solve.cpp:281-286 / 342-347 */
      int blk1[2] = {ns, ne};
      const int *blk = H->blk[Alevel];
      int nb = H->nblk[Alevel];
      if (all_levels && (ns != 0 || ne != A->nrows)) { blk = blk1; nb = 1; }
      or_async_gs(A, f, u, blk, nb, sweeps, 0);
      return;
   }
   if (all_levels) {
      if (o->smoother == OR_HYBRID_JACOBI_GAUSS_SEIDEL) {
         int blk1[2] = {ns, ne};
         const int *blk = H->blk[Alevel];
         int nb = H->nblk[Alevel];
         if (ns != 0 || ne != A->nrows) { blk = blk1; nb = 1; }
         or_hybrid_jgs(A, f, u, y, blk, nb, NULL, 1.0, sweeps, zf, 0);
      } else if (o->smoother == OR_L1_JACOBI) {
         if (sym) or_smem_sym_l1jacobi(A, f, u, y, r, H->L1[Alevel], sweeps, zf, ns, ne);
         else or_smem_l1jacobi(A, f, u, y, H->L1[Alevel], sweeps, zf, ns, ne);
      } else {
         if (sym) or_smem_sym_jacobi(A, f, u, y, r, o->smooth_weight, sweeps, zf, ns, ne);
         else or_smem_jacobi(A, f, u, y, o->smooth_weight, sweeps, zf, ns, ne);
      }
   } else {
      if (o->smoother == OR_HYBRID_JACOBI_GAUSS_SEIDEL ||
          o->smoother == OR_L1_HYBRID_JACOBI_GAUSS_SEIDEL) {
         /* Parfor variant: diag_scale = A_diag (a_ii/omega) or L1 norms, weight 1 */
         const double *ds = (o->smoother == OR_L1_HYBRID_JACOBI_GAUSS_SEIDEL) ? H->L1[Alevel]
                                                                               : H->A_diag[Alevel];
         or_hybrid_jgs(A, f, u, y, H->blk[Alevel], H->nblk[Alevel], ds, 1.0, sweeps, zf, 0);
      } else if (o->smoother == OR_L1_JACOBI) {
         or_smem_l1jacobi(A, f, u, y, H->L1[Alevel], sweeps, zf, 0, A->nrows);
      } else {
         or_smem_jacobi(A, f, u, y, o->smooth_weight, sweeps, zf, 0, A->nrows);
      }
   }
}

/* SMEM_Sync_AMG.cpp:8-145 SMEM_Sync_Parfor_Vcycle (ONE_LEVEL) */
void or_vcycle(or_hier *H)
{
   int L = H->L;
   const or_opts *o = &H->o;
   for (int level = 0; level < L - 1; level++) {
      int fg = level, cg = level + 1;
      H->zero_flags[level] = 1;
      if (level == 0 && H->precond_flag == 0) H->zero_flags[level] = 0;
      double *f_fine = (fg == 0 && H->precond_flag == 1) ? H->r[fg] : H->f[fg];
      smooth(H, fg, f_fine, H->u[fg], H->u_prev[fg], H->y[fg], o->num_pre, fg, 0, 0, 0);
      /* SMEM_Sync_Residual -> SpGEMV(alpha=-1, beta=1) */
      or_smem_spgemv(&H->A[fg], H->u[fg], f_fine, -1.0, 1.0, H->r_fine[fg], 0, H->n[fg]);
      /* SMEM_Sync_Parfor_Restrict, construct_R_flag = 1 */
      or_smem_matvec(&H->R[fg], H->r_fine[fg], H->f[cg], 0, H->n[cg]);
   }
   int cl = L - 1;
   smooth(H, cl, H->f[cl], H->u[cl], H->u_prev[cl], H->y[cl], o->num_pre + o->num_post, cl, 0, 0, 0);
   for (int level = L - 2; level > -1; level--) {
      H->zero_flags[level] = 0;
      int fg = level, cg = level + 1;
      or_smem_spgemv(&H->P[fg], H->u[cg], H->u[fg], 1.0, 1.0, H->u[fg], 0, H->n[fg]);
      double *f_fine = (fg == 0 && H->precond_flag == 1) ? H->r[fg] : H->f[fg];
      smooth(H, fg, f_fine, H->u[fg], H->u_prev[fg], H->y[fg], o->num_post, fg, 0, 0, 0);
   }
}

/* SMEM_Sync_AMG.cpp:147-294 SMEM_Sync_Parfor_BPXcycle (solver BPX, ONE_LEVEL):
 * restrict r[0] to every level, smooth every level (coarsest included) from a
 * zero guess with num_pre sweeps into e[l] (ONE_LEVEL smoothers), prolong
 * e_fine += P e_coarse upwards, then u += e[0] (u = e[0] as a preconditioner). */
void or_bpx_cycle(or_hier *H)
{
   int L = H->L;
   const or_opts *o = &H->o;
   for (int level = 0; level < L - 1; level++)
      or_smem_matvec(&H->R[level], H->r[level], H->r[level + 1], 0, H->n[level + 1]);
   for (int level = 0; level < L; level++) {
      H->zero_flags[level] = 1;
      smooth(H, level, H->r[level], H->e[level], H->u_prev[level], H->y[level], o->num_pre, level,
             0, 0, 0);
   }
   for (int level = L - 2; level > -1; level--)
      or_smem_spgemv(&H->P[level], H->e[level + 1], H->e[level], 1.0, 1.0, H->e[level], 0,
                     H->n[level]);
   int n0 = H->n[0];
   if (H->precond_flag == 1)
      memcpy(H->u[0], H->e[0], (size_t)n0 * sizeof(double));
   else
      for (int i = 0; i < n0; i++) H->u[0][i] += H->e[0][i];
}

/* SMEM_Sync_AMG.cpp:408-621 SMEM_Sync_Add_Vcycle (ALL_LEVELS, res LOCAL).
 * Level corrections are added to u in level order (the reference adds them
 * from concurrent thread groups without atomics). */
void or_sync_add_vcycle(or_hier *H)
{
   int L = H->L;
   const or_opts *o = &H->o;
   int multadd = (o->solver == OR_MULTADD || o->solver == OR_ASYNC_MULTADD);
   for (int k = 0; k < L; k++) {
      H->zero_flags[k] = 1;
      int coarsest = multadd ? k : k + 1;
      memcpy(H->lv_r[k][0], H->r[0], (size_t)H->n[0] * sizeof(double));
      for (int level = 0; level < coarsest; level++) {
         if (level < L - 1)
            xfer_restrict(H, level, H->lv_r[k][level], H->lv_r[k][level + 1], H->xt ? H->xt[k] : NULL,
                          H->xy ? H->xy[k] : NULL);
      }
      if (k == L - 1) {
         /* hypre_GaussElimSolve writes hypre's own U_array, which the cycle
          * never reads: the coarsest correction stays at its initial zero. */
      } else if (multadd) {
         memset(H->lv_e[k][k], 0, (size_t)H->n[k] * sizeof(double));
         smooth(H, k, H->lv_r[k][k], H->lv_e[k][k], H->lv_u_prev[k][k], H->lv_y[k][k],
                o->num_fine, k, 1, 0, H->n[k]);
      } else {
         int fg = k, cg = k + 1;
         memset(H->lv_u_fine[k][fg], 0, (size_t)H->n[fg] * sizeof(double));
         memset(H->lv_u_coarse[k][cg], 0, (size_t)H->n[cg] * sizeof(double));
         smooth(H, cg, H->lv_r[k][cg], H->lv_u_coarse[k][cg], H->lv_u_coarse_prev[k][cg],
                H->lv_y[k][cg], o->num_coarse, k, 1, 0, H->n[cg]);
         or_smem_matvec(&H->P[fg], H->lv_u_coarse[k][cg], H->lv_e[k][fg], 0, H->n[fg]);
         or_smem_residual(&H->A[fg], H->lv_r[k][fg], H->lv_e[k][fg], H->lv_y[k][fg],
                          H->lv_r_fine[k][fg], 0, H->n[fg]);
         smooth(H, fg, H->lv_r_fine[k][fg], H->lv_u_fine[k][fg], H->lv_u_fine_prev[k][fg],
                H->lv_y[k][fg], o->num_fine, k, 1, 0, H->n[fg]);
         memcpy(H->lv_e[k][k], H->lv_u_fine[k][k], (size_t)H->n[k] * sizeof(double));
      }
      for (int level = k - 1; level > -1; level--)
         xfer_prolong(H, level, H->lv_e[k][level + 1], H->lv_e[k][level], H->xy ? H->xy[k] : NULL);
      for (int i = 0; i < H->n[0]; i++) H->u[0][i] += H->lv_e[k][0][i];
   }
}

static void init_vectors(or_hier *H)
{
   /* Misc.cpp:565-692 InitVectors + InitSolve: every level vector to zero */
   for (int l = 0; l < H->L; l++) {
      size_t b = (size_t)H->n[l] * sizeof(double);
      if (l > 0) memset(H->f[l], 0, b);
      memset(H->u[l], 0, b); memset(H->u_prev[l], 0, b); memset(H->y[l], 0, b);
      memset(H->r[l], 0, b); memset(H->r_fine[l], 0, b); memset(H->e[l], 0, b);
      H->zero_flags[l] = 0;
   }
   for (int k = 0; k < H->L; k++)
      for (int l = 0; l < H->L && l < k + 2; l++) {
         if (!H->lv_r[k][l]) continue;
         size_t b = (size_t)H->n[l] * sizeof(double);
         memset(H->lv_r[k][l], 0, b); memset(H->lv_e[k][l], 0, b);
         memset(H->lv_u_prev[k][l], 0, b); memset(H->lv_y[k][l], 0, b);
         memset(H->lv_rr[k][l], 0, b); memset(H->lv_u_fine[k][l], 0, b);
         memset(H->lv_u_coarse[k][l], 0, b); memset(H->lv_u_fine_prev[k][l], 0, b);
         memset(H->lv_u_coarse_prev[k][l], 0, b); memset(H->lv_r_fine[k][l], 0, b);
      }
}

static double g_loop_seconds = 0.0;
double or_last_loop_seconds(void) { return g_loop_seconds; }

/* SMEM_Solve.cpp:11-262, synchronous branch (async_flag == 0) */
int or_solve(or_hier *H, const double *f, double *u, double *reshist)
{
   const or_opts *o = &H->o;
   int n0 = H->n[0];
   init_vectors(H);
   memcpy(H->f[0], f, (size_t)n0 * sizeof(double));
   memcpy(H->u[0], u, (size_t)n0 * sizeof(double));
   memset(H->u_outer, 0, (size_t)n0 * sizeof(double));
   memset(H->y_outer, 0, (size_t)n0 * sizeof(double));
   double mu24 = 4.0 * pow(o->cheby_mu, 2.0);
   double delta = o->cheby_delta;
   double *r = H->r[0];
   or_smem_spgemv(&H->A[0], H->u[0], H->f[0], -1.0, 1.0, r, 0, n0);
   double r0 = or_norm2(r, n0);
   if (reshist) reshist[0] = r0;
   double omega = 2.0;
   int done = 0;
   int all_levels = !(o->solver == OR_MULT || o->solver == OR_BPX);
#ifdef _OPENMP
   double t_start = omp_get_wtime();
#endif
   for (int k = 1; k <= o->num_cycles; k++) {
      if (o->solver == OR_BPX) or_bpx_cycle(H); /* SMEM_Solve.cpp:161-163 */
      else if (all_levels) or_sync_add_vcycle(H);
      else or_vcycle(H);
      if (o->cheby_flag == 1) {
         double *uu = H->u[0], *uo = H->u_outer, *yo = H->y_outer;
#pragma omp parallel for schedule(static) if (n0 > OMP_MIN_ROWS)
         for (int i = 0; i < n0; i++) {
            double u_outer_prev = uo[i];
            uo[i] = yo[i] + omega * (delta * uu[i] + uo[i] - yo[i]);
            yo[i] = u_outer_prev;
            uu[i] = uo[i];
         }
         omega = 1.0 / (1.0 - omega / mu24);
      }
      or_smem_spgemv(&H->A[0], H->u[0], H->f[0], -1.0, 1.0, r, 0, n0);
      done = k;
      if (o->check_resnorm == 1) {
         double rn = or_norm2(r, n0);
         if (reshist) reshist[k] = rn;
         if (rn / r0 < o->tol) break;
      }
   }
#ifdef _OPENMP
   g_loop_seconds = omp_get_wtime() - t_start;
#endif
   memcpy(u, H->u[0], (size_t)n0 * sizeof(double));
   return done;
}

/* ------------------------------------------------------------------------- */
/* SMEM_Async_Add_AMG (SMEM_Async_AMG.cpp:7-437) on real OpenMP threads        */
/* ------------------------------------------------------------------------- */
/* The reference's asynchronous additive cycle restated on T threads, so its
 * nondeterminism is the reference's own: nt[k] threads own level k (every
 * level at least one: the thread-to-level map PartitionLevels computes,
 * SMEM_Setup.cpp:590-868, given here as input); each group loops restrict ->
 * smooth -> prolong -> update of the shared fine iterate with no
 * synchronisation between groups; inside a group the threads split each
 * level's rows nnz-balanced (PartitionGrids, SMEM_Setup.cpp:945-978) and meet at
 * the group barrier (SMEM_LevelBarrier, Misc.cpp:485-533).  FULL_ASYNC adds
 * with `omp atomic` (:284-301; the private copy takes the value after this
 * thread's add), SEMI_ASYNC under one lock held by the group root (:238-283).
 * READ_SOL or READ_RES (:227-236, 270-295: the groups subtract A e from the
 * shared residual and keep private correction sums, joined at the end,
 * :416-426), res_compute LOCAL or GLOBAL (below), converge LOCAL (:317-322: a group stops after
 * num_cycles corrections) or GLOBAL (:323-337: the finest group's root sets
 * the converge flag once every level has num_cycles corrections -- CheckConverge,
 * Misc.cpp:418-442 -- and each group barrier hands it to the group).  The
 * smoothers are the ALL_LEVELS ones of the dispatcher (SMEM_Solve.cpp:277-321):
 * hybrid JGS (:533-586), Jacobi / L1 (:365-443), symmetric Jacobi / L1
 * (:643-762) with their barriers.  Test infrastructure: relres bands. */
typedef struct {
   int n, count, gen, flag;
} or_gbar;

/* schedule of the groups: 0 free (the OS's); 1 / 2 (converge LOCAL only) the
 * groups one after another, finest / coarsest first -- the extreme speed
 * ratios of the race, for the band's ends; 3 round robin: a token passes
 * from group to group (ascending level, cyclic, skipping groups that have
 * stopped), each holding it for one whole correction -- the equal-speed
 * schedule with a fixed update order.  1-3 make the race deterministic. */
static int g_async_schedule = 0;
void or_set_async_schedule(int s) { g_async_schedule = s; }

/* schedule 4 (timed): the race with fixed level speeds.  Group k
 * takes d[k] per correction; its j-th correction ends (and updates the shared
 * vectors) at j * d[k]; the corrections run whole, in the order of those end
 * times (ties: the finer group first) -- the race of level groups running
 * concurrently at those speeds, each update applied at its end.  Fed with
 * the device's measured per-level correction times, it is the oracle's model
 * of the device's free race. */
#define OR_MAX_LEVELS 64
static double g_async_dur[OR_MAX_LEVELS];
static double *g_async_t[OR_MAX_LEVELS]; /* or_set_async_times: end time of every correction */
static int g_async_tn[OR_MAX_LEVELS];
static int g_async_exact = 0; /* or_set_async_exact: a replay runs exactly the table's corrections */
void or_set_async_exact(int on) { g_async_exact = on; }
void or_set_async_durations(const double *d, int n)
{
   for (int k = 0; k < OR_MAX_LEVELS; k++) {
      g_async_dur[k] = k < n ? d[k] : 1.0;
      free(g_async_t[k]);
      g_async_t[k] = NULL;
      g_async_tn[k] = 0;
   }
}

/* schedule 4 with recorded end times: group k's j-th correction ends at
 * t[off_k + j] (j < n[k]; past the table the last interval repeats) -- the
 * replay of a measured race's update order */
void or_set_async_times(const double *t, const int *n, int L)
{
   or_set_async_durations(NULL, 0);
   for (int k = 0, off = 0; k < L && k < OR_MAX_LEVELS; off += n[k], k++) {
      if (n[k] <= 0) continue;
      g_async_t[k] = (double *)malloc((size_t)n[k] * sizeof(double));
      memcpy(g_async_t[k], t + off, (size_t)n[k] * sizeof(double));
      g_async_tn[k] = n[k];
   }
}

/* end time of group c's correction j (0-based) */
static double timed_end(int c, int j)
{
   const int n = g_async_tn[c];
   if (n == 0) return (double)(j + 1) * g_async_dur[c];
   const double *t = g_async_t[c];
   if (j < n) return t[j];
   const double dt = n > 1 ? t[n - 1] - t[n - 2] : t[0];
   return t[n - 1] + (double)(j - n + 1) * dt;
}

/* the next group of the timed schedule: the smallest end time of its next
 * correction among the groups that have not stopped (-1: none) */
static int timed_next(const int *count, const int *done, int k_lo, int k_hi)
{
   int best = -1;
   double tb = 0.0;
   for (int c = k_lo; c < k_hi; c++) {
      if (done[c]) continue;
      const double t = timed_end(c, __atomic_load_n(&count[c], __ATOMIC_ACQUIRE));
      if (best < 0 || t < tb) {
         best = c;
         tb = t;
      }
   }
   return best;
}

/* res_compute_type GLOBAL (ASYNC_MULTADD, SMEM_Main.cpp:650-660): no group owns
 * level 0 (PartitionLevels' finest_level = 1, SMEM_Setup.cpp:609-615); every
 * thread first smooths its global slice of the fine grid (A_ns_global: equal
 * row splits over all threads, SMEM_Setup.cpp:923-937) from its group's
 * residual and adds that into u (:35-77, SEMI_ASYNC under the lock :258-265),
 * and each iteration ends with the thread's slice of the global residual
 * f - A u_k written into the shared r and the group's rows of r read back
 * (:356-414) */
static int g_async_res_global = 0;
void or_set_async_res_global(int on) { g_async_res_global = on; }

/* DMEM acceleration of the asynchronous additive cycle (DMEM_Add.cpp:319-324):
 * ChebyUpdate(gridk.d, U_array[0]) on each level's prolonged fine correction
 * before it is added, async branch (DMEM_Misc.cpp:650-663): level `grid` (the
 * cheby_grid) carries d, the others scale their correction by omega * delta;
 * each level counts its own cycles.  Restated here per level group on the
 * group's rows, so the distributed solve's acceleration gets a band too. */
static int g_acc_type = 0, g_acc_grid = 0;
static double g_acc_mu = 0.0, g_acc_delta = 0.0;
void or_set_async_accel(int accel, int grid, double mu, double delta)
{
   g_acc_type = accel;
   g_acc_grid = grid;
   g_acc_mu = mu;
   g_acc_delta = delta;
}

static int gbar_wait(or_gbar *b, const int *conv)
{
   int g = __atomic_load_n(&b->gen, __ATOMIC_ACQUIRE);
   if (__atomic_add_fetch(&b->count, 1, __ATOMIC_ACQ_REL) == b->n) {
      __atomic_store_n(&b->count, 0, __ATOMIC_RELAXED);
      __atomic_store_n(&b->flag, conv ? __atomic_load_n(conv, __ATOMIC_ACQUIRE) : 0, __ATOMIC_RELAXED);
      __atomic_store_n(&b->gen, g + 1, __ATOMIC_RELEASE);
   } else {
      while (__atomic_load_n(&b->gen, __ATOMIC_ACQUIRE) == g) sched_yield();
   }
   return __atomic_load_n(&b->flag, __ATOMIC_RELAXED);
}

/* the ALL_LEVELS smoother of level `level` on A = A[Alevel], this thread's rows
 * [ns, ne) (SMEM_Smooth's argument order: f, u, y (u_prev), r (y)) */
static void async_smooth(or_hier *H, int Alevel, const double *f, double *u, double *up, double *yy,
                         int sweeps, int level, int ns, int ne, or_gbar *b)
{
   const or_csr *A = &H->A[Alevel];
   const or_opts *o = &H->o;
   const int *Ai = A->i, *Aj = A->j;
   const double *Ad = A->data;
   const double w = o->smooth_weight;
   const int zf = H->zero_flags[level];
   const int multadd = (o->solver == OR_MULTADD || o->solver == OR_ASYNC_MULTADD);
   const int sym = multadd && o->num_post > 0 && o->num_pre > 0;
   /* the smoothed operator's L1 norms.  The reference reads
    * L1_row_norm[level] with the GROUP's level (SMEM_Smooth.cpp:426,438), which
    * for AFACx's coarse-grid smoothing (SMEM_Async_AMG.cpp:164-173) are the
    * fine level's norms -- a quirk that makes AFACx + L1 diverge; the sync
    * additive restatement (smooth() above) and the device use A[Alevel]'s */
   const double *l1 = H->L1[Alevel];
   if (o->smoother == OR_HYBRID_JACOBI_GAUSS_SEIDEL) {
      /* SMEM_Sync_HybridJacobiGaussSeidel :533-586 (weight 1, divisor a_ii): the
       * GS block is the thread's rows [ns, ne); a hierarchy with an explicit
       * block partition of this level (or_hier_set_blocks: the device's 64-row
       * blocks) runs every block whose first row is in [ns, ne) -- the
       * reference with one thread per block, each block's rows in order */
      const int *hb = H->blk[Alevel];
      const int nhb = H->nblk[Alevel];
      const int many = nhb > 1;
      int b0 = 0, b1 = 1, one[2] = {ns, ne};
      if (many) {
         while (b0 < nhb && hb[b0] < ns) b0++;
         b1 = b0;
         while (b1 < nhb && hb[b1] < ne) b1++;
      }
      for (int k = 0; k < sweeps; k++) {
         const int zero = (k == 0 && zf == 1);
         if (!zero) {
            for (int i = ns; i < ne; i++) up[i] = u[i];
            gbar_wait(b, NULL);
         }
         for (int q = b0; q < b1; q++) {
            const int bs = many ? hb[q] : one[0], be = many ? hb[q + 1] : one[1];
            if (zero)
               for (int i = bs; i < be; i++) u[i] = 0.0;
            for (int i = bs; i < be; i++) {
               if (Ad[Ai[i]] == 0.0) continue;
               double res = f[i];
               for (int jj = Ai[i]; jj < Ai[i + 1]; jj++) {
                  int ii = Aj[jj];
                  if (ii >= bs && ii < be) res -= Ad[jj] * u[ii];
                  else if (!zero) res -= Ad[jj] * up[ii];
               }
               if (zero) u[i] = 1.0 * res / Ad[Ai[i]];
               else u[i] += 1.0 * res / Ad[Ai[i]];
            }
         }
         gbar_wait(b, NULL);
      }
      return;
   }
   const int use_l1 = o->smoother == OR_L1_JACOBI;
   if (sym) {
      /* SMEM_Sync_Symmetric[L1]Jacobi :643-762 (res_compute LOCAL); r = yy, y = up */
      double *r = yy, *y = up;
      int k = 0;
      if (zf == 1) for (int i = ns; i < ne; i++) r[i] = f[i];
      else or_smem_residual(A, f, u, y, r, ns, ne);
      while (1) {
         for (int i = ns; i < ne; i++) {
            if (use_l1) r[i] /= l1[i];
            else r[i] *= w / Ad[Ai[i]];
         }
         gbar_wait(b, NULL);
         or_smem_matvec(A, r, y, ns, ne);
         gbar_wait(b, NULL);
         for (int i = ns; i < ne; i++) {
            if (use_l1) {
               r[i] = (2.0 * l1[i] * r[i]) - y[i];
               r[i] /= l1[i];
            } else {
               r[i] = (2.0 * Ad[Ai[i]] * r[i] / w) - y[i];
               r[i] *= w / Ad[Ai[i]];
            }
         }
         if (zf == 1) for (int i = ns; i < ne; i++) u[i] = r[i];
         else for (int i = ns; i < ne; i++) u[i] += r[i];
         gbar_wait(b, NULL);
         if (++k == sweeps) break;
         or_smem_residual(A, f, u, y, r, ns, ne);
      }
      return;
   }
   /* SMEM_Sync_[L1]Jacobi :365-443 */
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zf == 1) {
         for (int i = ns; i < ne; i++) {
            if (use_l1) u[i] = f[i] / l1[i];
            else if (Ad[Ai[i]] != 0.0) u[i] = w * f[i] / Ad[Ai[i]];
         }
      } else {
         for (int i = ns; i < ne; i++) up[i] = u[i];
         gbar_wait(b, NULL);
         for (int i = ns; i < ne; i++) {
            if (!use_l1 && Ad[Ai[i]] == 0.0) continue;
            double res = f[i];
            for (int jj = Ai[i]; jj < Ai[i + 1]; jj++) res -= Ad[jj] * up[Aj[jj]];
            if (use_l1) u[i] += res / l1[i];
            else u[i] += w * res / Ad[Ai[i]];
         }
      }
      gbar_wait(b, NULL);
   }
}

int or_async_add(or_hier *H, const double *f, double *u, const int *nt, int async_type, int read_type,
                 int converge_type, int *corrections, double *relres)
{
   const or_opts *o = &H->o;
   const int L = H->L, n0 = H->n[0];
   const int multadd = (o->solver == OR_MULTADD || o->solver == OR_ASYNC_MULTADD);
   const int gres = g_async_res_global && multadd;
   const int k_lo = gres ? 1 : 0; /* the finest level with a group */
   if (gres && (L < 2 || read_type != OR_READ_SOL)) return -1; /* READ_RES needs LOCAL residuals (:227, 270, 288) */
   /* a sequential schedule never ends under converge GLOBAL (the first group
    * would wait for the others' counts forever) */
   if ((g_async_schedule == 1 || g_async_schedule == 2) && converge_type != OR_CONVERGE_LOCAL) return -1;
   if (L > OR_MAX_LEVELS) return -1;
   int T = 0;
   for (int k = 0; k < L; k++) {
      if (k < k_lo ? nt[k] != 0 : nt[k] < 1) return -1;
      T += nt[k];
   }
   init_vectors(H);
   memcpy(H->f[0], f, (size_t)n0 * sizeof(double));
   memcpy(H->u[0], u, (size_t)n0 * sizeof(double));
   /* SMEM_Solve: r = f - A u, its norm (SMEM_Solve.cpp:60-70) */
   or_smem_spgemv(&H->A[0], H->u[0], H->f[0], -1.0, 1.0, H->r[0], 0, n0);
   const double r0 = or_norm2(H->r[0], n0);
   for (int k = 0; k < L; k++) {
      H->zero_flags[k] = 1;
      memcpy(H->lv_r[k][0], H->r[0], (size_t)n0 * sizeof(double)); /* :10-15 */
   }
   /* groups: thread -> level, rank inside the group; row ranges per level */
   int *lev = (int *)malloc(T * sizeof(int)), *gi = (int *)malloc(T * sizeof(int));
   int *root = (int *)malloc(L * sizeof(int));
   for (int k = 0, t = 0; k < L; k++) {
      root[k] = t;
      for (int g = 0; g < nt[k]; g++, t++) {
         lev[t] = k;
         gi[t] = g;
      }
   }
   /* GLOBAL residuals: thread t's global fine slice [gs[t], gs[t + 1]) */
   int *gs = (int *)malloc((T + 1) * sizeof(int));
   if (H->nblk[0] > 1) {
      /* an explicit block partition of level 0 (the device's GS blocks): the
       * slices are equal splits of the blocks, so no block straddles two
       * threads' slices (the reference's GS block is the thread's slice) */
      const int nb = H->nblk[0];
      for (int t = 0; t <= T; t++) gs[t] = H->blk[0][(int)((long long)nb * t / T)];
   } else {
      const int size = n0 / T, rest = n0 - size * T;
      for (int t = 0; t <= T; t++) gs[t] = t * size + (t < rest ? t : rest);
   }
   /* blkA[k][l]: level-l row partition among group k (nt[k] + 1 entries); P / R likewise */
   int ***blk = (int ***)malloc(3 * sizeof(int **));
   for (int m = 0; m < 3; m++) {
      blk[m] = (int **)malloc((size_t)L * L * sizeof(int *));
      for (int k = 0; k < L; k++)
         for (int l = 0; l < L; l++) {
            int *b = (int *)malloc((nt[k] + 1) * sizeof(int));
            const or_csr *M = m == 0 ? &H->A[l] : (l < L - 1 ? (m == 1 ? &H->P[l] : &H->R[l]) : NULL);
            if (M && nt[k] > 0) or_partition_nnz(M, nt[k], b);
            else for (int g = 0; g <= nt[k]; g++) b[g] = 0;
            blk[m][k * L + l] = b;
         }
   }
   or_gbar *bar = (or_gbar *)calloc(L, sizeof(or_gbar));
   int *count = (int *)calloc(L, sizeof(int));
   double **uk = (double **)malloc(L * sizeof(double *)), **facc = (double **)malloc(L * sizeof(double *));
   double **dacc = (double **)malloc(L * sizeof(double *));
   for (int k = 0; k < L; k++) {
      bar[k].n = nt[k];
      uk[k] = dvec(n0);
      facc[k] = dvec(n0);
      dacc[k] = dvec(n0);
   }
   int conv_flag = 0;
   omp_lock_t lock;
   omp_init_lock(&lock);
   double *U = H->u[0];
   const double *F = H->f[0];
   const int rr = g_async_schedule == 3 || g_async_schedule == 4;
   const int timed = g_async_schedule == 4;
   int *gdone = (int *)calloc(L, sizeof(int)); /* round robin: groups that have stopped */
   /* round robin / timed: the group holding the token */
   int turn = timed ? timed_next(count, gdone, k_lo, L) : k_lo;
#pragma omp parallel num_threads(T)
   {
      const int tid = omp_get_thread_num();
      const int k = lev[tid], g = gi[tid];
      or_gbar *b = &bar[k];
#define RNG(m, l, s, e) const int s = blk[m][k * L + (l)][g], e = blk[m][k * L + (l)][g + 1]
      int tid_converge = 0;
      const int coarsest = multadd ? k : k + 1;
      if (g_async_schedule == 1 || g_async_schedule == 2) {
         const int prev = g_async_schedule == 1 ? k - 1 : k + 1; /* the group that runs before this one */
         if (prev >= k_lo && prev < L)
            while (__atomic_load_n(&count[prev], __ATOMIC_ACQUIRE) < o->num_cycles) sched_yield();
      }
      /* round robin: the group's whole correction runs while it holds the
       * token; the root hands it on (next group up, cyclic, skipping stopped
       * groups) after the group's last barrier of the correction */
#define RR_PASS(stop)                                                                 \
      do {                                                                           \
         if (rr) {                                                                   \
            gbar_wait(b, NULL);                                                      \
            if (tid == root[k]) {                                                    \
               if (stop) gdone[k] = 1;                                               \
               int nx = k;                                                           \
               if (timed) {                                                          \
                  const int c = timed_next(count, gdone, k_lo, L);                   \
                  if (c >= 0) nx = c;                                                \
               } else {                                                              \
                  for (int q = 1; q <= L - k_lo; q++) {                              \
                     const int c = k_lo + (k - k_lo + q) % (L - k_lo);               \
                     if (!gdone[c]) { nx = c; break; }                               \
                  }                                                                  \
               }                                                                     \
               __atomic_store_n(&turn, nx, __ATOMIC_RELEASE);                        \
            }                                                                        \
            gbar_wait(b, NULL); /* no thread of the group re-tests turn before */    \
         }                                                                           \
      } while (0)
      const int gns = gs[tid], gne = gs[tid + 1];
      int acc_cycle = 0;
      double acc_state[2] = {g_acc_mu, 1.0}; /* every thread of the group advances it alike */
      while (1) {
         if (rr)
            while (__atomic_load_n(&turn, __ATOMIC_ACQUIRE) != k) sched_yield();
         if (gres) {
            /* :35-77: smooth the global slice of A_0 u = r_k from zero */
            async_smooth(H, 0, H->lv_r[k][0], H->lv_u_fine[k][0], H->lv_u_prev[k][0], H->lv_y[k][0], o->num_fine,
                         k, gns, gne, b);
            if (async_type != OR_SEMI_ASYNC)
               for (int i = gns; i < gne; i++) {
#pragma omp atomic
                  U[i] += H->lv_u_fine[k][0][i];
               }
         }
         /* restriction :93-108 */
         for (int l = 0; l < coarsest; l++) {
            if (l >= L - 1) continue;
            if (composed_r(H)) { /* the group's first thread applies R~ (composed) */
               if (g == 0) xfer_restrict(H, l, H->lv_r[k][l], H->lv_r[k][l + 1], H->xt[k], H->xy[k]);
            } else {
               RNG(2, l, rs, re);
               or_smem_matvec(&H->R[l], H->lv_r[k][l], H->lv_r[k][l + 1], rs, re);
            }
            gbar_wait(b, NULL);
         }
         if (k == L - 1) {
            gbar_wait(b, NULL); /* :112-132: the coarsest solve is commented out */
         } else if (multadd) {
            RNG(0, k, ns, ne);
            for (int i = ns; i < ne; i++) H->lv_e[k][k][i] = 0.0;
            gbar_wait(b, NULL);
            async_smooth(H, k, H->lv_r[k][k], H->lv_e[k][k], H->lv_u_prev[k][k], H->lv_y[k][k], o->num_fine, k,
                         ns, ne, b);
         } else {
            const int fg = k, cg = k + 1;
            {
               RNG(0, fg, ns, ne);
               for (int i = ns; i < ne; i++) H->lv_u_fine[k][fg][i] = 0.0;
            }
            {
               RNG(0, cg, ns, ne);
               for (int i = ns; i < ne; i++) H->lv_u_coarse[k][cg][i] = 0.0;
               gbar_wait(b, NULL);
               async_smooth(H, cg, H->lv_r[k][cg], H->lv_u_coarse[k][cg], H->lv_u_coarse_prev[k][cg],
                            H->lv_y[k][cg], o->num_coarse, k, ns, ne, b);
            }
            RNG(0, fg, ns, ne);
            or_smem_matvec(&H->P[fg], H->lv_u_coarse[k][cg], H->lv_e[k][fg], ns, ne);
            gbar_wait(b, NULL);
            or_smem_residual(&H->A[fg], H->lv_r[k][fg], H->lv_e[k][fg], H->lv_y[k][fg], H->lv_r_fine[k][fg], ns,
                             ne);
            gbar_wait(b, NULL);
            async_smooth(H, fg, H->lv_r_fine[k][fg], H->lv_u_fine[k][fg], H->lv_u_fine_prev[k][fg],
                         H->lv_y[k][fg], o->num_fine, k, ns, ne, b);
            for (int i = ns; i < ne; i++) H->lv_e[k][k][i] = H->lv_u_fine[k][k][i];
            gbar_wait(b, NULL);
         }
         /* prolongation :211-224 */
         for (int l = k - 1; l > -1; l--) {
            if (composed_p(H)) {
               if (g == 0) xfer_prolong(H, l, H->lv_e[k][l + 1], H->lv_e[k][l], H->xy[k]);
            } else {
               RNG(1, l, ps, pe);
               or_smem_matvec(&H->P[l], H->lv_e[k][l + 1], H->lv_e[k][l], ps, pe);
            }
            gbar_wait(b, NULL);
         }
         RNG(0, 0, ns, ne);
         if (g_acc_type != OR_NO_ACCEL) {
            or_dmem_cheby_update(dacc[k] + ns, H->lv_e[k][0] + ns, ne - ns, acc_cycle, g_acc_type,
                                 k == g_acc_grid ? OR_CHEBY_GRID : OR_CHEBY_OTHER, g_acc_mu, g_acc_delta, acc_state);
            acc_cycle++;
         }
         const double *e0 = H->lv_e[k][0];
         double *ukk = uk[k];
         const int rres = read_type == OR_READ_RES;
         /* READ_RES: y = A e on the group's rows (:227-236) */
         if (rres) or_smem_matvec(&H->A[0], e0, H->lv_y[k][0], ns, ne);
         const double *y0 = H->lv_y[k][0];
         double *R0 = H->r[0], *rk = H->lv_r[k][0], *fk = facc[k];
         /* update of the shared iterate (READ_SOL) or residual (READ_RES) :238-301 */
         if (async_type == OR_SEMI_ASYNC) {
            if (tid == root[k]) omp_set_lock(&lock);
            gbar_wait(b, NULL);
            if (gres) /* :258-265 */
               for (int i = gns; i < gne; i++) U[i] += H->lv_u_fine[k][0][i];
         }
         for (int i = ns; i < ne; i++) {
            double v;
            if (rres) {
               if (async_type != OR_SEMI_ASYNC) fk[i] += e0[i];
               else {
#pragma omp atomic
                  U[i] += e0[i];
               }
#pragma omp atomic capture
               {
                  R0[i] -= y0[i];
                  v = R0[i];
               }
               rk[i] = v;
            } else {
#pragma omp atomic capture
               {
                  U[i] += e0[i];
                  v = U[i];
               }
               ukk[i] = v;
            }
         }
         if (async_type == OR_SEMI_ASYNC && tid == root[k]) omp_unset_lock(&lock);
         if (tid == root[k]) __atomic_add_fetch(&count[k], 1, __ATOMIC_ACQ_REL);
         if (timed && g_async_exact && g_async_tn[k] > 0) {
            /* a replay (or_set_async_times + or_set_async_exact) runs exactly the
             * recorded corrections: under converge GLOBAL the race's stopping
             * point is in the table */
            gbar_wait(b, NULL);
            if (__atomic_load_n(&count[k], __ATOMIC_ACQUIRE) >= g_async_tn[k]) tid_converge = 1;
         } else if (converge_type == OR_CONVERGE_LOCAL) {
            gbar_wait(b, NULL);
            if (__atomic_load_n(&count[k], __ATOMIC_ACQUIRE) == o->num_cycles) tid_converge = 1;
         } else {
            if (tid == root[k_lo] && __atomic_load_n(&conv_flag, __ATOMIC_ACQUIRE) == 0) {
               int all = 1;
               for (int l = k_lo; l < L; l++)
                  if (__atomic_load_n(&count[l], __ATOMIC_ACQUIRE) < o->num_cycles) all = 0;
               if (all) __atomic_store_n(&conv_flag, 1, __ATOMIC_RELEASE);
            }
            if (gbar_wait(b, &conv_flag) == 1) tid_converge = 1;
         }
         if (!gres) {
            /* LOCAL residual, READ_SOL :338-351 */
            if (!rres) or_smem_residual(&H->A[0], F, ukk, H->lv_y[k][0], H->lv_r[k][0], ns, ne);
            gbar_wait(b, NULL);
         }
         if (tid_converge == 1) {
            RR_PASS(1);
            break;
         }
         if (gres) {
            /* :356-414: u_k = u on the group's rows; the slice's residual
             * into the shared r; the group's rows of r back into r_k */
            for (int i = ns; i < ne; i++) {
               double v;
#pragma omp atomic read
               v = U[i];
               ukk[i] = v;
            }
            gbar_wait(b, NULL);
            or_smem_residual(&H->A[0], F, ukk, H->lv_y[k][0], H->lv_r[k][0], gns, gne);
            if (async_type == OR_SEMI_ASYNC && tid == root[k]) omp_set_lock(&lock);
            gbar_wait(b, NULL);
            for (int i = gns; i < gne; i++) {
#pragma omp atomic write
               R0[i] = rk[i];
            }
            for (int i = ns; i < ne; i++) {
               double v;
#pragma omp atomic read
               v = R0[i];
               rk[i] = v;
            }
            if (async_type == OR_SEMI_ASYNC && tid == root[k]) omp_unset_lock(&lock);
         }
         RR_PASS(0);
      }
#undef RNG
#undef RR_PASS
   }
   omp_destroy_lock(&lock);
   free(gdone);
   /* FULL_ASYNC READ_RES: the private correction sums join u (:416-426) */
   if (read_type == OR_READ_RES && async_type != OR_SEMI_ASYNC)
      for (int k = 0; k < L; k++)
         for (int i = 0; i < n0; i++) H->u[0][i] += facc[k][i];
   /* SMEM_Solve.cpp:82-91: the final residual */
   or_smem_spgemv(&H->A[0], H->u[0], H->f[0], -1.0, 1.0, H->r[0], 0, n0);
   if (relres) *relres = r0 > 0 ? or_norm2(H->r[0], n0) / r0 : 0.0;
   if (corrections)
      for (int k = 0; k < L; k++) corrections[k] = count[k];
   memcpy(u, H->u[0], (size_t)n0 * sizeof(double));
   for (int m = 0; m < 3; m++) {
      for (int q = 0; q < L * L; q++) free(blk[m][q]);
      free(blk[m]);
   }
   free(blk);
   for (int k = 0; k < L; k++) {
      free(uk[k]);
      free(facc[k]);
      free(dacc[k]);
   }
   free(uk);
   free(dacc);
   free(facc); free(bar); free(count); free(lev); free(gi); free(root); free(gs);
   return 0;
}

/* Replay of a DISTRIBUTED free race (the row-sliced event model of
 * amg_dist_async_solve, FULL_ASYNC / READ_SOL / LOCAL residuals, converge
 * LOCAL).  Every rank holds slice [rs[r], rs[r+1]) of the fine rows; level k's
 * correction j is one collective computation (its restrictions, smoothing and
 * prolongations exchange halos inside level k only), but its update of the
 * shared iterate -- u += e on the slice, the private copy u_k = u there -- runs
 * on every rank at that rank's own time t[k][j][r], in between the other
 * levels' updates of the same slice, and the level's next residual
 * r_k = f - A u_k takes each slice from its own rank's copy.  The replay
 * applies the slice updates in the order of the recorded times (ties: lower
 * level, then lower rank) and forms e_{k,j} from r_k as left by every slice of
 * correction j - 1 -- so it reproduces the blend of per-rank update orders a
 * single global order cannot.  t: for each level k in 0..L-1, nc[k] * R times
 * (correction-major); levels with nc[k] = 0 do not correct.  One thread; the
 * arithmetic of each correction is or_async_add's group body with one thread
 * per group. */
typedef struct {
   double t;
   int k, r, x;
} replay_ev;

static int replay_ev_cmp(const void *pa, const void *pb)
{
   const replay_ev *a = (const replay_ev *)pa, *b = (const replay_ev *)pb;
   if (a->t != b->t) return a->t < b->t ? -1 : 1;
   if (a->k != b->k) return a->k < b->k ? -1 : 1;
   if (a->r != b->r) return a->r < b->r ? -1 : 1;
   return a->x < b->x ? -1 : a->x > b->x;
}

int or_async_add_replay(or_hier *H, const double *f, double *u, int R, const int *rs, const double *t,
                        const int *nc, int *corrections, double *relres)
{
   const or_opts *o = &H->o;
   const int L = H->L, n0 = H->n[0];
   const int multadd = (o->solver == OR_MULTADD || o->solver == OR_ASYNC_MULTADD);
   if (R < 1 || rs[0] != 0 || rs[R] != n0 || L > OR_MAX_LEVELS) return -1;
   init_vectors(H);
   memcpy(H->f[0], f, (size_t)n0 * sizeof(double));
   memcpy(H->u[0], u, (size_t)n0 * sizeof(double));
   or_smem_spgemv(&H->A[0], H->u[0], H->f[0], -1.0, 1.0, H->r[0], 0, n0);
   const double r0 = or_norm2(H->r[0], n0);
   for (int k = 0; k < L; k++) {
      H->zero_flags[k] = 1;
      memcpy(H->lv_r[k][0], H->r[0], (size_t)n0 * sizeof(double));
   }
   double *U = H->u[0];
   const double *F = H->f[0];
   /* the event list (k, j, r) sorted by time */
   int ne = 0, off[OR_MAX_LEVELS + 1];
   for (int k = 0; k < L; k++) {
      off[k] = ne;
      ne += nc[k] * R;
   }
   off[L] = ne;
   int *ev = (int *)malloc((size_t)(ne > 0 ? ne : 1) * sizeof(int));
   /* sorted by (time, k, r, j) */
   replay_ev *key = (replay_ev *)malloc((size_t)(ne > 0 ? ne : 1) * sizeof(replay_ev));
   for (int k = 0; k < L; k++)
      for (int q = off[k]; q < off[k + 1]; q++) {
         key[q].t = t[q];
         key[q].k = k;
         key[q].r = (q - off[k]) % R;
         key[q].x = q;
      }
   qsort(key, (size_t)ne, sizeof(replay_ev), replay_ev_cmp);
   for (int q = 0; q < ne; q++) ev[q] = key[q].x;
   free(key);
   double **E = (double **)malloc(L * sizeof(double *)), **uk = (double **)malloc(L * sizeof(double *));
   double **dacc = (double **)malloc(L * sizeof(double *));
   int *jc = (int *)calloc(L, sizeof(int));    /* corrections whose e is formed */
   int *nup = (int *)calloc(L, sizeof(int));   /* slices updated of the current correction */
   int *done = (int *)calloc((size_t)(ne > 0 ? ne : 1), sizeof(int));
   int *acc_cycle = (int *)calloc(L, sizeof(int));
   double (*acc_state)[2] = malloc((size_t)L * sizeof(*acc_state));
   for (int k = 0; k < L; k++) {
      E[k] = dvec(n0);
      uk[k] = dvec(n0);
      dacc[k] = dvec(n0);
      acc_state[k][0] = g_acc_mu;
      acc_state[k][1] = 1.0;
   }
   or_gbar one = {1, 0, 0, 0};
   or_gbar *b = &one;
   /* e_{k, jc[k]}: or_async_add's group body, one thread */
   #define FORM_E(k)                                                                                          \
   do {                                                                                                      \
      const int coarsest = multadd ? (k) : (k) + 1;                                                          \
      for (int l = 0; l < coarsest; l++) {                                                                   \
         if (l >= L - 1) continue;                                                                           \
         if (composed_r(H)) xfer_restrict(H, l, H->lv_r[k][l], H->lv_r[k][l + 1], H->xt[k], H->xy[k]);      \
         else or_smem_matvec(&H->R[l], H->lv_r[k][l], H->lv_r[k][l + 1], 0, H->n[l + 1]);                     \
      }                                                                                                      \
      if ((k) == L - 1) {                                                                                    \
      } else if (multadd) {                                                                                  \
         memset(H->lv_e[k][k], 0, (size_t)H->n[k] * sizeof(double));                                         \
         async_smooth(H, k, H->lv_r[k][k], H->lv_e[k][k], H->lv_u_prev[k][k], H->lv_y[k][k], o->num_fine, k, \
                      0, H->n[k], b);                                                                       \
      } else {                                                                                               \
         const int fg = (k), cg = (k) + 1;                                                                   \
         memset(H->lv_u_fine[k][fg], 0, (size_t)H->n[fg] * sizeof(double));                                 \
         memset(H->lv_u_coarse[k][cg], 0, (size_t)H->n[cg] * sizeof(double));                               \
         async_smooth(H, cg, H->lv_r[k][cg], H->lv_u_coarse[k][cg], H->lv_u_coarse_prev[k][cg],             \
                      H->lv_y[k][cg], o->num_coarse, k, 0, H->n[cg], b);                                     \
         or_smem_matvec(&H->P[fg], H->lv_u_coarse[k][cg], H->lv_e[k][fg], 0, H->n[fg]);                      \
         or_smem_residual(&H->A[fg], H->lv_r[k][fg], H->lv_e[k][fg], H->lv_y[k][fg], H->lv_r_fine[k][fg], 0, \
                          H->n[fg]);                                                                        \
         async_smooth(H, fg, H->lv_r_fine[k][fg], H->lv_u_fine[k][fg], H->lv_u_fine_prev[k][fg],            \
                      H->lv_y[k][fg], o->num_fine, k, 0, H->n[fg], b);                                       \
         memcpy(H->lv_e[k][k], H->lv_u_fine[k][k], (size_t)H->n[k] * sizeof(double));                        \
      }                                                                                                      \
      for (int l = (k) - 1; l > -1; l--) {                                                                   \
         if (composed_p(H)) xfer_prolong(H, l, H->lv_e[k][l + 1], H->lv_e[k][l], H->xy[k]);                 \
         else or_smem_matvec(&H->P[l], H->lv_e[k][l + 1], H->lv_e[k][l], 0, H->n[l]);                         \
      }                                                                                                      \
      if (g_acc_type != OR_NO_ACCEL) {                                                                       \
         or_dmem_cheby_update(dacc[k], H->lv_e[k][0], n0, acc_cycle[k], g_acc_type,                          \
                              (k) == g_acc_grid ? OR_CHEBY_GRID : OR_CHEBY_OTHER, g_acc_mu, g_acc_delta,     \
                              acc_state[k]);                                                                 \
         acc_cycle[k]++;                                                                                     \
      }                                                                                                      \
      memcpy(E[k], H->lv_e[k][0], (size_t)n0 * sizeof(double));                                              \
      jc[k]++;                                                                                               \
   } while (0)
   for (int q = 0; q < ne; q++) {
      const int x = ev[q];
      if (done[x]) continue;
      int k = 0;
      while (k < L && off[k + 1] <= x) k++;
      const int j = (x - off[k]) / R;
      /* a slice of correction j before correction j - 1 finished on every
       * rank (timer skew): the earlier correction's remaining slices first */
      while (jc[k] < j + 1) {
         if (jc[k] > 0 && nup[k] > 0) {
            const int jp = jc[k] - 1;
            for (int r = 0; r < R; r++) {
               const int y = off[k] + jp * R + r;
               if (done[y]) continue;
               for (int i = rs[r]; i < rs[r + 1]; i++) {
                  U[i] += E[k][i];
                  uk[k][i] = U[i];
               }
               done[y] = 1;
               nup[k]++;
            }
            or_smem_residual(&H->A[0], F, uk[k], H->lv_y[k][0], H->lv_r[k][0], 0, n0);
            nup[k] = 0;
         }
         FORM_E(k);
      }
      const int r = (x - off[k]) % R;
      for (int i = rs[r]; i < rs[r + 1]; i++) {
         U[i] += E[k][i];
         uk[k][i] = U[i];
      }
      done[x] = 1;
      if (++nup[k] == R) {
         /* SMEM_Residual on every slice's own copy: the level's next residual */
         or_smem_residual(&H->A[0], F, uk[k], H->lv_y[k][0], H->lv_r[k][0], 0, n0);
         nup[k] = 0;
      }
   }
   #undef FORM_E
   or_smem_spgemv(&H->A[0], H->u[0], H->f[0], -1.0, 1.0, H->r[0], 0, n0);
   if (relres) *relres = r0 > 0 ? or_norm2(H->r[0], n0) / r0 : 0.0;
   if (corrections)
      for (int k = 0; k < L; k++) corrections[k] = jc[k];
   memcpy(u, H->u[0], (size_t)n0 * sizeof(double));
   for (int k = 0; k < L; k++) {
      free(E[k]);
      free(uk[k]);
      free(dacc[k]);
   }
   free(E); free(uk); free(dacc); free(jc); free(nup); free(done); free(acc_cycle); free(acc_state); free(ev);
   return 0;
}

/* M^{-1} = one V-cycle in preconditioner mode from a zero state (the
 * reference uses HYPRE_BoomerAMGSolve here, SMEM_Cheby.cpp:458-459). */
static void precond_apply(or_hier *H, const double *fin, double *out)
{
   int saved = H->precond_flag;
   H->precond_flag = 1;
   for (int l = 0; l < H->L; l++) {
      memset(H->u[l], 0, (size_t)H->n[l] * sizeof(double));
      H->zero_flags[l] = 0;
   }
   memcpy(H->r[0], fin, (size_t)H->n[0] * sizeof(double));
   or_vcycle(H);
   memcpy(out, H->u[0], (size_t)H->n[0] * sizeof(double));
   H->precond_flag = saved;
}

static double dot(const double *a, const double *b, int n)
{
   double s = 0;
   for (int i = 0; i < n; i++) s += a[i] * b[i];
   return s;
}

/* SMEM_Cheby.cpp:410-518 EigsPower */
void or_eigs_power(or_hier *H, int iters, double *eig_max, double *eig_min)
{
   int n = H->n[0];
   double *u = dvec(n), *e = dvec(n), *fv = dvec(n), *v = dvec(n);
   for (int i = 0; i < n; i++) u[i] = 1.0;
   int it = 0;
   while (1) {
      double un = sqrt(dot(u, u, n));
      for (int i = 0; i < n; i++) u[i] *= 1.0 / un;
      for (int i = 0; i < n; i++) e[i] = u[i];
      or_seq_matvec(&H->A[0], u, fv);
      precond_apply(H, fv, u);
      it++;
      if (it == iters) break;
   }
   for (int i = 0; i < n; i++) v[i] = e[i];
   double emax = dot(v, u, n);
   for (int i = 0; i < n; i++) u[i] = 1.0;
   it = 0;
   while (1) {
      double un = sqrt(dot(u, u, n));
      for (int i = 0; i < n; i++) u[i] *= 1.0 / un;
      for (int i = 0; i < n; i++) e[i] = u[i];
      or_seq_matvec(&H->A[0], u, fv);
      precond_apply(H, fv, u);
      for (int i = 0; i < n; i++) v[i] = e[i];
      it++;
      if (it == iters) break;
      for (int i = 0; i < n; i++) u[i] += -emax * v[i];
   }
   *eig_min = dot(v, u, n);
   *eig_max = emax;
   free(u); free(e); free(fv); free(v);
}

/* SMEM_Cheby.cpp:48-49 */
void or_cheby_setup(double eig_min, double eig_max, double *mu, double *delta)
{
   *mu = (eig_max + eig_min) / (eig_max - eig_min);
   *delta = 2.0 / (eig_max + eig_min);
}

/* ------------------------------------------------------------------------- */
/* DMEM outer acceleration and drivers                                        */
/* ------------------------------------------------------------------------- */

/* DMEM_Misc.cpp:612-666 DMEM_ChebyUpdate */
void or_dmem_cheby_update(double *d, double *u, int n, int cycle, int accel, int branch, double mu,
                          double delta, double *state)
{
   if (cycle == 0) { /* :627-631 DMEM_HypreParVector_Copy(d, u) */
      memcpy(d, u, (size_t)n * sizeof(double));
      return;
   }
   double omega;
   if (accel == OR_RICHARD_ACCEL) { /* :634-636 */
      omega = 2.0 / (1.0 + sqrt(1.0 - pow(mu, -2.0)));
   } else { /* :637-642 */
      double c_temp = state[0];
      state[0] = 2.0 * mu * state[0] - state[1];
      state[1] = c_temp;
      omega = 2.0 * mu * state[1] / state[0];
   }
   if (branch == OR_CHEBY_SYNC) { /* :645-649 */
      for (int i = 0; i < n; i++) d[i] = (omega - 1.0) * d[i] + omega * delta * u[i];
   } else if (branch == OR_CHEBY_GRID) { /* :651-657 */
      for (int i = 0; i < n; i++) {
         double d_prev = d[i];
         d[i] = (omega - 1.0) * d[i] + omega * delta * u[i];
         u[i] = (omega - 1.0) * d_prev + omega * delta * u[i];
      }
   } else { /* :658-662 */
      for (int i = 0; i < n; i++) u[i] = omega * delta * u[i];
   }
}

/* DMEM_Mult.cpp:13-93 */
int or_dmem_mult_solve(or_hier *H, const double *b, double *x, double *reshist, int accel, double mu,
                       double delta)
{
   const or_opts *o = &H->o;
   int n0 = H->n[0];
   if (o->num_cycles <= 0) return 0;
   init_vectors(H);
   memcpy(H->f[0], b, (size_t)n0 * sizeof(double));
   double *r = H->r[0], *e = H->u[0];
   double *d = dvec(n0);
   double state[2] = {mu, 1.0};
   /* ResetNorms, DMEM_Setup.cpp:1455-1461: r = b - A x, r0 = ||r|| */
   or_smem_spgemv(&H->A[0], x, b, -1.0, 1.0, r, 0, n0);
   double r0 = or_norm2(r, n0);
   if (reshist) reshist[0] = r0;
   int saved = H->precond_flag;
   H->precond_flag = 1; /* precond_zero_init_guess = 1: the cycle acts on r from e = 0 */
   int cycle = 0;
   while (1) {
      memset(e, 0, (size_t)n0 * sizeof(double)); /* :41 Set(e, 0) */
      or_vcycle(H);                                 /* :42-45 DMEM_MultCycle(r -> e) */
      for (int i = 0; i < n0; i++) x[i] += 1.0 * e[i]; /* :46-48 Axpy(x, e, 1) */
      if (accel != OR_NO_ACCEL) {                   /* :50-55 */
         or_dmem_cheby_update(d, e, n0, cycle, accel, OR_CHEBY_SYNC, mu, delta, state);
         for (int i = 0; i < n0; i++) x[i] += 1.0 * d[i];
      }
      or_smem_spgemv(&H->A[0], x, b, -1.0, 1.0, r, 0, n0); /* :68-73 */
      double rn = or_norm2(r, n0);
      cycle++;
      if (reshist) reshist[cycle] = rn;
      if (rn / r0 < o->tol || cycle == o->num_cycles) break; /* :84 */
   }
   H->precond_flag = saved;
   free(d);
   return cycle;
}

/* DMEM_Smooth.cpp:16-313, one rank, one grid */
double or_dmem_async_jacobi(const or_csr *A, const double *b, double *x, int sweeps, double omega,
                            const double *l1, int accel, double mu, double delta)
{
   int n = A->nrows;
   double *s = dvec(n), *u = dvec(n), *e = dvec(n), *r = dvec(n), *d = dvec(n);
   double state[2] = {mu, 1.0};
   for (int i = 0; i < n; i++) {
      double a = A->data[A->i[i]];
      s[i] = l1 ? l1[i] : (a == 0 ? 1.0 : a / omega); /* DMEM_Setup.cpp:474-480 */
      x[i] = 0.0;
      r[i] = b[i];
   }
   for (int k = 0; k < sweeps; k++) {
      for (int i = 0; i < n; i++) u[i] = 0.0 + r[i] / s[i]; /* :100-106 Set(u, 0); Ivaxpy(u, r, s) */
      if (accel != OR_NO_ACCEL)                            /* :110-112 */
         or_dmem_cheby_update(d, u, n, k, accel, OR_CHEBY_GRID, mu, delta, state);
      for (int i = 0; i < n; i++) e[i] = 0.0 + 1.0 * u[i]; /* :171-183 Set(e, 0); Axpy(e, u, 1) */
      or_smem_spgemv(A, e, r, -1.0, 1.0, r, 0, n);         /* :218-224 r -= A_diag e */
      for (int i = 0; i < n; i++) x[i] += 1.0 * e[i];      /* :229 Axpy(x, e, 1) */
   }
   or_smem_spgemv(A, x, b, -1.0, 1.0, r, 0, n);
   double rn = or_norm2(r, n);
   free(s); free(u); free(e); free(r); free(d);
   return rn;
}

/* ------------------------------------------------------------------------- */
/* DMEM_Add (DMEM_Add.cpp:20-944) with its message engine (DMEM_Comm.cpp:11-382) */
/* ------------------------------------------------------------------------- */
/* The reference's level-grouped asynchronous additive solver restated with
 * OpenMP threads standing in for the MPI ranks, one rank per grid (grid k
 * computes level k's correction): every grid holds the whole fine problem,
 * AddCycle (:180-329) restricts its residual F[0] to level k with R,
 * DMEM_AddSmooth's 2-step symmetric Jacobi there (DMEM_Smooth.cpp:574-638, s =
 * a_ii / w or 1 where a_ii = 0, DMEM_Setup.cpp:471-482) -- or, on the coarsest
 * grid, the exact solve of hypre_GaussElimSolve (:263; dense LU with partial
 * pivoting here) -- and prolongs with P; DMEM_AddCorrect_LocalRes / AddCheckComm
 * (:391-528) send the accumulated correction y to every other grid
 * (gridjToGridk_Correct_outsideSend, ACCUMULATE, every async_comm_save_divisor
 * cycles and on convergence) and add what arrived into x (payloads of
 * messages received alone with a done flag are dropped, as in the reference:
 * SendRecv breaks before raising the receive flag, DMEM_Comm.cpp:292-305);
 * CheckInFlight / SetNextInFlight keep max_inflight sends per destination;
 * CheckConverge LOCAL / GLOBAL (:906-944), AddResNorm's InnerProdFlag (one rank
 * per grid: local), AsyncRecvCleanup + CompleteInFlight (:827-890).
 *
 * Messages: an in-process mailbox with MPI point-to-point matching (per source,
 * destination, in order); a receive completes when matched, a send when the
 * receiver has taken its payload (the device hub's completion: the slot is
 * released by the receiver's read).
 *
 * sched 0: the free race (the OS schedules the grid threads).  sched 1: round
 * robin -- a token passes from grid to grid (ascending, cyclic, skipping
 * finished grids) at fixed points: the end of every main-loop iteration, every
 * pass of CheckInFlight's wait, every iteration of AsyncRecvCleanup, every
 * failed test of the final waits.  The device's amg_grid_add_solve with
 * async_schedule = AMG_SCHED_ROUND_ROBIN yields at the same points.
 * sched 2 / 3 (converge LOCAL): the race's extreme speed ratios -- the token
 * starts at the finest (2) / coarsest (3) grid and a grid keeps it through its
 * main loop, handing it on (ascending / descending) only where a reference rank
 * would block (CheckInFlight's wait, AsyncRecvCleanup, the final waits): each
 * grid runs its cycles as if the others were stalled. */
typedef struct or_rec {
   double *pay;          /* payload copy (send) */
   int n;
   double flag;          /* the done flag slot data[len] */
   int matched, consumed;
   struct or_rec *peer;  /* receive: the matched send */
   struct or_rec *qnext; /* mailbox queue */
   struct or_rec *all;   /* every record (freed at the end) */
} or_rec;

typedef struct {
   int G;
   or_rec **sendq, **recvq; /* [src * G + dst] unmatched sends / posted receives */
   or_rec *all;
   omp_lock_t lock;
   /* round robin */
   int sched, token;
   int *finished;
} or_mbox;

static or_rec *mb_new(or_mbox *M)
{
   or_rec *r = (or_rec *)calloc(1, sizeof(or_rec));
   r->all = M->all;
   M->all = r;
   return r;
}

static void q_push(or_rec **q, or_rec *r)
{
   r->qnext = NULL;
   while (*q) q = &(*q)->qnext;
   *q = r;
}

static or_rec *q_pop(or_rec **q)
{
   or_rec *r = *q;
   if (r) *q = r->qnext;
   return r;
}

static or_rec *mb_isend(or_mbox *M, int src, int dst, const double *data, int n, double flag)
{
   omp_set_lock(&M->lock);
   or_rec *s = mb_new(M);
   s->pay = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
   memcpy(s->pay, data, (size_t)n * sizeof(double));
   s->n = n;
   s->flag = flag;
   or_rec *r = q_pop(&M->recvq[src * M->G + dst]);
   if (r) {
      r->matched = s->matched = 1;
      r->peer = s;
   } else {
      q_push(&M->sendq[src * M->G + dst], s);
   }
   omp_unset_lock(&M->lock);
   return s;
}

static or_rec *mb_irecv(or_mbox *M, int dst, int src)
{
   omp_set_lock(&M->lock);
   or_rec *r = mb_new(M);
   or_rec *s = q_pop(&M->sendq[src * M->G + dst]);
   if (s) {
      r->matched = s->matched = 1;
      r->peer = s;
   } else {
      q_push(&M->recvq[src * M->G + dst], r);
   }
   omp_unset_lock(&M->lock);
   return r;
}

static int mb_matched(or_mbox *M, or_rec *r)
{
   omp_set_lock(&M->lock);
   const int m = r->matched;
   omp_unset_lock(&M->lock);
   return m;
}

static void mb_consume(or_mbox *M, or_rec *r)
{
   omp_set_lock(&M->lock);
   r->peer->consumed = 1;
   omp_unset_lock(&M->lock);
}

static int mb_sent(or_mbox *M, or_rec *s)
{
   omp_set_lock(&M->lock);
   const int c = s->consumed;
   omp_unset_lock(&M->lock);
   return c;
}

/* round robin: hand the token to the next unfinished grid and wait for it */
static void rr_wait(or_mbox *M, int g)
{
   if (!M->sched) return;
   while (__atomic_load_n(&M->token, __ATOMIC_ACQUIRE) != g) sched_yield();
}

static void rr_pass(or_mbox *M, int g, int finished)
{
   if (!M->sched) return;
   if (finished) M->finished[g] = 1;
   int nx = -1;
   for (int q = 1; q <= M->G; q++) {
      const int c = M->sched == 3 ? ((g - q) % M->G + M->G) % M->G : (g + q) % M->G;
      if (!M->finished[c]) {
         nx = c;
         break;
      }
   }
   __atomic_store_n(&M->token, nx, __ATOMIC_RELEASE);
}

static void rr_yield(or_mbox *M, int g)
{
   if (!M->sched) return;
   rr_pass(M, g, 0);
   rr_wait(M, g);
}

/* the end of a main-loop iteration: round robin hands the token on, the
 * sequential schedules keep it */
static void rr_yield_main(or_mbox *M, int g)
{
   if (M->sched == 1) rr_yield(M, g);
}

enum { OR_MSG_ACCUMULATE = 0, OR_MSG_WRITE = 1 };

/* DMEM_CommData of one grid: the other grids, all rows overlapping */
typedef struct {
   int send, np, len, max_inflight;
   int *procs, *done_flags, *recv_flags, *message_count;
   double **data;
   or_rec **requests;
   int *num_inflight, *next_inflight;
   double ***data_inflight;
   or_rec ***requests_inflight;
   int **inflight_flags;
} or_cls;

typedef struct {
   or_hier *H;
   or_mbox *M;
   int k, L, n0;
   int converge_local, semi, save, accel, cheby_mine;
   double tol, mu, delta;
   int num_cycles;
   or_cls send, recv;
   /* iter / comm flags (DMEM_AllData) */
   int all_done_flag, outside_done_flag, grid_done_flag, converge_flag, r_local_converge_flag, cycle;
   double r0_norm2, r_local;
   long long sent, rcvd;
   /* numerics */
   double *x, *b, *r, *y, *e, *d, *z, *vt;
   double **F, **U;
   double *sc, *nsc; /* DMEM_AddSmooth scales of level k */
   double *lu;
   int *piv, nc;
   double acc_state[2];
   int acc_cycle;
} or_grid;

static void cls_init(or_cls *c, int send, int G, int me, int n0, int mi)
{
   memset(c, 0, sizeof(*c));
   c->send = send;
   c->np = G - 1;
   c->len = n0;
   c->max_inflight = mi;
   c->procs = (int *)malloc(G * sizeof(int));
   for (int p = 0, i = 0; p < G; p++)
      if (p != me) c->procs[i++] = p;
   c->done_flags = (int *)calloc(G, sizeof(int));
   c->recv_flags = (int *)calloc(G, sizeof(int));
   c->message_count = (int *)calloc(G, sizeof(int));
   c->data = (double **)malloc(G * sizeof(double *));
   for (int i = 0; i < c->np; i++) c->data[i] = dvec(n0 + 2);
   c->requests = (or_rec **)calloc(G, sizeof(or_rec *));
   if (send) {
      c->num_inflight = (int *)calloc(G, sizeof(int));
      c->next_inflight = (int *)calloc(G, sizeof(int));
      c->data_inflight = (double ***)malloc(G * sizeof(double **));
      c->requests_inflight = (or_rec ***)malloc(G * sizeof(or_rec **));
      c->inflight_flags = (int **)malloc(G * sizeof(int *));
      for (int i = 0; i < c->np; i++) {
         c->data_inflight[i] = (double **)malloc(mi * sizeof(double *));
         for (int j = 0; j < mi; j++) c->data_inflight[i][j] = dvec(n0 + 2);
         c->requests_inflight[i] = (or_rec **)calloc(mi, sizeof(or_rec *));
         c->inflight_flags[i] = (int *)calloc(mi, sizeof(int));
      }
   }
}

static void cls_free(or_cls *c)
{
   for (int i = 0; i < c->np; i++) {
      free(c->data[i]);
      if (c->send) {
         for (int j = 0; j < c->max_inflight; j++) free(c->data_inflight[i][j]);
         free(c->data_inflight[i]);
         free(c->requests_inflight[i]);
         free(c->inflight_flags[i]);
      }
   }
   free(c->procs); free(c->done_flags); free(c->recv_flags); free(c->message_count); free(c->data);
   free(c->requests);
   if (c->send) {
      free(c->num_inflight); free(c->next_inflight); free(c->data_inflight); free(c->requests_inflight);
      free(c->inflight_flags);
   }
}

/* CheckInFlight (DMEM_Comm.cpp:25-67) */
static void check_inflight(or_grid *g, or_cls *c, int i)
{
   while (1) {
      int break_flag = 0;
      if (g->all_done_flag == 0)
         break_flag = 1;
      else if (c->num_inflight[i] < c->max_inflight)
         break;
      for (int j = 0; j < c->max_inflight; j++) {
         if (c->inflight_flags[i][j] == 1) {
            if (mb_sent(g->M, c->requests_inflight[i][j])) {
               c->inflight_flags[i][j] = 0;
               c->num_inflight[i]--;
               if (j < c->next_inflight[i]) c->next_inflight[i] = j;
               if (g->all_done_flag == 1) {
                  break_flag = 1;
                  break;
               }
            }
         } else if (g->all_done_flag == 1) {
            break_flag = 1;
            break;
         }
      }
      if (break_flag) break;
      rr_yield(g->M, g->k);
   }
}

/* SetNextInFlight (DMEM_Comm.cpp:69-79) */
static void set_next_inflight(or_cls *c, int i)
{
   for (int j = 0; j < c->max_inflight; j++)
      if (c->inflight_flags[i][j] == 0) {
         c->next_inflight[i] = j;
         return;
      }
   c->next_inflight[i] = c->max_inflight;
}

/* SendRecv, asynchronous outside classes (DMEM_Comm.cpp:81-348) */
static int send_recv(or_grid *g, or_cls *c, double *v, int op)
{
   int return_flag = 0;
   const int len = c->len;
   for (int i = 0; i < c->np; i++) {
      const int ip = c->procs[i];
      c->recv_flags[i] = 0;
      if (c->send) {
         if (c->done_flags[i] >= 2) continue;
         if (op == OR_MSG_WRITE)
            memcpy(c->data[i], v, (size_t)len * sizeof(double));
         else
            for (int j = 0; j < len; j++) c->data[i][j] += 1.0 * v[j];
         check_inflight(g, c, i);
         if (c->num_inflight[i] >= c->max_inflight) continue;
         const int nx = c->next_inflight[i];
         double *slot = c->data_inflight[i][nx];
         memcpy(slot, c->data[i], (size_t)len * sizeof(double));
         for (int j = 0; j < len; j++) c->data[i][j] = 0.0;
         slot[len] = 0.0;
         if (g->grid_done_flag == 1) {
            slot[len] = 1.0;
            if (g->converge_local) {
               c->done_flags[i] = 2;
            } else {
               c->done_flags[i] = 1;
               if (g->all_done_flag == 1) {
                  c->done_flags[i] = 2;
                  slot[len] = 2.0;
               }
            }
         }
         c->requests_inflight[i][nx] = mb_isend(g->M, g->k, ip, slot, len, slot[len]);
         c->inflight_flags[i][nx] = 1;
         c->num_inflight[i]++;
         set_next_inflight(c, i);
         c->message_count[i]++;
         g->sent++;
         return_flag = 1;
      } else {
         if (c->done_flags[i] >= 2) continue;
         while (1) {
            or_rec *rq = c->requests[i];
            if (!mb_matched(g->M, rq)) break;
            c->message_count[i]++;
            g->rcvd++;
            const or_rec *s = rq->peer;
            for (int j = 0; j < len; j++) v[j] += 1.0 * s->pay[j];
            const double fl = s->flag;
            mb_consume(g->M, rq);
            if (g->converge_local) {
               if (fl == 1.0) {
                  c->done_flags[i] = 2;
                  break;
               }
            } else {
               if (fl == 1.0) {
                  c->done_flags[i] = 1;
               } else if (fl == 2.0) {
                  c->done_flags[i] = 2;
                  break;
               }
            }
            c->requests[i] = mb_irecv(g->M, g->k, ip);
            c->recv_flags[i] = 1;
            return_flag = 1;
            if (g->semi && g->all_done_flag == 0) break;
         }
      }
   }
   return return_flag;
}

/* AddCycle (DMEM_Add.cpp:180-329), NUMLEVELS_INTERPOLANTS, grid k; u = U[0] */
static void add_cycle(or_grid *g)
{
   or_hier *H = g->H;
   const int k = g->k, L = g->L;
   memcpy(g->F[0], g->r, (size_t)g->n0 * sizeof(double));
   for (int l = 0; l < k; l++) or_smem_matvec(&H->R[l], g->F[l], g->F[l + 1], 0, H->n[l + 1]);
   if (k == L - 1) {
      /* hypre_GaussElimSolve: A_c u = f_c, dense LU with partial pivoting */
      const int n = g->nc;
      double *x = g->U[k];
      memcpy(x, g->F[k], (size_t)n * sizeof(double));
      for (int c = 0; c < n; c++)
         if (g->piv[c] != c) {
            double t = x[c];
            x[c] = x[g->piv[c]];
            x[g->piv[c]] = t;
         }
      for (int i = 0; i < n; i++)
         for (int j = 0; j < i; j++) x[i] -= g->lu[(size_t)i * n + j] * x[j];
      for (int i = n - 1; i >= 0; i--) {
         for (int j = i + 1; j < n; j++) x[i] -= g->lu[(size_t)i * n + j] * x[j];
         const double dd = g->lu[(size_t)i * n + i];
         x[i] = dd != 0.0 ? x[i] / dd : 0.0;
      }
   } else {
      /* DMEM_AddSmooth (DMEM_Smooth.cpp:574-638), simple_jacobi_flag = -1:
       * u = 0 + f ./ s;  v = A u;  u = 2 u;  u = u + v ./ (-s) */
      const int n = H->n[k];
      double *u = g->U[k];
      for (int i = 0; i < n; i++) u[i] = 0.0;
      for (int i = 0; i < n; i++) u[i] += g->F[k][i] / g->sc[i];
      or_smem_matvec(&H->A[k], u, g->vt, 0, n);
      for (int i = 0; i < n; i++) u[i] = 2.0 * u[i];
      for (int i = 0; i < n; i++) u[i] += g->vt[i] / g->nsc[i];
   }
   for (int l = k - 1; l >= 0; l--) or_smem_matvec(&H->P[l], g->U[l + 1], g->U[l], 0, H->n[l]);
   if (g->accel != OR_NO_ACCEL) {
      /* :320-324 DMEM_ChebyUpdate(gridk.d, U_array[0]), async branch */
      or_dmem_cheby_update(g->d, g->U[0], g->n0, g->acc_cycle, g->accel, g->cheby_mine ? OR_CHEBY_GRID : OR_CHEBY_OTHER,
                           g->mu, g->delta, g->acc_state);
      g->acc_cycle++;
   }
}

/* r = b - A x (DMEM_AddResidual_LocalRes, :530-556); returns r.r */
static double add_residual(or_grid *g)
{
   or_smem_spgemv(&g->H->A[0], g->x, g->b, -1.0, 1.0, g->r, 0, g->n0);
   double s = 0.0;
   for (int i = 0; i < g->n0; i++) s += g->r[i] * g->r[i];
   return s;
}

/* DMEM_AddCheckComm (:460-528) */
static void add_check_comm(or_grid *g)
{
   for (int i = 0; i < g->n0; i++) g->e[i] = 0.0;
   const int recv_flag = send_recv(g, &g->recv, g->e, OR_MSG_ACCUMULATE);
   if (recv_flag == 1) {
      for (int i = 0; i < g->n0; i++) g->x[i] += 1.0 * g->e[i];
      if (g->accel != OR_NO_ACCEL && g->cheby_mine)
         for (int i = 0; i < g->n0; i++) g->d[i] += 1.0 * g->e[i];
   }
   for (int i = 0; i < g->send.np; i++) check_inflight(g, &g->send, i);
}

/* DMEM_AddCorrect_LocalRes (:391-458) */
static void add_correct(or_grid *g)
{
   double *u = g->U[0];
   for (int i = 0; i < g->n0; i++) g->y[i] += 1.0 * u[i];
   if (g->converge_flag == 1 || g->cycle % g->save == 0) {
      send_recv(g, &g->send, g->y, OR_MSG_ACCUMULATE);
      for (int i = 0; i < g->n0; i++) g->y[i] = 0.0;
   }
   for (int i = 0; i < g->n0; i++) g->x[i] += 1.0 * u[i];
   add_check_comm(g);
}

static int all_flags(const or_cls *c, int v)
{
   for (int i = 0; i < c->np; i++)
      if (c->done_flags[i] != v) return 0;
   return 1;
}

/* CheckConverge (:906-944) with DMEM_CheckOutsideDoneFlag (:795-803) */
static int check_converge(or_grid *g)
{
   if (!g->converge_local) {
      if (g->all_done_flag == 0) {
         if (g->grid_done_flag == 0 && (g->cycle >= g->num_cycles - 1 || g->r_local_converge_flag == 1))
            g->grid_done_flag = 1;
         if (g->grid_done_flag == 1 && g->outside_done_flag == 0) {
            int ok = 1;
            for (int i = 0; i < g->send.np; i++)
               if (g->send.done_flags[i] == 0) ok = 0;
            for (int i = 0; i < g->recv.np; i++)
               if (g->recv.done_flags[i] == 0) ok = 0;
            if (ok) g->outside_done_flag = 1;
         }
         return 0;
      }
      return 1;
   }
   if (g->cycle >= g->num_cycles - 1 || g->r_local_converge_flag == 1) {
      g->grid_done_flag = 1;
      return 1;
   }
   return 0;
}

/* the grid's solve: DMEM_Add's asynchronous branch (:20-178) */
static void grid_run(or_grid *g)
{
   or_mbox *M = g->M;
   for (int i = 0; i < g->n0; i++) g->y[i] = g->e[i] = g->d[i] = 0.0;
   g->r0_norm2 = sqrt(add_residual(g));
   if (g->r0_norm2 == 0.0) g->r0_norm2 = 1.0;
   g->r_local = 1.0;
   for (int i = 0; i < g->recv.np; i++) g->recv.requests[i] = mb_irecv(M, g->k, g->recv.procs[i]); /* AsyncStart */
   rr_wait(M, g->k);
   while (1) {
      g->converge_flag = check_converge(g);
      add_cycle(g);
      add_correct(g);
      const double rr = add_residual(g);
      if (g->all_done_flag == 0 && !g->semi) {
         /* AddResNorm: InnerProdFlag over the grid (one rank: local) */
         g->r_local = sqrt(rr) / g->r0_norm2;
         if (g->r_local < g->tol) g->r_local_converge_flag = 1;
         if (g->outside_done_flag == 1) g->all_done_flag = 1;
      }
      g->cycle++;
      rr_yield_main(M, g->k);
      if (g->converge_flag == 1) break;
   }
   /* AsyncEnd: AsyncRecvCleanup (:827-890) */
   for (int i = 0; i < g->n0; i++) g->e[i] = 0.0;
   double *zero = dvec(g->n0);
   while (1) {
      if (g->converge_local ? (all_flags(&g->recv, 2) && all_flags(&g->send, 2)) : all_flags(&g->recv, 2)) break;
      send_recv(g, &g->recv, g->e, OR_MSG_ACCUMULATE);
      if (g->converge_local) send_recv(g, &g->send, zero, OR_MSG_ACCUMULATE);
      rr_yield(M, g->k);
   }
   free(zero);
   for (int i = 0; i < g->n0; i++) g->x[i] += 1.0 * g->e[i];
   /* CompleteInFlight (DMEM_Comm.cpp:11-23) */
   for (int i = 0; i < g->send.np; i++)
      for (int j = 0; j < g->send.max_inflight; j++)
         if (g->send.inflight_flags[i][j] == 1) {
            while (!mb_sent(M, g->send.requests_inflight[i][j])) {
               if (M->sched)
                  rr_yield(M, g->k);
               else
                  sched_yield();
            }
            g->send.inflight_flags[i][j] = 0;
         }
   rr_pass(M, g->k, 1);
}

int or_dmem_add(or_hier *H, const double *b, double *x_out, int sched, int converge_type, int async_type,
                int max_inflight, int save_divisor, double tol, int accel, int cheby_grid, double mu, double delta,
                int *cycles, double *relres, long long *messages)
{
   const int L = H->L, n0 = H->n[0], G = L;
   if (G < 2 || max_inflight < 1) return -1;
   if (async_type == OR_SEMI_ASYNC && converge_type == OR_CONVERGE_GLOBAL) return -1; /* :346-358 */
   if (sched < 0 || sched > 3 || (sched >= 2 && converge_type != OR_CONVERGE_LOCAL)) return -1;
   or_mbox M;
   memset(&M, 0, sizeof(M));
   M.G = G;
   M.sendq = (or_rec **)calloc((size_t)G * G, sizeof(or_rec *));
   M.recvq = (or_rec **)calloc((size_t)G * G, sizeof(or_rec *));
   omp_init_lock(&M.lock);
   M.sched = sched;
   M.token = sched == 3 ? G - 1 : 0;
   M.finished = (int *)calloc(G, sizeof(int));
   or_grid *gs = (or_grid *)calloc(G, sizeof(or_grid));
   const int cg = cheby_grid < L - 1 ? cheby_grid : L - 1; /* DMEM_Setup.cpp:1911-1913 */
   for (int k = 0; k < G; k++) {
      or_grid *g = &gs[k];
      g->H = H;
      g->M = &M;
      g->k = k;
      g->L = L;
      g->n0 = n0;
      g->converge_local = converge_type == OR_CONVERGE_LOCAL;
      g->semi = async_type == OR_SEMI_ASYNC;
      g->save = save_divisor > 0 ? save_divisor : 1;
      g->tol = tol;
      g->num_cycles = H->o.num_cycles;
      g->accel = accel;
      g->cheby_mine = k == cg;
      g->mu = mu;
      g->delta = delta;
      g->acc_state[0] = mu;
      g->acc_state[1] = 1.0;
      cls_init(&g->send, 1, G, k, n0, max_inflight);
      cls_init(&g->recv, 0, G, k, n0, max_inflight);
      g->x = dvec(n0); g->b = dvec(n0); g->r = dvec(n0); g->y = dvec(n0); g->e = dvec(n0); g->d = dvec(n0);
      memcpy(g->b, b, (size_t)n0 * sizeof(double));
      g->F = (double **)malloc((k + 1) * sizeof(double *));
      g->U = (double **)malloc((k + 1) * sizeof(double *));
      for (int l = 0; l <= k; l++) {
         g->F[l] = dvec(H->n[l]);
         g->U[l] = dvec(H->n[l]);
      }
      g->vt = dvec(H->n[k]);
      if (k == L - 1) {
         /* hypre_GaussElimSetup: the coarsest operator dense, LU with partial pivoting */
         const or_csr *A = &H->A[k];
         const int n = A->nrows;
         g->nc = n;
         g->lu = (double *)calloc((size_t)n * n, sizeof(double));
         g->piv = (int *)calloc(n, sizeof(int));
         for (int i = 0; i < n; i++)
            for (int q = A->i[i]; q < A->i[i + 1]; q++) g->lu[(size_t)i * n + A->j[q]] += A->data[q];
         for (int c = 0; c < n; c++) {
            int p = c;
            for (int i = c + 1; i < n; i++)
               if (fabs(g->lu[(size_t)i * n + c]) > fabs(g->lu[(size_t)p * n + c])) p = i;
            g->piv[c] = p;
            if (p != c)
               for (int j = 0; j < n; j++) {
                  double t = g->lu[(size_t)c * n + j];
                  g->lu[(size_t)c * n + j] = g->lu[(size_t)p * n + j];
                  g->lu[(size_t)p * n + j] = t;
               }
            const double dd = g->lu[(size_t)c * n + c];
            if (dd == 0.0) continue;
            for (int i = c + 1; i < n; i++) {
               const double m = (g->lu[(size_t)i * n + c] /= dd);
               for (int j = c + 1; j < n; j++) g->lu[(size_t)i * n + j] -= m * g->lu[(size_t)c * n + j];
            }
         }
      } else {
         /* wJacobi_scale_gridk / symmwJacobi_scale_gridk (DMEM_Setup.cpp:471-482) */
         const or_csr *A = &H->A[k];
         const int n = A->nrows;
         g->sc = dvec(n);
         g->nsc = dvec(n);
         for (int i = 0; i < n; i++) {
            const double a = A->data[A->i[i]];
            g->sc[i] = a == 0.0 ? 1.0 : a / H->o.smooth_weight;
            g->nsc[i] = -g->sc[i];
         }
      }
   }
#pragma omp parallel num_threads(G)
   grid_run(&gs[omp_get_thread_num()]);
   for (int k = 0; k < G; k++) {
      or_grid *g = &gs[k];
      const double rr = add_residual(g);
      memcpy(x_out + (size_t)k * n0, g->x, (size_t)n0 * sizeof(double));
      if (cycles) cycles[k] = g->cycle;
      if (relres) relres[k] = sqrt(rr) / g->r0_norm2;
      if (messages) {
         messages[2 * k] = g->sent;
         messages[2 * k + 1] = g->rcvd;
      }
      cls_free(&g->send);
      cls_free(&g->recv);
      free(g->x); free(g->b); free(g->r); free(g->y); free(g->e); free(g->d); free(g->vt);
      for (int l = 0; l <= k; l++) {
         free(g->F[l]);
         free(g->U[l]);
      }
      free(g->F); free(g->U); free(g->sc); free(g->nsc); free(g->lu); free(g->piv);
   }
   while (M.all) {
      or_rec *r = M.all;
      M.all = r->all;
      free(r->pay);
      free(r);
   }
   omp_destroy_lock(&M.lock);
   free(M.sendq); free(M.recvq); free(M.finished); free(gs);
   return 0;
}
