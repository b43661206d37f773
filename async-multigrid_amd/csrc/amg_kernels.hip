// amg_kernels.hip -- hand-written gfx950 kernels of the AMG solve phase.
//
// Hot kernel: the CSR "tile" kernel.  A 256-lane workgroup owns 256
// consecutive rows (one row per lane).  The workgroup streams the tile's
// contiguous [rowptr[r0], rowptr[r0+256]) slice of col/val with 16-byte
// vector loads (int4 col, 2 x double2 val per lane: fully coalesced), gathers
// x[col] for those entries, and writes the rounded products a_ij*x_j into an
// LDS chunk.  Each lane then accumulates its own row's products from LDS in
// the CSR order.  This keeps every HBM stream coalesced while reproducing
// the reference's sequential per-row sum (`tempx += A_data[jj]*x[A_j[jj]]`)
// bit for bit: no re-association, products rounded before accumulation (the
// library is built with -ffp-contract=off).  Rows of any length work: a tile
// whose slice exceeds one LDS chunk is processed in several chunks while each
// lane carries its partial sum in a register.
//
// The kernels are HBM-bound (≈0.17 flop/byte); no MFMA.
#include "amg_internal.h"

#include <algorithm>

namespace amgk {

// ---------------------------------------------------------------------------
// deterministic workgroup reduction of one double per lane (256 lanes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double block_sum_256(double v, double *lds4)
{
#pragma unroll
   for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
   const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
   __syncthreads();
   if (lane == 0) lds4[wid] = v;
   __syncthreads();
   double s = 0.0;
   if (threadIdx.x == 0) s = ((lds4[0] + lds4[1]) + lds4[2]) + lds4[3];
   return s;
}

// ---------------------------------------------------------------------------
// CSR tile kernel
// ---------------------------------------------------------------------------
template <int NEG, bool NEED_DIAG, class Epi>
__global__ __launch_bounds__(AMG_TILE_ROWS) void csr_tile_kernel(
   const int *__restrict__ rowptr, const int *__restrict__ col, const double *__restrict__ val,
   const double *__restrict__ x, int rb, int re, Epi epi, double *__restrict__ partials)
{
   __shared__ __attribute__((aligned(16))) double prod[AMG_CHUNK];
   __shared__ double red[4];
   const int r0 = rb + blockIdx.x * AMG_TILE_ROWS;
   const int r1 = min(r0 + AMG_TILE_ROWS, re);
   const int row = r0 + (int)threadIdx.x;
   const bool active = row < r1;
   const int tb = rowptr[r0];
   const int te = rowptr[r1];
   int rs = 0, rend = 0;
   if (active) {
      rs = rowptr[row];
      rend = rowptr[row + 1];
   }
   double acc = active ? epi.init(row) : 0.0;
   const int base = tb & ~3;
   for (int cs = base; cs < te; cs += AMG_CHUNK) {
      const int ce = min(cs + AMG_CHUNK, te);
      for (int k = cs + 4 * (int)threadIdx.x; k < ce; k += 4 * AMG_TILE_ROWS) {
         const int4 c4 = *reinterpret_cast<const int4 *>(col + k);
         const double2 v01 = *reinterpret_cast<const double2 *>(val + k);
         const double2 v23 = *reinterpret_cast<const double2 *>(val + k + 2);
         const double x0 = x[c4.x];
         const double x1 = x[c4.y];
         const double x2 = x[c4.z];
         const double x3 = x[c4.w];
         double2 p01, p23;
         p01.x = v01.x * x0;
         p01.y = v01.y * x1;
         p23.x = v23.x * x2;
         p23.y = v23.y * x3;
         double2 *dst = reinterpret_cast<double2 *>(prod + (k - cs));
         dst[0] = p01;
         dst[1] = p23;
      }
      __syncthreads();
      const int a = max(rs, cs), e = min(rend, ce);
      for (int k = a; k < e; ++k) {
         if (NEG)
            acc -= prod[k - cs];
         else
            acc += prod[k - cs];
      }
      __syncthreads();
   }
   double out = 0.0;
   if (active) {
      double d = 0.0;
      if (NEED_DIAG) d = val[rs];
      out = epi.finish(row, acc, d);
   }
   if (partials) {
      const double s = block_sum_256(out * out, red);
      if (threadIdx.x == 0) partials[blockIdx.x] = s;
   }
}

// y = SpGEMV epilogue (SMEM_MatVec.cpp:140-258)
struct EpiGemv {
   const double *b;
   double *y;
   int imode;
   int scale;
   double alpha, temp;
   __device__ __forceinline__ double init_val(int i) const
   {
      switch (imode) {
      case 0: return 0.0;
      case 1: return b[i];
      case 2: return -b[i];
      case 3: return b[i] * temp;
      default: return -b[i] * temp;
      }
   }
   __device__ __forceinline__ double init(int i) const { return init_val(i); }
   __device__ __forceinline__ double finish(int i, double acc, double) const
   {
      const double v = scale ? alpha * acc : acc;
      y[i] = v;
      return v;
   }
};

// Jacobi sweep epilogue (SMEM_Smooth.cpp:35-45): res = f - sum; u_new = u + w*res/a
struct EpiJacobi {
   const double *f;
   const double *x;
   double *out;
   double omega;
   __device__ __forceinline__ double init(int i) const { return f[i]; }
   __device__ __forceinline__ double finish(int i, double res, double a) const
   {
      const double xi = x[i];
      const double v = (a != 0.0) ? xi + omega * res / a : xi;
      out[i] = v;
      return v;
   }
};

// L1 Jacobi sweep epilogue (SMEM_Smooth.cpp:122-130): u_new = u + res/l1
struct EpiL1Jacobi {
   const double *f;
   const double *x;
   const double *l1;
   double *out;
   __device__ __forceinline__ double init(int i) const { return f[i]; }
   __device__ __forceinline__ double finish(int i, double res, double) const
   {
      const double v = x[i] + res / l1[i];
      out[i] = v;
      return v;
   }
};

int tile_blocks(int rb, int re) { return (re - rb + AMG_TILE_ROWS - 1) / AMG_TILE_ROWS; }

Gemv gemv_mode(double alpha, double beta)
{
   Gemv g;
   const double temp = beta / alpha;
   const int acase = (alpha == 1) ? 0 : (alpha == -1) ? 1 : 2;
   if (temp == 0)
      g.init = 0;
   else if (temp == -1)
      g.init = (acase == 1) ? 1 : 2;
   else if (temp == 1)
      g.init = (acase == 1) ? 2 : 1;
   else
      g.init = (acase == 1) ? 4 : 3;
   g.negacc = (acase == 1);
   g.scale = (acase == 2);
   g.alpha = alpha;
   g.temp = temp;
   return g;
}

void spgemv(hipStream_t s, const amg_mat *A, const double *x, const double *b, const Gemv &g,
            double *y, int rb, int re, double *partials)
{
   if (re <= rb) return;
   EpiGemv e{b, y, g.init, g.scale, g.alpha, g.temp};
   const int nb = tile_blocks(rb, re);
   if (g.negacc)
      csr_tile_kernel<1, false, EpiGemv>
         <<<nb, AMG_TILE_ROWS, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, partials);
   else
      csr_tile_kernel<0, false, EpiGemv>
         <<<nb, AMG_TILE_ROWS, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, partials);
}

void jacobi_sweep(hipStream_t s, const amg_mat *A, const double *f, const double *x,
                  const double *l1, double omega, double *out, int rb, int re)
{
   if (re <= rb) return;
   const int nb = tile_blocks(rb, re);
   if (l1) {
      EpiL1Jacobi e{f, x, l1, out};
      csr_tile_kernel<1, false, EpiL1Jacobi>
         <<<nb, AMG_TILE_ROWS, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, nullptr);
   } else {
      EpiJacobi e{f, x, out, omega};
      csr_tile_kernel<1, true, EpiJacobi>
         <<<nb, AMG_TILE_ROWS, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, nullptr);
   }
}

// ---------------------------------------------------------------------------
// element-wise kernels
// ---------------------------------------------------------------------------
static inline int ew_blocks(int n)
{
   const int b = (n + 255) / 256;
   return std::max(1, std::min(b, 65536));
}

#define EW_LOOP(i, rb, re)                                                                  \
   for (int i = (rb) + blockIdx.x * blockDim.x + threadIdx.x; i < (re);                    \
        i += gridDim.x * blockDim.x)

// SMEM_Smooth.cpp:25-29 / SEQ_Smooth.cpp:24-29 / SMEM_Smooth.cpp:114-116 / SEQ_Smooth.cpp:67-72
__global__ void jacobi_zero_k(const double *__restrict__ diag, const double *__restrict__ f,
                              const double *__restrict__ l1, double omega, double *__restrict__ u,
                              int rb, int re, int variant)
{
   EW_LOOP(i, rb, re)
   {
      const double a = diag[i];
      if (l1) {
         if (variant == 0)
            u[i] = f[i] / l1[i];
         else if (a != 0.0)
            u[i] += f[i] / l1[i];
      } else if (a != 0.0) {
         if (variant == 0)
            u[i] = omega * f[i] / a;
         else
            u[i] += omega * f[i] / a;
      }
   }
}

void jacobi_zero(hipStream_t s, const double *diag, const double *f, const double *l1,
                 double omega, double *u, int rb, int re, int variant)
{
   if (re <= rb) return;
   jacobi_zero_k<<<ew_blocks(re - rb), 256, 0, s>>>(diag, f, l1, omega, u, rb, re, variant);
}

__global__ void jacobi_from_res_k(const double *__restrict__ diag, const double *__restrict__ r,
                                  const double *__restrict__ l1, double omega,
                                  double *__restrict__ u, int rb, int re)
{
   EW_LOOP(i, rb, re)
   {
      if (l1) {
         u[i] = u[i] + r[i] / l1[i];
      } else {
         const double a = diag[i];
         if (a != 0.0) u[i] = u[i] + omega * r[i] / a;
      }
   }
}

void jacobi_from_residual(hipStream_t s, const double *diag, const double *r, const double *l1,
                          double omega, double *u, int rb, int re)
{
   if (re <= rb) return;
   jacobi_from_res_k<<<ew_blocks(re - rb), 256, 0, s>>>(diag, r, l1, omega, u, rb, re);
}

// hybrid Jacobi / Gauss-Seidel, one lane per block (SMEM_Smooth.cpp:265-304 / 548-585)
__global__ void hybrid_jgs_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                             const double *__restrict__ val, const double *__restrict__ f,
                             double *u, const double *__restrict__ u_prev,
                             const int *__restrict__ blk, int nblk,
                             const double *__restrict__ ds, double weight, int zero, int reverse)
{
   // A lane re-reads values of u it stored earlier in this sweep.  Plain
   // global loads may be served by a stale line of the CU's vector L1 (gfx950
   // stores write through to L2 without refreshing L1), so every access to u
   // is a relaxed atomic: same-location coherence then holds by the memory
   // model (agent-scope loads are L2-served).
   auto ld = [u](int k) { return __hip_atomic_load(u + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
   auto st = [u](int k, double v) {
      __hip_atomic_store(u + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   };
   const int b = blockIdx.x * blockDim.x + threadIdx.x;
   if (b >= nblk) return;
   const int ns = blk[b], ne = blk[b + 1];
   if (zero)
      for (int i = ns; i < ne; i++) st(i, 0.0);
   for (int c = 0; c < ne - ns; c++) {
      const int i = reverse ? ne - 1 - c : ns + c;
      const int rs = rowptr[i], rend = rowptr[i + 1];
      const double a = val[rs];
      if (a == 0.0) continue;
      const double d = ds ? ds[i] : a;
      double res = f[i];
      for (int jj = rs; jj < rend; jj++) {
         const int ii = col[jj];
         if (ii >= ns && ii < ne)
            res -= val[jj] * ld(ii);
         else if (!zero)
            res -= val[jj] * u_prev[ii];
      }
      if (zero)
         st(i, weight * res / d);
      else
         st(i, ld(i) + weight * res / d);
   }
}

void hybrid_jgs(hipStream_t s, const amg_mat *A, const double *f, double *u, const double *u_prev,
                const int *d_blk, int nblk, const double *diag_scale, double weight, int zero,
                int reverse)
{
   if (nblk <= 0) return;
   const int tpb = 64;
   hybrid_jgs_k<<<(nblk + tpb - 1) / tpb, tpb, 0, s>>>(A->rowptr, A->col, A->val, f, u, u_prev,
                                                       d_blk, nblk, diag_scale, weight, zero,
                                                       reverse);
}

// y = A^T x in SMEM_Sync_Parfor_MatVecT order (SMEM_MatVec.cpp:42-57): for each
// output j the contributions of source rows are summed per static chunk of
// T threads, then the chunk sums are added in thread order.  T = 1 is
// SEQ_MatVecT (SEQ_MatVec.cpp:40-45).
__global__ void matvec_t_chunked_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                                   const double *__restrict__ val, const double *__restrict__ x,
                                   double *__restrict__ y, int m, int n_src, int T)
{
   EW_LOOP(j, 0, m)
   {
      const int q = n_src / T, rem = n_src % T;
      const int split = rem * (q + 1);
      double total = 0.0, part = 0.0;
      int cur = -1;
      for (int k = rowptr[j]; k < rowptr[j + 1]; k++) {
         const int i = col[k];
         const int t = (i < split) ? i / (q + 1) : rem + (i - split) / (q > 0 ? q : 1);
         if (t != cur) {
            if (cur >= 0) total += part;
            part = 0.0;
            cur = t;
         }
         part += val[k] * x[i];
      }
      if (cur >= 0) total += part;
      y[j] = total;
   }
}

void matvec_t_chunked(hipStream_t s, const amg_mat *AT, const double *x, double *y, int n_src,
                      int T)
{
   if (AT->nrows <= 0) return;
   matvec_t_chunked_k<<<ew_blocks(AT->nrows), 256, 0, s>>>(AT->rowptr, AT->col, AT->val, x, y,
                                                          AT->nrows, n_src, T < 1 ? 1 : T);
}

__global__ void vcopy_k(const double *__restrict__ x, double *__restrict__ y, int rb, int re)
{
   EW_LOOP(i, rb, re) y[i] = x[i];
}
void vcopy(hipStream_t s, const double *x, double *y, int rb, int re)
{
   if (re > rb) vcopy_k<<<ew_blocks(re - rb), 256, 0, s>>>(x, y, rb, re);
}

__global__ void vset_k(double *__restrict__ y, double a, int rb, int re)
{
   EW_LOOP(i, rb, re) y[i] = a;
}
void vset(hipStream_t s, double *y, double a, int rb, int re)
{
   if (re > rb) vset_k<<<ew_blocks(re - rb), 256, 0, s>>>(y, a, rb, re);
}

__global__ void vaxpy_k(double a, const double *__restrict__ x, double *__restrict__ y, int rb,
                        int re)
{
   EW_LOOP(i, rb, re) y[i] += a * x[i];
}
void vaxpy(hipStream_t s, double a, const double *x, double *y, int rb, int re)
{
   if (re > rb) vaxpy_k<<<ew_blocks(re - rb), 256, 0, s>>>(a, x, y, rb, re);
}

// DMEM_HypreParVector_Ivaxpy DMEM_Misc.cpp:462-478: y += x ./ s
__global__ void vivaxpy_k(const double *__restrict__ x, const double *__restrict__ sc,
                          double *__restrict__ y, int rb, int re)
{
   EW_LOOP(i, rb, re) y[i] += x[i] / sc[i];
}
void vivaxpy(hipStream_t s, const double *x, const double *sc, double *y, int rb, int re)
{
   if (re > rb) vivaxpy_k<<<ew_blocks(re - rb), 256, 0, s>>>(x, sc, y, rb, re);
}

__global__ void vscale_k(double a, double *__restrict__ y, int rb, int re)
{
   EW_LOOP(i, rb, re) y[i] = a * y[i];
}
void vscale(hipStream_t s, double a, double *y, int rb, int re)
{
   if (re > rb) vscale_k<<<ew_blocks(re - rb), 256, 0, s>>>(a, y, rb, re);
}

__global__ void vsub_k(const double *__restrict__ b, const double *__restrict__ y,
                       double *__restrict__ r, int rb, int re)
{
   EW_LOOP(i, rb, re)
   {
      const double ri = b[i] - y[i];
      r[i] = ri;
   }
}
void vsub(hipStream_t s, const double *b, const double *y, double *r, int rb, int re)
{
   if (re > rb) vsub_k<<<ew_blocks(re - rb), 256, 0, s>>>(b, y, r, rb, re);
}

__global__ void vadd_into_k(const double *__restrict__ r, double *__restrict__ u, int rb, int re,
                            int overwrite)
{
   EW_LOOP(i, rb, re)
   {
      if (overwrite)
         u[i] = r[i];
      else
         u[i] += r[i];
   }
}
void vadd_into(hipStream_t s, const double *r, double *u, int rb, int re, int overwrite)
{
   if (re > rb) vadd_into_k<<<ew_blocks(re - rb), 256, 0, s>>>(r, u, rb, re, overwrite);
}

// SMEM_Setup.cpp:222-232: L1 = sum_j |a_ij| in CSR order
__global__ void l1_norms_k(const int *__restrict__ rowptr, const double *__restrict__ val,
                           double *__restrict__ out, int n)
{
   EW_LOOP(i, 0, n)
   {
      double s = 0;
      for (int k = rowptr[i]; k < rowptr[i + 1]; k++) s += fabs(val[k]);
      out[i] = s;
   }
}
void l1_norms(hipStream_t s, const amg_mat *A, double *out)
{
   if (A->nrows > 0) l1_norms_k<<<ew_blocks(A->nrows), 256, 0, s>>>(A->rowptr, A->val, out, A->nrows);
}

// SMEM_Setup.cpp:234-237: A_diag = a_ii / omega
__global__ void a_diag_k(const double *__restrict__ diag, double omega, double *__restrict__ out,
                         int n)
{
   EW_LOOP(i, 0, n) out[i] = diag[i] / omega;
}
void a_diag(hipStream_t s, const double *diag, double omega, double *out, int n)
{
   if (n > 0) a_diag_k<<<ew_blocks(n), 256, 0, s>>>(diag, omega, out, n);
}

__global__ void extract_diag_k(const int *__restrict__ rowptr, const double *__restrict__ val,
                               double *__restrict__ diag, int n)
{
   EW_LOOP(i, 0, n) diag[i] = (rowptr[i + 1] > rowptr[i]) ? val[rowptr[i]] : 0.0;
}
void extract_diag(hipStream_t s, const amg_mat *A)
{
   if (A->nrows > 0)
      extract_diag_k<<<ew_blocks(A->nrows), 256, 0, s>>>(A->rowptr, A->val, A->diag, A->nrows);
}

// symmetric Jacobi scale step: SMEM r *= w/a (SMEM_Smooth.cpp:665); SEQ adds the
// a != 0 test (SEQ_Smooth.cpp:135-137); L1: r /= l1 (:726)
__global__ void sym_scale_k(const double *__restrict__ diag, const double *__restrict__ l1,
                            double omega, double *__restrict__ r, int rb, int re, int seq)
{
   EW_LOOP(i, rb, re)
   {
      if (l1) {
         r[i] /= l1[i];
      } else {
         const double a = diag[i];
         if (!seq || a != 0.0) r[i] *= omega / a;
      }
   }
}
void sym_scale(hipStream_t s, const double *diag, const double *l1, double omega, double *r,
               int rb, int re, int seq)
{
   if (re > rb) sym_scale_k<<<ew_blocks(re - rb), 256, 0, s>>>(diag, l1, omega, r, rb, re, seq);
}

// SMEM_Smooth.cpp:681-694 / 741-754, SEQ_Smooth.cpp:142-148 / 178-182
__global__ void sym_update_k(const double *__restrict__ diag, const double *__restrict__ l1,
                             double omega, double *__restrict__ r, const double *__restrict__ y,
                             double *__restrict__ u, int rb, int re, int seq, int overwrite)
{
   EW_LOOP(i, rb, re)
   {
      double ri = r[i];
      if (l1) {
         ri = (2.0 * l1[i] * ri) - y[i];
         ri /= l1[i];
      } else {
         const double a = diag[i];
         if (!seq || a != 0.0) {
            ri = (2.0 * a * ri / omega) - y[i];
            ri *= omega / a;
         }
      }
      r[i] = ri;
      if (overwrite)
         u[i] = ri;
      else
         u[i] += ri;
   }
}
void sym_update(hipStream_t s, const double *diag, const double *l1, double omega, double *r,
                const double *y, double *u, int rb, int re, int seq, int overwrite)
{
   if (re > rb)
      sym_update_k<<<ew_blocks(re - rb), 256, 0, s>>>(diag, l1, omega, r, y, u, rb, re, seq,
                                                     overwrite);
}

// SMEM_Solve.cpp:179-186
__global__ void cheby_update_k(double *__restrict__ u, double *__restrict__ uo,
                               double *__restrict__ yo, double omega, double delta, int n)
{
   EW_LOOP(i, 0, n)
   {
      const double u_outer_prev = uo[i];
      const double v = yo[i] + omega * (delta * u[i] + uo[i] - yo[i]);
      uo[i] = v;
      yo[i] = u_outer_prev;
      u[i] = v;
   }
}
void cheby_update(hipStream_t s, double *u, double *u_outer, double *y_outer, double omega,
                  double delta, int n)
{
   if (n > 0) cheby_update_k<<<ew_blocks(n), 256, 0, s>>>(u, u_outer, y_outer, omega, delta, n);
}

// SMEM_Async_AMG.cpp:296-299 (FULL_ASYNC): omp atomic u[i] += e[i]; u_k[i] = u[i]
__global__ void atomic_correct_k(double *u, const double *__restrict__ e,
                                 double *__restrict__ u_priv, int n)
{
   EW_LOOP(i, 0, n)
   {
      const double ei = e[i];
      const double old = atomicAdd(u + i, ei);
      u_priv[i] = old + ei;
   }
}
void atomic_correct(hipStream_t s, double *u, const double *e, double *u_priv, int n)
{
   if (n > 0) atomic_correct_k<<<ew_blocks(n), 256, 0, s>>>(u, e, u_priv, n);
}

// ---------------------------------------------------------------------------
// deterministic reductions: fixed grid, fixed per-lane order, fixed tree
// ---------------------------------------------------------------------------
static inline int red_blocks(int n) { return std::max(1, std::min(1024, (n + 2047) / 2048)); }

template <bool DOT>
__global__ __launch_bounds__(256) void partials_k(const double *__restrict__ x,
                                                  const double *__restrict__ y, int n,
                                                  double *__restrict__ partials)
{
   __shared__ double red[4];
   double s = 0.0;
   for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
      s += DOT ? x[i] * y[i] : x[i] * x[i];
   s = block_sum_256(s, red);
   if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

void sumsq_partials(hipStream_t s, const double *x, int n, double *partials, int *nparts)
{
   const int nb = red_blocks(n);
   partials_k<false><<<nb, 256, 0, s>>>(x, nullptr, n, partials);
   *nparts = nb;
}

void dot_partials(hipStream_t s, const double *x, const double *y, int n, double *partials,
                  int *nparts)
{
   const int nb = red_blocks(n);
   partials_k<true><<<nb, 256, 0, s>>>(x, y, n, partials);
   *nparts = nb;
}

__global__ __launch_bounds__(256) void sum_partials_k(const double *__restrict__ p, int np,
                                                      double *__restrict__ out)
{
   __shared__ double red[4];
   double s = 0.0;
   for (int i = blockIdx.x * 256 + threadIdx.x; i < np; i += gridDim.x * 256) s += p[i];
   s = block_sum_256(s, red);
   if (threadIdx.x == 0) out[blockIdx.x] = s;
}

__global__ void finish_k(double *out, int do_sqrt)
{
   if (do_sqrt) out[0] = sqrt(out[0]);
}

void reduce_partials(hipStream_t s, const double *partials, int np, double *out, int do_sqrt,
                     double *scratch)
{
   // two fixed levels keep the single-workgroup tail short for large np
   if (np > 4096) {
      const int nb = std::min(1024, (np + 2047) / 2048);
      double *mid = scratch; // >= 1024 doubles
      sum_partials_k<<<nb, 256, 0, s>>>(partials, np, mid);
      sum_partials_k<<<1, 256, 0, s>>>(mid, nb, out);
   } else {
      sum_partials_k<<<1, 256, 0, s>>>(partials, np, out);
   }
   if (do_sqrt) finish_k<<<1, 1, 0, s>>>(out, do_sqrt);
}

} // namespace amgk
