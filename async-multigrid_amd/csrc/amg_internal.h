// amg_internal.h -- shared internals of libamg_mi355x (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <limits>
#include <vector>

#include "amg_mi355x.h"

// ---------------------------------------------------------------------------
// error plumbing: every C-ABI entry returns AMG_OK or a negative status and
// leaves a thread-local message for amg_last_error().
// ---------------------------------------------------------------------------
int amg_set_error(int code, const char *fmt, ...);

#define AMG_HIP(call)                                                                      \
   do {                                                                                    \
      hipError_t _e = (call);                                                              \
      if (_e != hipSuccess)                                                                \
         return amg_set_error(AMG_ERR_HIP, "%s:%d %s -> %s", __FILE__, __LINE__, #call,   \
                              hipGetErrorString(_e));                                      \
   } while (0)

#define AMG_TRY(call)                                                                      \
   do {                                                                                    \
      int _s = (call);                                                                     \
      if (_s != AMG_OK) return _s;                                                         \
   } while (0)

#define AMG_ARG(cond, ...)                                                                 \
   do {                                                                                    \
      if (!(cond)) return amg_set_error(AMG_ERR_ARG, __VA_ARGS__);                         \
   } while (0)

// rows handled by one workgroup of the CSR tile kernels (one row per lane)
constexpr int AMG_TILE_ROWS = 256;
// products staged per LDS chunk in the CSR tile kernels (16 KiB of fp64)
constexpr int AMG_CHUNK = 2048;
// device arrays of col/val are padded so 16-byte vector loads past nnz stay in bounds
constexpr int AMG_NNZ_PAD = 8;
// longest row the dictionary-coded kernel stages in LDS
constexpr int AMG_DC_MAXROW = 32;
// bytes per row pattern of the row-pattern-coded form: length + entries (x4 aligned)
constexpr int AMG_RP_STRIDE = 36;
// paired row patterns (rows 2t, 2t+1 of operators whose rows hold <= 32
// entries): one header word + up to 2 * maxrow merged entry words per pair
// pattern, maxrow = 8 (7-pt) or 32 (27-pt Galerkin); the table must fit
// AMG_PP_LDS bytes of LDS
constexpr int AMG_PP_MAXROW = 32;
constexpr int AMG_PP_LDS = 32 * 1024;
// rows of > 8 entries are pair-coded from this size up (a pair lane walks
// twice the entries: latency-bound grids below it run faster one row per lane)
constexpr int AMG_PP_LONG_MIN_ROWS = 1 << 22;
inline int amg_pp_stride(int maxrow) { return 1 + 2 * (maxrow <= 8 ? 8 : AMG_PP_MAXROW); }

// AMG_SCHED_TIMED: the end time of a level's correction j (0-based) -- its
// recorded end times t (the replay of a measured race; past the table the
// last interval repeats) or, without a table, (j + 1) dur.  The oracle's
// timed_end (or_set_async_durations / or_set_async_times), the same doubles.
inline double amg_timed_end(const std::vector<double> &t, double dur, int j)
{
   const int n = (int)t.size();
   if (n == 0) return (double)(j + 1) * dur;
   if (j < n) return t[j];
   const double dt = n > 1 ? t[n - 1] - t[n - 2] : t[0];
   return t[n - 1] + (double)(j - n + 1) * dt;
}

namespace amgk {
void stamp_init(hipStream_t s, unsigned long long *stamps, int n);
}

// per-correction end events of a free race (one pool per level, grown on use)
// (the update point of correction j: its start event `record_start`, before
// the kernel that adds it into the shared iterate, and its end event `record`,
// after it -- a window in which other levels' updates may interleave row by row)
struct AmgCorrTimes {
   std::vector<std::vector<hipEvent_t>> ev, ev0; // [level][correction]: update end / start
   std::vector<std::vector<double>> ms, ms0;     // [level][correction], after the solve
   static int rec(std::vector<hipEvent_t> &v, int j, hipStream_t s)
   {
      while ((int)v.size() <= j) {
         hipEvent_t e;
         if (hipEventCreate(&e) != hipSuccess) return -1;
         v.push_back(e);
      }
      return hipEventRecord(v[j], s) == hipSuccess ? 0 : -1;
   }
   int record(int k, int j, hipStream_t s) { return rec(ev[k], j, s); }
   int record_start(int k, int j, hipStream_t s) { return rec(ev0[k], j, s); }
   void reset(int L)
   {
      ev.resize(L);
      ev0.resize(L);
      ms.assign(L, {});
      ms0.assign(L, {});
   }
   // elapsed ms of the first cnt[k] events of every level from t0
   int collect(hipEvent_t t0, const std::vector<int> &cnt)
   {
      ms.assign(ev.size(), {});
      ms0.assign(ev.size(), {});
      for (size_t k = 0; k < ev.size() && k < cnt.size(); k++)
         for (int j = 0; j < cnt[k] && j < (int)ev[k].size(); j++) {
            float m = 0.f;
            if (hipEventElapsedTime(&m, t0, ev[k][j]) != hipSuccess) return -1;
            ms[k].push_back(m);
            if (j < (int)ev0[k].size()) {
               if (hipEventElapsedTime(&m, t0, ev0[k][j]) != hipSuccess) return -1;
               ms0[k].push_back(m);
            }
         }
      return 0;
   }
   // device execution windows of the update kernels (stamp_begin / stamp_end
   // in the kernel that adds correction j of level k into the shared vector):
   // [k][j] start / end in ms of the device wall clock (an arbitrary origin
   // common to every stream and process on the device); NaN: not stamped.
   // Record of correction (k, j): 4 words -- window start, window end, the
   // device address of its per-row stamp array (0: none), unused.
   unsigned long long *d_st = nullptr;
   int st_cap = 0, st_L = 0;
   std::vector<std::vector<double>> w0, w1;
   // per-row update times (stamp_row: the low 32 bits of the device wall clock
   // at which row i's add + read of the shared vector completed) of the first
   // rows_j corrections of every level; rows_ms[k][j]: nrow times in ms, on the
   // window clock (empty: not recorded)
   unsigned *d_rows = nullptr;
   double *d_vals = nullptr; // per row: the value each add replaced and the value it left
   size_t rows_alloc = 0;
   int nrow = 0, rows_j = 0;
   std::vector<std::vector<std::vector<double>>> rows_ms, rows_vals;
   std::vector<unsigned long long> h_init;
   // row stamps are taken while nrow * L * rows_j * 20 B stays within this
   static constexpr size_t kRowBudget = (size_t)512 << 20;
   // koff[k]: the index of owned row 0 in the vector the update kernel of
   // level k indexes (a slab level-0 vector with its ghost planes in front)
   int stamps_begin(hipStream_t s, int L, int cap, int n_rows = 0, const std::vector<long long> &koff = {})
   {
      if (!d_st || L * cap > st_L * st_cap) {
         if (d_st) hipFree(d_st);
         d_st = nullptr;
         if (hipMalloc((void **)&d_st, (size_t)4 * L * cap * sizeof(unsigned long long)) != hipSuccess) return -1;
      }
      st_L = L;
      st_cap = cap;
      nrow = n_rows > 0 ? n_rows : 0;
      rows_j = nrow > 0 ? (int)std::min<size_t>(cap, kRowBudget / ((size_t)nrow * L * 20)) : 0;
      const size_t need = (size_t)nrow * L * rows_j;
      if (need > rows_alloc) {
         if (d_rows) hipFree(d_rows);
         if (d_vals) hipFree(d_vals);
         d_rows = nullptr;
         d_vals = nullptr;
         rows_alloc = 0;
         if (hipMalloc((void **)&d_rows, need * sizeof(unsigned)) != hipSuccess ||
             hipMalloc((void **)&d_vals, 2 * need * sizeof(double)) != hipSuccess) {
            (void)hipGetLastError();
            rows_j = 0;
         } else {
            rows_alloc = need;
         }
      }
      if (rows_j == 0) {
         // no row arrays: the records set on the device, in stream order (a
         // pageable host copy per solve serialises the ranks sharing a GPU)
         amgk::stamp_init(s, d_st, L * cap);
         return 0;
      }
      h_init.assign((size_t)4 * L * cap, 0ull);
      for (int k = 0; k < L; k++)
         for (int j = 0; j < cap; j++) {
            unsigned long long *w = &h_init[4 * ((size_t)k * cap + j)];
            w[0] = ~0ull;
            if (j < rows_j) {
               const long long o = k < (int)koff.size() ? koff[k] : 0;
               w[2] = (unsigned long long)(uintptr_t)(d_rows + ((size_t)k * rows_j + j) * nrow - o);
               w[3] = (unsigned long long)(uintptr_t)(d_vals + 2 * (((size_t)k * rows_j + j) * nrow - o));
            }
         }
      if (hipMemcpyAsync(d_st, h_init.data(), h_init.size() * sizeof(unsigned long long), hipMemcpyHostToDevice,
                         s) != hipSuccess)
         return -1;
      if (rows_j > 0 && hipMemsetAsync(d_rows, 0, need * sizeof(unsigned), s) != hipSuccess) return -1;
      // NaN: a row whose update recorded no values (the no-return form)
      if (rows_j > 0 && hipMemsetAsync(d_vals, 0xff, 2 * need * sizeof(double), s) != hipSuccess) return -1;
      return 0;
   }
   unsigned long long *stamp(int k, int j) const
   {
      if (!(d_st && k >= 0 && k < st_L && j >= 0 && j < st_cap)) return nullptr;
      unsigned long long *p = d_st + 4 * ((size_t)k * st_cap + j);
      // low bit: the record carries row arrays (stamp_rows reads them only then)
      return (j < rows_j && nrow > 0) ? reinterpret_cast<unsigned long long *>(reinterpret_cast<uintptr_t>(p) | 1)
                                      : p;
   }
   // after the solve (the stream has finished): windows of the first cnt[k]
   // corrections of every level, and their row times where recorded
   int stamps_collect(const std::vector<int> &cnt, int wall_khz)
   {
      w0.assign(st_L, {});
      w1.assign(st_L, {});
      rows_ms.assign(st_L, {});
      rows_vals.assign(st_L, {});
      if (!d_st) return 0;
      std::vector<unsigned long long> h((size_t)4 * st_L * st_cap);
      if (hipMemcpy(h.data(), d_st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
         return -1;
      const double tpm = wall_khz > 0 ? (double)wall_khz : 1e5; // ticks per ms
      // the host copy of a correction's row times only where rows were
      // recorded (nrow is the level-0 row count: a per-solve zero-filled
      // buffer of that size cost 12 % of config 3's asynchronous cycle)
      std::vector<unsigned> hr;
      if (rows_j > 0) hr.resize((size_t)nrow);
      for (int k = 0; k < st_L && k < (int)cnt.size(); k++)
         for (int j = 0; j < cnt[k] && j < st_cap; j++) {
            const unsigned long long a = h[4 * ((size_t)k * st_cap + j)], b = h[4 * ((size_t)k * st_cap + j) + 1];
            const bool ok = a != ~0ull && b != 0ull;
            w0[k].push_back(ok ? (double)a / tpm : std::numeric_limits<double>::quiet_NaN());
            w1[k].push_back(ok ? (double)b / tpm : std::numeric_limits<double>::quiet_NaN());
            if (!ok || j >= rows_j || nrow == 0) continue;
            if (hipMemcpy(hr.data(), d_rows + ((size_t)k * rows_j + j) * nrow, (size_t)nrow * sizeof(unsigned),
                          hipMemcpyDeviceToHost) != hipSuccess)
               return -1;
            // unwrap the low 32 bits around the window start (|dt| < 21 s)
            if ((int)rows_ms[k].size() != j) continue;
            std::vector<double> t((size_t)nrow);
            for (int i = 0; i < nrow; i++) {
               const int d = (int)(hr[i] - (unsigned)a);
               t[i] = ((double)a + (double)d) / tpm;
            }
            rows_ms[k].push_back(std::move(t));
            std::vector<double> v((size_t)2 * nrow);
            if (hipMemcpy(v.data(), d_vals + 2 * ((size_t)k * rows_j + j) * nrow, v.size() * sizeof(double),
                          hipMemcpyDeviceToHost) != hipSuccess)
               return -1;
            rows_vals[k].push_back(std::move(v));
         }
      return 0;
   }
   // per-row times of correction j of level k: nrow values, or 0 if not
   // recorded; vals: the 2 nrow (old, new) values instead
   int rows_of(int k, int j, double *out, int cap, bool vals = false) const
   {
      const auto &src = vals ? rows_vals : rows_ms;
      if (k < 0 || k >= (int)src.size() || j < 0 || j >= (int)src[k].size()) return 0;
      const int n = std::min(cap, (int)src[k][j].size());
      if (out) std::copy(src[k][j].begin(), src[k][j].begin() + n, out);
      return n;
   }
   ~AmgCorrTimes()
   {
      for (auto *vv : {&ev, &ev0})
         for (auto &v : *vv)
            for (auto e : v) hipEventDestroy(e);
      if (d_st) hipFree(d_st);
      if (d_rows) hipFree(d_rows);
      if (d_vals) hipFree(d_vals);
   }
};
// anchored operators (interpolation, restriction): row 2t+1's anchor minus
// row 2t's, + AMG_PP_DA0, must lie in [0, AMG_PP_NDA)
constexpr int AMG_PP_NDA = 16;
constexpr int AMG_PP_DA0 = 8;
constexpr int AMG_PP_NK = 256 * 257 * AMG_PP_NDA; // pair keys
// pair-coded only if the merged lists are at most this factor longer than the
// longer row of each pair (summed over all row pairs)
constexpr double AMG_PP_MAXFILL = 1.15;
// paired kernel epilogue form (csr_rpp_kernel OPT, tools/tune_spmv.py ABL_jac_o*):
// bit 1 = a_ii from the header word
constexpr int AMG_RPP_OPT = 2;
// master-pattern form: longest master list, LDS budget of the per-pattern
// value table (pp_n * J * 16 bytes)
constexpr int AMG_MP_MAXJ = 32;
constexpr int AMG_MP_LDS = 48 * 1024;

struct amg_transport; // amg_dist.cpp: RCCL communicator or host-callback test transport

struct amg_ctx {
   amg_transport *xport = nullptr;
   long long replicate_rows = 1LL << 18;
   int device = 0;
   hipStream_t stream = nullptr;           // compute stream (all sync work)
   std::vector<hipStream_t> level_streams; // async additive: one per level
   hipStream_t comm_stream = nullptr;      // halo exchange (distributed)
   double *d_partials = nullptr;           // per-workgroup partial sums
   size_t partials_cap = 0;
   double *d_scalars = nullptr;            // device scalars (norms, dots)
   int *d_err = nullptr;                   // device-side range-check flags (amg_device_errors)
   double *h_pinned = nullptr;             // pinned host mirror of scalars
   int num_cus = 256;
   int wall_khz = 100000;  // device wall clock (wall_clock64) rate, for injected delays
   int value_index = 1; // build value-indexed CSR for matrices with <= 256 distinct values
   int dict_index = 1;  // build dictionary-coded CSR for stencil-like square operators
   int row_pattern = 1; // build row-pattern-coded CSR on top of the dictionary
   int pair_pattern = 1; // paired-row-pattern CSR: 0 off, 1 size-gated for long rows, 2 always
   int master_pattern = 1; // master-pattern form of square pair-coded operators
   int pair_anchor16 = 0;  // slab-compressed anchors of pair-coded P/R (measured slower: off)
   int plane_march = 1;    // plane-marching kernel for 7-pt box-grid masters (csr_mz_kernel)
   int mz_zc = 16;         // planes per workgroup chunk of the plane-marching kernel
   int mz_edge = 1;        // x-edge pair patterns on the 27-pt march's fast path
   int mz_zc_auto = 1;     // shorten the chunks of small levels to keep >= 2048 workgroups
   // 27-pt march: chunks sized so the grid is one round of resident
   // workgroups (mz27_occ > 0: workgroups per CU; 0: mz_chunk's rule) and the
   // prefetch distance in planes (1 or 2)
   // (> 0: that many per CU; < 0: the kernel's own occupancy from the runtime)
   int mz27_occ = -1;
   int mz_occ = 0; // the same for the 7-pt march (AMG_MZ_OCC; 0: mz_chunk's rule)
   int mz_pf = 3;  // 7-pt march prefetch distance in planes (AMG_MZ_PF: 1 or 2; 3: 1 + halo operands and rhs ahead)
   int mz27_pf = 2;
   int mz_xcd = 1;         // XCD-contiguous workgroup order of the plane-marching kernel
   int fuse_transfer = 1;  // fused level-0 residual + restriction on geometric hierarchies
   int bsr3 = 2;           // 3x3 block form of num_functions = 3 operators (1: lane per row; 2: lane per block row when value-indexed)
   unsigned knob_gen = 0;  // bumped by every amg_set_* knob: captured hipGraphs older than it are dropped
   int graphs = 0;         // hipGraphs of the additive cycles' launch-bound loops (AMG_GRAPHS)
   int fuse_xfer = 1;      // composed smoothed transfers of marched 7-pt levels in one pass each
   int fuse_xfp_slab = 0;  // ... and the slab async solve's fused prolongation + atomic (AMG_FUSE_XFP_SLAB)
   int fuse_prolong = 0;   // prolongation fused into the first post sweep (measured slower: off)
   int bsr3_xs = 1;        // 3x3 block kernel: one x load per lane, shared over the triplet (AMG_BSR3_XS)
   int fuse_outer = 0;     // level 0's last post sweep + the outer residual as one march (AMG_FUSE_OUTER;
                           // 1: u' stored every step, 2: only at the end of an iterate batch;
                           // 3: the two sweeps slab by slab over z through the Infinity Cache, u' as in 2)
   int outer_slab = 32;    // planes per z-slab of fuse_outer 3 (AMG_OUTER_SLAB): a slab's u, f and u'
                           // (3 x 32 x 2 MB at 512^2 planes) stay in the 256 MiB Infinity Cache
   int rr_lines = 1;       // coarse lines per lane of the fused residual + restriction (1 or 2)
   int mz_lines = 1;       // 7-pt plane march: lines per lane (1, 2 or 4, AMG_MZ_LINES)
   int mz_lines_gemv = 2;  // the same for SpMV / SpGEMV (AMG_MZ_LINES_GEMV; 2: -8 % on the 512^3 SpMV)
   int mz_nt = 0;          // streaming hints on > 512 MB levels: 1 NT stores, 2 NT rhs loads
   int rr_ring = 0;        // wave-edge residuals through a flag-ordered LDS ring (measured slower: off)
   int rr_occ = 0;         // 5: the fused residual + restriction compiled for 5 waves / SIMD
   int rr_fpf = 0;         // 1: its right-hand side a fine plane ahead (AMG_RR_FPF)
   int long_form = 0;      // long-row CSR kernel: 0 workgroup chunks (csr_long_kernel), 1 / 2 wave-independent
                           // chunks of 8 / 16 entries per lane (csr_longw_kernel; AMG_LONG_FORM)
   int long_xcd = 1;       // ... with XCD-contiguous row blocks (AMG_LONG_XCD)
   int rr_zc = 0;          // coarse planes per chunk of the fused residual + restriction (0: mz_zc / 2)
   int jgs_wave = 1;       // hybrid JGS form: 1 8 blocks per wave, 2 one wave per block, 0 one lane per block, 3 LDS tile
   int jgs_small = 2;      // small levels' hybrid JGS form (amg_set_jgs_small)
   int jgs_fold = 0;       // FULL_ASYNC level-0 correction folded into the last JGS sweep (amg_set_jgs_fold)
};

struct amg_mat {
   amg_ctx *ctx = nullptr;
   int nrows = 0, ncols = 0;
   long long nnz = 0;
   int *rowptr = nullptr;
   int *col = nullptr;
   double *val = nullptr;
   double *diag = nullptr; // val[rowptr[i]] (the reference's a_ii; the zero pad after the last row)
   int diag_first = 1;
   int maxrow = -1;          // longest row (amg_mat_finish)
   amg_mat *trans = nullptr; // lazily built transpose for amg_matvec_t
   // value-indexed form (the hot kernels' format when the matrix has at most
   // 256 distinct values): vidx[k] indexes vtab (256 doubles, sorted by bits)
   unsigned char *vidx = nullptr;
   double *vtab = nullptr;
   int vi_n = 0;
   // dictionary-coded form (operators whose (col - anchor, value) pairs fit
   // 256 entries and whose rows hold <= AMG_DC_MAXROW entries; the anchor of a
   // row is its first column -- the row itself for diag-first square operators,
   // then danch is null): col = anchor + doff[didx[k]], a_ik = dval[didx[k]]
   unsigned char *didx = nullptr;
   int *doff = nullptr;
   double *dval = nullptr;
   int *danch = nullptr;
   int dc_n = 0;
   int dc_maxrow = 0; // longest row (selects the LDS staging size)
   // row-pattern-coded form (dictionary-coded operators with <= 256 distinct
   // rows, none empty): rpat[i] names row i's dictionary sequence in ptab
   // (AMG_RP_STRIDE bytes per pattern: length, then the entries)
   unsigned char *rpat = nullptr;
   unsigned char *ptab = nullptr;
   int rp_n = 0;
   // paired-row-pattern form (row-pattern-coded operators with rows of <= 32
   // entries and <= 256 distinct (pattern of row 2t, pattern of row 2t+1,
   // anchor delta) pairs): ppat[t] names the pair's merged entry list in
   // pptab (pp_stride words per pair: header nel | first entry of row 2t << 8
   // | of row 2t+1 << 16 | row 2t+1 present << 24 | (da + 16) << 25, then
   // entries d0 | d1 << 8 | has0 << 16 | has1 << 17).  An entry present in
   // both rows reads x[base + off], x[base + off + 1] with one 16-byte load.
   unsigned char *ppat = nullptr;
   unsigned int *pptab = nullptr;
   int pp_n = 0;
   int pp_stride = 0; // words per pair pattern (amg_pp_stride)
   int pp_centre0 = 0; // every pair's first merged entry is both rows' diagonal
   // master-pattern form (square, diagonal-first pair-coded operators whose
   // rows are all ordered subsequences of one master list of column offsets:
   // the diagonal, then the offsets ascending).  The offsets are wave-uniform
   // kernel arguments; mpmask[p] holds pair pattern p's row-use bits (bit 2j:
   // row 2t uses master entry j, bit 2j+1: row 2t+1).  mp_uni: one value per
   // offset over the whole matrix (values are kernel arguments too), else
   // mpval[p * mp_J + j] = {row 2t's value, row 2t+1's value}.
   // slab-compressed anchors of pair-coded operators with an anchor array:
   // anchor(2t) = pbase[2t >> 9] + pdelta[t] (every 512-row slab's anchors
   // within 65535 of its least), 2 bytes per row pair instead of 4 per row
   int *pbase = nullptr;
   unsigned short *pdelta = nullptr;
   int mp_J = 0; // master length (0: not master-coded)
   int mp_uni = 0;
   // every row's diagonal (A->diag) is the same value diag_u (amg_mat_finish)
   int diag_uni = 0;
   double diag_u = 0.0;
   int mp_off[AMG_MP_MAXJ] = {};
   double mp_val[AMG_MP_MAXJ] = {};
   unsigned long long *mpmask = nullptr;
   double *mpval = nullptr;
   // plane-marching form (csr_mz_kernel): the master list is [0, -P, -S, -1, +1,
   // +S, +P] with P % 512 == 0 and nrows = nz * P (0: not applicable)
   int mz_P = 0, mz_S = 0;
   // 27-pt plane march (csr_mz27_kernel): master list [0, the 26 offsets
   // dz P + dy S + dx ascending]; mz_dom = the most frequent pair pattern that
   // uses every entry with one value per entry in both rows (-1: none), its
   // values in master order (wave-uniform fast path)
   int mz27 = 0;
   int mz_dom = -1;
   double mz_domval[27] = {};
   // x-edge pair patterns of the fast path: mz_xlo = row 2t at the box's low
   // x face (its dx = -1 entries unused, values the dominant ones), row 2t+1
   // dominant; mz_xhi = row 2t dominant, row 2t+1 at the high x face (dx = +1
   // unused, values mz_hival); -1: none
   int mz_xlo = -1, mz_xhi = -1;
   double mz_hival[27] = {};
   // 3x3 block form (num_functions = 3 operators, byVDIM): block row t = rows
   // 3t..3t+2 whose three rows hold the same block columns, each block dense;
   // bmode[t] = 1: the block row keeps the CSR form (identity rows of fixed
   // dofs, irregular rows).  Block values as value-table indices (bvi: 3 rows
   // x 4 bytes, the 4th unused) when the matrix is value-indexed, else fp64
   // (bval: 9 per block, row-major)
   // Sliced layout: slice s = block rows 21s..21s+20 (one wave), padded to
   // its longest block row; block k of the slice's block row q sits at slot
   // soff[s] + 21 k + q, so a wave's loads of block k are contiguous.
   // bcnt[t] = blocks of block row t (0: CSR form), bdiag[t] = its diagonal
   // block's index k
   int bsr3 = 0; // 1: value-indexed blocks, 2: fp64 blocks
   int bsl = 21; // block rows per slice: 21 (lane per row, bsr3_kernel) or 64 (lane per block row, bsr3_row_kernel)
   long long *soff = nullptr;
   int *bcol = nullptr, *bdiag = nullptr;
   unsigned char *bmode = nullptr;
   unsigned int *bvi = nullptr;
   double *bval = nullptr;
};

struct amg_vec {
   amg_ctx *ctx = nullptr;
   int n = 0;
   double *d = nullptr;
   bool owns = true;
};

// workspace
int amg_ctx_partials(amg_ctx *ctx, size_t n, double **out);
// device CSR allocation (+ diagonal extraction) for in-library builders
int amg_mat_create_device(amg_ctx *c, int nrows, int ncols, long long nnz, amg_mat **out);
int amg_mat_finish(amg_mat *A);
// coarse sub-cycle of a hierarchy whose level 0 is an inner level of a larger
// one: f_dev -> level-0 correction (zero start, SMEM_Sync_Parfor_Vcycle from
// that level down); returns the level-0 iterate pointer in *u_dev
int amg_hier_subcycle(amg_hier *H, hipStream_t s, const double *f_dev, const double **u_dev);
// InitVectors: zero every level vector of H (start of a new solve)
int amg_hier_reset(amg_hier *H);

// ---------------------------------------------------------------------------
// kernel launchers (amg_kernels.hip); all asynchronous on stream s
// ---------------------------------------------------------------------------
namespace amgk {

// SMEM_SpGEMV branch selection (SMEM_MatVec.cpp:140-258)
struct Gemv {
   int init;     // 0: 0.0, 1: b, 2: -b, 3: b*temp, 4: -b*temp
   int negacc;   // 1: tempx -= a*x ; 0: tempx += a*x
   int scale;    // 1: y = alpha*tempx
   double alpha, temp;
};
Gemv gemv_mode(double alpha, double beta);

// y[rb,re) per the Gemv mode; if partials != nullptr also writes per-workgroup
// sum of y_i^2 to partials[0..nblocks) (fixed order)
void spgemv(hipStream_t s, const amg_mat *A, const double *x, const double *b, const Gemv &g,
            double *y, int rb, int re, double *partials);
// r = b - (A x) over [0, n): SMEM_Residual's y = A x; r = b - y (the sum
// rounded first, then subtracted) in one pass without y where A is
// dictionary-coded, else the two passes through y (bit-identical either way)
void residual_fsub(hipStream_t s, const amg_mat *A, const double *x, const double *b, double *y, double *r, int n);
int tile_blocks(int rb, int re);

// Jacobi sweep out[i] = x[i] + (omega*(f_i - sum a_ij x_j))/a_ii  (a_ii != 0)
//   l1 != nullptr: out[i] = x[i] + (f_i - sum)/l1[i]   (no a_ii test)
void jacobi_sweep(hipStream_t s, const amg_mat *A, const double *f, const double *x,
                  const double *l1, double omega, double *out, int rb, int re);
// outer residual r = f - A x fused with the next cycle's first Jacobi sweep on
// the same x: unext = x + w r / a_ii (l1: x + r / l1); partials of sum r_i^2
void residual_jacobi(hipStream_t s, const amg_mat *A, const double *f, const double *x,
                     const double *l1, double omega, double *r, double *unext, int rb, int re,
                     double *partials);
// level 0's last post-smoothing sweep and the outer residual + next first
// sweep as ONE plane march (7-pt master form, S = 512): u1out = u' (null: not
// stored), rout = r (null: not stored), unext = u'', partials of sum r_i^2
bool mz_sweep_outer_ok(const amg_mat *A);
void mz_sweep_outer(hipStream_t s, const amg_mat *A, const double *f, const double *u, double *u1out,
                    double *rout, double *unext, double omega, double *partials);
// zero-guess sweep: variant 0 (SMEM) u = omega*f/a (a != 0) | u = f/l1
//                   variant 1 (SEQ)  u += omega*f/a (a != 0) | u += f/l1 (a != 0)
void jacobi_zero(hipStream_t s, const double *diag, const double *f, const double *l1,
                 double omega, double *u, int rb, int re, int variant);
// u_new = u + (omega*r)/a (a != 0): Jacobi sweep from a precomputed residual
void jacobi_from_residual(hipStream_t s, const double *diag, const double *r, const double *l1,
                          double omega, double *u, int rb, int re);
// hybrid JGS: one wave (rows <= 32 entries) or one lane per block, blocks d_blk[0..nblk] (device), in place on u.
// apply_u (the LDS tile form only): the FULL_ASYNC correction of the sweep's result folded into its
// write-out -- apply_u += u by device-scope atomics, apply_priv = the value after it (atomic_correct);
// returns whether it was applied
bool hybrid_jgs(hipStream_t s, const amg_mat *A, const double *f, double *u, const double *u_prev,
                const int *d_blk, int nblk, const double *diag_scale, double weight, int zero,
                int reverse, double *apply_u = nullptr, double *apply_priv = nullptr,
                unsigned long long *stamp = nullptr);
// *d_out = max(*d_out, longest row of A)
void row_max(hipStream_t s, const amg_mat *A, int *d_out);
// asynchronous / semi-asynchronous Gauss-Seidel, one lane per block, live u
void async_gs(hipStream_t s, const amg_mat *A, const double *f, double *u, const int *d_blk, int nblk,
              int sweeps, int semi, int reverse);
// geometric transfers of a marched level (R_0 = P_0^T of an nx*ny*nz box):
// coarse K couples to fine 2K + d, d in {0,1,2}^3, weight w[dz*9 + dy*3 + dx]
struct GeoT {
   double w[27];
   int nx, ny, nz;
};
// *bad |= 1 unless every row of M equals the geometric form (mode 0: M = R,
// coarse rows; mode 1: M = P, fine rows): lengths, columns, value bits
// z-slab forms (rows / columns of an extended slab operator): local rows [rb, re)
// are global rows + row_g0, local columns global columns + col_g0 (re < 0: all rows)
void geo_check(hipStream_t s, const amg_mat *M, int mode, const GeoT &g, int *bad, int rb = 0, int re = -1,
               long long row_g0 = 0, long long col_g0 = 0);
// fc = R (f - A u) for a plane-marched A with geometric R, without the fine
// residual vector (bit-identical to the residual SpGEMV + R SpMV).  Slab form:
// coarse planes [Kb, Ke) (Ke < 0: all), u / f plane 0 = fine plane fz0 (A's
// rows are those vectors' planes), fc plane 0 = coarse plane cz0
// the coarse level's zero-guess Jacobi sweep folded into a restriction: where
// u != null, u[i] = w fc[i] / d[i] for d[i] != 0 (jacobi_zero variant 0, no L1)
struct ZeroGuess {
   const double *d = nullptr;
   double w = 0.0;
   double *u = nullptr;
   // indices the fold may write: [lo, hi) (hi < 0: unchecked); a write outside
   // is dropped and flagged in *err (amg_device_errors)
   long long lo = 0, hi = -1;
   int *err = nullptr;
};
void mz_residual_restrict(hipStream_t s, const amg_mat *A, const double *f, const double *u, const GeoT &g,
                          const double *wdev, double *fc, int Kb = 0, int Ke = -1, int fz0 = 0, int cz0 = 0,
                          ZeroGuess zg = ZeroGuess());
// f_c = R r for the checked geometric R of GeoT g (bit-identical to the SpMV);
// coarse planes [Kb, Ke), r plane 0 = fine plane fz0, fc plane 0 = coarse cz0
void geo_restrict(hipStream_t s, const GeoT &g, const double *wdev, const double *r, double *fc, int Kb = 0,
                  int Ke = -1, int fz0 = 0, int cz0 = 0, ZeroGuess zg = ZeroGuess());
// u += P e for the checked geometric P of GeoT g (bit-identical to the SpGEMV);
// fine planes [zb, ze), u plane 0 = fine plane fz0, e plane 0 = coarse cz0;
// assign: u = P e (the SpMV, alpha 1 beta 0)
void geo_prolong(hipStream_t s, const GeoT &g, const double *wdev, const double *e, double *u, int zb = 0,
                 int ze = -1, int fz0 = 0, int cz0 = 0, int assign = 0);
// DMEM_AddSmooth scale vectors: s = a_ii / w (1 where a_ii = 0) or the L1 row
// norm l1 (l1 != nullptr), ns = -s (DMEM_Setup.cpp:423-482)
void dmem_scale(hipStream_t s, const double *diag, const double *l1, double omega, double *sc, double *nsc, int n);
// the stream waits usec microseconds (device wall clock at wall_khz)
void delay(hipStream_t s, double usec, int wall_khz);
// u_out = first Jacobi (l1 == nullptr) / L1 Jacobi sweep of A on uc = u + P e,
// P the checked geometric transfer of marched 7-pt level A (uc never stored)
void mz_prolong_sweep(hipStream_t s, const amg_mat *A, const double *f, const double *u, const double *ec,
                      const GeoT &g, const double *wdev, const double *l1, double omega, double *uout);
// composed smoothed transfers of a marched 7-pt level with geometric R / P in
// one pass each (bit-identical to xfer_div + SpMV + xfer_sub + R, and to
// P + SpMV + xfer_corr): rc = R (r + (-w) A (r ./ a)) (uniform operators only);
// ef = P ec + (-w) (A P ec) ./ a, then mode 0: out = ef; 1: atomic_correct(out =
// u, ef, u_priv); 2: out = u + ef
void mz_xfer_restrict(hipStream_t s, const amg_mat *A, const double *r, const GeoT &g, const double *wdev,
                      double omega, double *rc, int Kb = 0, int Ke = -1, int fz0 = 0, int cz0 = 0);
void mz_xfer_prolong(hipStream_t s, const amg_mat *A, const double *ec, const GeoT &g, const double *wdev,
                     double omega, int mode, double *out, double *u_priv, int zlo = 0, int zhi = -1, int fz0 = 0,
                     int cz0 = 0, unsigned long long *stamp = nullptr);
// transpose-product with the expansion-buffer order of T static chunks
void matvec_t_chunked(hipStream_t s, const amg_mat *AT, const double *x, double *y, int n_src,
                      int T);

// vector kernels
void vcopy(hipStream_t s, const double *x, double *y, int rb, int re);
void vset(hipStream_t s, double *y, double a, int rb, int re);
void vaxpy(hipStream_t s, double a, const double *x, double *y, int rb, int re);
void vivaxpy(hipStream_t s, const double *x, const double *sc, double *y, int rb, int re);
void vscale(hipStream_t s, double a, double *y, int rb, int re);
void vsub(hipStream_t s, const double *b, const double *y, double *r, int rb, int re); // r = b - y
// composed smoothed transfers: out = x ./ diag;  z = r + (-w) y;  e = e + (-w) (y ./ diag)
void xfer_div(hipStream_t s, const double *diag, const double *x, double *out, int rb, int re);
void xfer_sub(hipStream_t s, double w, const double *r, const double *y, double *z, int rb, int re);
void xfer_corr(hipStream_t s, double w, const double *y, const double *diag, double *e, int rb, int re);
void vadd_into(hipStream_t s, const double *r, double *u, int rb, int re, int overwrite);
void l1_norms(hipStream_t s, const amg_mat *A, double *out);
void a_diag(hipStream_t s, const double *diag, double omega, double *out, int n);
void extract_diag(hipStream_t s, const amg_mat *A);
// *d_flag = 1 unless every diag[i] has diag[0]'s bits
void diag_uniform(hipStream_t s, const amg_mat *A, int *d_flag);
// symmetric Jacobi pieces (SMEM_Smooth.cpp:665,682-683 / SEQ_Smooth.cpp:136,144-145)
void sym_scale(hipStream_t s, const double *diag, const double *l1, double omega, double *r,
               int rb, int re, int seq);
void sym_update(hipStream_t s, const double *diag, const double *l1, double omega, double *r,
                const double *y, double *u, int rb, int re, int seq, int overwrite);
// Chebyshev outer update SMEM_Solve.cpp:179-186
void cheby_update(hipStream_t s, double *u, double *u_outer, double *y_outer, double omega,
                  double delta, int n);
// DMEM_ChebyUpdate (DMEM_Misc.cpp:612-666) after the first cycle; branch 0 sync
// (d only), 1 async cheby_grid (d and u), 2 async other grid (u only)
void dmem_cheby_update(hipStream_t s, double *d, double *u, int n, int branch, double om1, double omd);
// DMEM_Mult accelerated update: x += e; d = first ? e : om1 d + omd e; x += d
void dmem_mult_accel(hipStream_t s, double *x, const double *e, double *d, int n, int first, double om1,
                     double omd);
// atomic correction: u += e (device-scope fp64 atomics), u_priv = value after the add
// stamp (nullable, every update kernel of a free race): stamp[0] = min, stamp[1] = max of the
// device wall clock over the kernel's workgroups -- its actual execution window (stamp_init)
void atomic_correct(hipStream_t s, double *u, const double *e, double *u_priv, int n,
                    unsigned long long *stamp = nullptr);
// stamps[0 .. 2n): starts ~0, ends 0
void stamp_init(hipStream_t s, unsigned long long *stamps, int n);
// serialised (SEMI_ASYNC) form: u += e; u_priv = u (u_priv may be null)
void semi_correct(hipStream_t s, double *u, const double *e, double *u_priv, int n);
// READ_RES: r -= y (atomic or serialised), r_priv = the updated value
void res_update(hipStream_t s, double *r, const double *y, double *r_priv, int n, int atomic,
                unsigned long long *stamp = nullptr);
// u[rb, re) += x[rb, re), device-scope atomics
void atomic_add(hipStream_t s, double *u, const double *x, int rb, int re);

// STREAM triad a = b + q c over n doubles (n even)
void stream_triad(hipStream_t s, double *a, const double *b, const double *c, double q, long long n);
// PMC calibration streams: mode 0/1/2/3 = read bytes with 16/8/4/1-byte lanes, 4 = 8-byte writes
void calib_stream(hipStream_t s, int mode, void *buf, long long bytes, double *out);

// value-indexed CSR construction
void vi_collect(hipStream_t s, const double *val, long long nnz, unsigned long long *slots, int nslots,
                int *count);
void vi_encode(hipStream_t s, const double *val, long long nnz, const unsigned long long *keys, int T,
               unsigned char *vidx);

// row-pattern construction (needs the dictionary index)
void rp_collect(hipStream_t s, const amg_mat *A, unsigned long long *slots, int *rep, int nslots, int *count,
                int *bad);
void rp_table(hipStream_t s, const amg_mat *A, const int *rep, int T, unsigned char *ptab);
void rp_encode(hipStream_t s, const amg_mat *A, const unsigned long long *keys, int T,
               const unsigned char *ptab, unsigned char *rpat, int *bad);
void pp_collect(hipStream_t s, const amg_mat *A, unsigned char *flags);
// slab-compressed anchors (pbase, pdelta); ok set to 0 when a slab's range
// exceeds 16 bits
void pp_anchor_compress(hipStream_t s, const amg_mat *A, int *pbase, unsigned short *pdelta, int *ok);
void pp_encode(hipStream_t s, const amg_mat *A, const unsigned char *map, unsigned char *ppat,
               unsigned long long *counts);

// dictionary-coded CSR construction (needs the value index)
void dc_collect(hipStream_t s, const amg_mat *A, unsigned long long *slots, int nslots, int *count,
                int *maxlen);
void dc_encode(hipStream_t s, const amg_mat *A, const unsigned long long *keys, int T,
               unsigned char *didx, int *anch);

// deterministic reductions
void sumsq_partials(hipStream_t s, const double *x, int n, double *partials, int *nparts);
void abssum_partials(hipStream_t s, const double *x, int n, double *partials, int *nparts);
void dot_partials(hipStream_t s, const double *x, const double *y, int n, double *partials,
                  int *nparts);
// out[0] = sum(partials[0..np)) in fixed order; if do_sqrt, out[0] = sqrt(sum)
void reduce_partials(hipStream_t s, const double *partials, int np, double *out, int do_sqrt,
                     double *scratch);

} // namespace amgk

// process-wide lock held by the teardown entry points (amg_api.cpp)
#include <mutex>
std::recursive_mutex &amg_teardown_mutex();
