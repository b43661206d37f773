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

#include <mutex>
#include <unordered_map>

#include <algorithm>
#include <type_traits>

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
typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));
// two consecutive doubles at an 8-byte aligned address (global_load_dwordx4)
typedef double v2du __attribute__((ext_vector_type(2), aligned(8)));

// Tile configuration: RPT rows per lane (tile = 256*RPT rows), CH products
// per LDS chunk, NT non-temporal val/col streams (read once; keep L2 for x),
// XCD contiguous-range tile remap (T1; speed only, any placement is correct).
template <int RPT, int CH, bool NT, bool XCD, bool UNR = false, bool SKIPSYNC = false,
          bool SHFL = false, bool STR = false, bool W8 = false>
struct TileCfg {
   static constexpr int rpt = RPT, ch = CH;
   static constexpr bool nt = NT, xcd = XCD;
   static constexpr bool unr = UNR;       // issue two staging groups' loads before storing
   static constexpr bool skipsync = SKIPSYNC; // no barrier after the tile's last chunk
   static constexpr bool shfl = SHFL;     // rowptr[row+1] from the neighbour lane
   static constexpr bool w8 = W8;         // 8 consecutive entries per lane, all loads up front
   static constexpr bool str = STR;       // lane-strided entries (dword loads): one gather
                                          // instruction covers 64 consecutive entries
};

template <bool NT>
__device__ __forceinline__ void stage4(const int *__restrict__ col, const double *__restrict__ val,
                                       int k, v4i &c4, v2d &v01, v2d &v23)
{
   if (NT) {
      c4 = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(col + k));
      v01 = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(val + k));
      v23 = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(val + k + 2));
   } else {
      c4 = *reinterpret_cast<const v4i *>(col + k);
      v01 = *reinterpret_cast<const v2d *>(val + k);
      v23 = *reinterpret_cast<const v2d *>(val + k + 2);
   }
}

// value-indexed CSR: 4 column ids (16 B) + 4 one-byte value indices (4 B);
// the values come from the matrix's table of distinct values held in LDS
template <bool NT>
__device__ __forceinline__ void stage4_vi(const int *__restrict__ col,
                                          const unsigned char *__restrict__ vidx,
                                          const double *vtab, int k, v4i &c4, v2d &v01, v2d &v23)
{
   unsigned int b;
   if (NT) {
      c4 = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(col + k));
      b = __builtin_nontemporal_load(reinterpret_cast<const unsigned int *>(vidx + k));
   } else {
      c4 = *reinterpret_cast<const v4i *>(col + k);
      b = *reinterpret_cast<const unsigned int *>(vidx + k);
   }
   v01.x = vtab[b & 0xff];
   v01.y = vtab[(b >> 8) & 0xff];
   v23.x = vtab[(b >> 16) & 0xff];
   v23.y = vtab[b >> 24];
}

// one 256*RPT-row tile (body shared by the one-tile-per-workgroup and the
// persistent launch); vtab: the value table (LDS or global)
template <class Cfg, int NEG, bool NEED_DIAG, class Epi, bool VI, bool STAGE_TAB = false>
__device__ __forceinline__ void tile_body(
   int tile, const int *__restrict__ rowptr, const int *__restrict__ col,
   const double *__restrict__ val, const double *__restrict__ x, int rb, int re, const Epi &epi,
   double *__restrict__ partials, const unsigned char *__restrict__ vidx, double *vtab,
   double *prod, double *red, const double *__restrict__ vtab_g = nullptr)
{
   constexpr int RPT = Cfg::rpt, CH = Cfg::ch, TROWS = 256 * RPT;
   const int r0 = rb + tile * TROWS;
   const int r1 = min(r0 + TROWS, re);
   const int tb = rowptr[r0];
   const int te = rowptr[r1];
   int rs[RPT], rend[RPT];
   double acc[RPT], dg[RPT], pf[RPT];
#pragma unroll
   for (int q = 0; q < RPT; q++) {
      const int row = r0 + q * 256 + (int)threadIdx.x;
      rs[q] = rend[q] = 0;
      acc[q] = dg[q] = pf[q] = 0.0;
      if (Cfg::shfl) {
         // rows r0+q*256+lane are consecutive within a wave: rowptr[row+1] is
         // the next lane's rowptr[row]; lane 63 loads its own
         const int rr = min(row, r1);
         const int v = rowptr[rr];
         int nxt = __shfl_down(v, 1, 64);
         if ((threadIdx.x & 63) == 63) nxt = rowptr[min(row + 1, r1)];
         if (row < r1) {
            rs[q] = v;
            rend[q] = nxt;
            acc[q] = epi.init(row);
         }
      } else if (row < r1) {
         rs[q] = rowptr[row];
         rend[q] = rowptr[row + 1];
         acc[q] = epi.init(row);
      }
      // epilogue operands issued before the stream so their latency hides
      if (row < r1) {
         if (NEED_DIAG && !VI) dg[q] = val[rs[q]];
         pf[q] = epi.pf(row);
      }
   }
   if (STAGE_TAB) {
      // the value table, staged after the prologue's loads so its latency
      // overlaps theirs (one barrier)
      vtab[threadIdx.x] = vtab_g[threadIdx.x];
      __syncthreads();
   }
   if (NEED_DIAG && VI) {
#pragma unroll
      for (int q = 0; q < RPT; q++)
         if (r0 + q * 256 + (int)threadIdx.x < r1) dg[q] = vtab[vidx[rs[q]]];
   }
   const int base = tb & ~3;
   for (int cs = base; cs < te; cs += CH) {
      const int ce = min(cs + CH, te);
      if (Cfg::w8) {
         for (int k = cs + 8 * (int)threadIdx.x; k < ce; k += 8 * 256) {
            v4i c4, d4;
            v2d v01, v23, w01, w23;
            if (VI) {
               stage4_vi<Cfg::nt>(col, vidx, vtab, k, c4, v01, v23);
               stage4_vi<Cfg::nt>(col, vidx, vtab, k + 4, d4, w01, w23);
            } else {
               stage4<Cfg::nt>(col, val, k, c4, v01, v23);
               stage4<Cfg::nt>(col, val, k + 4, d4, w01, w23);
            }
            const double x0 = x[c4.x], x1 = x[c4.y], x2 = x[c4.z], x3 = x[c4.w];
            const double x4 = x[d4.x], x5 = x[d4.y], x6 = x[d4.z], x7 = x[d4.w];
            v2d *dst = reinterpret_cast<v2d *>(prod + (k - cs));
            dst[0] = v2d{v01.x * x0, v01.y * x1};
            dst[1] = v2d{v23.x * x2, v23.y * x3};
            dst[2] = v2d{w01.x * x4, w01.y * x5};
            dst[3] = v2d{w23.x * x6, w23.y * x7};
         }
      } else if (Cfg::str) {
         for (int k = cs + (int)threadIdx.x; k < ce; k += 256) {
            const int c = col[k];
            const double v = VI ? vtab[vidx[k]] : val[k];
            prod[k - cs] = v * x[c];
         }
      } else if (Cfg::unr) {
         for (int k = cs + 4 * (int)threadIdx.x; k < ce; k += 8 * 256) {
            const int k2 = k + 4 * 256;
            const bool has2 = k2 < ce;
            v4i c4, d4;
            v2d v01, v23, w01, w23;
            if (VI) {
               stage4_vi<Cfg::nt>(col, vidx, vtab, k, c4, v01, v23);
               if (has2) stage4_vi<Cfg::nt>(col, vidx, vtab, k2, d4, w01, w23);
            } else {
               stage4<Cfg::nt>(col, val, k, c4, v01, v23);
               if (has2) stage4<Cfg::nt>(col, val, k2, d4, w01, w23);
            }
            const double x0 = x[c4.x], x1 = x[c4.y], x2 = x[c4.z], x3 = x[c4.w];
            double y0 = 0, y1 = 0, y2 = 0, y3 = 0;
            if (has2) {
               y0 = x[d4.x];
               y1 = x[d4.y];
               y2 = x[d4.z];
               y3 = x[d4.w];
            }
            v2d p01, p23;
            p01.x = v01.x * x0;
            p01.y = v01.y * x1;
            p23.x = v23.x * x2;
            p23.y = v23.y * x3;
            v2d *dst = reinterpret_cast<v2d *>(prod + (k - cs));
            dst[0] = p01;
            dst[1] = p23;
            if (has2) {
               v2d q01, q23;
               q01.x = w01.x * y0;
               q01.y = w01.y * y1;
               q23.x = w23.x * y2;
               q23.y = w23.y * y3;
               v2d *dst2 = reinterpret_cast<v2d *>(prod + (k2 - cs));
               dst2[0] = q01;
               dst2[1] = q23;
            }
         }
      } else {
         for (int k = cs + 4 * (int)threadIdx.x; k < ce; k += 4 * 256) {
            v4i c4;
            v2d v01, v23;
            if (VI)
               stage4_vi<Cfg::nt>(col, vidx, vtab, k, c4, v01, v23);
            else
               stage4<Cfg::nt>(col, val, k, c4, v01, v23);
            const double x0 = x[c4.x];
            const double x1 = x[c4.y];
            const double x2 = x[c4.z];
            const double x3 = x[c4.w];
            v2d p01, p23;
            p01.x = v01.x * x0;
            p01.y = v01.y * x1;
            p23.x = v23.x * x2;
            p23.y = v23.y * x3;
            v2d *dst = reinterpret_cast<v2d *>(prod + (k - cs));
            dst[0] = p01;
            dst[1] = p23;
         }
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < RPT; q++) {
         const int a = max(rs[q], cs), e = min(rend[q], ce);
         for (int k = a; k < e; ++k) {
            if (NEG)
               acc[q] -= prod[k - cs];
            else
               acc[q] += prod[k - cs];
         }
      }
      if (!Cfg::skipsync || ce < te) __syncthreads(); // WAR on prod before the next chunk
   }
   double sq = 0.0;
#pragma unroll
   for (int q = 0; q < RPT; q++) {
      const int row = r0 + q * 256 + (int)threadIdx.x;
      if (row < r1) {
         const double out = epi.finish(row, acc[q], dg[q], pf[q]);
         sq += out * out;
      }
   }
   if (partials) {
      const double s = block_sum_256(sq, red);
      if (threadIdx.x == 0) partials[tile] = s;
   }
}

template <class Cfg, int NEG, bool NEED_DIAG, class Epi, bool VI = false, bool GTAB = false>
__global__ __launch_bounds__(256) void csr_tile_kernel(
   const int *__restrict__ rowptr, const int *__restrict__ col, const double *__restrict__ val,
   const double *__restrict__ x, int rb, int re, Epi epi, double *__restrict__ partials,
   const unsigned char *__restrict__ vidx = nullptr, const double *__restrict__ vtab_g = nullptr)
{
   __shared__ __attribute__((aligned(16))) double prod[Cfg::ch];
   __shared__ double red[4];
   __shared__ double vtab[(VI && !GTAB) ? 256 : 1];
   int tile = blockIdx.x;
   if (Cfg::xcd) {
      // bijective remap: the blocks dealt to one XCD (b % 8) get a contiguous tile range
      const int nb = gridDim.x, q = nb >> 3, r = nb & 7, xg = tile & 7, idx = tile >> 3;
      tile = (xg < r ? xg * (q + 1) : r * (q + 1) + (xg - r) * q) + idx;
   }

   tile_body<Cfg, NEG, NEED_DIAG, Epi, VI, VI && !GTAB>(tile, rowptr, col, val, x, rb, re, epi,
                                                        partials, vidx,
                                                        GTAB ? const_cast<double *>(vtab_g) : vtab,
                                                        prod, red, vtab_g);
}

// persistent form: gridDim.x workgroups walk the tiles t, t + gridDim.x, ...
template <class Cfg, int NEG, bool NEED_DIAG, class Epi, bool VI = false>
__global__ __launch_bounds__(256) void csr_ptile_kernel(
   const int *__restrict__ rowptr, const int *__restrict__ col, const double *__restrict__ val,
   const double *__restrict__ x, int rb, int re, Epi epi, double *__restrict__ partials,
   const unsigned char *__restrict__ vidx, const double *__restrict__ vtab_g, int ntiles)
{
   __shared__ __attribute__((aligned(16))) double prod[Cfg::ch];
   __shared__ double red[4];
   __shared__ double vtab[VI ? 256 : 1];
   if (VI) {
      vtab[threadIdx.x] = vtab_g[threadIdx.x];
      __syncthreads();
   }
   for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      tile_body<Cfg, NEG, NEED_DIAG, Epi, VI>(tile, rowptr, col, val, x, rb, re, epi, partials, vidx,
                                              vtab, prod, red);
      __syncthreads();
   }
}

// Dictionary-coded CSR (CSR-DC) kernel, lane per row.  For operators whose
// (column - row, value) pairs fit a 256-entry dictionary (stencil and
// structured Galerkin operators) every entry is one byte: col = row +
// off[b], a_ij = val[b].  The tile's entry bytes are staged into LDS with
// coalesced 8-byte loads; each lane then walks its own row in CSR order,
// issuing up to 8 independent x loads at a time -- and because neighbouring
// lanes own neighbouring rows, the j-th load of a wave reads x[row + off]
// for 64 consecutive rows: a coalesced gather.  Each lane sums its row
// sequentially: bit-identical to the other kernels.  Rows of at most
// AMG_DC_MAXROW entries (checked at registration).
template <int NEG, bool NEED_DIAG, class Epi, int RPL = 2, bool STAGE = true, int MAXR = AMG_DC_MAXROW>
__global__ __launch_bounds__(256) void csr_dc_kernel(
   const int *__restrict__ rowptr, const unsigned char *__restrict__ didx,
   const int *__restrict__ doff_g, const double *__restrict__ dval_g, const double *__restrict__ x,
   int rb, int re, Epi epi, double *__restrict__ partials, int T, const int *__restrict__ anch)
{
   // RPL rows per lane (lane owns rows r0 + q*256 + lane); STAGE: the tile's
   // entry bytes go through LDS (coalesced 8-byte loads) instead of each lane
   // reading its row's bytes from global memory
   __shared__ int otab[256];
   __shared__ double vtab[256];
   __shared__ __attribute__((aligned(16))) unsigned char ent[STAGE ? 256 * RPL * MAXR + 32 : 8];
   __shared__ double red[4];
   const int tid = (int)threadIdx.x;
   const int wg = (int)blockIdx.x;
   const int r0 = rb + wg * 256 * RPL, r1 = min(r0 + 256 * RPL, re);
   int rs[RPL], rend[RPL], an[RPL];
   double acc[RPL], pf[RPL];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = r0 + q * 256 + tid;
      rs[q] = rend[q] = 0;
      an[q] = row;
      acc[q] = pf[q] = 0.0;
      if (row < r1) {
         rs[q] = rowptr[row];
         rend[q] = rowptr[row + 1];
         if (anch) an[q] = anch[row];
         acc[q] = epi.init(row);
         pf[q] = epi.pf(row);
      }
   }
   if (tid < T) {
      otab[tid] = doff_g[tid];
      vtab[tid] = dval_g[tid];
   }
   int base = 0;
   if (STAGE) {
      const int tb = rowptr[r0], te = rowptr[r1];
      base = tb & ~7;
      const int nw = (te - base + 8 + 7) >> 3; // one extra word: a_ii of an empty last row
      const unsigned long long *src = reinterpret_cast<const unsigned long long *>(didx + base);
      unsigned long long *dst = reinterpret_cast<unsigned long long *>(ent);
      for (int w = tid; w < nw; w += 256) dst[w] = src[w];
   }
   __syncthreads();
   double sq[RPL];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = r0 + q * 256 + tid;
      sq[q] = 0.0;
      if (row >= r1) continue;
      auto eb = [&](int k) -> int { return STAGE ? ent[k - base] : didx[k]; };
      double dg = 0.0;
      if (NEED_DIAG) dg = vtab[eb(rs[q])]; // a_ii := A_data[A_i[i]]
      for (int k = rs[q]; k < rend[q]; k += 8) {
         const int m = rend[q] - k;
         double xv[8], vv[8];
#pragma unroll
         for (int j = 0; j < 8; j++) {
            xv[j] = 0.0;
            vv[j] = 0.0;
            if (j < m) {
               const int bb = eb(k + j);
               vv[j] = vtab[bb];
               xv[j] = x[an[q] + otab[bb]];
            }
         }
#pragma unroll
         for (int j = 0; j < 8; j++)
            if (j < m) {
               if (NEG)
                  acc[q] -= vv[j] * xv[j];
               else
                  acc[q] += vv[j] * xv[j];
            }
      }
      const double out = epi.finish(row, acc[q], dg, pf[q]);
      sq[q] = out * out;
   }
   if (partials) {
      // one partial per 256-row tile, the layout of the tile kernel
#pragma unroll
      for (int q = 0; q < RPL; q++) {
         const double sblk = block_sum_256(sq[q], red);
         if (tid == 0 && r0 + q * 256 < r1) partials[wg * RPL + q] = sblk;
      }
   }
}

// Row-pattern-coded CSR (on top of the dictionary): every row is one byte
// naming its sequence of dictionary entries (the pattern table holds <= 256
// distinct sequences of <= MAXR entries), so the kernel streams one byte per
// ROW and no row pointer.  Lane owns rows r0 + q*256 + tid; the row's entries
// are walked in CSR order from the LDS pattern table, exactly as the
// dictionary-coded kernel walks its staged bytes.  Every row is non-empty.
template <int NEG, bool NEED_DIAG, class Epi, int RPL>
__global__ __launch_bounds__(256) void csr_rp_kernel(
   const unsigned char *__restrict__ rpat, const unsigned char *__restrict__ ptab_g, int np,
   const int *__restrict__ doff_g, const double *__restrict__ dval_g, const double *__restrict__ x,
   int rb, int re, Epi epi, double *__restrict__ partials, int T, const int *__restrict__ anch)
{
   constexpr int PS = AMG_RP_STRIDE; // bytes per pattern: length, then the entries
   __shared__ int otab[256];
   __shared__ double vtab[256];
   __shared__ __attribute__((aligned(16))) unsigned char ptab[256 * PS];
   __shared__ double red[4];
   const int tid = (int)threadIdx.x;
   if (tid < T) {
      otab[tid] = doff_g[tid];
      vtab[tid] = dval_g[tid];
   }
   {
      const int nw = (np * PS) >> 2;
      const unsigned int *src = reinterpret_cast<const unsigned int *>(ptab_g);
      unsigned int *dst = reinterpret_cast<unsigned int *>(ptab);
      for (int w = tid; w < nw; w += 256) dst[w] = src[w];
   }
   const int wg = (int)blockIdx.x;
   const int r0 = rb + wg * 256 * RPL, r1 = min(r0 + 256 * RPL, re);
   int pid[RPL], an[RPL];
   double acc[RPL], pf[RPL];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = r0 + q * 256 + tid;
      pid[q] = 0;
      an[q] = row;
      acc[q] = pf[q] = 0.0;
      if (row < r1) {
         pid[q] = rpat[row];
         if (anch) an[q] = anch[row];
         acc[q] = epi.init(row);
         pf[q] = epi.pf(row);
      }
   }
   __syncthreads();
   double sq[RPL];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = r0 + q * 256 + tid;
      sq[q] = 0.0;
      if (row >= r1) continue;
      const unsigned char *pp = ptab + pid[q] * PS;
      const int len = pp[0];
      double dg = 0.0;
      if (NEED_DIAG) dg = vtab[pp[1]]; // a_ii := A_data[A_i[i]]
      for (int k = 0; k < len; k += 8) {
         const int m = len - k;
         double xv[8], vv[8];
#pragma unroll
         for (int j = 0; j < 8; j++) {
            xv[j] = 0.0;
            vv[j] = 0.0;
            if (j < m) {
               const int bb = pp[1 + k + j];
               vv[j] = vtab[bb];
               xv[j] = x[an[q] + otab[bb]];
            }
         }
#pragma unroll
         for (int j = 0; j < 8; j++)
            if (j < m) {
               if (NEG)
                  acc[q] -= vv[j] * xv[j];
               else
                  acc[q] += vv[j] * xv[j];
            }
      }
      const double out = epi.finish(row, acc[q], dg, pf[q]);
      sq[q] = out * out;
   }
   if (partials) {
#pragma unroll
      for (int q = 0; q < RPL; q++) {
         const double sblk = block_sum_256(sq[q], red);
         if (tid == 0 && r0 + q * 256 < r1) partials[wg * RPL + q] = sblk;
      }
   }
}

// Paired-row-pattern kernel: lane owns the row pair (2t, 2t+1) and reads the
// pair's merged entry list (ps words in LDS).  Columns are relative to the
// pair's base: row 2t itself for square diagonal-first operators, else row
// 2t's anchor (its first column; interpolation / restriction), with row 2t+1's
// anchor at base + da (da = 1 for square operators, from the header word for
// anchored ones).  An entry of row 2t at column c matched with an entry of row
// 2t+1 at column c + 1 reads both x values with ONE 16-byte load (half the
// vector-memory instructions of one lane per row, which bounds the single-row
// kernel: DESIGN.md Sec.4); an entry of one row alone reads its x value by
// itself.  Each row still sums its own entries in its CSR order (the merge
// keeps both orders), so results are bit-identical.  The header word also
// carries each row's first dictionary entry (a_ii, no scan).  Workgroup slab
// q covers 512 rows = two 256-row norm tiles; the tiles' sums are reduced
// after every slab is done (no barrier between slabs), in the single-row
// kernel's lane order.  rb must be even.
// OPT bit 1: a_ii from the header word (else scanned from the entry list)
// Jacobi-form epilogues read x[i] of the gathered vector itself: when every
// pair's first merged entry is both rows' diagonal (c0, square diag-first
// operators), that operand is the first gather, not a load of its own.
struct EpiJacobi;
struct EpiL1Jacobi;
struct EpiResJacobi;
template <class Epi>
struct pf_is_x {
   static constexpr bool value = false;
};
template <>
struct pf_is_x<EpiJacobi> {
   static constexpr bool value = true;
};
template <>
struct pf_is_x<EpiL1Jacobi> {
   static constexpr bool value = true;
};
template <>
struct pf_is_x<EpiResJacobi> {
   static constexpr bool value = true;
};
// the epilogue's operand vector (found by ADL at instantiation)
template <class Epi>
__device__ __forceinline__ const double *epi_pf_vec(const Epi &)
{
   return nullptr;
}

template <int NEG, bool NEED_DIAG, class Epi, int RPL, int OPT = AMG_RPP_OPT>
__global__ __launch_bounds__(256) void csr_rpp_kernel(
   const unsigned char *__restrict__ ppat, const unsigned int *__restrict__ pptab_g, int np,
   const int *__restrict__ doff_g, const double *__restrict__ dval_g, const double *__restrict__ x,
   int rb, int re, Epi epi, double *__restrict__ partials, int T, int PS, const int *__restrict__ anch,
   int c0, const int *__restrict__ pbase = nullptr, const unsigned short *__restrict__ pdelta = nullptr)
{
   const bool xc = pf_is_x<Epi>::value && c0 && epi_pf_vec(epi) == x;
   __shared__ int otab[256];
   __shared__ double vtab[256];
   extern __shared__ unsigned int ptab[]; // np * PS words (dynamic)
   __shared__ double red[RPL * 8];
   const int tid = (int)threadIdx.x;
   if (tid < T) {
      otab[tid] = doff_g[tid];
      vtab[tid] = dval_g[tid];
   }
   for (int w = tid; w < np * PS; w += 256) ptab[w] = pptab_g[w];
   const int wg = (int)blockIdx.x;
   int pid[RPL], base[RPL];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = rb + (wg * RPL + q) * 512 + 2 * tid;
      pid[q] = row < re ? ppat[row >> 1] : 0;
      base[q] = row;
      if (pdelta) {
         if (row < re) base[q] = pbase[row >> 9] + (int)pdelta[row >> 1];
      } else if (anch && row < re) {
         base[q] = anch[row];
      }
   }
   __syncthreads();
   double sq[RPL][2];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int s0 = rb + (wg * RPL + q) * 512;
      const int row = s0 + 2 * tid;
      const bool a0 = row < re, a1 = row + 1 < re;
      sq[q][0] = sq[q][1] = 0.0;
      if (a0) {
         const unsigned int *pp = ptab + pid[q] * PS;
         const unsigned int hd = pp[0];
         const int nel = hd & 0xff;
         // row 2t+1's columns: base + da + offset
         const int b1 = base[q] + (anch ? (int)(hd >> 25) - 16 : 1);
         v2d acc, pf{0.0, 0.0};
         if (a1) {
            acc = epi.init2(row);
            if (!xc) pf = epi.pf2(row);
         } else {
            acc = v2d{epi.init(row), 0.0};
            if (!xc) pf = v2d{epi.pf(row), 0.0};
         }
         for (int k = 0; k < nel; k += 8) {
            const int m = nel - k;
            v2d xv[8];
            unsigned int ew[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
               ew[j] = 0;
               xv[j] = v2d{0.0, 0.0};
               if (j < m) {
                  const unsigned int w = pp[1 + k + j];
                  ew[j] = w;
                  const int d0 = w & 0xff, d1 = (w >> 8) & 0xff;
                  if ((w >> 16 & 3) == 3)
                     xv[j] = *reinterpret_cast<const v2du *>(x + base[q] + otab[d0]);
                  else if (w >> 16 & 1)
                     xv[j].x = x[base[q] + otab[d0]];
                  else
                     xv[j].y = x[b1 + otab[d1]];
               }
            }
            if (xc && k == 0) pf = xv[0]; // x[2t], x[2t+1]: the diagonal entry
#pragma unroll
            for (int j = 0; j < 8; j++)
               if (j < m) {
                  const unsigned int w = ew[j];
                  if (w >> 16 & 1) {
                     const double v = vtab[w & 0xff];
                     if (NEG)
                        acc.x -= v * xv[j].x;
                     else
                        acc.x += v * xv[j].x;
                  }
                  if (w >> 17 & 1) {
                     const double v = vtab[(w >> 8) & 0xff];
                     if (NEG)
                        acc.y -= v * xv[j].y;
                     else
                        acc.y += v * xv[j].y;
                  }
               }
         }
         // a_ii := A_data[A_i[i]]: each row's first dictionary entry
         double dg0 = 0.0, dg1 = 0.0;
         if (NEED_DIAG && (OPT & 2)) {
            dg0 = vtab[(hd >> 8) & 0xff];
            dg1 = a1 ? vtab[(hd >> 16) & 0xff] : 0.0;
         } else if (NEED_DIAG) {
            bool f0 = false, f1 = false;
            for (int e = 0; e < nel && !(f0 && f1); e++) {
               const unsigned int w = pp[1 + e];
               if (!f0 && (w >> 16 & 1)) {
                  dg0 = vtab[w & 0xff];
                  f0 = true;
               }
               if (!f1 && (w >> 17 & 1)) {
                  dg1 = vtab[(w >> 8) & 0xff];
                  f1 = true;
               }
            }
         }
         if (a1) {
            const v2d out = epi.finish2(row, acc, v2d{dg0, dg1}, pf);
            sq[q][0] = out.x * out.x;
            sq[q][1] = out.y * out.y;
         } else {
            const double out = epi.finish(row, acc.x, dg0, pf.x);
            sq[q][0] = out * out;
         }
      }
   }
   if (partials) {
      // the 256-row tiles' sums in block_sum_256's order (single-row kernel):
      // its wave tree over 64 rows v[r] += v[r + off], off = 32 .. 1, is run
      // on the 32 lanes holding those rows (lane l: rows 2l, 2l+1), so every
      // addition has the same operands; then ((g0 + g1) + g2) + g3 over the
      // tile's four 64-row groups
#pragma unroll
      for (int q = 0; q < RPL; q++) {
         double a = sq[q][0], b = sq[q][1];
#pragma unroll
         for (int off = 16; off > 0; off >>= 1) {
            a += __shfl_down(a, off, 32);
            b += __shfl_down(b, off, 32);
         }
         if ((tid & 31) == 0) red[q * 8 + (tid >> 5)] = a + b;
      }
      __syncthreads();
      if (tid < 2 * RPL) {
         const int tile = wg * RPL * 2 + tid;
         if (rb + tile * 256 < re)
            partials[tile] = ((red[tid * 4] + red[tid * 4 + 1]) + red[tid * 4 + 2]) + red[tid * 4 + 3];
      }
   }
}

// Master-pattern kernel (square diagonal-first operators, amg_internal.h):
// the lane/row mapping, epilogues and norm partials of csr_rpp_kernel, but the
// entry walk is over the master list, whose column offsets (and, when
// UNI, values) are wave-uniform kernel arguments.  Per pair only the 64-bit
// use mask (and, without UNI, the pattern's value pairs) comes from LDS.  An
// entry both rows use is one 16-byte load of x[i+o], x[i+1+o]; each row adds
// its used entries in master order = its CSR order (bit-identical).
struct MpSten {
   int off[AMG_MP_MAXJ];
   double val[AMG_MP_MAXJ];
};

// exact per-entry gather (csr_mp_kernel FORM 1): row 2t's operand loaded only
// when it uses the entry, row 2t+1's likewise, one 16-byte load when both do
template <int NEG, int JM, bool UNI>
__device__ __forceinline__ v2d mp_gather_exact(v2d acc, v2d &pf, bool xc, unsigned long long mk,
                                               const v2d *vp, int J, const MpSten &S,
                                               const double *__restrict__ x, int row)
{
#pragma unroll
   for (int k = 0; k < JM; k += 8) {
      if (k < J) {
         v2d xv[8];
#pragma unroll
         for (int j = 0; j < 8; j++) {
            xv[j] = v2d{0.0, 0.0};
            if (k + j < J) {
               const unsigned int b = (unsigned int)(mk >> (2 * (k + j))) & 3u;
               const double *xp = x + row + S.off[k + j];
               if (b == 3)
                  xv[j] = *reinterpret_cast<const v2du *>(xp);
               else if (b == 1)
                  xv[j].x = xp[0];
               else if (b == 2)
                  xv[j].y = xp[1];
            }
         }
         if (k == 0 && xc) pf = xv[0]; // master entry 0: both rows' diagonal
#pragma unroll
         for (int j = 0; j < 8; j++)
            if (k + j < J) {
               const unsigned int b = (unsigned int)(mk >> (2 * (k + j))) & 3u;
               const v2d v = UNI ? v2d{S.val[k + j], S.val[k + j]} : vp[k + j];
               if (b & 1) acc.x = NEG ? acc.x - v.x * xv[j].x : acc.x + v.x * xv[j].x;
               if (b & 2) acc.y = NEG ? acc.y - v.y * xv[j].y : acc.y + v.y * xv[j].y;
            }
      }
   }
   return acc;
}

// FORM 3 (default): 16-byte gather of every entry, unused entries re-read the
// pair's own x (no branches), edge waves through mp_gather_exact; FORM 1:
// mp_gather_exact everywhere; FORM 0: branch-free clamped gather; FORM 2: as
// FORM 3 with a branch per entry (tools/tune_spmv.py mp_*)
template <int NEG, bool NEED_DIAG, class Epi, int JM, bool UNI, int FORM = 3, int RPL = 2>
__global__ __launch_bounds__(256) void csr_mp_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, int J, MpSten S, const double *__restrict__ x, int N, int rb, int re, Epi epi,
   double *__restrict__ partials)
{
   const bool xc = pf_is_x<Epi>::value && epi_pf_vec(epi) == x;
   __shared__ unsigned long long mtab[256];
   extern __shared__ v2d mval[]; // np * J value pairs (UNI: unused)
   __shared__ double red[RPL * 8];
   const int tid = (int)threadIdx.x;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (!UNI)
      for (int w = tid; w < np * J; w += 256) mval[w] = mval_g[w];
   const int wg = (int)blockIdx.x;
   int pid[RPL];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = rb + (wg * RPL + q) * 512 + 2 * tid;
      pid[q] = row < re ? ppat[row >> 1] : 0;
   }
   __syncthreads();
   double sq[RPL][2];
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = rb + (wg * RPL + q) * 512 + 2 * tid;
      const bool a0 = row < re, a1 = row + 1 < re;
      sq[q][0] = sq[q][1] = 0.0;
      if (a0) {
         const unsigned long long mk = mtab[pid[q]];
         const v2d *vp = mval + pid[q] * J;
         v2d acc, pf{0.0, 0.0};
         if (a1) {
            acc = epi.init2(row);
            if (!xc) pf = epi.pf2(row);
         } else {
            acc = v2d{epi.init(row), 0.0};
            if (!xc) pf = v2d{epi.pf(row), 0.0};
         }
         if constexpr (FORM == 1) {
            acc = mp_gather_exact<NEG, JM, UNI>(acc, pf, xc, mk, vp, J, S, x, row);
         } else if constexpr (FORM == 2 || FORM == 3) {
         // A used entry is one 16-byte load of x[row + o], x[row + o + 1]
         // whichever of the pair's rows use it: inside x whenever
         // row + omin >= 0 and row + omax + 2 <= N (omin/omax over the master
         // offsets; FORM 3's unused entries read x[row], x[row + 1]).  Waves
         // holding a row outside that window (for the 7-pt stencil the first
         // and last two planes) take the exact per-entry form.
         int omin = 0, omax = 0;
         for (int j = 0; j < J; j++) {
            omin = min(omin, S.off[j]);
            omax = max(omax, S.off[j]);
         }
         const bool edge = (long long)row + omin < 0 || (long long)row + omax + 2 > N;
         if (__any(edge)) {
            acc = mp_gather_exact<NEG, JM, UNI>(acc, pf, xc, mk, vp, J, S, x, row);
         } else {
#pragma unroll
         for (int k = 0; k < JM; k += 8) {
            if (k < J) {
               v2d xv[8];
#pragma unroll
               for (int j = 0; j < 8; j++) {
                  if (FORM == 3) {
                     // unused entries re-read the pair's own x[row], x[row+1]
                     const int o = ((mk >> (2 * (k + j))) & 3u) ? S.off[k + j] : 0;
                     xv[j] = *reinterpret_cast<const v2du *>(x + row + o);
                  } else {
                     xv[j] = v2d{0.0, 0.0};
                     if ((mk >> (2 * (k + j))) & 3u) xv[j] = *reinterpret_cast<const v2du *>(x + row + S.off[k + j]);
                  }
               }
               if (k == 0 && xc) pf = xv[0];
#pragma unroll
               for (int j = 0; j < 8; j++) {
                  const unsigned int b = (unsigned int)(mk >> (2 * (k + j))) & 3u;
                  const v2d v = UNI ? v2d{S.val[k + j], S.val[k + j]} : vp[min(k + j, J - 1)];
                  if (b & 1) acc.x = NEG ? acc.x - v.x * xv[j].x : acc.x + v.x * xv[j].x;
                  if (b & 2) acc.y = NEG ? acc.y - v.y * xv[j].y : acc.y + v.y * xv[j].y;
               }
            }
         }
         }
         } else {
#pragma unroll
         for (int k = 0; k < JM; k += 8) {
            if (k < J) {
               // branch-free gather: every entry issues one 16-byte load at
               // s = clamp(row + o, 0, N - 2), which covers the element(s) the
               // pair's used rows need (row 2t: row + o, row 2t+1: row + 1 + o,
               // both in [0, N)); unused entries load a harmless in-range word.
               // All loads of a chunk are in flight together.
               v2d xv[8];
               bool lo[8];
#pragma unroll
               for (int j = 0; j < 8; j++) {
                  const int base = row + S.off[k + j];
                  const int sidx = min(max(base, 0), N - 2);
                  lo[j] = sidx == base;
                  xv[j] = *reinterpret_cast<const v2du *>(x + sidx);
               }
               // entries past J: offset 0 (a valid load), use bits 0
#pragma unroll
               for (int j = 0; j < 8; j++) {
                     const unsigned int b = (unsigned int)(mk >> (2 * (k + j))) & 3u;
                     const double x0 = lo[j] ? xv[j].x : xv[j].y; // row 2t's operand
                     const double x1 = lo[j] ? xv[j].y : xv[j].x; // row 2t+1's operand
                     if (k + j == 0 && xc) pf = v2d{x0, x1}; // master entry 0: both rows' diagonal
                     const v2d v = UNI ? v2d{S.val[k + j], S.val[k + j]} : vp[min(k + j, J - 1)];
                     const double s0 = NEG ? acc.x - v.x * x0 : acc.x + v.x * x0;
                     const double s1 = NEG ? acc.y - v.y * x1 : acc.y + v.y * x1;
                     acc.x = (b & 1) ? s0 : acc.x;
                     acc.y = (b & 2) ? s1 : acc.y;
               }
            }
         }
         }
         // a_ii := A_data[A_i[i]]: master entry 0 (every row's first entry)
         v2d dg{0.0, 0.0};
         if (NEED_DIAG) {
            dg = UNI ? v2d{S.val[0], S.val[0]} : vp[0];
            if (!a1) dg.y = 0.0;
         }
         if (a1) {
            const v2d out = epi.finish2(row, acc, dg, pf);
            sq[q][0] = out.x * out.x;
            sq[q][1] = out.y * out.y;
         } else {
            const double out = epi.finish(row, acc.x, dg.x, pf.x);
            sq[q][0] = out * out;
         }
      }
   }
   if (partials) {
      // csr_rpp_kernel's tile sums (block_sum_256's order)
#pragma unroll
      for (int q = 0; q < RPL; q++) {
         double a = sq[q][0], b = sq[q][1];
#pragma unroll
         for (int off = 16; off > 0; off >>= 1) {
            a += __shfl_down(a, off, 32);
            b += __shfl_down(b, off, 32);
         }
         if ((tid & 31) == 0) red[q * 8 + (tid >> 5)] = a + b;
      }
      __syncthreads();
      if (tid < 2 * RPL) {
         const int tile = wg * RPL * 2 + tid;
         if (rb + tile * 256 < re)
            partials[tile] = ((red[tid * 4] + red[tid * 4 + 1]) + red[tid * 4 + 2]) + red[tid * 4 + 3];
      }
   }
}

template <int NEG, bool NEED_DIAG, class Epi>
static void launch_mp(hipStream_t s, const amg_mat *A, const double *x, int rb, int re, const Epi &e,
                      double *partials)
{
   MpSten S;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      S.off[j] = A->mp_off[j];
      S.val[j] = A->mp_val[j];
   }
   const int nb = (re - rb + 1023) / 1024;
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
   const size_t lds = A->mp_uni ? 0 : (size_t)A->pp_n * A->mp_J * sizeof(v2d);
   if (A->mp_J <= 8) {
      if (A->mp_uni)
         csr_mp_kernel<NEG, NEED_DIAG, Epi, 8, true><<<nb, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, A->mp_J,
                                                                      S, x, A->ncols, rb, re, e, partials);
      else
         csr_mp_kernel<NEG, NEED_DIAG, Epi, 8, false><<<nb, 256, lds, s>>>(A->ppat, A->mpmask, A->pp_n, mv,
                                                                         A->mp_J, S, x, A->ncols, rb, re, e, partials);
   } else {
      if (A->mp_uni)
         csr_mp_kernel<NEG, NEED_DIAG, Epi, AMG_MP_MAXJ, true><<<nb, 256, 0, s>>>(
            A->ppat, A->mpmask, A->pp_n, mv, A->mp_J, S, x, A->ncols, rb, re, e, partials);
      else
         csr_mp_kernel<NEG, NEED_DIAG, Epi, AMG_MP_MAXJ, false><<<nb, 256, lds, s>>>(
            A->ppat, A->mpmask, A->pp_n, mv, A->mp_J, S, x, A->ncols, rb, re, e, partials);
   }
}

// ---------------------------------------------------------------------------
// Plane-marching master kernel (csr_mz_kernel): master-coded operators whose
// 7-entry master list is [0, -P, -S, -1, +1, +S, +P] with N = nz * P and
// P % 512 == 0 -- the 7-pt stencil of an nx * ny * nz box (S = nx, P = nx ny)
// in the reference's diagonal-first row order.  The use masks (ppat + mpmask)
// still decide which entries every row adds, so the result is exact for ANY
// matrix with that master list; the geometry only decides where the operands
// come from:
//   * a workgroup owns 512 consecutive in-plane positions (lane t: rows
//     pos = 2t, 2t + 1) and marches over a chunk of ZC planes;
//   * x of planes k - 1, k, k + 1 stay in registers (the +-P entries and the
//     diagonal), plane k + 2 is prefetched one iteration ahead, so every x
//     element is loaded from HBM once per chunk instead of three times;
//   * +-1 come from the neighbour lanes (ds_bpermute), the wave's two edge
//     operands from one two-lane load; +-S are 16-byte loads of the lines the
//     neighbouring workgroups stream at the same time (L2 hits with the
//     XCD-contiguous workgroup order below).
// Each row adds its used entries in master order = its CSR order, and the
// norm partials are csr_mp_kernel's (one per 256-row tile, block_sum_256's
// operand order), so every output and every partial is bit-identical.
// Per pair of rows: 6 memory instructions (f, x[k+2], x[-S], x[+S], the
// pattern byte, the store) against 10 in csr_mp_kernel.
// ---------------------------------------------------------------------------
constexpr int AMG_MZ_MAXZC = 64;

// 16-byte / 8-byte loads at a 32-bit element index from a wave-uniform base:
// the byte offset stays a zero-extended 32-bit VGPR (global_load ... off,
// s[base] addressing: one VGPR per address, no 64-bit address arithmetic);
// callers guarantee 8 * index < 2^32
__device__ __forceinline__ v2d ld2u(const double *b, unsigned i)
{
   return *reinterpret_cast<const v2du *>(reinterpret_cast<const char *>(b) + (size_t)(i * 8u));
}
__device__ __forceinline__ double ld1u(const double *b, unsigned i)
{
   return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(b) + (size_t)(i * 8u));
}

// 16-byte load; nt bit 1: nontemporal (a streamed right-hand side)
__device__ __forceinline__ v2d ld2nt(const double *p, int nt)
{
   if (nt & 2) return __builtin_nontemporal_load(reinterpret_cast<const v2du *>(p));
   return *reinterpret_cast<const v2du *>(p);
}

// streaming hints (st2 / ld2nt bits) for levels whose vectors exceed the
// Infinity Cache (ctx->mz_nt, AMG_MZ_NT)
static int stream_hint(const amg_mat *A)
{
   return (long long)A->nrows * 8 > (512LL << 20) ? A->ctx->mz_nt : 0;
}

// the 7 master entries of a row pair in master (= CSR) order; a wave whose
// pairs all use every entry (the box interior) skips the per-entry use tests
template <int NEG, bool UNI>
__device__ __forceinline__ v2d mz_acc7(v2d acc, const v2d (&xv)[7], unsigned long long mk, const MpSten &Sv,
                                       const v2d *mvp)
{
   if (__all(mk == 0x3FFFull)) {
#pragma unroll
      for (int j = 0; j < 7; j++) {
         const v2d v = UNI ? v2d{Sv.val[j], Sv.val[j]} : mvp[j];
         acc.x = NEG ? acc.x - v.x * xv[j].x : acc.x + v.x * xv[j].x;
         acc.y = NEG ? acc.y - v.y * xv[j].y : acc.y + v.y * xv[j].y;
      }
   } else {
#pragma unroll
      for (int j = 0; j < 7; j++) {
         const unsigned int b = (unsigned int)(mk >> (2 * j)) & 3u;
         const v2d v = UNI ? v2d{Sv.val[j], Sv.val[j]} : mvp[j];
         if (b & 1) acc.x = NEG ? acc.x - v.x * xv[j].x : acc.x + v.x * xv[j].x;
         if (b & 2) acc.y = NEG ? acc.y - v.y * xv[j].y : acc.y + v.y * xv[j].y;
      }
   }
   return acc;
}

// NLN lines per lane (register blocking in y): the workgroup holds NLN
// adjacent lines of 512 positions, a lane keeps x of its NLN lines for planes
// k - 1, k, k + 1, so the +-S operands of its inner lines come from registers
// and only the two halo lines are loaded per plane (2 / NLN line loads per line
// instead of 2).  NLN > 1 needs S % 512 == 0 and NLN | P / S.
//
// HPF (halo prefetch, ctx->mz_pf == 3): the +-S lines, wave-edge elements and
// pattern bytes of plane k + 2 are loaded in iteration k, together with the
// workgroup's own line of that plane -- the three workgroups that read a line
// of x (as their own line and as the +-S operands of the lines beside it) then
// read it in the same iteration instead of two iterations apart, when the
// 2.3 MB per iteration that an XCD's resident workgroups stream has evicted
// it from the 4 MB L2 (two PlaneIn sets held: planes k and k + 1)
template <int NEG, bool NEED_DIAG, class Epi, bool UNI, int NLN = 1, int PF = 1, int WPE = 0, int HPF = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1))) void csr_mz_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, MpSten Sv, const double *__restrict__ x, int P, int S, int nz, int zc,
   int npb, int xcd, Epi epi, double *__restrict__ partials, int kb, int ke)
{
   const bool xc_pf = pf_is_x<Epi>::value && epi_pf_vec(epi) == x;
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 256 * 7];
   __shared__ double red[AMG_MZ_MAXZC * 8 * NLN];
   const int tid = (int)threadIdx.x, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (!UNI)
      for (int w = tid; w < np * 7; w += 256) mval[w] = mval_g[w];
   // XCD-contiguous order: hardware workgroup w runs on XCD w % 8; give XCD j
   // the logical range [j G/8, (j+1) G/8) so neighbouring lines (the +-S
   // operands) are streamed by the same L2
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   // planes [kb, ke) of the nz-plane operator (a z-slab's owned planes; the
   // planes outside stay readable as x operands)
   const int k0 = kb + chunk * zc, k1 = min(k0 + zc, ke);
   int blk0 = pblk * 512; // plane offset of the workgroup's first line block
   if (NLN > 1) {
      const int nbx = S / 512;
      blk0 = (pblk / nbx) * NLN * S + (pblk % nbx) * 512;
   }
   const int pos = blk0 + 2 * tid;
   const unsigned Nu = (unsigned)((long long)nz * P);
   v2d xm[NLN], xc[NLN], xq[NLN];
#pragma unroll
   for (int i = 0; i < NLN; i++) {
      const unsigned p = (unsigned)(pos + i * S);
      xm[i] = k0 > 0 ? ld2u(x, (unsigned)(k0 - 1) * P + p) : v2d{0.0, 0.0};
      xc[i] = ld2u(x, (unsigned)k0 * P + p);
      xq[i] = k0 + 1 < nz ? ld2u(x, (unsigned)(k0 + 1) * P + p) : v2d{0.0, 0.0};
   }
   // PF = 2: plane k + 2 arrives one iteration early (q2), plane k + 3 is in
   // flight while plane k is computed
   v2d q2[PF == 2 ? NLN : 1];
#pragma unroll
   for (int i = 0; i < (PF == 2 ? NLN : 1); i++) {
      q2[i] = v2d{0.0, 0.0};
      if (PF == 2 && k0 + 2 < nz && k0 + 1 < k1) q2[i] = ld2u(x, (unsigned)(k0 + 2) * P + (unsigned)(pos + i * S));
   }
   // HPF 1 / 2: halo operands one / two planes ahead; 3 / 4: the same with the
   // epilogue's first operand (the right-hand side) too
   constexpr int HD = HPF > 2 ? HPF - 2 : HPF;
   constexpr bool HF = HPF > 2;
   struct PlaneIn {
      v2d ym, yp; // halo lines: below the first, above the last
      double e[NLN];
      int pid[NLN];
      v2d a0[NLN]; // HF: epi.init2
   };
   auto fetch = [&](int k, PlaneIn &in) {
      const unsigned row = (unsigned)k * P + pos;
      if (HF)
#pragma unroll
         for (int i = 0; i < NLN; i++) in.a0[i] = epi.init2((int)(row + (unsigned)(i * S)));
      in.ym = ld2u(x, row >= (unsigned)S ? row - S : 0u);
      const unsigned rp = row + (unsigned)(NLN * S);
      in.yp = ld2u(x, rp + 2 <= Nu ? rp : Nu - 2);
#pragma unroll
      for (int i = 0; i < NLN; i++) {
         const unsigned ri = row + (unsigned)(i * S);
         in.pid[i] = ppat[ri >> 1];
         in.e[i] = 0.0;
         if (lane == 0 && ri > 0) in.e[i] = ld1u(x, ri - 1);
         if (lane == 63 && ri + 2 < Nu) in.e[i] = ld1u(x, ri + 2);
      }
   };
   PlaneIn h0{}, h1{}; // HD 2: planes k, k + 1; HD 1: plane k in h0
   if (HD) fetch(k0, h0);
   if (HD == 2 && k0 + 1 < k1) fetch(k0 + 1, h1);
   __syncthreads();
   for (int k = k0; k < k1; k++) {
      const unsigned row0 = (unsigned)k * P + pos;
      // prefetch plane k + PF + 1 (this chunk's last iteration needs plane k1)
      v2d xn[NLN];
#pragma unroll
      for (int i = 0; i < NLN; i++) {
         xn[i] = v2d{0.0, 0.0};
         if (k + PF + 1 < nz && k + PF < k1) xn[i] = ld2u(x, row0 + (unsigned)(i * S) + (PF + 1u) * P);
      }
      PlaneIn cur;
      if (HD == 2) {
         cur = h0;
         h0 = h1;
         if (k + 2 < k1) fetch(k + 2, h1);
      } else if (HD == 1) {
         cur = h0;
         if (k + 1 < k1) fetch(k + 1, h0);
      } else {
         fetch(k, cur);
      }
#pragma unroll
      for (int i = 0; i < NLN; i++) {
         const unsigned row = row0 + (unsigned)(i * S);
         const int pid = cur.pid[i];
         v2d acc = HF ? cur.a0[i] : epi.init2((int)row);
         v2d pf = xc_pf ? xc[i] : epi.pf2((int)row);
         const double e = cur.e[i];
         double lft = __shfl_up(xc[i].y, 1, 64);
         double rgt = __shfl_down(xc[i].x, 1, 64);
         if (lane == 0) lft = e;
         if (lane == 63) rgt = e;
         const unsigned long long mk = mtab[pid];
         v2d xv[7];
         xv[0] = xc[i];
         xv[1] = xm[i];
         xv[2] = i == 0 ? cur.ym : xc[i == 0 ? 0 : i - 1];
         xv[3] = v2d{lft, xc[i].x};
         xv[4] = v2d{xc[i].y, rgt};
         xv[5] = i == NLN - 1 ? cur.yp : xc[i == NLN - 1 ? 0 : i + 1];
         xv[6] = xq[i];
         acc = mz_acc7<NEG, UNI>(acc, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
         v2d dg{0.0, 0.0};
         if (NEED_DIAG) dg = UNI ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 7];
         const v2d out = epi.finish2((int)row, acc, dg, pf);
         if (partials) {
            // csr_mp_kernel's 64-row group sums
            double a = out.x * out.x, b = out.y * out.y;
#pragma unroll
            for (int off = 16; off > 0; off >>= 1) {
               a += __shfl_down(a, off, 32);
               b += __shfl_down(b, off, 32);
            }
            if ((tid & 31) == 0) red[((k - k0) * NLN + i) * 8 + (tid >> 5)] = a + b;
         }
      }
#pragma unroll
      for (int i = 0; i < NLN; i++) {
         xm[i] = xc[i];
         xc[i] = xq[i];
         if (PF == 2) {
            xq[i] = q2[i];
            q2[i] = xn[i];
         } else {
            xq[i] = xn[i];
         }
      }
   }
   if (partials) {
      __syncthreads();
      for (int w = tid; w < 2 * NLN * (k1 - k0); w += 256) {
         const int it = w / (2 * NLN), i = (w >> 1) % NLN, h = w & 1;
         const double *g = red + (it * NLN + i) * 8 + 4 * h;
         partials[((long long)(k0 + it - kb) * P + blk0 + i * S) / 256 + h] = ((g[0] + g[1]) + g[2]) + g[3];
      }
   }
}

// planes per workgroup chunk: the context's, shortened on small levels (when
// automatic) so the launch keeps >= 2048 workgroups
static int mz_chunk(const amg_mat *A, int nz, int npb)
{
   int zc = std::max(1, std::min(A->ctx->mz_zc, AMG_MZ_MAXZC));
   if (A->ctx->mz_zc_auto) zc = (int)std::max(1LL, std::min((long long)zc, (long long)nz * npb / 2048));
   return zc;
}

// planes per chunk sized so the launch is a whole number of rounds of `occ`
// resident workgroups per CU (occ: the kernel's VGPR-limited occupancy; 0: off,
// mz_chunk's rule), each chunk at most AMG_MZ_MAXZC planes
// resident 256-thread workgroups per CU of a kernel (its VGPR / LDS limits),
// from the runtime's occupancy calculator, cached per kernel
static int kernel_occ(const void *fn)
{
   static std::mutex mu;
   static std::unordered_map<const void *, int> cache;
   std::lock_guard<std::mutex> g(mu);
   auto it = cache.find(fn);
   if (it != cache.end()) return it->second;
   int nb = 0;
   if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, 0) != hipSuccess) {
      (void)hipGetLastError();
      nb = 0;
   }
   cache[fn] = nb;
   return nb;
}

// occ < 0: the kernel's own occupancy (kernel_occ)
static int occ_chunk(const amg_mat *A, int nk, int npb, int occ, const void *fn)
{
   if (occ < 0) occ = fn ? kernel_occ(fn) : 0;
   int zc = mz_chunk(A, nk, npb);
   const long long slots = (long long)occ * A->ctx->num_cus, work = (long long)nk * npb;
   if (!A->ctx->mz_zc_auto || occ <= 0 || work < slots) return zc;
   const long long rounds = (work + slots * AMG_MZ_MAXZC - 1) / (slots * AMG_MZ_MAXZC);
   zc = (int)((work + slots * rounds - 1) / (slots * rounds));
   return std::max(1, std::min(zc, AMG_MZ_MAXZC));
}

struct EpiGemv; // below

template <int NEG, bool NEED_DIAG, class Epi>
static void launch_mz(hipStream_t s, const amg_mat *A, const double *x, const Epi &e, double *partials, int kb,
                      int ke)
{
   MpSten S;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      S.off[j] = A->mp_off[j];
      S.val[j] = A->mp_val[j];
   }
   const int P = A->mz_P, nz = A->nrows / P, Sx = A->mz_S, nk = ke - kb;
   if (nk <= 0) return;
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
   // two or four lines per lane (ctx->mz_lines; SpMV / SpGEMV: ctx->mz_lines_gemv)
   // where the plane splits into line groups; ctx->mz_pf: prefetch distance
   const int lines = std::is_same<Epi, EpiGemv>::value ? A->ctx->mz_lines_gemv : A->ctx->mz_lines;
   const bool pf2 = A->ctx->mz_pf == 2;
   // AMG_MZ_WPE=8: registers capped for 8 waves per SIMD (one line, prefetch 1)
   static const int wpe = [] {
      const char *v = std::getenv("AMG_MZ_WPE");
      return v ? std::atoi(v) : 0;
   }();
   // ctx->mz_pf == 3: prefetch 1 with the halo operands two planes ahead (HPF, one line per lane)
   const int pfk = A->ctx->mz_pf == 3 && lines == 1 ? 3 : (pf2 ? 2 : 1);
   auto go = [&](auto uni, auto nln, auto pf) {
      constexpr bool U = decltype(uni)::value;
      constexpr int N = decltype(nln)::value, F = decltype(pf)::value;
      if constexpr (N == 1 && F == 1) {
         if (pfk == 3) {
            auto hpf = [&](auto wv, auto dv) {
               constexpr int W = decltype(wv)::value, D = decltype(dv)::value;
               const void *fnh = (const void *)csr_mz_kernel<NEG, NEED_DIAG, Epi, U, N, F, W, D>;
               const int npb = P / 512, zc = occ_chunk(A, nk, npb, A->ctx->mz_occ, fnh), nch = (nk + zc - 1) / zc;
               csr_mz_kernel<NEG, NEED_DIAG, Epi, U, N, F, W, D><<<npb * nch, 256, 0, s>>>(
                  A->ppat, A->mpmask, A->pp_n, mv, S, x, P, Sx, nz, zc, npb, A->ctx->mz_xcd, e, partials, kb, ke);
            };
            using W0 = std::integral_constant<int, 0>;
            using W5 = std::integral_constant<int, 5>;
            // AMG_MZ_HPF: 1 / 2 the halo operands one / two planes ahead, 3 / 4
            // with the right-hand side too (default 3: 90 VGPRs, 5 waves per
            // SIMD; profiles/r05/hpf/); AMG_MZ_WPE=5: held to 5 waves per SIMD
            static const int hd = [] {
               const char *v = std::getenv("AMG_MZ_HPF");
               const int d = v ? std::atoi(v) : 3;
               return d >= 1 && d <= 4 ? d : 3;
            }();
            switch (hd * 2 + (wpe == 5)) {
            case 2: hpf(W0{}, std::integral_constant<int, 1>{}); break;
            case 3: hpf(W5{}, std::integral_constant<int, 1>{}); break;
            case 5: hpf(W5{}, std::integral_constant<int, 2>{}); break;
            case 6: hpf(W0{}, std::integral_constant<int, 3>{}); break;
            case 7: hpf(W5{}, std::integral_constant<int, 3>{}); break;
            case 8: hpf(W0{}, std::integral_constant<int, 4>{}); break;
            case 9: hpf(W5{}, std::integral_constant<int, 4>{}); break;
            default: hpf(W0{}, std::integral_constant<int, 2>{}); break;
            }
            return;
         }
      }
      if constexpr (N == 1 && F == 1) {
         if (wpe == 8) {
            const void *fn8 = (const void *)csr_mz_kernel<NEG, NEED_DIAG, Epi, U, N, F, 8>;
            const int npb = P / 512, zc = occ_chunk(A, nk, npb, A->ctx->mz_occ, fn8), nch = (nk + zc - 1) / zc;
            csr_mz_kernel<NEG, NEED_DIAG, Epi, U, N, F, 8><<<npb * nch, 256, 0, s>>>(
               A->ppat, A->mpmask, A->pp_n, mv, S, x, P, Sx, nz, zc, npb, A->ctx->mz_xcd, e, partials, kb, ke);
            return;
         }
      }
      const void *fn = (const void *)csr_mz_kernel<NEG, NEED_DIAG, Epi, U, N, F>;
      const int npb = P / (512 * N), zc = occ_chunk(A, nk, npb, A->ctx->mz_occ, fn), nch = (nk + zc - 1) / zc;
      // AMG_MZ_LDSPAD: dynamic LDS bytes per workgroup that cap the resident
      // workgroups per CU (an occupancy experiment; the kernel does not use them)
      static const int ldspad = [] {
         const char *v = std::getenv("AMG_MZ_LDSPAD");
         return v ? std::atoi(v) : 0;
      }();
      csr_mz_kernel<NEG, NEED_DIAG, Epi, U, N, F><<<npb * nch, 256, (size_t)ldspad, s>>>(
         A->ppat, A->mpmask, A->pp_n, mv, S, x, P, Sx, nz, zc, npb, A->ctx->mz_xcd, e, partials, kb, ke);
   };
   using T = std::true_type;
   using F = std::false_type;
   using I1 = std::integral_constant<int, 1>;
   using I2 = std::integral_constant<int, 2>;
   using I4 = std::integral_constant<int, 4>;
   if (A->mp_uni && lines > 1 && Sx % 512 == 0 && (P / Sx) % lines == 0) {
      if (lines == 4) {
         if (pf2) go(T{}, I4{}, I2{});
         else go(T{}, I4{}, I1{});
      } else {
         if (pf2) go(T{}, I2{}, I2{});
         else go(T{}, I2{}, I1{});
      }
      return;
   }
   if (A->mp_uni) {
      if (pf2) go(T{}, I1{}, I2{});
      else go(T{}, I1{}, I1{});
   } else {
      if (pf2) go(F{}, I1{}, I2{});
      else go(F{}, I1{}, I1{});
   }
}

// ---------------------------------------------------------------------------
// 27-point plane-marching kernel (csr_mz27_kernel): master-coded operators
// whose master list is [0, then the 26 offsets dz P + dy S + dx (dz, dy, dx in
// {-1, 0, 1}, not all 0) ascending] -- the Galerkin coarse operators R A P of
// the box hierarchy (27-pt stencils, diagonal-first rows).  As in
// csr_mz_kernel a lane owns rows (2t, 2t + 1) of a workgroup's 512 in-plane
// positions and marches over a chunk of planes, but here it keeps the three
// lines y - 1, y, y + 1 of planes k - 1, k, k + 1 in registers, each with its
// +-1 neighbours (ds_bpermute from the adjacent lanes, the wave's edges from
// one scalar load): per plane step three 16-byte x loads (the new plane k + 2)
// replace the master kernel's 27 gathers.  The use masks decide which entries
// each row adds; a wave whose pairs all have the dominant interior pattern
// (every entry used, one value per entry in both rows) takes the values from
// kernel arguments (SGPRs) and skips the use tests.  Each row adds its used
// entries in master (= CSR) order: bit-identical to every other form.
// ---------------------------------------------------------------------------
struct Ln4 {
   double l, a, b, r; // x at the pair's positions - 1, + 0, + 1, + 2 (one line)
};

// master entry j -> lexicographic stencil slot (dz + 1) 9 + (dy + 1) 3 + dx + 1
__device__ __forceinline__ constexpr int mz27_slot(int j)
{
   return j == 0 ? 13 : (j <= 13 ? j - 1 : j);
}

__device__ __forceinline__ v2d mz27_opnd(const Ln4 (&X)[3][3], int L)
{
   const Ln4 &q = X[L / 9][(L / 3) % 3];
   const int dx = L % 3;
   return dx == 0 ? v2d{q.l, q.a} : (dx == 1 ? v2d{q.a, q.b} : v2d{q.b, q.r});
}

// one line of plane data at element index idx (even; lines wholly outside the
// box are clamped, their entries unused): the pair's 16-byte load plus the
// wave-edge neighbours, then the +-1 shuffles
__device__ __forceinline__ void mz27_load(const double *__restrict__ x, long long idx, unsigned Nu, int lane,
                                          v2d &v, double &e)
{
   const unsigned i = idx < 0 ? 0u : (idx + 2 > (long long)Nu ? Nu - 2 : (unsigned)idx);
   v = ld2u(x, i);
   e = 0.0;
   if (lane == 0 && i > 0) e = ld1u(x, i - 1);
   if (lane == 63 && i + 2 < Nu) e = ld1u(x, i + 2);
}

__device__ __forceinline__ Ln4 mz27_line(v2d v, double e, int lane)
{
   double l = __shfl_up(v.y, 1, 64);
   double r = __shfl_down(v.x, 1, 64);
   if (lane == 0) l = e;
   if (lane == 63) r = e;
   return Ln4{l, v.x, v.y, r};
}

struct Val27 {
   double v[27];
};

template <int NEG, bool NEED_DIAG, class Epi, bool UNI, int PF = 1>
__global__ __launch_bounds__(256) void csr_mz27_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, MpSten Sv, int dom, int xlo, int xhi, Val27 Hv, const double *__restrict__ x,
   int P, int S, int nz, int zc, int npb, int xcd, Epi epi, double *__restrict__ partials, int kb, int ke)
{
   constexpr unsigned long long FULL = (1ull << 54) - 1;
   const bool xc_pf = pf_is_x<Epi>::value && epi_pf_vec(epi) == x;
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 64 * 27];
   __shared__ double red[AMG_MZ_MAXZC * 8];
   const int tid = (int)threadIdx.x, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (!UNI)
      for (int w = tid; w < np * 27; w += 256) mval[w] = mval_g[w];
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = kb + chunk * zc, k1 = min(k0 + zc, ke); // planes [kb, ke) (csr_mz_kernel)
   const int pos = pblk * 512 + 2 * tid;
   const unsigned Nu = (unsigned)((long long)nz * P);
   Ln4 X[3][3];
#pragma unroll
   for (int m = 0; m < 3; m++) {
      const int p = k0 - 1 + m;
#pragma unroll
      for (int d = 0; d < 3; d++) {
         v2d v{0.0, 0.0};
         double e = 0.0;
         if (p >= 0 && p < nz) mz27_load(x, (long long)p * P + pos + (d - 1) * S, Nu, lane, v, e);
         X[m][d] = mz27_line(v, e, lane);
      }
   }
   // PF = 2: plane k + 2 arrives one iteration early (qv / qe), plane k + 3 is
   // in flight while plane k is computed
   v2d qv[3] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
   double qe[3] = {0.0, 0.0, 0.0};
   if (PF == 2 && k0 + 2 < nz && k0 + 1 < k1) {
#pragma unroll
      for (int d = 0; d < 3; d++)
         mz27_load(x, (long long)(k0 + 2) * P + pos + (d - 1) * S, Nu, lane, qv[d], qe[d]);
   }
   __syncthreads();
   for (int k = k0; k < k1; k++) {
      const unsigned row = (unsigned)k * P + pos;
      // prefetch plane k + PF + 1 (the chunk's last iteration needs plane k1)
      v2d nv[3] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
      double ne[3] = {0.0, 0.0, 0.0};
      if (k + PF + 1 < nz && k + PF < k1) {
#pragma unroll
         for (int d = 0; d < 3; d++)
            mz27_load(x, (long long)row + (PF + 1LL) * P + (d - 1) * S, Nu, lane, nv[d], ne[d]);
      }
      const int pid = ppat[row >> 1];
      const v2d acc0 = epi.init2((int)row);
      v2d acc = acc0;
      const v2d pf = xc_pf ? v2d{X[1][1].a, X[1][1].b} : epi.pf2((int)row);
      // fast path: every pair of the wave dominant, or an x-edge pair whose
      // edge row is then recomputed on its own (its entries in master order,
      // the dx = -1 / +1 ones skipped, its own values) -- the ends of every
      // line, which otherwise send every wave of a short line to the LDS path
      const bool fast = UNI ? __all(mtab[pid] == FULL) : __all(pid == dom || pid == xlo || pid == xhi);
      if (fast) {
#pragma unroll
         for (int j = 0; j < 27; j++) {
            const v2d o = mz27_opnd(X, mz27_slot(j));
            const double v = Sv.val[j];
            acc.x = NEG ? acc.x - v * o.x : acc.x + v * o.x;
            acc.y = NEG ? acc.y - v * o.y : acc.y + v * o.y;
         }
         if (!UNI && pid == xlo) {
            acc.x = acc0.x;
#pragma unroll
            for (int j = 0; j < 27; j++) {
               const int L = mz27_slot(j);
               if (L % 3 == 0) continue; // dx = -1
               const double o = mz27_opnd(X, L).x, v = Sv.val[j];
               acc.x = NEG ? acc.x - v * o : acc.x + v * o;
            }
         }
         if (!UNI && pid == xhi) {
            acc.y = acc0.y;
#pragma unroll
            for (int j = 0; j < 27; j++) {
               const int L = mz27_slot(j);
               if (L % 3 == 2) continue; // dx = +1
               const double o = mz27_opnd(X, L).y, v = Hv.v[j];
               acc.y = NEG ? acc.y - v * o : acc.y + v * o;
            }
         }
      } else {
         const unsigned long long mk = mtab[pid];
         const v2d *vp = mval + (UNI ? 0 : pid * 27);
#pragma unroll
         for (int j = 0; j < 27; j++) {
            const unsigned int b = (unsigned int)(mk >> (2 * j)) & 3u;
            const v2d o = mz27_opnd(X, mz27_slot(j));
            const v2d v = UNI ? v2d{Sv.val[j], Sv.val[j]} : vp[j];
            if (b & 1) acc.x = NEG ? acc.x - v.x * o.x : acc.x + v.x * o.x;
            if (b & 2) acc.y = NEG ? acc.y - v.y * o.y : acc.y + v.y * o.y;
         }
      }
      v2d dg{0.0, 0.0};
      if (NEED_DIAG) {
         dg = (UNI || fast) ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 27];
         if (!UNI && fast && pid == xhi) dg.y = Hv.v[0];
      }
      const v2d out = epi.finish2((int)row, acc, dg, pf);
      if (partials) {
         double a = out.x * out.x, b = out.y * out.y;
#pragma unroll
         for (int off = 16; off > 0; off >>= 1) {
            a += __shfl_down(a, off, 32);
            b += __shfl_down(b, off, 32);
         }
         if ((tid & 31) == 0) red[(k - k0) * 8 + (tid >> 5)] = a + b;
      }
#pragma unroll
      for (int d = 0; d < 3; d++) {
         X[0][d] = X[1][d];
         X[1][d] = X[2][d];
         if (PF == 2) {
            X[2][d] = mz27_line(qv[d], qe[d], lane);
            qv[d] = nv[d];
            qe[d] = ne[d];
         } else {
            X[2][d] = mz27_line(nv[d], ne[d], lane);
         }
      }
   }
   if (partials) {
      __syncthreads();
      for (int w = tid; w < 2 * (k1 - k0); w += 256) {
         const int it = w >> 1, h = w & 1;
         const double *g = red + it * 8 + 4 * h;
         partials[((long long)(k0 + it - kb) * P + pblk * 512) / 256 + h] = ((g[0] + g[1]) + g[2]) + g[3];
      }
   }
}

// LDS plane-ring form of the 27-point march (ctx->mz27_pf 3).  The workgroup's
// 512 in-plane positions plus S + 2 on each side (its +-S lines and the
// wave-edge neighbours: one contiguous range of the plane) are staged once per
// plane into a 4-slot LDS ring -- 16-byte loads, two planes ahead in
// registers, one barrier per plane step -- and every lane reads the nine
// lines of its 3 x 3 x 3 neighbourhood (x - 1 .. x + 2 of each) from the ring
// instead of carrying them in registers across the march (no +-1 shuffles,
// no wave-edge loads).  The row arithmetic is csr_mz27_kernel's: the same
// fast / edge / masked paths, the same operands in master order
// (bit-identical); the non-dominant patterns' values come from global memory
// (L1 / L2) so the ring and mask table fit four workgroups per CU.  Staged
// elements outside the box (clamped or zero planes) feed only masked entries.
template <int NEG, bool NEED_DIAG, class Epi, bool UNI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void csr_mz27l_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval, MpSten Sv, int dom, int xlo, int xhi, Val27 Hv, const double *__restrict__ x,
   int P, int S, int nz, int zc, int npb, int xcd, Epi epi, double *__restrict__ partials, int kb, int ke)
{
   constexpr unsigned long long FULL = (1ull << 54) - 1;
   extern __shared__ v2d ring[]; // 4 slots of NPR pairs
   __shared__ unsigned long long mtab[256];
   __shared__ double red[AMG_MZ_MAXZC * 8];
   const bool xc_pf = pf_is_x<Epi>::value && epi_pf_vec(epi) == x;
   const int tid = (int)threadIdx.x;
   if (tid < np) mtab[tid] = mmask_g[tid];
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = kb + chunk * zc, k1 = min(k0 + zc, ke);
   const int pos = pblk * 512 + 2 * tid;
   const unsigned Nu = (unsigned)((long long)nz * P);
   const int NPR = 258 + S;                            // pairs per slot: 512 + 2 S + 4 elements
   const long long e0 = (long long)pblk * 512 - S - 2; // in-plane position of a slot's element 0
   // plane p's staged pairs of this lane (pairs tid, tid + 256, tid + 512)
   auto stage_ld = [&](int p, v2d (&st)[3]) {
#pragma unroll
      for (int r = 0; r < 3; r++) {
         st[r] = v2d{0.0, 0.0};
         const int q = tid + 256 * r;
         if (q < NPR && p >= 0 && p < nz) {
            long long i = (long long)p * P + e0 + 2 * q;
            i = i < 0 ? 0 : (i + 2 > (long long)Nu ? (long long)Nu - 2 : i);
            st[r] = ld2u(x, (unsigned)i);
         }
      }
   };
   auto stage_st = [&](int p, const v2d (&st)[3]) {
      v2d *sl = ring + (p & 3) * NPR;
#pragma unroll
      for (int r = 0; r < 3; r++) {
         const int q = tid + 256 * r;
         if (q < NPR) sl[q] = st[r];
      }
   };
   {
      v2d st[3];
      for (int p = k0 - 1; p <= k0 + 1 && p <= k1; p++) {
         stage_ld(p, st);
         stage_st(p, st);
      }
   }
   v2d sa[3], sb[3]; // planes k + 2 (loaded one step ago) and k + 3
   stage_ld(k0 + 2 <= k1 ? k0 + 2 : -1, sa);
   __syncthreads();
   for (int k = k0; k < k1; k++) {
      stage_ld(k + 3 <= k1 ? k + 3 : -1, sb);
      const unsigned row = (unsigned)k * P + pos;
      // line d of plane k - 1 + m at the pair's x - 1 .. x + 2, from the ring
      auto ldline = [&](int m, int d) {
         const double *rl = reinterpret_cast<const double *>(ring + ((k - 1 + m) & 3) * NPR);
         const int e = 2 * tid + d * S + 2;
         return Ln4{rl[e - 1], rl[e], rl[e + 1], rl[e + 2]};
      };
      auto opnd4 = [](const Ln4 &q, int dx) {
         return dx == 0 ? v2d{q.l, q.a} : (dx == 1 ? v2d{q.a, q.b} : v2d{q.b, q.r});
      };
      // f(j, operand pair) for the 27 master entries in master order (j = 0:
      // the centre, then the lexicographic slots), each line read once
      auto visit = [&](auto &&f) {
         const Ln4 c = ldline(1, 1);
         f(0, opnd4(c, 1));
         Ln4 q = c;
#pragma unroll
         for (int L = 0; L < 27; L++) {
            if (L == 13) continue;
            if (L % 3 == 0) q = (L / 3 == 4) ? c : ldline(L / 9, (L / 3) % 3);
            f(L < 13 ? L + 1 : L, opnd4(q, L % 3));
         }
      };
      const int pid = ppat[row >> 1];
      const v2d acc0 = epi.init2((int)row);
      v2d acc = acc0;
      v2d pf;
      if (xc_pf) {
         const Ln4 c = ldline(1, 1);
         pf = v2d{c.a, c.b};
      } else {
         pf = epi.pf2((int)row);
      }
      const bool fast = UNI ? __all(mtab[pid] == FULL) : __all(pid == dom || pid == xlo || pid == xhi);
      if (fast) {
         visit([&](int jj, v2d o) {
            const double v = Sv.val[jj];
            acc.x = NEG ? acc.x - v * o.x : acc.x + v * o.x;
            acc.y = NEG ? acc.y - v * o.y : acc.y + v * o.y;
         });
         if (!UNI && pid == xlo) {
            acc.x = acc0.x;
            visit([&](int jj, v2d o) {
               if (mz27_slot(jj) % 3 == 0) return; // dx = -1
               const double v = Sv.val[jj];
               acc.x = NEG ? acc.x - v * o.x : acc.x + v * o.x;
            });
         }
         if (!UNI && pid == xhi) {
            acc.y = acc0.y;
            visit([&](int jj, v2d o) {
               if (mz27_slot(jj) % 3 == 2) return; // dx = +1
               const double v = Hv.v[jj];
               acc.y = NEG ? acc.y - v * o.y : acc.y + v * o.y;
            });
         }
      } else {
         const unsigned long long mk = mtab[pid];
         const v2d *vp = mval + (UNI ? 0 : pid * 27);
         visit([&](int jj, v2d o) {
            const unsigned int b = (unsigned int)(mk >> (2 * jj)) & 3u;
            const v2d v = UNI ? v2d{Sv.val[jj], Sv.val[jj]} : vp[jj];
            if (b & 1) acc.x = NEG ? acc.x - v.x * o.x : acc.x + v.x * o.x;
            if (b & 2) acc.y = NEG ? acc.y - v.y * o.y : acc.y + v.y * o.y;
         });
      }
      v2d dg{0.0, 0.0};
      if (NEED_DIAG) {
         dg = (UNI || fast) ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 27];
         if (!UNI && fast && pid == xhi) dg.y = Hv.v[0];
      }
      const v2d out = epi.finish2((int)row, acc, dg, pf);
      if (partials) {
         double a = out.x * out.x, b = out.y * out.y;
#pragma unroll
         for (int off = 16; off > 0; off >>= 1) {
            a += __shfl_down(a, off, 32);
            b += __shfl_down(b, off, 32);
         }
         if ((tid & 31) == 0) red[(k - k0) * 8 + (tid >> 5)] = a + b;
      }
      // plane k + 2 into the slot of plane k - 2 (read by no lane this step)
      if (k + 2 <= k1) stage_st(k + 2, sa);
#pragma unroll
      for (int r = 0; r < 3; r++) sa[r] = sb[r];
      __syncthreads();
   }
   if (partials) {
      for (int w = tid; w < 2 * (k1 - k0); w += 256) {
         const int it = w >> 1, h = w & 1;
         const double *g = red + it * 8 + 4 * h;
         partials[((long long)(k0 + it - kb) * P + pblk * 512) / 256 + h] = ((g[0] + g[1]) + g[2]) + g[3];
      }
   }
}

template <int NEG, bool NEED_DIAG, class Epi>
static void launch_mz27(hipStream_t s, const amg_mat *A, const double *x, const Epi &e, double *partials, int kb,
                        int ke)
{
   MpSten S;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      S.off[j] = A->mp_off[j];
      S.val[j] = A->mp_uni ? A->mp_val[j] : A->mz_domval[j];
   }
   const int P = A->mz_P, nz = A->nrows / P, nk = ke - kb;
   if (nk <= 0) return;
   const int npb = P / 512;
   // whole rounds of resident workgroups (mz27_occ per CU, the VGPR-limited
   // occupancy of this kernel)
   const void *fn;
   if (A->ctx->mz27_pf == 2)
      fn = A->mp_uni ? (const void *)csr_mz27_kernel<NEG, NEED_DIAG, Epi, true, 2>
                     : (const void *)csr_mz27_kernel<NEG, NEED_DIAG, Epi, false, 2>;
   else
      fn = A->mp_uni ? (const void *)csr_mz27_kernel<NEG, NEED_DIAG, Epi, true, 1>
                     : (const void *)csr_mz27_kernel<NEG, NEED_DIAG, Epi, false, 1>;
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
   Val27 H;
   for (int j = 0; j < 27; j++) H.v[j] = A->mz_hival[j];
   // the x-edge fast path needs the dominant pattern (ctx->mz_edge: on)
   const int xlo = A->ctx->mz_edge ? A->mz_xlo : -1, xhi = A->ctx->mz_edge ? A->mz_xhi : -1;
   if (A->ctx->mz27_pf == 3 && A->mz_S <= 512) {
      // the LDS plane-ring form: four workgroups per CU at S = 256 (33 KB ring)
      const size_t lds = (size_t)4 * (258 + A->mz_S) * sizeof(v2d);
      const void *fl = A->mp_uni ? (const void *)csr_mz27l_kernel<NEG, NEED_DIAG, Epi, true>
                                 : (const void *)csr_mz27l_kernel<NEG, NEED_DIAG, Epi, false>;
      int occ = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fl, 256, lds) != hipSuccess) {
         (void)hipGetLastError();
         occ = 0;
      }
      const int zcl = occ_chunk(A, nk, npb, occ > 0 ? occ : 0, nullptr);
      const int nchl = (nk + zcl - 1) / zcl;
      if (A->mp_uni)
         csr_mz27l_kernel<NEG, NEED_DIAG, Epi, true><<<npb * nchl, 256, lds, s>>>(
            A->ppat, A->mpmask, A->pp_n, mv, S, -1, -1, -1, H, x, P, A->mz_S, nz, zcl, npb, A->ctx->mz_xcd, e,
            partials, kb, ke);
      else
         csr_mz27l_kernel<NEG, NEED_DIAG, Epi, false><<<npb * nchl, 256, lds, s>>>(
            A->ppat, A->mpmask, A->pp_n, mv, S, A->mz_dom, A->mz_dom >= 0 ? xlo : -1, A->mz_dom >= 0 ? xhi : -1,
            H, x, P, A->mz_S, nz, zcl, npb, A->ctx->mz_xcd, e, partials, kb, ke);
      return;
   }
   const int zc = occ_chunk(A, nk, npb, A->ctx->mz27_occ, fn);
   const int nch = (nk + zc - 1) / zc;
   auto go = [&](auto pf) {
      constexpr int PF = decltype(pf)::value;
      if (A->mp_uni)
         csr_mz27_kernel<NEG, NEED_DIAG, Epi, true, PF><<<npb * nch, 256, 0, s>>>(
            A->ppat, A->mpmask, A->pp_n, mv, S, -1, -1, -1, H, x, P, A->mz_S, nz, zc, npb, A->ctx->mz_xcd, e,
            partials, kb, ke);
      else
         csr_mz27_kernel<NEG, NEED_DIAG, Epi, false, PF><<<npb * nch, 256, 0, s>>>(
            A->ppat, A->mpmask, A->pp_n, mv, S, A->mz_dom, A->mz_dom >= 0 ? xlo : -1, A->mz_dom >= 0 ? xhi : -1,
            H, x, P, A->mz_S, nz, zc, npb, A->ctx->mz_xcd, e, partials, kb, ke);
   };
   if (A->ctx->mz27_pf == 2)
      go(std::integral_constant<int, 2>{});
   else
      go(std::integral_constant<int, 1>{});
}

// ---------------------------------------------------------------------------
// Geometric transfers of a marched level (SMEM_Sync_Parfor_Restrict /
// SMEM_SpGEMV prolongation, SMEM_MatVec.cpp:380-392 / 140-258, on the
// hierarchy's R_0 = P_0^T of the nx * ny * nz box): coarse point K couples to
// the fine points 2K + d, d in {0,1,2}^3, with weight w[dz][dy][dx].  Both
// matrices are checked entry for entry against this form at hierarchy
// creation (geo_check_k), so the fused kernels below compute exactly what the
// CSR kernels would.
// ---------------------------------------------------------------------------
// every row of R (mode 0, coarse rows) or P (mode 1, fine rows) equals the
// geometric form: same length, same columns in CSR order, same value bits
__global__ __launch_bounds__(256) void geo_check_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                   const double *__restrict__ val, int rb, int re, int mode, GeoT g,
                                                   long long row_g0, long long col_g0, int *__restrict__ bad)
{
   // local rows [rb, re) are global rows + row_g0, local columns global + col_g0
   // (a z-slab's extended operator); the full operator: 0, nrows, 0, 0
   const int li = rb + (int)(blockIdx.x * 256 + threadIdx.x);
   if (li >= re) return;
   const long long gi = li + row_g0;
   const int cx_n = g.nx / 2, cy_n = g.ny / 2, cz_n = g.nz / 2;
   int k = rowptr[li];
   const int e = rowptr[li + 1];
   bool ok = true;
   if (mode == 0) {
      const int Kx = (int)(gi % cx_n), Ky = (int)((gi / cx_n) % cy_n), Kz = (int)(gi / ((long long)cx_n * cy_n));
      for (int dz = 0; dz < 3; dz++)
         for (int dy = 0; dy < 3; dy++)
            for (int dx = 0; dx < 3; dx++) {
               const int fz = 2 * Kz + dz, fy = 2 * Ky + dy, fx = 2 * Kx + dx;
               if (fz >= g.nz || fy >= g.ny || fx >= g.nx) continue;
               const long long c = ((long long)fz * g.ny + fy) * g.nx + fx;
               if (k >= e || col[k] + col_g0 != c ||
                   __double_as_longlong(val[k]) != __double_as_longlong(g.w[dz * 9 + dy * 3 + dx]))
                  ok = false;
               k++;
            }
   } else {
      const int fx = (int)(gi % g.nx), fy = (int)((gi / g.nx) % g.ny), fz = (int)(gi / ((long long)g.nx * g.ny));
      // coarse candidates of one axis, ascending: odd f -> (f-1)/2; even f -> f/2-1, f/2
      auto cand = [](int f, int nc, int *c) {
         int m = 0;
         if (f & 1) {
            c[m++] = (f - 1) / 2;
         } else {
            if (f / 2 - 1 >= 0) c[m++] = f / 2 - 1;
            if (f / 2 < nc) c[m++] = f / 2;
         }
         return m;
      };
      int czs[2], cys[2], cxs[2];
      const int mz = cand(fz, cz_n, czs), my = cand(fy, cy_n, cys), mx = cand(fx, cx_n, cxs);
      for (int a = 0; a < mz; a++)
         for (int b = 0; b < my; b++)
            for (int q = 0; q < mx; q++) {
               const int dz = fz - 2 * czs[a], dy = fy - 2 * cys[b], dx = fx - 2 * cxs[q];
               const long long c = ((long long)czs[a] * cy_n + cys[b]) * cx_n + cxs[q];
               if (k >= e || col[k] + col_g0 != c ||
                   __double_as_longlong(val[k]) != __double_as_longlong(g.w[dz * 9 + dy * 3 + dx]))
                  ok = false;
               k++;
            }
   }
   if (k != e) ok = false;
   if (!ok) atomicOr(bad, 1);
}

void geo_check(hipStream_t s, const amg_mat *M, int mode, const GeoT &g, int *bad, int rb, int re,
               long long row_g0, long long col_g0)
{
   if (re < 0) re = M->nrows;
   if (re <= rb) return;
   geo_check_k<<<(re - rb + 255) / 256, 256, 0, s>>>(M->rowptr, M->col, M->val, rb, re, mode, g, row_g0, col_g0,
                                                      bad);
}

// Fused level-0 residual + restriction: f_c = R (f - A u) without the fine
// residual vector.  A lane owns fine columns 2cx, 2cx + 1 of the 2 LC + 1 fine
// lines 2Ky0 .. 2Ky0 + 2 LC that LC consecutive coarse lines Ky0 .. Ky0 + LC - 1
// restrict from (a workgroup holds 512 / nx such line groups) and marches
// through the fine planes of a chunk of coarse planes, keeping x of planes
// k - 1, k, k + 1 of its lines in registers (csr_mz_kernel's scheme; the halo
// lines 2Ky0 - 1, 2Ky0 + 2 LC + 1 are loaded).  Each fine residual is
// r = f - sum a_ij x_j in the row's master (= CSR) order, then coarse point
// (Kz, Ky, cx) accumulates its 27 terms w * r in R's CSR order (fine column
// ascending: dz, dy, dx), one fine plane at a time: even plane 2Kz closes
// coarse plane Kz - 1 (dz = 2) and opens Kz (dz = 0), odd plane 2Kz + 1 adds
// dz = 1.  r at fine column 2cx + 2 comes from lane t + 1 (the wave's last
// lane reads it from LDS).  Line 2Ky0 + 2 LC is shared with the next group
// (computed twice: (2 LC + 1) / 2 LC of the residual work).  Bit-identical to
// the residual kernel followed by R's SpMV.
struct Val7 {
   double v[7];
};

// RING: the wave-edge residuals travel through an LDS ring of RR planes
// between adjacent waves, ordered by per-wave produced / consumed plane
// counters (release fence + flag, acquire spin) instead of a workgroup
// barrier per plane, so the four waves march loosely coupled
constexpr int AMG_RR_RING = 4;

// execution window of an update kernel (a free race's replay checks): the
// first start and last end on the device wall clock over a sample of its
// workgroups -- every 64th and the last (workgroups dispatch in index order;
// a stamp from every workgroup would queue tens of thousands of atomics on one
// word and slow the kernel it measures several-fold); vector atomics
__device__ __forceinline__ bool stamp_wg() { return (blockIdx.x & 63) == 0 || blockIdx.x == gridDim.x - 1; }
// a record pointer's low bit (AmgCorrTimes::stamp) says whether the record
// carries row arrays: without it the update kernels never read the record
// (its line takes the window atomics; loading the row pointers from it in
// every wave cost config 4's asynchronous cycle 18 %)
__device__ __forceinline__ unsigned long long *stamp_rec(unsigned long long *st)
{
   return reinterpret_cast<unsigned long long *>(reinterpret_cast<uintptr_t>(st) & ~(uintptr_t)7);
}
__device__ __forceinline__ void stamp_begin(unsigned long long *st)
{
   st = stamp_rec(st);
   if (st && threadIdx.x == 0 && stamp_wg()) atomicMin(st, (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void stamp_end(unsigned long long *st)
{
   st = stamp_rec(st);
   if (st && stamp_wg()) {
      __syncthreads();
      if (threadIdx.x == 0) atomicMax(st + 1, (unsigned long long)wall_clock64());
   }
}
// per-row update times (AmgCorrTimes::stamps_begin: word 2 of the record is the
// row array, indexed like the updated vector, or 0): the low 32 bits of the
// device wall clock when the row's add + read of the shared vector completed,
// so a free race's replay can order every row's updates exactly
// Word 3: the row values array -- [2i] the value the add replaced, [2i + 1]
// the value it left (the capture form's returned value and that + e_i): per
// row they chain the updates of all levels in their actual order (each add's
// old value is the previous add's new value), which the replay follows
// where two levels' updates of one row came too close for the clock
struct RowRec {
   unsigned *t;
   double *v;
};
__device__ __forceinline__ RowRec stamp_rows(const unsigned long long *st)
{
   if (!(reinterpret_cast<uintptr_t>(st) & 1)) return RowRec{nullptr, nullptr};
   st = reinterpret_cast<const unsigned long long *>(reinterpret_cast<uintptr_t>(st) & ~(uintptr_t)7);
   return RowRec{reinterpret_cast<unsigned *>(static_cast<uintptr_t>(st[2])),
                 reinterpret_cast<double *>(static_cast<uintptr_t>(st[3]))};
}
__device__ __forceinline__ void stamp_row(const RowRec &r, long long i)
{
   if (r.t) r.t[i] = (unsigned)wall_clock64();
}
__device__ __forceinline__ void stamp_row(const RowRec &r, long long i, double old, double nw)
{
   if (r.t) r.t[i] = (unsigned)wall_clock64();
   if (r.v) *reinterpret_cast<v2du *>(r.v + 2 * i) = v2d{old, nw};
}

// The FULL_ASYNC update u_i += e_i with the level's copy of the updated row.
// The reference's form (SMEM_Async_AMG.cpp:296-299): an atomic add, then a
// read of u_i.  Default (AMG_ATOMIC_NORET=0): the capture form -- the
// device-scope add returns the value it replaced, and the level's copy is
// that value + e_i, i.e. u_i right after this add: the interleaving of the
// reference's race in which no other group's add falls between a thread's
// add and its read.  Every row's copy then matches one order of whole adds,
// which the per-row stamps record, so a free race replays exactly
// (tests/async_band.py row_replay).  AMG_ATOMIC_NORET=1 keeps the literal
// form: a no-return add, the wave's wait for it, an L1-bypassing read.  On
// gfx950 that read is not ordered after the add's completion at the memory
// side (the wait covers its acknowledgement): one-rank races with the read
// form ended 0.02-3.95x their exact replay, the capture form 0.91-1.00
// (profiles/r06/races).  Alone (one stream) both give the same bits.
static int atomic_noret_mode()
{
   static const int m = [] {
      const char *v = std::getenv("AMG_ATOMIC_NORET");
      return v ? std::atoi(v) : 0;
   }();
   return m;
}
__device__ __forceinline__ void add_noret(double *p, double v)
{
   (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every vector-memory operation this wave issued (stores and no-return atomics too) has completed
__device__ __forceinline__ void wait_vm_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ double read_agent(const double *p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ZeroGuess epilogue of a restriction: the coarse level's first pre-smoothing
// sweep from a zero guess, u = w f / a (jacobi_zero_k variant 0, same
// expression, a == 0 rows untouched), from the restricted value in registers
__device__ __forceinline__ void zg_apply(const ZeroGuess &zg, long long i, double fv)
{
   if (zg.u) {
      if (zg.hi >= 0 && (i < zg.lo || i >= zg.hi)) {
         if (zg.err) *zg.err = 1;
         return;
      }
      const double a = zg.d[i];
      if (a != 0.0) zg.u[i] = zg.w * fv / a;
   }
}

// XF: the composed smoothed restriction instead of the residual (UNI operators,
// xfer_restrict of the solver): x is the fine residual r, the operands are
// t = r ./ a (a = the uniform diagonal, divided once per loaded element), the
// fine value is z = r + (-w) (A t) (xfer_div, SpMV, xfer_sub: same operations,
// same order) and f_c = R z; f is not read
// FPF: the right-hand side of fine plane k + 1 loaded in iteration k (12 more
// VGPRs, still 4 waves per SIMD)
template <bool UNI, int LC, int OCC = 1, bool RING = false, bool XF = false, bool FPF = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void mz_res_restrict_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, Val7 Sv7, const double *__restrict__ x, const double *__restrict__ f,
   const double *__restrict__ wg, int nx, int ny, int nz, int zcc, int nlb, int xcd, int ntf,
   double *__restrict__ fc, int Kb, int Ke, int fz0, int cz0, int nzm, ZeroGuess zg, double mw = 0.0)
{
   // coarse planes [Kb, Ke) of the nx * ny * nz box; x / f (and the pattern
   // bytes) hold nzm planes from fine plane fz0, fc's plane 0 is coarse plane
   // cz0 (a z-slab's extended vectors; the whole box: 0, ncz, 0, 0, nz)
   constexpr int NL = 2 * LC + 1; // fine lines per lane
   MpSten Sv;
#pragma unroll
   for (int j = 0; j < 7; j++) Sv.val[j] = Sv7.v[j];
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 256 * 7];
   __shared__ double xr[RING ? AMG_RR_RING : 2][4][NL];
   __shared__ int prod[4], cons[4]; // RING: planes produced by wave w's lane 0, consumed by wave w's lane 63
   __shared__ double wl[27]; // R's weights (uniform LDS reads)
   const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (tid < 27) wl[tid] = wg[tid];
   if (!UNI)
      for (int w = tid; w < np * 7; w += 256) mval[w] = mval_g[w];
   const int S = nx, P = nx * ny;
   const long long N = (long long)nzm * P;
   const int lpl = nx >> 1; // lanes per line group
   const int ncy = ny >> 1;
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int lb = lg % nlb, chunk = lg / nlb;
   const int Ky0 = (lb * (256 / lpl) + tid / lpl) * LC, cx = tid % lpl;
   const int Kc0 = Kb + chunk * zcc, Kc1 = min(Kc0 + zcc, Ke);
   const int kf0 = 2 * Kc0, kf1 = min(2 * Kc1, nz - 1); // fine planes, inclusive
   const int y0 = 2 * Ky0;
   const bool lastl = y0 + 2 * LC >= ny; // the group's last line is outside the box
   const bool d2x = 2 * cx + 2 < nx;     // dx = 2 inside
   const int pos0 = y0 * S + 2 * cx;      // line 0 offset in the plane
   const unsigned Nu = (unsigned)N;
   const double d0 = Sv.val[0];
   auto sc = [&](v2d v) { return XF ? v2d{v.x / d0, v.y / d0} : v; };
   v2d xm[NL], xc[NL], xq[NL];
   v2d xcr[XF ? NL : 1], xqr[XF ? NL : 1]; // XF: the unscaled r of planes k, k + 1
#pragma unroll
   for (int i = 0; i < NL; i++) {
      const unsigned p = (unsigned)pos0 + (unsigned)i * S;
      const bool ok = i < NL - 1 || !lastl;
      xm[i] = (ok && kf0 > 0) ? ld2u(x, p + (unsigned)(kf0 - 1 - fz0) * P) : v2d{0.0, 0.0};
      xc[i] = ok ? ld2u(x, p + (unsigned)(kf0 - fz0) * P) : v2d{0.0, 0.0};
      xq[i] = (ok && kf0 + 1 < nz) ? ld2u(x, p + (unsigned)(kf0 + 1 - fz0) * P) : v2d{0.0, 0.0};
      if (XF) {
         xcr[i] = xc[i];
         xqr[i] = xq[i];
         xm[i] = sc(xm[i]);
         xc[i] = sc(xc[i]);
         xq[i] = sc(xq[i]);
      }
   }
   double acc[LC];
#pragma unroll
   for (int c = 0; c < LC; c++) acc[c] = 0.0;
   if (RING && tid < 4) prod[tid] = cons[tid] = kf0 - 1;
   // wave wv reads from wave wv + 1 when both hold the same line group
   const int wpl = lpl >> 6; // waves per line group (lpl > 64)
   const bool has_next = lpl > 64 && (wv + 1) % wpl != 0;
   const bool has_prev = lpl > 64 && wv % wpl != 0;
   // one plane's operands other than the marched x, all loads issued before
   // any row computes (interleaving them with the rows ran 0.71 against 0.60 ms)
   struct PlaneIn {
      v2d hm, hp, a2[NL];
      double e[NL];
      int pid[NL];
   };
   auto fetch = [&](int k, PlaneIn &in) {
      const unsigned base = (unsigned)(k - fz0) * P + pos0;
      // halo lines 2Ky0 - 1 and 2Ky0 + 2 LC + 1 (entries outside the box are unused)
      in.hm = ld2u(x, base >= (unsigned)S ? base - S : 0u);
      const unsigned hp_i = base + (unsigned)NL * S;
      in.hp = ld2u(x, hp_i + 2 <= Nu ? hp_i : Nu - 2);
#pragma unroll
      for (int i = 0; i < NL; i++) {
         const unsigned row = base + (unsigned)i * S;
         in.pid[i] = 0;
         in.a2[i] = v2d{0.0, 0.0};
         in.e[i] = 0.0;
         if (i == NL - 1 && lastl) continue;
         in.pid[i] = ppat[row >> 1];
         if (!XF && !FPF) in.a2[i] = ld2nt(f + row, ntf);
         if (lane == 0 && row > 0) in.e[i] = ld1u(x, row - 1);
         if (lane == 63 && row + 2 < Nu) in.e[i] = ld1u(x, row + 2);
      }
   };
   // FPF: f of the next fine plane (lines outside the box stay zero)
   auto fetch_f = [&](int k, v2d (&fa)[NL]) {
      const unsigned base = (unsigned)(k - fz0) * P + pos0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
         fa[i] = v2d{0.0, 0.0};
         if (i == NL - 1 && lastl) continue;
         fa[i] = ld2nt(f + base + (unsigned)i * S, ntf);
      }
   };
   v2d fcur[FPF ? NL : 1];
   if constexpr (FPF) fetch_f(kf0, fcur);
   __syncthreads();
   for (int k = kf0; k <= kf1; k++) {
      const unsigned base = (unsigned)(k - fz0) * P + pos0;
      v2d r[NL];
      PlaneIn cur;
      fetch(k, cur);
      v2d fnx[FPF ? NL : 1];
      if constexpr (FPF) {
#pragma unroll
         for (int i = 0; i < NL; i++) {
            cur.a2[i] = fcur[i];
            fnx[i] = v2d{0.0, 0.0};
         }
         if (k + 1 <= kf1) fetch_f(k + 1, fnx);
      }
      const v2d hm = sc(cur.hm), hp = sc(cur.hp);
#pragma unroll
      for (int i = 0; i < NL; i++) {
         r[i] = v2d{0.0, 0.0};
         if (i == NL - 1 && lastl) continue;
         const int pid = cur.pid[i];
         v2d a2 = cur.a2[i];
         const double e = XF ? cur.e[i] / d0 : cur.e[i];
         double lft = __shfl_up(xc[i].y, 1, 64);
         double rgt = __shfl_down(xc[i].x, 1, 64);
         if (lane == 0) lft = e;
         if (lane == 63) rgt = e;
         const unsigned long long mk = mtab[pid];
         v2d xv[7];
         xv[0] = xc[i];
         xv[1] = xm[i];
         xv[2] = i == 0 ? hm : xc[i == 0 ? 0 : i - 1];
         xv[3] = v2d{lft, xc[i].x};
         xv[4] = v2d{xc[i].y, rgt};
         xv[5] = i == NL - 1 ? hp : xc[i == NL - 1 ? NL - 1 : i + 1];
         xv[6] = xq[i];
         if (XF) {
            const v2d y = mz_acc7<0, UNI>(v2d{0.0, 0.0}, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
            r[i] = v2d{xcr[i].x + mw * y.x, xcr[i].y + mw * y.y};
         } else {
            r[i] = mz_acc7<1, UNI>(a2, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
         }
      }
      if constexpr (FPF)
#pragma unroll
         for (int i = 0; i < NL; i++) fcur[i] = fnx[i];
      // next plane's operands: load plane k + 2 while the restriction runs
#pragma unroll
      for (int i = 0; i < NL; i++) {
         xm[i] = xc[i];
         xc[i] = xq[i];
         v2d raw{0.0, 0.0};
         if ((i < NL - 1 || !lastl) && k + 2 < nz && k + 1 <= kf1)
            raw = ld2u(x, base + (unsigned)i * S + 2u * P);
         if (XF) {
            xcr[i] = xqr[i];
            xqr[i] = raw;
         }
         xq[i] = sc(raw);
      }
      // r at fine column 2cx + 2: lane t + 1 (LDS across waves for line groups
      // of more than 64 lanes)
      double r2[NL];
#pragma unroll
      for (int i = 0; i < NL; i++) r2[i] = __shfl_down(r[i].x, 1, 64);
      if (RING && lpl > 64) {
         volatile int *vp = prod, *vc = cons;
         const int slot = (k - kf0) % AMG_RR_RING;
         if (has_prev && lane == 0) {
            // slot free once wave wv - 1 consumed plane k - RING
            while (vc[wv - 1] < k - AMG_RR_RING) __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int i = 0; i < NL; i++) xr[slot][wv][i] = r[i].x;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            vp[wv] = k;
         }
         if (has_next && lane == 63) {
            while (vp[wv + 1] < k) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
            for (int i = 0; i < NL; i++) r2[i] = xr[slot][wv + 1][i];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            vc[wv] = k;
         }
      } else if (lpl > 64) {
         if (lane == 0)
#pragma unroll
            for (int i = 0; i < NL; i++) xr[k & 1][wv][i] = r[i].x;
         __syncthreads();
         if (lane == 63 && wv < 3)
#pragma unroll
            for (int i = 0; i < NL; i++) r2[i] = xr[k & 1][wv + 1][i];
      }
      const int Kz = k >> 1;
      // coarse line c of the group reads fine lines 2c .. 2c + 2
      auto add = [&](int c, int dzz) {
#pragma unroll
         for (int dy = 0; dy < 3; dy++) {
            const int i = 2 * c + dy;
            if (i == NL - 1 && lastl) continue;
            acc[c] = acc[c] + wl[dzz * 9 + dy * 3 + 0] * r[i].x;
            acc[c] = acc[c] + wl[dzz * 9 + dy * 3 + 1] * r[i].y;
            if (d2x) acc[c] = acc[c] + wl[dzz * 9 + dy * 3 + 2] * r2[i];
         }
      };
#pragma unroll
      for (int c = 0; c < LC; c++) {
         const long long ci = ((long long)(Ky0 + c)) * lpl + cx;
         if (k & 1) {
            add(c, 1);
            if (k + 1 >= nz) {
               fc[(long long)(Kz - cz0) * ncy * lpl + ci] = acc[c];
               zg_apply(zg, (long long)(Kz - cz0) * ncy * lpl + ci, acc[c]);
            }
         } else {
            if (k > kf0) {
               add(c, 2);
               fc[(long long)(Kz - 1 - cz0) * ncy * lpl + ci] = acc[c];
               zg_apply(zg, (long long)(Kz - 1 - cz0) * ncy * lpl + ci, acc[c]);
            }
            if (Kz < Kc1) {
               acc[c] = 0.0;
               add(c, 0);
            }
         }
      }
   }
}

// coarse planes per chunk: ctx->rr_zc (AMG_RR_ZC), else half the march chunk;
// a chunk re-reads fine planes 2 Kc0 - 1 and 2 Kc1 + 1 of its neighbours
static int rr_chunk(const amg_mat *A)
{
   const int z = A->ctx->rr_zc > 0 ? A->ctx->rr_zc : A->ctx->mz_zc / 2;
   return std::max(1, std::min(z, 32));
}

void mz_residual_restrict(hipStream_t s, const amg_mat *A, const double *f, const double *u, const GeoT &g,
                          const double *wdev, double *fc, int Kb, int Ke, int fz0, int cz0, ZeroGuess zg)
{
   if (Ke < 0) Ke = g.nz / 2;
   if (Ke <= Kb) return;
   const int nzm = A->nrows / (g.nx * g.ny);
   Val7 S;
   for (int j = 0; j < 7; j++) S.v[j] = A->mp_val[j];
   const int lpl = g.nx / 2, groups = 256 / lpl;
   const int LC = ((g.ny / 2) % (2 * groups) == 0 && A->ctx->rr_lines == 2) ? 2 : 1;
   const int nlb = (g.ny / 2) / (groups * LC);
   const int zcc = rr_chunk(A);
   const int nch = (Ke - Kb + zcc - 1) / zcc;
   const int nb = nlb * nch;
   const int xcd = A->ctx->mz_xcd;
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
#define AMG_RR(U, L, ...) \
   mz_res_restrict_kernel<U, L, ##__VA_ARGS__><<<nb, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, S, u, f, wdev, g.nx, g.ny, \
                                                   g.nz, zcc, nlb, xcd, stream_hint(A), fc, Kb, Ke, fz0, cz0, nzm, zg)
   if (A->mp_uni) {
      if (LC == 2) AMG_RR(true, 2);
      else if (A->ctx->rr_fpf == 3) AMG_RR(true, 1, 1, false, false, true); // 136 VGPRs, 3 waves / SIMD
      else if (A->ctx->rr_fpf) AMG_RR(true, 1, 4, false, false, true);      // held to 4 waves (128, 5 spilled)
      else if (A->ctx->rr_occ == 5) AMG_RR(true, 1, 5);
      else if (A->ctx->rr_ring) AMG_RR(true, 1, 1, true);
      else AMG_RR(true, 1);
   } else {
      if (LC == 2) AMG_RR(false, 2);
      else AMG_RR(false, 1);
   }
#undef AMG_RR
}

// rc = R (r + (-w) A (r ./ a)) for a marched uniform 7-pt level with geometric
// R (the composed smoothed restriction of xfer_restrict in one pass)
void mz_xfer_restrict(hipStream_t s, const amg_mat *A, const double *r, const GeoT &g, const double *wdev,
                      double omega, double *rc, int Kb, int Ke, int fz0, int cz0)
{
   if (Ke < 0) Ke = g.nz / 2;
   if (Ke <= Kb) return;
   const int nzm = A->nrows / (g.nx * g.ny);
   Val7 S;
   for (int j = 0; j < 7; j++) S.v[j] = A->mp_val[j];
   const int lpl = g.nx / 2, groups = 256 / lpl;
   const int LC = ((g.ny / 2) % (2 * groups) == 0 && A->ctx->rr_lines == 2) ? 2 : 1;
   const int nlb = (g.ny / 2) / (groups * LC);
   const int zcc = rr_chunk(A);
   const int nb = nlb * ((Ke - Kb + zcc - 1) / zcc);
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
   if (LC == 2)
      mz_res_restrict_kernel<true, 2, 1, false, true><<<nb, 256, 0, s>>>(
         A->ppat, A->mpmask, A->pp_n, mv, S, r, nullptr, wdev, g.nx, g.ny, g.nz, zcc, nlb, A->ctx->mz_xcd, 0, rc, Kb,
         Ke, fz0, cz0, nzm, ZeroGuess(), -omega);
   else
      mz_res_restrict_kernel<true, 1, 1, false, true><<<nb, 256, 0, s>>>(
         A->ppat, A->mpmask, A->pp_n, mv, S, r, nullptr, wdev, g.nx, g.ny, g.nz, zcc, nlb, A->ctx->mz_xcd, 0, rc, Kb,
         Ke, fz0, cz0, nzm, ZeroGuess(), -omega);
}

// Geometric prolongation + correction u += P e (SMEM_Sync_SpGEMV(P, e, u, 1, 1,
// u), SMEM_Sync_AMG.cpp:118-123) for the checked geometric P_0 of a marched
// level: lane t owns fine rows (2t, 2t + 1) of a line; per coarse (plane, line)
// pair of the row's interpolation stencil one 16-byte load brings coarse
// columns cx - 1, cx.  Each row sums u_i + w * e_c over its coarse columns
// ascending (P's CSR order: cz, cy, cx), the SpGEMV's (alpha = beta = 1) order.
// rows (i, i + 1) = fine (x, y, z), x even: u_i + sum w e_c over the coarse
// columns of P's rows in CSR order (cz, cy, cx ascending), from the pair's u
__device__ __forceinline__ v2d geo_prolong_pair(v2d acc, const double *__restrict__ e, const double *wl, int x,
                                                int y, int z, int ncx, int ncy, int ncz, int czoff = 0)
{
   const int t = x >> 1;
   // coarse candidates of one axis (ascending) and their offsets d = f - 2c
   int cz[2], dz[2], cy[2], dy[2];
   int mz = 0, my = 0;
   if (z & 1) {
      cz[mz] = (z - 1) >> 1, dz[mz++] = 1;
   } else {
      if (z >= 2) cz[mz] = (z >> 1) - 1, dz[mz++] = 2;
      if ((z >> 1) < ncz) cz[mz] = z >> 1, dz[mz++] = 0;
   }
   if (y & 1) {
      cy[my] = (y - 1) >> 1, dy[my++] = 1;
   } else {
      if (y >= 2) cy[my] = (y >> 1) - 1, dy[my++] = 2;
      if ((y >> 1) < ncy) cy[my] = y >> 1, dy[my++] = 0;
   }
   const bool lo = t >= 1, hi = t < ncx; // row 2t: coarse t - 1 (dx = 2), t (dx = 0)
   // every (plane, line) candidate's load issued first (absent candidates read
   // the first one's, unused), then the terms added in P's CSR order
   if (my < 2) cy[1] = cy[0];
   if (mz < 2) cz[1] = cz[0];
   v2d ev[2][2];
#pragma unroll
   for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++) {
         const long long cb = ((long long)(cz[a] - czoff) * ncy + cy[b]) * ncx + t; // e plane 0 = coarse czoff
         // e[cb - 1], e[cb]; the first is unused (and clamped) at t = 0
         ev[a][b] = *reinterpret_cast<const v2du *>(e + (lo ? cb - 1 : cb));
      }
#pragma unroll
   for (int a = 0; a < 2; a++) {
      if (a >= mz) break;
#pragma unroll
      for (int b = 0; b < 2; b++) {
         if (b >= my) break;
         const double em = lo ? ev[a][b].x : 0.0, ec = lo ? ev[a][b].y : ev[a][b].x;
         const double *w = wl + dz[a] * 9 + dy[b] * 3;
         if (lo) acc.x = acc.x + w[2] * em;
         if (hi) acc.x = acc.x + w[0] * ec;
         acc.y = acc.y + w[1] * ec;
      }
   }
   return acc;
}

// one fine point (x, y, z): u_i + sum w e_c in P's CSR order (scalar form of
// geo_prolong_pair, for the marching kernels' wave-edge neighbours)
__device__ __forceinline__ double geo_prolong_point(double acc, const double *__restrict__ e, const double *wl,
                                                    int x, int y, int z, int ncx, int ncy, int ncz)
{
   int c[3][2], d[3][2], m[3];
   const int f[3] = {z, y, x}, nc[3] = {ncz, ncy, ncx};
#pragma unroll
   for (int q = 0; q < 3; q++) {
      m[q] = 0;
      if (f[q] & 1) {
         c[q][m[q]] = (f[q] - 1) >> 1, d[q][m[q]++] = 1;
      } else {
         if (f[q] >= 2) c[q][m[q]] = (f[q] >> 1) - 1, d[q][m[q]++] = 2;
         if ((f[q] >> 1) < nc[q]) c[q][m[q]] = f[q] >> 1, d[q][m[q]++] = 0;
      }
   }
   for (int a = 0; a < m[0]; a++)
      for (int b = 0; b < m[1]; b++)
         for (int q = 0; q < m[2]; q++)
            acc = acc + wl[d[0][a] * 9 + d[1][b] * 3 + d[2][q]] *
                           e[((long long)c[0][a] * ncy + c[1][b]) * ncx + c[2][q]];
   return acc;
}

// fine planes [zb, zb + npairs / (nx ny / 2)) of the nx * ny * nz box; u's
// plane 0 is fine plane fz0, e's plane 0 coarse plane cz0 (z-slab vectors)
__global__ __launch_bounds__(256) void geo_prolong_k(const double *__restrict__ e, double *__restrict__ u,
                                                     const double *__restrict__ wg, int nx, int ny, int nz,
                                                     long long npairs, int zb, int fz0, int cz0, int asg)
{
   __shared__ double wl[27];
   const int tid = (int)threadIdx.x;
   if (tid < 27) wl[tid] = wg[tid];
   __syncthreads();
   const long long q = (long long)blockIdx.x * 256 + tid;
   if (q >= npairs) return;
   const long long i = 2 * q;
   int x, y, z;
   if (npairs < (1LL << 30)) { // 32-bit index arithmetic (the 64-bit divisions are emulated)
      const unsigned iu = (unsigned)i, yz = iu / (unsigned)nx;
      x = (int)(iu - yz * (unsigned)nx);
      y = (int)(yz % (unsigned)ny);
      z = (int)(yz / (unsigned)ny);
   } else {
      x = (int)(i % nx);
      const long long yz = i / nx;
      y = (int)(yz % ny);
      z = (int)(yz / ny);
   }
   z += zb;
   double *ui = u + (long long)(z - fz0) * nx * ny + (i - (long long)(z - zb) * nx * ny);
   // asg: u = P e (from 0.0, the SpMV's start) instead of u += P e
   const v2d acc = asg ? v2d{0.0, 0.0} : *reinterpret_cast<const v2du *>(ui);
   *reinterpret_cast<v2du *>(ui) = geo_prolong_pair(acc, e, wl, x, y, z, nx >> 1, ny >> 1, nz >> 1, cz0);
}

// coarse candidates of fine coordinate y on an axis of nc coarse points, in
// ascending order: (y - 1) / 2 (d 1) when odd; y / 2 - 1 (d 2) and y / 2 (d 0)
// when even, inside [0, nc).  Constant-index stores only (a runtime-indexed
// store would put the arrays in scratch); an absent second candidate repeats
// the first
__device__ __forceinline__ void line_cands(int y, int nc, int &m, int (&c)[2], int (&d)[2])
{
   if (y & 1) {
      m = 1, c[0] = c[1] = (y - 1) >> 1, d[0] = d[1] = 1;
   } else if (y >= 2) {
      c[0] = (y >> 1) - 1, d[0] = 2;
      const bool h = (y >> 1) < nc;
      m = h ? 2 : 1, c[1] = h ? y >> 1 : c[0], d[1] = h ? 0 : 2;
   } else {
      m = (y >> 1) < nc ? 1 : 0, c[0] = c[1] = y >> 1, d[0] = d[1] = 0;
   }
}

// The same prolongation as a plane march: a lane owns one fine pair (x = 2t,
// 2t + 1, y) and walks fine planes [z0, z1) of its chunk.  Fine planes 2c and
// 2c + 1 read coarse plane c (and 2c plane c - 1 too), so a lane loads each
// coarse plane's e[t - 1], e[t] of its (one or two) coarse lines once, at the
// even plane, and keeps the last two in registers: <= 1 coarse 16-byte load
// per fine pair and plane instead of geo_prolong_k's 4.  u of plane z + 1 is
// loaded before plane z is stored.  Terms and order as geo_prolong_pair
// (bit-identical).  Workgroups are mapped XCD-contiguously (csr_mz_kernel).
template <int PF>
__global__ __launch_bounds__(256) void geo_prolong_march_k(const double *__restrict__ e, double *__restrict__ u,
                                                           const double *__restrict__ wg, int nx, int ny, int nz,
                                                           int zb, int ze, int fz0, int cz0, int zc, int nseg,
                                                           int xcd, int asg, int nt = 0)
{
   __shared__ double wl[27];
   const int tid = (int)threadIdx.x;
   if (tid < 27) wl[tid] = wg[tid];
   __syncthreads();
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int seg = lg % nseg, chunk = lg / nseg;
   const unsigned ph = (unsigned)nx >> 1, npp = ph * (unsigned)ny; // pairs per line / plane
   const unsigned pp = (unsigned)seg * 256u + (unsigned)tid;
   const int z0 = zb + chunk * zc, z1 = min(z0 + zc, ze);
   if (pp >= npp || z0 >= z1) return;
   const int t = (int)(pp % ph), y = (int)(pp / ph);
   const int ncx = nx >> 1, ncy = ny >> 1, ncz = nz >> 1;
   int cy[2], dy[2], my;
   line_cands(y, ncy, my, cy, dy);
   const bool lo = t >= 1, hi = t < ncx;
   const long long fpl = (long long)nx * ny, cpl = (long long)ncx * ncy;
   // this lane's e[t - 1] (clamped to e[t] at t = 0) on coarse lines cy[0], cy[1] of plane 0
   const double *eb0 = e + (long long)cy[0] * ncx + (lo ? t - 1 : t);
   const double *eb1 = e + (long long)cy[1] * ncx + (lo ? t - 1 : t);
   auto load_c = [&](int c, v2d (&ev)[2]) {
      const long long o = (long long)(c - cz0) * cpl;
      ev[0] = *reinterpret_cast<const v2du *>(eb0 + o);
      ev[1] = *reinterpret_cast<const v2du *>(eb1 + o);
   };
   auto add_plane = [&](v2d acc, const v2d (&ev)[2], int d) {
#pragma unroll
      for (int b = 0; b < 2; b++) {
         if (b >= my) break;
         const double em = lo ? ev[b].x : 0.0, ec = lo ? ev[b].y : ev[b].x;
         const double *w = wl + d * 9 + dy[b] * 3;
         if (lo) acc.x = acc.x + w[2] * em;
         if (hi) acc.x = acc.x + w[0] * ec;
         acc.y = acc.y + w[1] * ec;
      }
      return acc;
   };
   v2d eprev[2], ecur[2];
   // coarse planes held on entry: z0 odd -> (z0 - 1) / 2; z0 even -> z0 / 2 - 1 (as
   // the "current" plane; the loop's even step shifts it to "previous")
   if (z0 & 1) {
      load_c((z0 - 1) >> 1, ecur);
   } else if (z0 >= 2) {
      load_c((z0 >> 1) - 1, ecur);
   }
   double *up = u + (long long)(z0 - fz0) * fpl + (long long)y * nx + 2 * t;
   // PF u pairs in flight ahead of the plane being stored
   v2d uq[PF];
#pragma unroll
   for (int i = 0; i < PF; i++)
      uq[i] = (!asg && z0 + i < z1) ? ld2nt(up + i * fpl, nt) : v2d{0.0, 0.0};
   for (int z = z0; z < z1; z++, up += fpl) {
      v2d un{0.0, 0.0};
      if (!asg && z + PF < z1) un = ld2nt(up + PF * fpl, nt);
      v2d acc = uq[0];
      if (z & 1) {
         acc = add_plane(acc, ecur, 1);
      } else {
         eprev[0] = ecur[0], eprev[1] = ecur[1];
         const bool has_lo = z >= 2, has_hi = (z >> 1) < ncz;
         if (has_hi) load_c(z >> 1, ecur);
         if (has_lo) acc = add_plane(acc, eprev, 2);
         if (has_hi) acc = add_plane(acc, ecur, 0);
      }
      if (nt & 1)
         __builtin_nontemporal_store(acc, reinterpret_cast<v2du *>(up));
      else
         *reinterpret_cast<v2du *>(up) = acc;
#pragma unroll
      for (int i = 0; i + 1 < PF; i++) uq[i] = uq[i + 1];
      uq[PF - 1] = un;
   }
}

void geo_prolong(hipStream_t s, const GeoT &g, const double *wdev, const double *e, double *u, int zb, int ze,
                 int fz0, int cz0, int assign)
{
   if (ze < 0) ze = g.nz;
   const long long np = (long long)g.nx * g.ny * (ze - zb) / 2;
   if (np <= 0) return;
   static const int march = [] {
      const char *v = std::getenv("AMG_PROLONG_MARCH");
      return v ? std::atoi(v) : 1;
   }();
   // tuning switches: planes per chunk (16) and u pairs in flight (1)
   static const int zc0 = [] {
      const char *v = std::getenv("AMG_PROLONG_ZC");
      return v ? std::max(2, std::min(64, std::atoi(v))) : 16;
   }();
   static const int pf = [] {
      const char *v = std::getenv("AMG_PROLONG_PF");
      return v && std::atoi(v) == 2 ? 2 : 1;
   }();
   // AMG_PROLONG_NT: bit 0 non-temporal stores of u, bit 1 non-temporal loads
   // (default 2: u read once, streamed past the caches -- 512^3 V-cycle
   // 3.018 -> 2.971 ms, profiles/r06/abnt; the stores stay cacheable: the
   // post-sweep reads them next)
   static const int pnt = [] {
      const char *v = std::getenv("AMG_PROLONG_NT");
      return v ? std::atoi(v) & 3 : 2;
   }();
   const long long npp = (long long)g.nx * g.ny / 2;
   if (march && (g.nx & 1) == 0 && npp >= 256 && npp < (1LL << 31)) {
      // fine planes per chunk: 16, fewer when the launch would have < 2048 workgroups
      const int nseg = (int)((npp + 255) / 256);
      const int nzl = ze - zb;
      int zc = zc0;
      while (zc > 2 && (long long)nseg * ((nzl + zc - 1) / zc) < 2048) zc >>= 1;
      const long long G = (long long)nseg * ((nzl + zc - 1) / zc);
      if (pf == 2)
         geo_prolong_march_k<2><<<(unsigned)G, 256, 0, s>>>(e, u, wdev, g.nx, g.ny, g.nz, zb, ze, fz0, cz0, zc, nseg,
                                                            1, assign, pnt);
      else
         geo_prolong_march_k<1><<<(unsigned)G, 256, 0, s>>>(e, u, wdev, g.nx, g.ny, g.nz, zb, ze, fz0, cz0, zc, nseg,
                                                            1, assign, pnt);
      return;
   }
   geo_prolong_k<<<(unsigned)((np + 255) / 256), 256, 0, s>>>(e, u, wdev, g.nx, g.ny, g.nz, np, zb, fz0, cz0, assign);
}

// Prolongation + correction fused with the first post-smoothing sweep of a
// marched 7-pt level (SMEM_Sync_AMG.cpp:118-134: SMEM_Sync_SpGEMV(P, e, u, 1, 1,
// u) then the Jacobi / L1 Jacobi sweep of SMEM_Smooth.cpp:35-45 / 122-130):
// u_out = uc + w (f - A uc) / a_ii with uc = u + P e never stored.  The
// csr_mz_kernel march over the corrected iterate: every uc operand (the
// pair's own line of plane k + 2, lines y -+ 1 of plane k, the wave-edge
// neighbours) is formed in registers from u and the coarse e exactly as
// geo_prolong_k forms it (same terms, same order), so the output is
// bit-identical to geo_prolong_k followed by csr_mz_kernel.  One pass over
// the fine level instead of two (reads f, u and e, writes u_out).
template <bool UNI, bool L1>
__global__ __launch_bounds__(256) void mz_prolong_sweep_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, MpSten Sv, const double *__restrict__ u, const double *__restrict__ e,
   const double *__restrict__ f, const double *__restrict__ l1, const double *__restrict__ wg, double omega,
   int nx, int ny, int nz, int zc, int npb, int xcd, double *__restrict__ uout)
{
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 256 * 7];
   __shared__ double wl[27];
   const int tid = (int)threadIdx.x, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (tid < 27) wl[tid] = wg[tid];
   if (!UNI)
      for (int w = tid; w < np * 7; w += 256) mval[w] = mval_g[w];
   const int S = nx, P = nx * ny;
   const int ncx = nx >> 1, ncy = ny >> 1, ncz = nz >> 1;
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   const int pos = pblk * 512 + 2 * tid;
   const int fx = pos % nx, fy = pos / nx;
   __syncthreads();
   // The operands follow csr_mz_kernel's element indices exactly (row -+ S,
   // row - 1, row + 2 may wrap into the neighbouring line / plane, as they do
   // for any matrix with this master list); only indices outside [0, N) are
   // dropped (no row can use them).  Coordinates one step outside a line or
   // plane carry into the next one.
   auto norm3 = [&](int &x, int &y, int &z) {
      if (x < 0) x += nx, y--;
      if (x >= nx) x -= nx, y++;
      if (y < 0) y += ny, z--;
      if (y >= ny) y -= ny, z++;
   };
   // corrected pair at (fx, fy + dy, p)
   auto uc2 = [&](int p, int dy) -> v2d {
      int x = fx, y = fy + dy, z = p;
      norm3(x, y, z);
      if (z < 0 || z >= nz) return v2d{0.0, 0.0};
      const unsigned i = (unsigned)z * P + (unsigned)(y * S + x);
      return geo_prolong_pair(ld2u(u, i), e, wl, x, y, z, ncx, ncy, ncz);
   };
   // wave-edge neighbour of the own line (lane 0: element - 1, lane 63: + 2)
   auto edge = [&](int p) -> double {
      if (lane != 0 && lane != 63) return 0.0;
      int x = lane == 0 ? fx - 1 : fx + 2, y = fy, z = p;
      norm3(x, y, z);
      if (z < 0 || z >= nz) return 0.0;
      const unsigned i = (unsigned)z * P + (unsigned)(y * S + x);
      return geo_prolong_point(ld1u(u, i), e, wl, x, y, z, ncx, ncy, ncz);
   };
   v2d xm = uc2(k0 - 1, 0);
   v2d xc = uc2(k0, 0);
   double ec = edge(k0);
   v2d xq = uc2(k0 + 1, 0);
   double eq = edge(k0 + 1);
   for (int k = k0; k < k1; k++) {
      const unsigned row = (unsigned)k * P + pos;
      // prefetch plane k + 2 (this chunk's last iteration needs plane k1)
      v2d xn{0.0, 0.0};
      double en = 0.0;
      if (k + 2 < nz && k + 1 < k1) {
         xn = uc2(k + 2, 0);
         en = edge(k + 2);
      }
      const int pid = ppat[row >> 1];
      const v2d fr = ld2u(f, row);
      const v2d ym = uc2(k, -1);
      const v2d yp = uc2(k, 1);
      double lft = __shfl_up(xc.y, 1, 64);
      double rgt = __shfl_down(xc.x, 1, 64);
      if (lane == 0) lft = ec;
      if (lane == 63) rgt = ec;
      const unsigned long long mk = mtab[pid];
      v2d xv[7];
      xv[0] = xc;
      xv[1] = xm;
      xv[2] = ym;
      xv[3] = v2d{lft, xc.x};
      xv[4] = v2d{xc.y, rgt};
      xv[5] = yp;
      xv[6] = xq;
      const v2d res = mz_acc7<1, UNI>(fr, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
      v2d o;
      if (L1) {
         const v2d l = ld2u(l1, row);
         o = v2d{xc.x + res.x / l.x, xc.y + res.y / l.y};
      } else {
         const v2d a = UNI ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 7];
         o = v2d{(a.x != 0.0) ? xc.x + omega * res.x / a.x : xc.x, (a.y != 0.0) ? xc.y + omega * res.y / a.y : xc.y};
      }
      *reinterpret_cast<v2du *>(uout + row) = o;
      xm = xc;
      xc = xq;
      ec = eq;
      xq = xn;
      eq = en;
   }
}

// The composed smoothed prolongation of a marched 7-pt level with geometric P
// (xfer_prolong of the solver: ef = P ec; y = A ef; ef = ef + (-w) (y ./ a))
// in one pass, mz_prolong_sweep_kernel's march over ef = P ec formed in
// registers (from 0.0, the SpMV's start; same terms, same order), then
//   OUT 0: ef stored;
//   OUT 1: atomic_correct: u += ef by device-scope fp64 atomics, u_priv = the
//          value after this level's update (old + ef);
//   OUT 2: u = u + ef (the synchronous cycle's vaxpy with a = 1).
// a_ii := master entry 0 (the diagonal-first rows' first value, = diag).
// held to 5 waves per SIMD (<= 96 VGPRs): the per-row race records took the
// non-uniform forms to 97-99 VGPRs and 4 waves, and config 4's asynchronous
// cycle from 23.4 to 19.0 cycles/s (profiles/r06/bisect*)
template <bool UNI, int OUT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void mz_xfer_prolong_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, MpSten Sv, const double *__restrict__ e, const double *__restrict__ wg,
   double mw, int nx, int ny, int nz, int zc, int npb, int xcd, double *__restrict__ out, double *__restrict__ u_priv,
   int zlo, int zhi, int fz0, int cz0, unsigned long long *stamp)
{
   // OUT 3: OUT 1 in the reference's add-then-read form; OUT 4: the same with
   // the reads batched per workgroup -- every plane's no-return adds issued
   // as the march goes, one wait, then the chunk's rows read back (a wave
   // stalls once per chunk instead of twice per plane; another level's adds
   // may land between a row's add and its read, as in the per-row form)
   constexpr bool noret = OUT == 3 || OUT == 4;
   stamp_begin(stamp);
   const RowRec rst = stamp_rows(stamp);
   // fine planes [zlo, zhi) of the nx * ny * nz box; out / u_priv / the
   // operator's rows (pattern bytes) have plane 0 = fine plane fz0, e plane 0
   // = coarse plane cz0 (a z-slab's extended vectors; the whole box: 0, nz, 0, 0)
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 256 * 7];
   __shared__ double wl[27];
   const int tid = (int)threadIdx.x, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (tid < 27) wl[tid] = wg[tid];
   if (!UNI)
      for (int w = tid; w < np * 7; w += 256) mval[w] = mval_g[w];
   const int P = nx * ny;
   const int ncx = nx >> 1, ncy = ny >> 1, ncz = nz >> 1;
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = zlo + chunk * zc, k1 = min(k0 + zc, zhi);
   const int pos = pblk * 512 + 2 * tid;
   const int fx = pos % nx, fy = pos / nx;
   __syncthreads();
   auto norm3 = [&](int &x, int &y, int &z) {
      if (x < 0) x += nx, y--;
      if (x >= nx) x -= nx, y++;
      if (y < 0) y += ny, z--;
      if (y >= ny) y -= ny, z++;
   };
   auto ef2 = [&](int p, int dy) -> v2d {
      int x = fx, y = fy + dy, z = p;
      norm3(x, y, z);
      if (z < 0 || z >= nz) return v2d{0.0, 0.0};
      return geo_prolong_pair(v2d{0.0, 0.0}, e, wl, x, y, z, ncx, ncy, ncz, cz0);
   };
   auto edge = [&](int p) -> double {
      if (lane != 0 && lane != 63) return 0.0;
      int x = lane == 0 ? fx - 1 : fx + 2, y = fy, z = p;
      norm3(x, y, z);
      if (z < 0 || z >= nz) return 0.0;
      return geo_prolong_point(0.0, e - (long long)cz0 * ncx * ncy, wl, x, y, z, ncx, ncy, ncz);
   };
   v2d xm = ef2(k0 - 1, 0);
   v2d xc = ef2(k0, 0);
   double ec = edge(k0);
   v2d xq = ef2(k0 + 1, 0);
   double eq = edge(k0 + 1);
   for (int k = k0; k < k1; k++) {
      const unsigned row = (unsigned)(k - fz0) * P + pos;
      v2d xn{0.0, 0.0};
      double en = 0.0;
      if (k + 2 < nz && k + 1 < k1) {
         xn = ef2(k + 2, 0);
         en = edge(k + 2);
      }
      const int pid = ppat[row >> 1];
      v2d uo{0.0, 0.0};
      if (OUT == 2) uo = ld2u(out, row);
      const v2d ym = ef2(k, -1);
      const v2d yp = ef2(k, 1);
      double lft = __shfl_up(xc.y, 1, 64);
      double rgt = __shfl_down(xc.x, 1, 64);
      if (lane == 0) lft = ec;
      if (lane == 63) rgt = ec;
      const unsigned long long mk = mtab[pid];
      v2d xv[7];
      xv[0] = xc;
      xv[1] = xm;
      xv[2] = ym;
      xv[3] = v2d{lft, xc.x};
      xv[4] = v2d{xc.y, rgt};
      xv[5] = yp;
      xv[6] = xq;
      const v2d y = mz_acc7<0, UNI>(v2d{0.0, 0.0}, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
      const v2d a = UNI ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 7];
      const double t0 = y.x / a.x, t1 = y.y / a.y;
      const v2d o{xc.x + mw * t0, xc.y + mw * t1};
      if (OUT == 0) {
         *reinterpret_cast<v2du *>(out + row) = o;
      } else if (OUT == 1 || OUT == 3 || OUT == 4) {
         if (noret) {
            add_noret(out + row, o.x);
            add_noret(out + row + 1, o.y);
            if (OUT == 3) {
               wait_vm_all();
               *reinterpret_cast<v2du *>(u_priv + row) = v2d{read_agent(out + row), read_agent(out + row + 1)};
               stamp_row(rst, row);
               stamp_row(rst, row + 1);
            }
         } else {
            const double q0 = atomicAdd(out + row, o.x);
            const double q1 = atomicAdd(out + row + 1, o.y);
            *reinterpret_cast<v2du *>(u_priv + row) = v2d{q0 + o.x, q1 + o.y};
            stamp_row(rst, row, q0, q0 + o.x);
            stamp_row(rst, row + 1, q1, q1 + o.y);
         }
      } else {
         *reinterpret_cast<v2du *>(out + row) = v2d{uo.x + 1.0 * o.x, uo.y + 1.0 * o.y};
      }
      xm = xc;
      xc = xq;
      ec = eq;
      xq = xn;
      eq = en;
   }
   if (OUT == 4) {
      wait_vm_all();
#pragma unroll 4
      for (int k = k0; k < k1; k++) {
         const unsigned row = (unsigned)(k - fz0) * P + pos;
         *reinterpret_cast<v2du *>(u_priv + row) = v2d{read_agent(out + row), read_agent(out + row + 1)};
         stamp_row(rst, row);
         stamp_row(rst, row + 1);
      }
   }
   stamp_end(stamp);
}

void mz_xfer_prolong(hipStream_t s, const amg_mat *A, const double *ec, const GeoT &g, const double *wdev,
                     double omega, int mode, double *out, double *u_priv, int zlo, int zhi, int fz0, int cz0,
                     unsigned long long *stamp)
{
   MpSten S;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      S.off[j] = A->mp_off[j];
      S.val[j] = A->mp_val[j];
   }
   const int P = A->mz_P;
   if (zhi < 0) zhi = g.nz;
   const int nk = zhi - zlo;
   if (nk <= 0) return;
   const int zc = mz_chunk(A, nk, P / 512);
   const int npb = P / 512, nch = (nk + zc - 1) / zc;
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
#define AMG_XP(U, O)                                                                                           \
   mz_xfer_prolong_kernel<U, O><<<npb * nch, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, S, ec, wdev, -omega, \
                                                          g.nx, g.ny, g.nz, zc, npb, A->ctx->mz_xcd, out, u_priv, \
                                                          zlo, zhi, fz0, cz0, mode == 1 ? stamp : nullptr)
#define AMG_XP2(U)                 \
   if (mode == 1 && atomic_noret_mode() == 2) AMG_XP(U, 4); \
   else if (mode == 1 && atomic_noret_mode()) AMG_XP(U, 3); \
   else if (mode == 1) AMG_XP(U, 1); \
   else if (mode == 2) AMG_XP(U, 2); \
   else AMG_XP(U, 0);
   if (A->mp_uni) {
      AMG_XP2(true)
   } else {
      AMG_XP2(false)
   }
#undef AMG_XP2
#undef AMG_XP
}

// The same fused sweep with NL lines per workgroup (lines of nx % 512 == 0
// points; lane t owns the pair (xs + 2t, xs + 2t + 1) of NL consecutive lines
// y0 .. y0 + NL - 1): the corrected iterate of the workgroup's own lines is
// formed ONCE per point (plane k + 2, carried through k + 1, k, k - 1 in
// registers, as csr_mz_kernel's NLN lines), and only the two halo lines
// y0 - 1, y0 + NL of plane k and the wave-edge points are formed on the side:
// (NL + 2) / NL prolongations per point instead of 3.  Same terms, same order:
// bit-identical to geo_prolong_k + csr_mz_kernel.
template <bool UNI, bool L1, int NL>
__global__ __launch_bounds__(256) void mz_prolong_sweep_nl_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, MpSten Sv, const double *__restrict__ u, const double *__restrict__ e,
   const double *__restrict__ f, const double *__restrict__ l1, const double *__restrict__ wg, double omega,
   int nx, int ny, int nz, int zc, int npb, int xcd, double *__restrict__ uout)
{
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 256 * 7];
   __shared__ double wl[27];
   const int tid = (int)threadIdx.x, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (tid < 27) wl[tid] = wg[tid];
   if (!UNI)
      for (int w = tid; w < np * 7; w += 256) mval[w] = mval_g[w];
   const int S = nx, P = nx * ny;
   const int ncx = nx >> 1, ncy = ny >> 1, ncz = nz >> 1;
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int nsx = nx / 512;                          // 512-point segments per line
   const int y0 = (pblk / nsx) * NL, fx = (pblk % nsx) * 512 + 2 * tid;
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   __syncthreads();
   // operands as csr_mz_kernel's element indices (coordinates one step
   // outside a line / plane carry into the next one; outside [0, N) dropped)
   auto norm3 = [&](int &x, int &y, int &z) {
      if (x < 0) x += nx, y--;
      if (x >= nx) x -= nx, y++;
      if (y < 0) y += ny, z--;
      if (y >= ny) y -= ny, z++;
   };
   auto uc2 = [&](int p, int yy) -> v2d {
      int x = fx, y = yy, z = p;
      norm3(x, y, z);
      if (z < 0 || z >= nz) return v2d{0.0, 0.0};
      const unsigned i = (unsigned)z * P + (unsigned)(y * S + x);
      return geo_prolong_pair(ld2u(u, i), e, wl, x, y, z, ncx, ncy, ncz);
   };
   auto edge = [&](int p, int yy) -> double {
      if (lane != 0 && lane != 63) return 0.0;
      int x = lane == 0 ? fx - 1 : fx + 2, y = yy, z = p;
      norm3(x, y, z);
      if (z < 0 || z >= nz) return 0.0;
      const unsigned i = (unsigned)z * P + (unsigned)(y * S + x);
      return geo_prolong_point(ld1u(u, i), e, wl, x, y, z, ncx, ncy, ncz);
   };
   v2d xm[NL], xc[NL], xq[NL];
   double ec[NL], eq[NL];
#pragma unroll
   for (int i = 0; i < NL; i++) {
      xm[i] = uc2(k0 - 1, y0 + i);
      xc[i] = uc2(k0, y0 + i);
      ec[i] = edge(k0, y0 + i);
      xq[i] = uc2(k0 + 1, y0 + i);
      eq[i] = edge(k0 + 1, y0 + i);
   }
   for (int k = k0; k < k1; k++) {
      // plane k + 2 of the own lines (this chunk's last iteration needs k1)
      v2d xn[NL];
      double en[NL];
      const bool nxt = k + 2 < nz && k + 1 < k1;
#pragma unroll
      for (int i = 0; i < NL; i++) {
         xn[i] = v2d{0.0, 0.0};
         en[i] = 0.0;
         if (nxt) {
            xn[i] = uc2(k + 2, y0 + i);
            en[i] = edge(k + 2, y0 + i);
         }
      }
      const v2d ym = uc2(k, y0 - 1), yp = uc2(k, y0 + NL); // halo lines of plane k
#pragma unroll
      for (int i = 0; i < NL; i++) {
         const unsigned row = (unsigned)k * P + (unsigned)((y0 + i) * S + fx);
         const int pid = ppat[row >> 1];
         const v2d fr = ld2u(f, row);
         double lft = __shfl_up(xc[i].y, 1, 64);
         double rgt = __shfl_down(xc[i].x, 1, 64);
         if (lane == 0) lft = ec[i];
         if (lane == 63) rgt = ec[i];
         const unsigned long long mk = mtab[pid];
         v2d xv[7];
         xv[0] = xc[i];
         xv[1] = xm[i];
         xv[2] = i == 0 ? ym : xc[i == 0 ? 0 : i - 1];
         xv[3] = v2d{lft, xc[i].x};
         xv[4] = v2d{xc[i].y, rgt};
         xv[5] = i == NL - 1 ? yp : xc[i == NL - 1 ? 0 : i + 1];
         xv[6] = xq[i];
         const v2d res = mz_acc7<1, UNI>(fr, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
         v2d o;
         if (L1) {
            const v2d l = ld2u(l1, row);
            o = v2d{xc[i].x + res.x / l.x, xc[i].y + res.y / l.y};
         } else {
            const v2d a = UNI ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 7];
            o = v2d{(a.x != 0.0) ? xc[i].x + omega * res.x / a.x : xc[i].x,
                    (a.y != 0.0) ? xc[i].y + omega * res.y / a.y : xc[i].y};
         }
         *reinterpret_cast<v2du *>(uout + row) = o;
      }
#pragma unroll
      for (int i = 0; i < NL; i++) {
         xm[i] = xc[i];
         xc[i] = xq[i];
         ec[i] = eq[i];
         xq[i] = xn[i];
         eq[i] = en[i];
      }
   }
}

// The fused sweep with the coarse correction read from LDS (fuse_prolong 4 /
// 5: NL = 2 / 4 lines per workgroup): the workgroup's coarse lines of the
// coarse planes in use sit in a 4-slot LDS ring (coarse lines y0 / 2 - 1 ..
// y0 / 2 + NL / 2 of the 512-point segment plus one coarse point either side),
// so every corrected operand -- the own lines' plane k + 2, the halo lines
// y0 - 1 / y0 + NL of plane k, the wave-edge points -- is u plus LDS terms, no
// coarse gathers from memory and no coarse values held in registers.  A
// coarse plane enters the ring every second fine plane (one workgroup barrier
// per two planes).  Terms and order as geo_prolong_march_k / geo_prolong_pair:
// bit-identical to geo_prolong + csr_mz_kernel.
template <bool UNI, bool L1, int NL, int OCC = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void mz_prolong_sweep_lds_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np,
   const v2d *__restrict__ mval_g, MpSten Sv, const double *__restrict__ u, const double *__restrict__ e,
   const double *__restrict__ f, const double *__restrict__ l1, const double *__restrict__ wg, double omega,
   int nx, int ny, int nz, int zc, int npb, int xcd, double *__restrict__ uout)
{
   constexpr int NCL = NL / 2 + 2; // coarse lines per ring slot
   constexpr int CW = 258;         // coarse points per line: t0 - 1 .. t0 + 256
   constexpr int NLD = (NCL * CW + 255) / 256;
   __shared__ unsigned long long mtab[256];
   __shared__ v2d mval[UNI ? 1 : 256 * 7];
   __shared__ double wl[27];
   __shared__ double ring[4][NCL][CW];
   const int tid = (int)threadIdx.x, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   if (tid < 27) wl[tid] = wg[tid];
   if (!UNI)
      for (int w = tid; w < np * 7; w += 256) mval[w] = mval_g[w];
   const int S = nx, P = nx * ny;
   const int ncx = nx >> 1, ncy = ny >> 1, ncz = nz >> 1;
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int nsx = nx / 512;
   const int y0 = (pblk / nsx) * NL, seg = pblk % nsx, fx = seg * 512 + 2 * tid;
   const int t = fx >> 1;                   // the pair's coarse x
   const int ct0 = seg * 256 - 1, cy0 = (y0 >> 1) - 1; // ring[.][0][0] = coarse (cy0, ct0)
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   const bool lo = t >= 1, hi = t < ncx;
   // coarse plane c (its NCL lines of CW points; outside the box 0.0) into registers / a slot
   auto fetch_c = [&](int c, double (&v)[NLD]) {
#pragma unroll
      for (int j = 0; j < NLD; j++) {
         const int idx = tid + 256 * j, li = idx / CW, xi = idx - li * CW;
         const int cy = cy0 + li, cx = ct0 + xi;
         v[j] = (idx < NCL * CW && c >= 0 && c < ncz && cy >= 0 && cy < ncy && cx >= 0 && cx < ncx)
                   ? e[((long long)c * ncy + cy) * ncx + cx]
                   : 0.0;
      }
   };
   auto store_c = [&](int c, const double (&v)[NLD]) {
      double *sl = &ring[c & 3][0][0];
#pragma unroll
      for (int j = 0; j < NLD; j++) {
         const int idx = tid + 256 * j;
         if (idx < NCL * CW) sl[idx] = v[j];
      }
   };
   // line candidates of fine line y (line_cands; ring line indices)
   struct LC {
      int m, c[2], d[2];
   };
   auto cands = [&](int y) {
      LC r;
      line_cands(y, ncy, r.m, r.c, r.d);
      r.c[0] -= cy0;
      r.c[1] -= cy0;
      return r;
   };
   // coarse terms of fine plane z for the pair (acc.x: coarse t - 1, t; acc.y: t)
   auto add_pair = [&](v2d acc, int z, const LC &lc) {
      auto plane = [&](int c, int d) {
#pragma unroll
         for (int b = 0; b < 2; b++) {
            if (b >= lc.m) break;
            const double *E = &ring[c & 3][lc.c[b]][0];
            const double em = lo ? E[tid] : 0.0, ec = E[tid + 1];
            const double *w = wl + d * 9 + lc.d[b] * 3;
            if (lo) acc.x = acc.x + w[2] * em;
            if (hi) acc.x = acc.x + w[0] * ec;
            acc.y = acc.y + w[1] * ec;
         }
      };
      if (z & 1) {
         plane((z - 1) >> 1, 1);
      } else {
         if (z >= 2) plane((z >> 1) - 1, 2);
         if ((z >> 1) < ncz) plane(z >> 1, 0);
      }
      return acc;
   };
   // corrected pair of line y, plane z (outside the box: 0.0, no row uses it)
   auto uc2 = [&](int z, int y, const LC &lc) -> v2d {
      if (z < 0 || z >= nz || y < 0 || y >= ny) return v2d{0.0, 0.0};
      return add_pair(ld2u(u, (unsigned)z * P + (unsigned)(y * S + fx)), z, lc);
   };
   // wave-edge neighbour of the own line: lane 0 the point fx - 1 (the .y of
   // pair t - 1), lane 63 the point fx + 2 (the .x of pair t + 1)
   auto edge = [&](int z, int y, const LC &lc) -> double {
      if (lane != 0 && lane != 63) return 0.0;
      if (z < 0 || z >= nz) return 0.0;
      const bool left = lane == 0;
      if (left ? fx == 0 : fx + 2 >= nx) return 0.0;
      double acc = ld1u(u, (unsigned)z * P + (unsigned)(y * S + (left ? fx - 1 : fx + 2)));
      const int q = left ? tid : tid + 1; // ring index of coarse t - 1 / t
      const bool hi2 = t + 1 < ncx;
      auto plane = [&](int c, int d) {
#pragma unroll
         for (int b = 0; b < 2; b++) {
            if (b >= lc.m) break;
            const double *E = &ring[c & 3][lc.c[b]][0];
            const double *w = wl + d * 9 + lc.d[b] * 3;
            if (left) {
               acc = acc + w[1] * E[q];
            } else {
               acc = acc + w[2] * E[q];
               if (hi2) acc = acc + w[0] * E[q + 1];
            }
         }
      };
      if (z & 1) {
         plane((z - 1) >> 1, 1);
      } else {
         if (z >= 2) plane((z >> 1) - 1, 2);
         if ((z >> 1) < ncz) plane(z >> 1, 0);
      }
      return acc;
   };
   LC lcs[NL];
#pragma unroll
   for (int i = 0; i < NL; i++) lcs[i] = cands(y0 + i);
   const LC lcm = cands(y0 - 1), lcp = cands(y0 + NL);
   // the ring holds coarse planes (k >> 1) - 1 .. (k >> 1) + 1 at step k, and
   // (k >> 1) + 2 from the barrier of the even step before it is needed
   {
      const int cb = (k0 >> 1) - 1, ce = (k0 >> 1) + 1 + (k0 & 1);
      double v[NLD];
      for (int c = cb; c <= ce; c++) {
         fetch_c(c, v);
         store_c(c, v);
      }
   }
   __syncthreads();
   v2d xm[NL], xc[NL], xq[NL];
   double ec[NL], eq[NL];
#pragma unroll
   for (int i = 0; i < NL; i++) {
      xm[i] = uc2(k0 - 1, y0 + i, lcs[i]);
      xc[i] = uc2(k0, y0 + i, lcs[i]);
      ec[i] = edge(k0, y0 + i, lcs[i]);
      xq[i] = uc2(k0 + 1, y0 + i, lcs[i]);
      eq[i] = edge(k0 + 1, y0 + i, lcs[i]);
   }
   for (int k = k0; k < k1; k++) {
      double cv[NLD];
      if ((k & 1) == 0) {
         if (k != k0) __syncthreads(); // slot (k >> 1) - 2 free, plane (k >> 1) + 1 visible
         fetch_c((k >> 1) + 2, cv);
      }
      v2d xn[NL];
      double en[NL];
      const bool nxt = k + 2 < nz && k + 1 < k1;
#pragma unroll
      for (int i = 0; i < NL; i++) {
         xn[i] = v2d{0.0, 0.0};
         en[i] = 0.0;
         if (nxt) {
            xn[i] = uc2(k + 2, y0 + i, lcs[i]);
            en[i] = edge(k + 2, y0 + i, lcs[i]);
         }
      }
      const v2d ym = uc2(k, y0 - 1, lcm), yp = uc2(k, y0 + NL, lcp); // halo lines of plane k
#pragma unroll
      for (int i = 0; i < NL; i++) {
         const unsigned row = (unsigned)k * P + (unsigned)((y0 + i) * S + fx);
         const int pid = ppat[row >> 1];
         const v2d fr = ld2u(f, row);
         double lft = __shfl_up(xc[i].y, 1, 64);
         double rgt = __shfl_down(xc[i].x, 1, 64);
         if (lane == 0) lft = ec[i];
         if (lane == 63) rgt = ec[i];
         const unsigned long long mk = mtab[pid];
         v2d xv[7];
         xv[0] = xc[i];
         xv[1] = xm[i];
         xv[2] = i == 0 ? ym : xc[i == 0 ? 0 : i - 1];
         xv[3] = v2d{lft, xc[i].x};
         xv[4] = v2d{xc[i].y, rgt};
         xv[5] = i == NL - 1 ? yp : xc[i == NL - 1 ? 0 : i + 1];
         xv[6] = xq[i];
         const v2d res = mz_acc7<1, UNI>(fr, xv, mk, Sv, UNI ? nullptr : mval + pid * 7);
         v2d o;
         if (L1) {
            const v2d l = ld2u(l1, row);
            o = v2d{xc[i].x + res.x / l.x, xc[i].y + res.y / l.y};
         } else {
            const v2d a = UNI ? v2d{Sv.val[0], Sv.val[0]} : mval[pid * 7];
            o = v2d{(a.x != 0.0) ? xc[i].x + omega * res.x / a.x : xc[i].x,
                    (a.y != 0.0) ? xc[i].y + omega * res.y / a.y : xc[i].y};
         }
         *reinterpret_cast<v2du *>(uout + row) = o;
      }
#pragma unroll
      for (int i = 0; i < NL; i++) {
         xm[i] = xc[i];
         xc[i] = xq[i];
         ec[i] = eq[i];
         xq[i] = xn[i];
         eq[i] = en[i];
      }
      if ((k & 1) == 0) store_c((k >> 1) + 2, cv);
   }
}

void mz_prolong_sweep(hipStream_t s, const amg_mat *A, const double *f, const double *u, const double *ec,
                      const GeoT &g, const double *wdev, const double *l1, double omega, double *uout)
{
   MpSten S;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      S.off[j] = A->mp_off[j];
      S.val[j] = A->mp_val[j];
   }
   const int P = A->mz_P, nz = A->nrows / P;
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
   // fuse_prolong 1: four lines per workgroup, 3: two, 2: one (mz_prolong_sweep_kernel);
   // 4 / 5: two / four lines, the coarse correction from an LDS ring (mz_prolong_sweep_lds_kernel)
   const int fp = A->ctx->fuse_prolong;
   if (fp >= 6 && g.nx % 512 == 0 && g.ny % 2 == 0) {
      // two lines, the kernel held to 5 / 6 waves per SIMD (register budget)
      const int npb = P / 1024, zc = mz_chunk(A, nz, npb), nch = (nz + zc - 1) / zc;
#define AMG_PSO(U, L, O)                                                                                           \
   mz_prolong_sweep_lds_kernel<U, L, 2, O><<<npb * nch, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, S, u, ec, f, l1, \
                                                                     wdev, omega, g.nx, g.ny, g.nz, zc, npb,           \
                                                                     A->ctx->mz_xcd, uout)
      if (A->mp_uni && !l1) {
         if (fp == 6) AMG_PSO(true, false, 5);
         else AMG_PSO(true, false, 6);
         return;
      }
#undef AMG_PSO
   }
   if ((fp == 4 || fp == 5) && g.nx % 512 == 0 && g.ny % (fp == 4 ? 2 : 4) == 0) {
      const int NLs = fp == 4 ? 2 : 4;
      const int npb = P / (512 * NLs), zc = mz_chunk(A, nz, npb), nch = (nz + zc - 1) / zc;
#define AMG_PSL(U, L, N)                                                                                               \
   mz_prolong_sweep_lds_kernel<U, L, N><<<npb * nch, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, S, u, ec, f, l1, wdev, \
                                                                  omega, g.nx, g.ny, g.nz, zc, npb, A->ctx->mz_xcd, uout)
#define AMG_PSL2(N)                           \
   if (A->mp_uni) {                           \
      if (l1) AMG_PSL(true, true, N);         \
      else AMG_PSL(true, false, N);           \
   } else {                                   \
      if (l1) AMG_PSL(false, true, N);        \
      else AMG_PSL(false, false, N);          \
   }
      if (NLs == 2) {
         AMG_PSL2(2)
      } else {
         AMG_PSL2(4)
      }
#undef AMG_PSL2
#undef AMG_PSL
      return;
   }
   const int NL = fp == 3 ? 2 : 4;
   if (fp != 2 && g.nx % 512 == 0 && g.ny % NL == 0) {
      const int npb = P / (512 * NL), zc = mz_chunk(A, nz, npb), nch = (nz + zc - 1) / zc;
#define AMG_PSN(U, L, N)                                                                                              \
   mz_prolong_sweep_nl_kernel<U, L, N><<<npb * nch, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, S, u, ec, f, l1, wdev, \
                                                                 omega, g.nx, g.ny, g.nz, zc, npb, A->ctx->mz_xcd, uout)
#define AMG_PSN2(N)                           \
   if (A->mp_uni) {                           \
      if (l1) AMG_PSN(true, true, N);         \
      else AMG_PSN(true, false, N);           \
   } else {                                   \
      if (l1) AMG_PSN(false, true, N);        \
      else AMG_PSN(false, false, N);          \
   }
      if (NL == 2) {
         AMG_PSN2(2)
      } else {
         AMG_PSN2(4)
      }
#undef AMG_PSN2
#undef AMG_PSN
      return;
   }
   const int zc = mz_chunk(A, nz, P / 512);
   const int npb = P / 512, nch = (nz + zc - 1) / zc;
#define AMG_PS(U, L) \
   mz_prolong_sweep_kernel<U, L><<<npb * nch, 256, 0, s>>>(A->ppat, A->mpmask, A->pp_n, mv, S, u, ec, f, l1, wdev, \
                                                           omega, g.nx, g.ny, g.nz, zc, npb, A->ctx->mz_xcd, uout)
   if (A->mp_uni) {
      if (l1) AMG_PS(true, true);
      else AMG_PS(true, false);
   } else {
      if (l1) AMG_PS(false, true);
      else AMG_PS(false, false);
   }
#undef AMG_PS
}

// Geometric restriction f_c = R r (SMEM_Sync_Parfor_Restrict,
// SMEM_MatVec.cpp:380-392) for a checked geometric R: coarse point K sums
// w * r over fine 2K + d in R's CSR order (dz, dy, dx), from 0.
// coarse planes [Kb, Kb + nc / (ncx ncy)); r's plane 0 is fine plane fz0, fc's
// plane 0 coarse plane cz0 (z-slab vectors)
__global__ __launch_bounds__(256) void geo_restrict_k(const double *__restrict__ r, double *__restrict__ fc,
                                                      const double *__restrict__ wg, int nx, int ny, int nz,
                                                      long long nc, int Kb, int fz0, int cz0, ZeroGuess zg)
{
   __shared__ double wl[27];
   const int tid = (int)threadIdx.x;
   if (tid < 27) wl[tid] = wg[tid];
   __syncthreads();
   const long long K = (long long)blockIdx.x * 256 + tid;
   if (K >= nc) return;
   const int ncx = nx >> 1, ncy = ny >> 1;
   int Kx, Ky, Kz;
   if (nc < (1LL << 31)) { // 32-bit index arithmetic (the 64-bit divisions are emulated)
      const unsigned t = (unsigned)K / (unsigned)ncx;
      Kx = (int)((unsigned)K - t * (unsigned)ncx);
      Ky = (int)(t % (unsigned)ncy);
      Kz = (int)(t / (unsigned)ncy);
   } else {
      Kx = (int)(K % ncx);
      const long long t = K / ncx;
      Ky = (int)(t % ncy);
      Kz = (int)(t / ncy);
   }
   Kz += Kb;
   const bool dx2 = 2 * Kx + 2 < nx;
   // the nine fine (plane, line) loads issued first (lines outside the box
   // read the last inside one, unused), then the terms in R's CSR order
   v2d a[3][3];
   double c[3][3];
#pragma unroll
   for (int dz = 0; dz < 3; dz++)
#pragma unroll
      for (int dy = 0; dy < 3; dy++) {
         const int fz = min(2 * Kz + dz, nz - 1), fy = min(2 * Ky + dy, ny - 1);
         const double *p = r + ((long long)(fz - fz0) * ny + fy) * nx + 2 * Kx;
         a[dz][dy] = *reinterpret_cast<const v2du *>(p);
         c[dz][dy] = dx2 ? p[2] : 0.0;
      }
   double acc = 0.0;
#pragma unroll
   for (int dz = 0; dz < 3; dz++) {
      if (2 * Kz + dz >= nz) break;
#pragma unroll
      for (int dy = 0; dy < 3; dy++) {
         if (2 * Ky + dy >= ny) break;
         const double *w = wl + dz * 9 + dy * 3;
         acc = acc + w[0] * a[dz][dy].x;
         acc = acc + w[1] * a[dz][dy].y;
         if (dx2) acc = acc + w[2] * c[dz][dy];
      }
   }
   const long long ci = ((long long)(Kz - cz0) * ncy + Ky) * ncx + Kx;
   fc[ci] = acc;
   zg_apply(zg, ci, acc);
}

void geo_restrict(hipStream_t s, const GeoT &g, const double *wdev, const double *r, double *fc, int Kb, int Ke,
                  int fz0, int cz0, ZeroGuess zg)
{
   if (Ke < 0) Ke = g.nz / 2;
   const long long nc = (long long)(g.nx / 2) * (g.ny / 2) * (Ke - Kb);
   if (nc <= 0) return;
   geo_restrict_k<<<(unsigned)((nc + 255) / 256), 256, 0, s>>>(r, fc, wdev, g.nx, g.ny, g.nz, nc, Kb, fz0, cz0, zg);
}

// dictionary-coded launches: rows of <= 8 entries (7-pt stencil, interpolation)
// take four 256-row tiles per workgroup, longer rows (27-pt Galerkin,
// restriction) two (tools/tune_spmv.py, profiles/r01/tune_spmv.log); the
// row-pattern form when the matrix has one
template <int NEG, bool NEED_DIAG, class Epi>
static void launch_dc_op(hipStream_t s, const amg_mat *A, const double *x, int rb, int re,
                         const Epi &e, double *partials, int tiles)
{
   // plane-aligned row ranges march over their planes (a z-slab's owned planes)
   const bool march = A->mz_P && rb % A->mz_P == 0 && re % A->mz_P == 0;
   if (march && A->mz27)
      launch_mz27<NEG, NEED_DIAG>(s, A, x, e, partials, rb / A->mz_P, re / A->mz_P);
   else if (march)
      launch_mz<NEG, NEED_DIAG>(s, A, x, e, partials, rb / A->mz_P, re / A->mz_P);
   else if (A->mp_J && (rb & 1) == 0)
      launch_mp<NEG, NEED_DIAG>(s, A, x, rb, re, e, partials);
   else if (A->ppat && (rb & 1) == 0)
      csr_rpp_kernel<NEG, NEED_DIAG, Epi, 2><<<(re - rb + 1023) / 1024, 256, A->pp_n * A->pp_stride * 4, s>>>(
         A->ppat, A->pptab, A->pp_n, A->doff, A->dval, x, rb, re, e, partials, A->dc_n, A->pp_stride, A->danch,
         A->pp_centre0, A->pbase, A->pdelta);
   else if (A->rpat && A->dc_maxrow <= 8)
      csr_rp_kernel<NEG, NEED_DIAG, Epi, 4><<<(tiles + 3) / 4, 256, 0, s>>>(
         A->rpat, A->ptab, A->rp_n, A->doff, A->dval, x, rb, re, e, partials, A->dc_n, A->danch);
   else if (A->rpat)
      csr_rp_kernel<NEG, NEED_DIAG, Epi, 2><<<(tiles + 1) / 2, 256, 0, s>>>(
         A->rpat, A->ptab, A->rp_n, A->doff, A->dval, x, rb, re, e, partials, A->dc_n, A->danch);
   else if (A->dc_maxrow <= 8)
      csr_dc_kernel<NEG, NEED_DIAG, Epi, 4, true, 8><<<(tiles + 3) / 4, 256, 0, s>>>(
         A->rowptr, A->didx, A->doff, A->dval, x, rb, re, e, partials, A->dc_n, A->danch);
   else
      csr_dc_kernel<NEG, NEED_DIAG, Epi, 2, true, AMG_DC_MAXROW><<<(tiles + 1) / 2, 256, 0, s>>>(
         A->rowptr, A->didx, A->doff, A->dval, x, rb, re, e, partials, A->dc_n, A->danch);
}

// Long-row operators (dense coarse levels of classical hierarchies: hundreds of
// entries per row, few rows): a 256-row tile leaves most of the chip idle.
// Here a workgroup of TB threads owns RW rows: all TB threads stream the rows'
// entries in chunks and form the rounded products into LDS, then lane r < RW
// adds its row's products in CSR order -- the tile kernel's exact summation
// with many more workgroups and loads in flight.  Norm partials (one per
// 256-row tile, the tile kernel's layout) only with RW = TB = 256.
template <int NEG, bool NEED_DIAG, class Epi, bool VI, int TB, int RW>
__global__ __launch_bounds__(TB) void csr_long_kernel(
   const int *__restrict__ rowptr, const int *__restrict__ col, const double *__restrict__ val,
   const unsigned char *__restrict__ vidx, const double *__restrict__ vtab_g, const double *__restrict__ x,
   int rb, int re, Epi epi, double *__restrict__ partials = nullptr)
{
   constexpr int CH = 2048;
   __shared__ double prod[CH];
   __shared__ double vtab[VI ? 256 : 1];
   __shared__ double red[4];
   const int tid = (int)threadIdx.x;
   const int r0 = rb + (int)blockIdx.x * RW, r1 = min(r0 + RW, re);
   const int row = r0 + tid;
   const bool own = tid < RW && row < r1;
   int rs = 0, rend = 0;
   double acc = 0.0, pf = 0.0, dg = 0.0;
   if (own) {
      rs = rowptr[row];
      rend = rowptr[row + 1];
      acc = epi.init(row);
      pf = epi.pf(row);
      if (NEED_DIAG && !VI) dg = val[rs];
   }
   const int tb = rowptr[r0], te = rowptr[r1];
   if (VI) {
      for (int t = tid; t < 256; t += TB) vtab[t] = vtab_g[t];
      __syncthreads();
      if (NEED_DIAG && own) dg = vtab[vidx[rs]];
   }
   for (int cs = tb; cs < te; cs += CH) {
      const int ce = min(cs + CH, te);
#pragma unroll 8
      for (int k = cs + tid; k < ce; k += TB) {
         const double a = VI ? vtab[vidx[k]] : val[k];
         prod[k - cs] = a * x[col[k]];
      }
      __syncthreads();
      if (own) {
         // in CSR order; the LDS reads of 8 products are issued together so
         // only the add chain is sequential
         const int a0 = max(rs, cs), a1 = min(rend, ce);
         int k = a0;
         for (; k + 8 <= a1; k += 8) {
            double p[8];
#pragma unroll
            for (int j = 0; j < 8; j++) p[j] = prod[k + j - cs];
#pragma unroll
            for (int j = 0; j < 8; j++) {
               if (NEG)
                  acc -= p[j];
               else
                  acc += p[j];
            }
         }
         for (; k < a1; k++) {
            if (NEG)
               acc -= prod[k - cs];
            else
               acc += prod[k - cs];
         }
      }
      __syncthreads();
   }
   double out = 0.0;
   if (own) out = epi.finish(row, acc, dg, pf);
   if (RW == 256 && TB == 256 && partials) {
      const double sblk = block_sum_256(out * out, red);
      if (tid == 0) partials[blockIdx.x] = sblk;
   }
}

// Wave-independent long-row form (ctx->long_form 1 / 2: CW = 8 / 16).  Each
// wave owns RPW consecutive rows (lane r < RPW: row r0 + r) and streams their
// entries itself in chunks of 64 CW (entry k of the chunk on lane k % 64, all
// CW column / value loads and then all CW gathers of a lane in flight), rounds
// the products into its own LDS slab, and each lane then adds its row's
// products in CSR order -- csr_long_kernel's exact summation, but with no
// workgroup barrier: the slab is the wave's own (the LDS executes a wave's
// operations in issue order, so the next chunk's stores follow this chunk's
// reads), and the waves' load and summation phases overlap.  XCD-contiguous
// row blocks (xcd) keep a block's gathered x in its XCD's L2.  Norm partials
// (one per 256-row tile) only with RPW = 64.
template <int NEG, bool NEED_DIAG, class Epi, bool VI, int CW>
__global__ __launch_bounds__(256) void csr_longw_kernel(
   const int *__restrict__ rowptr, const int *__restrict__ col, const double *__restrict__ val,
   const unsigned char *__restrict__ vidx, const double *__restrict__ vtab_g, const double *__restrict__ x,
   int rb, int re, int rpw, int xcd, Epi epi, double *__restrict__ partials)
{
   __shared__ double prod[4][64 * CW];
   __shared__ double vtab[VI ? 256 : 1];
   __shared__ double red[4];
   const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
   int blk = (int)blockIdx.x;
   if (xcd) {
      // bijective: the blocks dealt to one XCD (b % 8) get a contiguous range
      const int nb = (int)gridDim.x, q = nb >> 3, r = nb & 7, xg = blk & 7, idx = blk >> 3;
      blk = (xg < r ? xg * (q + 1) : r * (q + 1) + (xg - r) * q) + idx;
   }
   if (VI) {
      vtab[tid] = vtab_g[tid];
      __syncthreads();
   }
   const long long r0l = (long long)rb + ((long long)blk * 4 + w) * rpw;
   const int r0 = (int)min(r0l, (long long)re), r1 = min(r0 + rpw, re);
   const int row = r0 + lane;
   const bool own = lane < rpw && row < r1;
   int rs = 0, rend = 0;
   double acc = 0.0, pf = 0.0, dg = 0.0;
   if (own) {
      rs = rowptr[row];
      rend = rowptr[row + 1];
      acc = epi.init(row);
      pf = epi.pf(row);
      if (NEED_DIAG) dg = VI ? vtab[vidx[rs]] : val[rs];
   }
   if (r0 < r1) {
      const int tb = rowptr[r0], te = rowptr[r1];
      double *pw = prod[w];
      for (int cs = tb; cs < te; cs += 64 * CW) {
         const int ce = min(cs + 64 * CW, te);
         int cj[CW];
         double av[CW];
#pragma unroll
         for (int j = 0; j < CW; j++) {
            const int k = cs + j * 64 + lane;
            const int kk = k < ce ? k : cs; // past the chunk: a valid entry, never summed
            cj[j] = col[kk];
            av[j] = VI ? vtab[vidx[kk]] : val[kk];
         }
         double xv[CW];
#pragma unroll
         for (int j = 0; j < CW; j++) xv[j] = x[cj[j]];
#pragma unroll
         for (int j = 0; j < CW; j++) pw[j * 64 + lane] = av[j] * xv[j];
         __builtin_amdgcn_wave_barrier();
         if (own) {
            const int a0 = max(rs, cs), a1 = min(rend, ce);
            int k = a0;
            for (; k + 8 <= a1; k += 8) {
               double p[8];
#pragma unroll
               for (int j = 0; j < 8; j++) p[j] = pw[k + j - cs];
#pragma unroll
               for (int j = 0; j < 8; j++) {
                  if (NEG)
                     acc -= p[j];
                  else
                     acc += p[j];
               }
            }
            for (; k < a1; k++) {
               if (NEG)
                  acc -= pw[k - cs];
               else
                  acc += pw[k - cs];
            }
         }
         __builtin_amdgcn_wave_barrier();
      }
   }
   double out = 0.0;
   if (own) out = epi.finish(row, acc, dg, pf);
   if (partials) {
      const double sblk = block_sum_256(out * out, red);
      if (tid == 0) partials[blk] = sblk;
   }
}

// long rows: at least 64 entries per row on average
static inline bool long_rows(const amg_mat *A) { return A->nnz >= 64LL * A->nrows; }

template <int NEG, bool NEED_DIAG, int TB, int RW, class Epi>
static void launch_long_cfg(hipStream_t s, const amg_mat *A, const double *x, int rb, int re, const Epi &e,
                            double *partials = nullptr)
{
   const int nb = (re - rb + RW - 1) / RW;
   if (A->vidx)
      csr_long_kernel<NEG, NEED_DIAG, Epi, true, TB, RW><<<nb, TB, 0, s>>>(A->rowptr, A->col, A->val, A->vidx,
                                                                          A->vtab, x, rb, re, e, partials);
   else
      csr_long_kernel<NEG, NEED_DIAG, Epi, false, TB, RW><<<nb, TB, 0, s>>>(A->rowptr, A->col, A->val, nullptr,
                                                                           nullptr, x, rb, re, e, partials);
}

// rows per workgroup: the most that still gives >= 4096 workgroups (64 .. 8);
// with norm partials one 256-row tile per workgroup (tools/tune_spmv.py -5)
template <int NEG, bool NEED_DIAG, class Epi>
static void launch_long(hipStream_t s, const amg_mat *A, const double *x, int rb, int re, const Epi &e,
                        double *partials = nullptr)
{
   const int n = re - rb;
   if (A->ctx->long_form) {
      // rows per wave: the most that still gives >= 4096 workgroups (64 .. 8);
      // with norm partials 64 (one 256-row tile per workgroup)
      const int rpw = partials ? 64 : n >= 256 * 4096 ? 64 : n >= 128 * 4096 ? 32 : n >= 64 * 4096 ? 16 : 8;
      const int nb = (int)(((long long)n + 4 * rpw - 1) / (4 * rpw));
      auto go = [&](auto cw) {
         constexpr int W = decltype(cw)::value;
         if (A->vidx)
            csr_longw_kernel<NEG, NEED_DIAG, Epi, true, W><<<nb, 256, 0, s>>>(
               A->rowptr, A->col, A->val, A->vidx, A->vtab, x, rb, re, rpw, A->ctx->long_xcd, e, partials);
         else
            csr_longw_kernel<NEG, NEED_DIAG, Epi, false, W><<<nb, 256, 0, s>>>(
               A->rowptr, A->col, A->val, nullptr, nullptr, x, rb, re, rpw, A->ctx->long_xcd, e, partials);
      };
      if (A->ctx->long_form == 2)
         go(std::integral_constant<int, 16>{});
      else
         go(std::integral_constant<int, 8>{});
      return;
   }
   // AMG_LONG_RW=128 / 256: rows per workgroup on the largest levels (the rows'
   // sequential sums then spread over 2 / 4 waves instead of one)
   static const int lrw = [] {
      const char *v = std::getenv("AMG_LONG_RW");
      return v ? std::atoi(v) : 0;
   }();
   if (partials)
      launch_long_cfg<NEG, NEED_DIAG, 256, 256>(s, A, x, rb, re, e, partials);
   else if (lrw == 256 && n >= 256 * 2048)
      launch_long_cfg<NEG, NEED_DIAG, 256, 256>(s, A, x, rb, re, e);
   else if (lrw == 128 && n >= 128 * 2048)
      launch_long_cfg<NEG, NEED_DIAG, 256, 128>(s, A, x, rb, re, e);
   else if (n >= 64 * 4096)
      launch_long_cfg<NEG, NEED_DIAG, 256, 64>(s, A, x, rb, re, e);
   else if (n >= 32 * 4096)
      launch_long_cfg<NEG, NEED_DIAG, 256, 32>(s, A, x, rb, re, e);
   else if (n >= 16 * 4096)
      launch_long_cfg<NEG, NEED_DIAG, 256, 16>(s, A, x, rb, re, e);
   else
      launch_long_cfg<NEG, NEED_DIAG, 256, 8>(s, A, x, rb, re, e);
}

// production configuration (tools/tune_spmv.py picks it on the MI355X)
using ProdCfg = TileCfg<1, 2048, false, false>;
// value-indexed matrices with short rows (< 12 entries on average: 7-pt
// stencil, prolongation) stage 8 consecutive entries per lane with all loads
// issued up front (-3..6 % there; +2..5 % on 27-entry rows, which keep ProdCfg)
using ShortCfg = TileCfg<1, 2048, false, false, false, false, false, false, true>;
static inline bool short_rows(const amg_mat *A) { return A->nnz < 12LL * A->nrows; }

// Epilogue interface: init(i) -> accumulator start value; pf(i) -> one
// operand prefetched before the stream; finish(i, acc, a_ii, pf) writes the
// row's outputs and returns the value whose square feeds the norm partials.

// y = SpGEMV epilogue (SMEM_MatVec.cpp:140-258)
// 16-byte store of rows (i, i+1); nt bit 0: nontemporal (streamed past the
// caches, for fine-grid outputs far larger than L2 + Infinity Cache); bit 1
// (ld2nt): the same for the streamed right-hand side loads
__device__ __forceinline__ void st2(double *p, v2d v, int nt)
{
   if (nt & 1)
      __builtin_nontemporal_store(v, reinterpret_cast<v2du *>(p));
   else
      *reinterpret_cast<v2du *>(p) = v;
}

struct EpiGemv {
   const double *b;
   double *y;
   int imode;
   int scale;
   double alpha, temp;
   int nt = 0;
   __device__ __forceinline__ double init(int i) const
   {
      switch (imode) {
      case 0: return 0.0;
      case 1: return b[i];
      case 2: return -b[i];
      case 3: return b[i] * temp;
      default: return -b[i] * temp;
      }
   }
   __device__ __forceinline__ double pf(int) const { return 0.0; }
   __device__ __forceinline__ double finish(int i, double acc, double, double) const
   {
      const double v = scale ? alpha * acc : acc;
      y[i] = v;
      return v;
   }
   // rows i, i+1 (paired-row kernel)
   __device__ __forceinline__ v2d init2(int i) const
   {
      if (imode == 0) return v2d{0.0, 0.0};
      const v2d bb = *reinterpret_cast<const v2du *>(b + i);
      switch (imode) {
      case 1: return bb;
      case 2: return v2d{-bb.x, -bb.y};
      case 3: return v2d{bb.x * temp, bb.y * temp};
      default: return v2d{-bb.x * temp, -bb.y * temp};
      }
   }
   __device__ __forceinline__ v2d pf2(int) const { return v2d{0.0, 0.0}; }
   __device__ __forceinline__ v2d finish2(int i, v2d acc, v2d, v2d) const
   {
      const v2d v = scale ? v2d{alpha * acc.x, alpha * acc.y} : acc;
      st2(y + i, v, nt);
      return v;
   }
};

// r = b - sum (SMEM_Residual's y = A x then r = b - y, y not stored)
struct EpiFsub {
   const double *b;
   double *r;
   int nt = 0;
   __device__ __forceinline__ double init(int) const { return 0.0; }
   __device__ __forceinline__ double pf(int i) const { return b[i]; }
   __device__ __forceinline__ double finish(int i, double acc, double, double bi) const
   {
      const double v = bi - acc;
      r[i] = v;
      return v;
   }
   __device__ __forceinline__ v2d init2(int) const { return v2d{0.0, 0.0}; }
   __device__ __forceinline__ v2d pf2(int i) const { return *reinterpret_cast<const v2du *>(b + i); }
   __device__ __forceinline__ v2d finish2(int i, v2d acc, v2d, v2d bi) const
   {
      const v2d v{bi.x - acc.x, bi.y - acc.y};
      st2(r + i, v, nt);
      return v;
   }
};

// Division by a uniform diagonal d with its reciprocal y = RN(1/d) known:
// q0 = RN(x y), the exact remainder r = x - q0 d (fma), q1 = RN(q0 + r y) --
// the correctly rounded x / d, the same bits as the division, for x in the
// normal range (Markstein's correction step; host-checked divisor: fast_div_of;
// brute-forced against x / d over 10^9 operands incl. near-midpoint ones).
// A wave takes it only when every lane's divisor is d and operand in range
// (+0 included, -0 not: q1 would be +0), else the division itself.
__device__ __forceinline__ double div_rcp(double x, double d, double y)
{
   const double q0 = x * y;
   const double r = __builtin_fma(-q0, d, x);
   return __builtin_fma(r, y, q0);
}
__device__ __forceinline__ bool div_rcp_ok(double x)
{
   const double ax = fabs(x);
   return (ax >= 0x1p-960 && ax < 0x1p+960) || __double_as_longlong(x) == 0;
}
__device__ __forceinline__ v2d jac_div2(v2d num, v2d a, double dq, double rq)
{
   const bool ok = a.x == dq && a.y == dq && div_rcp_ok(num.x) && div_rcp_ok(num.y);
   if (dq != 0.0 && __all(ok)) return v2d{div_rcp(num.x, dq, rq), div_rcp(num.y, dq, rq)};
   return v2d{num.x / a.x, num.y / a.y};
}

__device__ __forceinline__ double jac_div1(double num, double a, double dq, double rq)
{
   const bool ok = a == dq && div_rcp_ok(num);
   if (dq != 0.0 && __all(ok)) return div_rcp(num, dq, rq);
   return num / a;
}

// Jacobi sweep epilogue (SMEM_Smooth.cpp:35-45): res = f - sum; u_new = u + w*res/a
// (dq, rq: a uniform diagonal and its reciprocal, jac_div2; dq = 0: off)
struct EpiJacobi {
   const double *f;
   const double *x;
   double *out;
   double omega;
   int nt = 0;
   double dq = 0.0, rq = 0.0;
   __device__ __forceinline__ double init(int i) const { return f[i]; }
   __device__ __forceinline__ double pf(int i) const { return x[i]; }
   __device__ __forceinline__ double finish(int i, double res, double a, double xi) const
   {
      const double q = jac_div1(omega * res, a, dq, rq);
      const double v = (a != 0.0) ? xi + q : xi;
      out[i] = v;
      return v;
   }
   __device__ __forceinline__ v2d init2(int i) const { return ld2nt(f + i, nt); }
   __device__ __forceinline__ v2d pf2(int i) const { return *reinterpret_cast<const v2du *>(x + i); }
   __device__ __forceinline__ v2d finish2(int i, v2d res, v2d a, v2d xi) const
   {
      const v2d q = jac_div2(v2d{omega * res.x, omega * res.y}, a, dq, rq);
      const v2d v{(a.x != 0.0) ? xi.x + q.x : xi.x, (a.y != 0.0) ? xi.y + q.y : xi.y};
      st2(out + i, v, nt);
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
   __device__ __forceinline__ double pf(int i) const { return x[i]; }
   __device__ __forceinline__ double finish(int i, double res, double, double xi) const
   {
      const double v = xi + res / l1[i];
      out[i] = v;
      return v;
   }
   __device__ __forceinline__ v2d init2(int i) const { return *reinterpret_cast<const v2du *>(f + i); }
   __device__ __forceinline__ v2d pf2(int i) const { return *reinterpret_cast<const v2du *>(x + i); }
   __device__ __forceinline__ v2d finish2(int i, v2d res, v2d, v2d xi) const
   {
      const v2d l = *reinterpret_cast<const v2du *>(l1 + i);
      const v2d v{xi.x + res.x / l.x, xi.y + res.y / l.y};
      *reinterpret_cast<v2du *>(out + i) = v;
      return v;
   }
};

// Outer residual r = f - A u (SMEM_Sync_Residual, SMEM_Solve.cpp:192-197) fused
// with the NEXT cycle's first level-0 Jacobi sweep, which on this same u
// computes res = f - A u in the same order (SMEM_Smooth.cpp:38-44):
// u_next = u + w*r/a_ii (L1: u + r/l1).  Writes r and u_next, returns r for
// the norm.
struct EpiResJacobi {
   const double *f;
   const double *x;
   const double *l1;
   double *r;
   double *unext;
   double omega;
   int nt = 0;
   double dq = 0.0, rq = 0.0;
   __device__ __forceinline__ double init(int i) const { return f[i]; }
   __device__ __forceinline__ double pf(int i) const { return x[i]; }
   __device__ __forceinline__ double finish(int i, double res, double a, double xi) const
   {
      if (r) r[i] = res;
      if (l1) {
         unext[i] = xi + res / l1[i];
      } else {
         const double q = jac_div1(omega * res, a, dq, rq);
         unext[i] = (a != 0.0) ? xi + q : xi;
      }
      return res;
   }
   __device__ __forceinline__ v2d init2(int i) const { return ld2nt(f + i, nt); }
   __device__ __forceinline__ v2d pf2(int i) const { return *reinterpret_cast<const v2du *>(x + i); }
   __device__ __forceinline__ v2d finish2(int i, v2d res, v2d a, v2d xi) const
   {
      if (r) st2(r + i, res, nt);
      v2d v;
      if (l1) {
         const v2d l = *reinterpret_cast<const v2du *>(l1 + i);
         v = v2d{xi.x + res.x / l.x, xi.y + res.y / l.y};
      } else {
         const v2d q = jac_div2(v2d{omega * res.x, omega * res.y}, a, dq, rq);
         v = v2d{(a.x != 0.0) ? xi.x + q.x : xi.x, (a.y != 0.0) ? xi.y + q.y : xi.y};
      }
      st2(unext + i, v, nt);
      return res;
   }
};

// ---------------------------------------------------------------------------
// Temporally fused pair of 7-pt marches (mz_sweep_outer_kernel).  A V-cycle
// ends with level 0's last post-smoothing sweep u' = u + w (f - A u) ./ a
// (csr_mz_kernel<EpiJacobi>); SMEM_Solve then forms the outer residual
// r = f - A u' with its norm, fused with the next cycle's first sweep
// u'' = u' + w r ./ a (csr_mz_kernel<EpiResJacobi>).  Here both run in ONE
// march, so u' never round-trips through HBM between them (f and u are read
// once, u' and u'' written once):
//   * a workgroup is NT = NL + 2 teams of 256 lanes; team t owns line
//     y = NL * group - 1 + t of the plane (512 positions; lane: rows 2l, 2l+1
//     as in csr_mz_kernel); teams 0 and NL + 1 carry the halo lines sweep 2
//     needs and store nothing;
//   * plane step k: every team computes u'(k) of its line exactly as
//     csr_mz_kernel<EpiJacobi> does (u of planes k-1, k, k+1 in registers, the
//     +-S lines loaded, +-1 from the neighbour lanes and one two-lane edge
//     load) and writes it to an LDS ring (2 planes); the inner teams then
//     compute sweep 2 at plane k - 1: u' of planes k-2, k-1, k of their own
//     pair from registers, the +-S and +-1 operands of plane k - 1 from the
//     ring; one barrier per plane step (the ring's RAW and WAR hazards both
//     fall on it);
//   * a chunk of ZC planes runs sweep 1 over k0-1 .. k1 (the z halo) and
//     sweep 2 over k0 .. k1-1;
//   * the next plane's operands (the +-S lines, f, the pattern byte, the edge)
//     are loaded before the barrier, so they are in flight across it.
// Every row adds its used entries in master (= CSR) order from the same
// operand values as the two separate marches, and the partials are
// csr_mz_kernel's (one per 256-row tile, the same operand order): u', u'' and
// every partial are bit-identical to the two launches.  Needs S = 512 (a team
// is one line) and NL | P / S.
// ---------------------------------------------------------------------------
constexpr int AMG_MZF_NL = 2;
constexpr int AMG_MZF_NT = AMG_MZF_NL + 2;

// PD: prefetch depth -- 1: u of plane k + 2 and the halo / f / pattern
// operands of plane k + 1 in flight during step k; 2: u of plane k + 3 and the
// operands of plane k + 2 (twice the bytes in flight per lane at one workgroup
// per CU).  dq / rq: the uniform diagonal and its reciprocal for the exact
// reciprocal division (jac_div2; dq = 0: the division itself).
template <bool STORE_U, int MINB, int PD = 1>
__global__ __launch_bounds__(256 * AMG_MZF_NT) __attribute__((amdgpu_waves_per_eu(MINB * 4))) void
mz_sweep_outer_kernel(
   const unsigned char *__restrict__ ppat, const unsigned long long *__restrict__ mmask_g, int np, MpSten Sv,
   const double *__restrict__ f, const double *__restrict__ u, double *__restrict__ u1out,
   double *__restrict__ rout, double *__restrict__ unext, double omega, int P, int nz, int zc, int npb, int xcd,
   double *__restrict__ partials, double dq, double rq)
{
   constexpr int NL = AMG_MZF_NL, NT = AMG_MZF_NT, S = 512;
   __shared__ unsigned long long mtab[256];
   __shared__ v2d ring[2][NT][256];
   __shared__ double red[AMG_MZ_MAXZC * NL * 8];
   const int tid = (int)threadIdx.x, team = tid >> 8, lt = tid & 255, lane = tid & 63;
   if (tid < np) mtab[tid] = mmask_g[tid];
   const int G = (int)gridDim.x;
   int lg = (int)blockIdx.x;
   if (xcd && (G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   const int ny = P / S;
   const int y = pblk * NL - 1 + team;
   const bool inner = team >= 1 && team <= NL;
   const int ly = y < 0 ? 0 : (y >= ny ? ny - 1 : y); // halo teams past the box: a valid line, never used
   const unsigned pos = (unsigned)(ly * S + 2 * lt);
   const unsigned Nu = (unsigned)((long long)nz * P);
   const double a0 = Sv.val[0];
   const v2d a2{a0, a0};
   auto ldp = [&](int k) { return (k >= 0 && k < nz) ? ld2u(u, (unsigned)k * P + pos) : v2d{0.0, 0.0}; };
   // u of planes k-1, k, k+1 (sweep 1 at plane k), then k + 2 (PD 2)
   v2d xm = ldp(k0 - 2), xc = ldp(k0 - 1), xq = ldp(k0), xn = PD == 2 ? ldp(k0 + 1) : v2d{0.0, 0.0};
   struct PlaneIn {
      v2d ym, yp, fv;
      double e;
      int pid;
   };
   auto fetch = [&](int k, PlaneIn &in) {
      const int kk = k < 0 ? 0 : (k >= nz ? nz - 1 : k);
      const unsigned row = (unsigned)kk * P + pos;
      in.ym = ld2u(u, row >= (unsigned)S ? row - S : 0u);
      const unsigned rp = row + (unsigned)S;
      in.yp = ld2u(u, rp + 2 <= Nu ? rp : Nu - 2);
      in.fv = ld2u(f, row);
      in.pid = ppat[row >> 1];
      in.e = 0.0;
      if (lane == 0 && row > 0) in.e = ld1u(u, row - 1);
      if (lane == 63 && row + 2 < Nu) in.e = ld1u(u, row + 2);
   };
   PlaneIn cur, nx1{};
   fetch(k0 - 1, cur);
   if (PD == 2 && k0 <= k1) fetch(k0, nx1);
   // sweep-2 state: u' of planes k-2, k-1 of the own pair; f and pattern of plane k-1
   v2d wm{0.0, 0.0}, wc{0.0, 0.0}, fm{0.0, 0.0};
   int pidm = 0;
   __syncthreads();
   for (int k = k0 - 1; k <= k1; k++) {
      const bool s1 = k >= 0 && k < nz;       // workgroup-uniform
      const v2d xnn = ldp(k + 1 + PD);        // u of plane k + 1 + PD, PD steps ahead
      // ---- sweep 1 at plane k: u' = u + w (f - A u) ./ a (EpiJacobi) ----
      v2d w1{0.0, 0.0};
      if (s1) {
         double lft = __shfl_up(xc.y, 1, 64);
         double rgt = __shfl_down(xc.x, 1, 64);
         if (lane == 0) lft = cur.e;
         if (lane == 63) rgt = cur.e;
         const unsigned long long mk = mtab[cur.pid];
         v2d xv[7];
         xv[0] = xc;
         xv[1] = xm;
         xv[2] = cur.ym;
         xv[3] = v2d{lft, xc.x};
         xv[4] = v2d{xc.y, rgt};
         xv[5] = cur.yp;
         xv[6] = xq;
         const v2d acc = mz_acc7<1, true>(cur.fv, xv, mk, Sv, nullptr);
         const v2d q = jac_div2(v2d{omega * acc.x, omega * acc.y}, a2, dq, rq);
         w1 = v2d{(a0 != 0.0) ? xc.x + q.x : xc.x, (a0 != 0.0) ? xc.y + q.y : xc.y};
         if (STORE_U && inner && y < ny && k >= k0 && k < k1)
            *reinterpret_cast<v2du *>(u1out + (size_t)((unsigned)k * P + pos)) = w1;
      }
      ring[k & 1][team][lt] = w1;
      const v2d fk = cur.fv;
      const int pidk = cur.pid;
      // the operands of plane k + PD, in flight across the barrier below
      PlaneIn nxt{};
      if (k + PD <= k1) fetch(k + PD, nxt);
      // ---- sweep 2 at plane k - 1 (inner teams): r = f - A u', u'' = u' + w r ./ a ----
      const int km = k - 1;
      if (km >= k0 && km < k1) {
         if (inner && y < ny) {
            const v2d *rg = ring[km & 1][0];
            // +-1 of the pair from the ring (line ends: clamped, masked out)
            const double *rl = reinterpret_cast<const double *>(ring[km & 1][team]);
            const double lft = rl[lt > 0 ? 2 * lt - 1 : 0];
            const double rgt = rl[lt < 255 ? 2 * lt + 2 : 511];
            const unsigned long long mk = mtab[pidm];
            v2d xv[7];
            xv[0] = wc;
            xv[1] = wm;
            xv[2] = rg[(team - 1) * 256 + lt];
            xv[3] = v2d{lft, wc.x};
            xv[4] = v2d{wc.y, rgt};
            xv[5] = rg[(team + 1) * 256 + lt];
            xv[6] = s1 ? w1 : v2d{0.0, 0.0};
            const v2d res = mz_acc7<1, true>(fm, xv, mk, Sv, nullptr);
            const unsigned row = (unsigned)km * P + pos;
            if (rout) *reinterpret_cast<v2du *>(rout + (size_t)row) = res;
            const v2d q = jac_div2(v2d{omega * res.x, omega * res.y}, a2, dq, rq);
            const v2d v{(a0 != 0.0) ? wc.x + q.x : wc.x, (a0 != 0.0) ? wc.y + q.y : wc.y};
            *reinterpret_cast<v2du *>(unext + (size_t)row) = v;
            if (partials) {
               double a = res.x * res.x, b = res.y * res.y;
#pragma unroll
               for (int off = 16; off > 0; off >>= 1) {
                  a += __shfl_down(a, off, 32);
                  b += __shfl_down(b, off, 32);
               }
               if ((lt & 31) == 0) red[((km - k0) * NL + (team - 1)) * 8 + (lt >> 5)] = a + b;
            }
         }
      }
      __syncthreads();
      wm = wc;
      wc = w1;
      fm = fk;
      pidm = pidk;
      xm = xc;
      xc = xq;
      if (PD == 2) {
         xq = xn;
         xn = xnn;
         cur = nx1;
         nx1 = nxt;
      } else {
         xq = xnn;
         cur = nxt;
      }
   }
   if (partials) {
      for (int w = tid; w < 2 * NL * (k1 - k0); w += 256 * NT) {
         const int it = w / (2 * NL), i = (w >> 1) % NL, h = w & 1;
         const int yl = pblk * NL + i;
         const double *g = red + (it * NL + i) * 8 + 4 * h;
         partials[((long long)(k0 + it) * P + (long long)yl * S) / 256 + h] = ((g[0] + g[1]) + g[2]) + g[3];
      }
   }
}

// can level 0's last post-sweep and the outer residual run as one march?
bool mz_sweep_outer_ok(const amg_mat *A)
{
   return A->mz_P && !A->mz27 && A->mp_uni && A->mz_S == 512 && A->mz_P % 512 == 0 &&
          (A->mz_P / 512) % AMG_MZF_NL == 0 && A->ppat && A->mpmask;
}

static bool fast_div_of(const amg_mat *A, double *d, double *y);

// the fused pair (see mz_sweep_outer_kernel): u1out = u' (when non-null),
// rout = r (when non-null), unext = u'', partials: the outer residual's
void mz_sweep_outer(hipStream_t s, const amg_mat *A, const double *f, const double *u, double *u1out,
                    double *rout, double *unext, double omega, double *partials)
{
   MpSten Sv;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      Sv.off[j] = A->mp_off[j];
      Sv.val[j] = A->mp_val[j];
   }
   const int P = A->mz_P, nz = A->nrows / P;
   const int npb = P / (512 * AMG_MZF_NL);
   int zc = std::max(1, std::min(A->ctx->mz_zc, AMG_MZ_MAXZC));
   if (A->ctx->mz_zc_auto) zc = (int)std::max(1LL, std::min((long long)zc, (long long)nz * npb / 1024));
   const int nch = (nz + zc - 1) / zc;
   // AMG_FUSE_OUTER_OCC=2: two workgroups per CU (<= 64 VGPRs; the compiler may spill)
   static const int occ2 = [] {
      const char *e = std::getenv("AMG_FUSE_OUTER_OCC");
      return e && std::atoi(e) == 2;
   }();
   // AMG_FUSE_OUTER_PD=2: operands two planes ahead
   static const int pd = [] {
      const char *e = std::getenv("AMG_FUSE_OUTER_PD");
      return e && std::atoi(e) == 2 ? 2 : 1;
   }();
   double dq = 0.0, rq = 0.0;
   if (!fast_div_of(A, &dq, &rq)) dq = rq = 0.0;
   auto go = [&](auto store, auto minb) {
      constexpr bool ST = decltype(store)::value;
      constexpr int MB = decltype(minb)::value;
      if (pd == 2)
         mz_sweep_outer_kernel<ST, MB, 2><<<npb * nch, 256 * AMG_MZF_NT, 0, s>>>(
            A->ppat, A->mpmask, A->pp_n, Sv, f, u, u1out, rout, unext, omega, P, nz, zc, npb, A->ctx->mz_xcd,
            partials, dq, rq);
      else
         mz_sweep_outer_kernel<ST, MB, 1><<<npb * nch, 256 * AMG_MZF_NT, 0, s>>>(
            A->ppat, A->mpmask, A->pp_n, Sv, f, u, u1out, rout, unext, omega, P, nz, zc, npb, A->ctx->mz_xcd,
            partials, dq, rq);
   };
   using T = std::true_type;
   using F = std::false_type;
   using M1 = std::integral_constant<int, 1>;
   using M2 = std::integral_constant<int, 2>;
   if (u1out) {
      if (occ2) go(T{}, M2{});
      else go(T{}, M1{});
   } else {
      if (occ2) go(F{}, M2{});
      else go(F{}, M1{});
   }
}

__device__ __forceinline__ const double *epi_pf_vec(const EpiJacobi &e) { return e.x; }
__device__ __forceinline__ const double *epi_pf_vec(const EpiL1Jacobi &e) { return e.x; }
__device__ __forceinline__ const double *epi_pf_vec(const EpiResJacobi &e) { return e.x; }

template <class Cfg>
static inline int cfg_blocks(int rb, int re)
{
   constexpr int T = 256 * Cfg::rpt;
   return (re - rb + T - 1) / T;
}

int tile_blocks(int rb, int re) { return cfg_blocks<ProdCfg>(rb, re); }

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

// 3x3 block kernel (bsr3_kernel) for num_functions = 3 operators (the DMEM
// elasticity problem, DMEM_BuildMatrix.cpp:442-719): lanes 3q, 3q+1, 3q+2 of
// a wave own the three rows of block row t (21 block rows per wave) and walk
// its blocks together -- per block one 4-byte load of the lane's three value
// indices (or its three fp64 values), the block column, and the node's three
// x values (shared by the three lanes).  Each row adds its diagonal first,
// then every other entry in ascending column order: its CSR order
// (bit-identical to the CSR kernels).  Block rows kept in CSR form (bmode 1:
// identity rows of fixed dofs) run the CSR row loop.  Per block row the
// value-indexed form streams 27 x (12 + 4) bytes against 81 x 5 for
// value-indexed CSR.
// Lane-per-block-row form (bsr3_row_kernel, ctx->bsr3 == 2, value-indexed):
// lane q of a wave owns block row t = 64 sl + q -- all three of its rows, three
// independent accumulators -- and walks its blocks: per block one 12-byte load of
// the three rows' value indices (a wave's 64 contiguous), one 4-byte block
// column (contiguous) and the node's three x values, no cross-lane shuffles.
// Each row adds its diagonal first, then its entries block by block in
// ascending column order (bsr3_kernel's order: bit-identical).
template <int NEG, bool NEED_DIAG, class Epi, int U = 4>
__global__ __launch_bounds__(256) void bsr3_row_kernel(const long long *__restrict__ soff,
                                                       const int *__restrict__ bcol, const int *__restrict__ bdiag,
                                                       const unsigned char *__restrict__ bcnt,
                                                       const unsigned int *__restrict__ bvi,
                                                       const double *__restrict__ vtab_g,
                                                       const int *__restrict__ rowptr, const int *__restrict__ col,
                                                       const double *__restrict__ val, const double *__restrict__ x,
                                                       int t0, int t1, Epi epi)
{
   __shared__ double vtab[256];
   vtab[threadIdx.x] = vtab_g[threadIdx.x];
   __syncthreads();
   const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
   const int sl = t0 / 64 + (int)blockIdx.x * 4 + wave;
   const int t = sl * 64 + lane;
   if (t < t0 || t >= t1) return;
   double acc[3], xi[3], a[3];
   auto madd = [&](double &ac, double v, double xv) { ac = NEG ? ac - v * xv : ac + v * xv; };
#pragma unroll
   for (int c = 0; c < 3; c++) {
      acc[c] = epi.init(3 * t + c);
      xi[c] = x[3 * t + c];
      a[c] = 0.0;
   }
   const int cnt = bcnt[t];
   if (cnt == 0) {
      // CSR form: each row's entries in order
#pragma unroll
      for (int c = 0; c < 3; c++) {
         const int i = 3 * t + c, b = rowptr[i], e = rowptr[i + 1];
         if (NEED_DIAG) a[c] = b < e ? val[b] : 0.0;
         for (int k = b; k < e; k++) madd(acc[c], val[k], x[col[k]]);
      }
   } else {
      const long long base = soff[sl] + lane;
      const int kd = bdiag[t];
      {
         const unsigned int *w = bvi + (base + 64LL * kd) * 3;
#pragma unroll
         for (int c = 0; c < 3; c++) {
            a[c] = vtab[(w[c] >> (8 * c)) & 0xff];
            madd(acc[c], a[c], xi[c]); // the diagonal first
         }
      }
      for (int kc = 0; kc < cnt; kc += U) {
         int jj[U];
         unsigned int wv[U][3];
#pragma unroll
         for (int u = 0; u < U; u++) {
            const long long sp = base + 64LL * min(kc + u, cnt - 1);
            jj[u] = bcol[sp];
#pragma unroll
            for (int c = 0; c < 3; c++) wv[u][c] = bvi[sp * 3 + c];
         }
         double xv[U][3];
#pragma unroll
         for (int u = 0; u < U; u++)
#pragma unroll
            for (int cc = 0; cc < 3; cc++) xv[u][cc] = x[3 * (size_t)jj[u] + cc];
#pragma unroll
         for (int u = 0; u < U; u++) {
            const int k = kc + u;
            if (k >= cnt) break;
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
               for (int cc = 0; cc < 3; cc++)
                  if (k != kd || c != cc) madd(acc[c], vtab[(wv[u][c] >> (8 * cc)) & 0xff], xv[u][cc]);
         }
      }
   }
#pragma unroll
   for (int c = 0; c < 3; c++)
      epi.finish(3 * t + c, acc[c], a[c], (pf_is_x<Epi>::value && epi_pf_vec(epi) == x) ? xi[c] : epi.pf(3 * t + c));
}

template <int NEG, bool NEED_DIAG, class Epi, bool VI, bool XS = false, int U = 9>
__global__ __launch_bounds__(256) void bsr3_kernel(const long long *__restrict__ soff, const int *__restrict__ bcol,
                                                   const int *__restrict__ bdiag,
                                                   const unsigned char *__restrict__ bcnt,
                                                   const unsigned int *__restrict__ bvi,
                                                   const double *__restrict__ bval, const double *__restrict__ vtab_g,
                                                   const int *__restrict__ rowptr, const int *__restrict__ col,
                                                   const double *__restrict__ val, const double *__restrict__ x,
                                                   int t0, int t1, Epi epi)
{
   __shared__ double vtab[VI ? 256 : 1];
   if (VI) vtab[threadIdx.x] = vtab_g[threadIdx.x];
   if (VI) __syncthreads();
   const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
   if (lane >= 63) return;
   const int sl = t0 / 21 + (int)blockIdx.x * 4 + wave, q = lane / 3, c = lane % 3;
   const int t = sl * 21 + q;
   if (t < t0 || t >= t1) return;
   const int i = 3 * t + c;
   double acc = epi.init(i);
   const double xi = x[i];
   double a = 0.0;
   auto madd = [&](double v, double xv) { acc = NEG ? acc - v * xv : acc + v * xv; };
   const int cnt = bcnt[t];
   if (cnt == 0) {
      // CSR form: the row's entries in order
      const int b = rowptr[i], e = rowptr[i + 1];
      if (NEED_DIAG) a = b < e ? val[b] : 0.0;
      for (int k = b; k < e; k++) madd(val[k], x[col[k]]);
   } else {
      const long long base = soff[sl] + q;
      auto row3 = [&](long long sp, double &v0, double &v1, double &v2) {
         if (VI) {
            const unsigned int w = bvi[sp * 3 + c];
            v0 = vtab[w & 0xff];
            v1 = vtab[(w >> 8) & 0xff];
            v2 = vtab[(w >> 16) & 0xff];
         } else {
            const double *p = bval + sp * 9 + 3 * c;
            v0 = p[0];
            v1 = p[1];
            v2 = p[2];
         }
      };
      const int kd = bdiag[t];
      double d0, d1, d2;
      row3(base + 21LL * kd, d0, d1, d2);
      a = c == 0 ? d0 : (c == 1 ? d1 : d2);
      madd(a, xi); // the diagonal first
      // blocks in chunks of U, the wave's loads of block k contiguous; every
      // load of a chunk in flight before its products are added in order
      for (int kc = 0; kc < cnt; kc += U) {
         int jj[U];
         double vv[U][3];
#pragma unroll
         for (int u = 0; u < U; u++) {
            const long long sp = base + 21LL * min(kc + u, cnt - 1);
            jj[u] = bcol[sp];
            row3(sp, vv[u][0], vv[u][1], vv[u][2]);
         }
         if (XS) {
            // XS: lane c of the triplet loads the node's component c (one
            // 8-byte load per lane and block instead of three), the other two
            // come from the triplet's lanes (ds_bpermute)
            double xl[U];
#pragma unroll
            for (int u = 0; u < U; u++) xl[u] = x[3 * (size_t)jj[u] + c];
            const int l0 = lane - c;
#pragma unroll
            for (int u = 0; u < U; u++) {
               const int k = kc + u;
               const double x0 = __shfl(xl[u], l0, 64), x1 = __shfl(xl[u], l0 + 1, 64),
                            x2 = __shfl(xl[u], l0 + 2, 64);
               if (k >= cnt) continue; // (every lane takes part in the shuffles)
               if (k != kd || c != 0) madd(vv[u][0], x0);
               if (k != kd || c != 1) madd(vv[u][1], x1);
               if (k != kd || c != 2) madd(vv[u][2], x2);
            }
            continue;
         }
#pragma unroll
         for (int u = 0; u < U; u++) {
            const int k = kc + u;
            if (k >= cnt) break;
            const double *xj = x + 3 * (size_t)jj[u];
            const double x0 = xj[0], x1 = xj[1], x2 = xj[2];
            if (k != kd || c != 0) madd(vv[u][0], x0);
            if (k != kd || c != 1) madd(vv[u][1], x1);
            if (k != kd || c != 2) madd(vv[u][2], x2);
         }
      }
   }
   epi.finish(i, acc, a, (pf_is_x<Epi>::value && epi_pf_vec(epi) == x) ? xi : epi.pf(i));
}

template <int NEG, bool NEED_DIAG, class Epi>
static void launch_bsr3(hipStream_t s, const amg_mat *A, const double *x, int rb, int re, const Epi &e)
{
   const int t0 = rb / 3, t1 = re / 3;
   if (A->bsl == 64) {
      // a lane per block row (value-indexed 64-row slices); AMG_BSR3_RU: blocks
      // per batch of in-flight loads (2, 4, 6 (default: 212 against 219 us for 4
      // at r = 6, profiles/r05/bsr3/ru/) or 8)
      static const int ru = [] {
         const char *v = std::getenv("AMG_BSR3_RU");
         return v ? std::atoi(v) : 6;
      }();
      const int nsl = (t1 - t0 + 63) / 64;
#define AMG_BR(UU)                                                                                            \
   bsr3_row_kernel<NEG, NEED_DIAG, Epi, UU><<<(nsl + 3) / 4, 256, 0, s>>>(A->soff, A->bcol, A->bdiag, A->bmode, \
                                                                          A->bvi, A->vtab, A->rowptr, A->col,    \
                                                                          A->val, x, t0, t1, e)
      if (ru == 2) AMG_BR(2);
      else if (ru == 4) AMG_BR(4);
      else if (ru == 8) AMG_BR(8);
      else AMG_BR(6);
#undef AMG_BR
      return;
   }
   const int nsl = (t1 - t0 + 20) / 21;
   const int nb = (nsl + 3) / 4;
   // ctx->bsr3_xs: the node's x shared across the block row's three lanes;
   // AMG_BSR3_U: blocks per batch of in-flight loads (2, 3, 4, 6, 9, 14 or 27)
   const bool xs = A->ctx->bsr3_xs != 0;
   static const int ub = [] {
      const char *v = std::getenv("AMG_BSR3_U");
      return v ? std::atoi(v) : 4; // 4: occupancy over loads in flight (0.425 against 0.40 at 9, r = 5)
   }();
   if (A->bsr3 == 1) {
      if (xs && ub == 3)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true, 3><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else if (xs && ub == 2)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true, 2><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else if (xs && ub == 6)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true, 6><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else if (xs && ub == 4)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true, 4><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else if (xs && ub == 27)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true, 27><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else if (xs && ub == 14)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true, 14><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else if (xs)
         bsr3_kernel<NEG, NEED_DIAG, Epi, true, true><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, A->bvi, nullptr, A->vtab, A->rowptr, A->col, A->val, x, t0, t1, e);
      else
         bsr3_kernel<NEG, NEED_DIAG, Epi, true><<<nb, 256, 0, s>>>(A->soff, A->bcol, A->bdiag, A->bmode, A->bvi,
                                                                    nullptr, A->vtab, A->rowptr, A->col, A->val, x,
                                                                    t0, t1, e);
   } else {
      if (xs)
         bsr3_kernel<NEG, NEED_DIAG, Epi, false, true><<<nb, 256, 0, s>>>(
            A->soff, A->bcol, A->bdiag, A->bmode, nullptr, A->bval, nullptr, A->rowptr, A->col, A->val, x, t0, t1, e);
      else
         bsr3_kernel<NEG, NEED_DIAG, Epi, false><<<nb, 256, 0, s>>>(A->soff, A->bcol, A->bdiag, A->bmode, nullptr,
                                                                     A->bval, nullptr, A->rowptr, A->col, A->val, x,
                                                                     t0, t1, e);
   }
}

// the block form serves row ranges that start on a slice (21 or 64 block rows)
// and end on a slice or at the last row
static inline bool use_bsr3(const amg_mat *A, int rb, int re, const double *partials)
{
   const int sr = 3 * A->bsl;
   return A->bsr3 && !partials && rb % sr == 0 && (re % sr == 0 || re == A->nrows) && A->nrows % 3 == 0;
}

void residual_fsub(hipStream_t s, const amg_mat *A, const double *x, const double *b, double *y, double *r, int n)
{
   if (n <= 0) return;
   if (A->didx && !use_bsr3(A, 0, n, nullptr)) {
      launch_dc_op<0, false>(s, A, x, 0, n, EpiFsub{b, r}, nullptr, tile_blocks(0, n));
      return;
   }
   spgemv(s, A, x, nullptr, gemv_mode(1.0, 0.0), y, 0, n, nullptr);
   vsub(s, b, y, r, 0, n);
}

void spgemv(hipStream_t s, const amg_mat *A, const double *x, const double *b, const Gemv &g,
            double *y, int rb, int re, double *partials)
{
   if (re <= rb) return;
   EpiGemv e{b, y, g.init, g.scale, g.alpha, g.temp};
   const int nb = tile_blocks(rb, re);
   if (use_bsr3(A, rb, re, partials)) {
      if (g.negacc)
         launch_bsr3<1, false>(s, A, x, rb, re, e);
      else
         launch_bsr3<0, false>(s, A, x, rb, re, e);
   } else if (A->didx) {
      if (g.negacc)
         launch_dc_op<1, false>(s, A, x, rb, re, e, partials, nb);
      else
         launch_dc_op<0, false>(s, A, x, rb, re, e, partials, nb);
   } else if (long_rows(A)) {
      if (g.negacc)
         launch_long<1, false>(s, A, x, rb, re, e, partials);
      else
         launch_long<0, false>(s, A, x, rb, re, e, partials);
   } else if (A->vidx && !partials && !g.negacc && A->nnz < 5LL * A->nrows && nb > 4096) {
      // short rows (prolongation): tiles carry little work, so 4096 persistent
      // workgroups walking the tiles beat one workgroup per tile
      csr_ptile_kernel<ShortCfg, 0, false, EpiGemv, true><<<4096, 256, 0, s>>>(
         A->rowptr, A->col, A->val, x, rb, re, e, nullptr, A->vidx, A->vtab, nb);
   } else if (A->vidx && short_rows(A)) {
      if (g.negacc)
         csr_tile_kernel<ShortCfg, 1, false, EpiGemv, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
      else
         csr_tile_kernel<ShortCfg, 0, false, EpiGemv, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
   } else if (A->vidx) {
      if (g.negacc)
         csr_tile_kernel<ProdCfg, 1, false, EpiGemv, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
      else
         csr_tile_kernel<ProdCfg, 0, false, EpiGemv, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
   } else if (g.negacc)
      csr_tile_kernel<ProdCfg, 1, false, EpiGemv>
         <<<nb, 256, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, partials);
   else
      csr_tile_kernel<ProdCfg, 0, false, EpiGemv>
         <<<nb, 256, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, partials);
}

// a marched operator's uniform diagonal d whose reciprocal divides exactly
// (div_rcp): normal, finite, 2^-40 <= |d| <= 2^40, the odd part of its significand below 2^30 (the
// distance of x / d from a rounding midpoint then dwarfs the correction's
// error); AMG_FAST_DIV=0: off
static bool fast_div_of(const amg_mat *A, double *d, double *y)
{
   static const bool on = [] {
      const char *v = std::getenv("AMG_FAST_DIV");
      return !v || std::atoi(v) != 0;
   }();
   // the uniform diagonal, or the 27-pt march's dominant pattern's (the
   // epilogue checks every wave's divisors against it)
   if (!on || !(A->mp_uni || A->diag_uni || (A->mz27 && A->mz_dom >= 0))) return false;
   const double a = A->mp_uni ? A->mp_val[0] : A->diag_uni ? A->diag_u : A->mz_domval[0];
   if (!std::isnormal(a)) return false;
   int e = 0;
   const double m = std::frexp(std::fabs(a), &e); // [0.5, 1)
   // |d| in [2^-40, 2^40]: with div_rcp_ok's |x| in [2^-960, 2^960) every
   // quotient x / d and product x * (1/d) stays normal and finite
   if (e < -39 || e > 40) return false;
   unsigned long long sig = (unsigned long long)std::ldexp(m, 53);
   while (sig && !(sig & 1)) sig >>= 1;
   if (sig >= (1ull << 30)) return false;
   *d = a;
   *y = 1.0 / a;
   return true;
}

void jacobi_sweep(hipStream_t s, const amg_mat *A, const double *f, const double *x,
                  const double *l1, double omega, double *out, int rb, int re)
{
   if (re <= rb) return;
   const int nb = tile_blocks(rb, re);
   if (use_bsr3(A, rb, re, nullptr)) {
      if (l1)
         launch_bsr3<1, false>(s, A, x, rb, re, EpiL1Jacobi{f, x, l1, out});
      else {
         EpiJacobi e{f, x, out, omega};
         fast_div_of(A, &e.dq, &e.rq);
         launch_bsr3<1, true>(s, A, x, rb, re, e);
      }
   } else if (A->didx) {
      if (l1)
         launch_dc_op<1, false>(s, A, x, rb, re, EpiL1Jacobi{f, x, l1, out}, nullptr, nb);
      else {
         EpiJacobi e{f, x, out, omega, stream_hint(A)};
         fast_div_of(A, &e.dq, &e.rq);
         launch_dc_op<1, true>(s, A, x, rb, re, e, nullptr, nb);
      }
   } else if (long_rows(A)) {
      if (l1)
         launch_long<1, false>(s, A, x, rb, re, EpiL1Jacobi{f, x, l1, out});
      else {
         EpiJacobi e{f, x, out, omega};
         fast_div_of(A, &e.dq, &e.rq);
         launch_long<1, true>(s, A, x, rb, re, e);
      }
   } else if (l1) {
      EpiL1Jacobi e{f, x, l1, out};
      if (A->vidx)
         csr_tile_kernel<ProdCfg, 1, false, EpiL1Jacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, nullptr, A->vidx, A->vtab);
      else
         csr_tile_kernel<ProdCfg, 1, false, EpiL1Jacobi>
            <<<nb, 256, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, nullptr);
   } else {
      EpiJacobi e{f, x, out, omega};
      fast_div_of(A, &e.dq, &e.rq);
      if (A->vidx && short_rows(A))
         csr_tile_kernel<ShortCfg, 1, true, EpiJacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, nullptr, A->vidx, A->vtab);
      else if (A->vidx)
         csr_tile_kernel<ProdCfg, 1, true, EpiJacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, nullptr, A->vidx, A->vtab);
      else
         csr_tile_kernel<ProdCfg, 1, true, EpiJacobi>
            <<<nb, 256, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, nullptr);
   }
}

void residual_jacobi(hipStream_t s, const amg_mat *A, const double *f, const double *x,
                     const double *l1, double omega, double *r, double *unext, int rb, int re,
                     double *partials)
{
   if (re <= rb) return;
   const int nb = tile_blocks(rb, re);
   EpiResJacobi e{f, x, l1, r, unext, omega};
   if (A->didx) e.nt = stream_hint(A);
   fast_div_of(A, &e.dq, &e.rq);
   if (use_bsr3(A, rb, re, partials)) {
      if (l1)
         launch_bsr3<1, false>(s, A, x, rb, re, e);
      else
         launch_bsr3<1, true>(s, A, x, rb, re, e);
   } else if (A->didx) {
      if (l1)
         launch_dc_op<1, false>(s, A, x, rb, re, e, partials, nb);
      else
         launch_dc_op<1, true>(s, A, x, rb, re, e, partials, nb);
   } else if (long_rows(A)) {
      if (l1)
         launch_long<1, false>(s, A, x, rb, re, e, partials);
      else
         launch_long<1, true>(s, A, x, rb, re, e, partials);
   } else if (A->vidx && short_rows(A)) {
      if (l1)
         csr_tile_kernel<ShortCfg, 1, false, EpiResJacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
      else
         csr_tile_kernel<ShortCfg, 1, true, EpiResJacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
   } else if (A->vidx) {
      if (l1)
         csr_tile_kernel<ProdCfg, 1, false, EpiResJacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
      else
         csr_tile_kernel<ProdCfg, 1, true, EpiResJacobi, true><<<nb, 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, rb, re, e, partials, A->vidx, A->vtab);
   } else if (l1)
      csr_tile_kernel<ProdCfg, 1, false, EpiResJacobi>
         <<<nb, 256, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, partials);
   else
      csr_tile_kernel<ProdCfg, 1, true, EpiResJacobi>
         <<<nb, 256, 0, s>>>(A->rowptr, A->col, A->val, x, rb, re, e, partials);
}

// ---------------------------------------------------------------------------
// tuning harness: time y = A x under several tile configurations, interleaved
// (development entry point used by tools/tune_spmv.py; not part of the C-ABI).
// Only in the development build (make dev -> lib/libamg_mi355x_dev.so with
// -DAMG_DEV_TUNE): the ablation kernels give wrong results by design and stay
// out of the product library.
// ---------------------------------------------------------------------------
#ifdef AMG_DEV_TUNE
template <class Cfg, bool VI = false>
static void launch_matvec_cfg(hipStream_t s, const amg_mat *A, const double *x, double *y)
{
   EpiGemv e{nullptr, y, 0, 0, 1.0, 0.0};
   if (VI && A->vidx)
      csr_tile_kernel<Cfg, 0, false, EpiGemv, true><<<cfg_blocks<Cfg>(0, A->nrows), 256, 0, s>>>(
         A->rowptr, A->col, A->val, x, 0, A->nrows, e, nullptr, A->vidx, A->vtab);
   else
      csr_tile_kernel<Cfg, 0, false, EpiGemv>
         <<<cfg_blocks<Cfg>(0, A->nrows), 256, 0, s>>>(A->rowptr, A->col, A->val, x, 0, A->nrows,
                                                      e, nullptr);
}

// ablations (wrong results, timing only): 1 = x gathered from a 64 KiB window
// (L1/L2 resident), 2 = no LDS round trip (lane sums its own products),
// 3 = pure stream of rowptr/col/val (no x, no LDS)
template <int ABL>
__global__ __launch_bounds__(256) void ablation_kernel(const int *__restrict__ rowptr,
                                                        const int *__restrict__ col,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x, int n,
                                                        double *__restrict__ y)
{
   __shared__ __attribute__((aligned(16))) double prod[2048];
   const int r0 = blockIdx.x * 256;
   const int r1 = min(r0 + 256, n);
   const int row = r0 + (int)threadIdx.x;
   const int tb = rowptr[r0], te = rowptr[r1];
   int rs = 0, rend = 0;
   if (row < r1) {
      rs = rowptr[row];
      rend = rowptr[row + 1];
   }
   double acc = 0.0;
   const int base = tb & ~3;
   for (int k = base + 4 * (int)threadIdx.x; k < te; k += 1024) {
      v4i c4 = *reinterpret_cast<const v4i *>(col + k);
      v2d v01 = *reinterpret_cast<const v2d *>(val + k);
      v2d v23 = *reinterpret_cast<const v2d *>(val + k + 2);
      double x0, x1, x2, x3;
      if (ABL == 1) {
         x0 = x[c4.x & 8191];
         x1 = x[c4.y & 8191];
         x2 = x[c4.z & 8191];
         x3 = x[c4.w & 8191];
      } else if (ABL == 3) {
         x0 = (double)c4.x;
         x1 = (double)c4.y;
         x2 = (double)c4.z;
         x3 = (double)c4.w;
      } else {
         x0 = x[c4.x];
         x1 = x[c4.y];
         x2 = x[c4.z];
         x3 = x[c4.w];
      }
      const double p0 = v01.x * x0, p1 = v01.y * x1, p2 = v23.x * x2, p3 = v23.y * x3;
      if (ABL == 1) {
         v2d *dst = reinterpret_cast<v2d *>(prod + (k - base));
         dst[0] = v2d{p0, p1};
         dst[1] = v2d{p2, p3};
      } else {
         acc += (p0 + p1) + (p2 + p3);
      }
   }
   if (ABL == 1) {
      __syncthreads();
      for (int k = rs; k < rend; ++k) acc += prod[k - base];
   }
   if (row < r1) y[row] = acc;
}

// tools/tune_spmv.py mp_* variants: y = A x (GEMV), r = x - A x (RES) or a
// Jacobi sweep (JAC, f = x) through csr_mp_kernel forms
template <int FORM, int RPL, int OP, int NT = 0>
static void launch_mp_tune(hipStream_t s, const amg_mat *A, const double *x, double *y)
{
   if (!A->mp_J || !A->mp_uni || A->mp_J > 8) return;
   MpSten S;
   for (int j = 0; j < AMG_MP_MAXJ; j++) {
      S.off[j] = A->mp_off[j];
      S.val[j] = A->mp_val[j];
   }
   const int nb = (A->nrows + 512 * RPL - 1) / (512 * RPL);
   const v2d *mv = reinterpret_cast<const v2d *>(A->mpval);
   if (OP == 2) {
      EpiJacobi e{x, x, y, 0.8, NT};
      csr_mp_kernel<1, true, EpiJacobi, 8, true, FORM, RPL><<<nb, 256, 0, s>>>(
         A->ppat, A->mpmask, A->pp_n, mv, A->mp_J, S, x, A->ncols, 0, A->nrows, e, nullptr);
   } else {
      EpiGemv e{x, y, OP == 1 ? 1 : 0, 0, 1.0, 0.0, NT};
      csr_mp_kernel<OP == 1 ? 1 : 0, false, EpiGemv, 8, true, FORM, RPL><<<nb, 256, 0, s>>>(
         A->ppat, A->mpmask, A->pp_n, mv, A->mp_J, S, x, A->ncols, 0, A->nrows, e, nullptr);
   }
}

int num_tune_variants() { return 71; }

template <int RPL, bool STAGE, int MAXR = AMG_DC_MAXROW>
static void launch_dc(hipStream_t s, const amg_mat *A, const double *x, double *y)
{
   EpiGemv e{nullptr, y, 0, 0, 1.0, 0.0};
   if (!A->didx || A->dc_maxrow > MAXR) return;
   const int nt = (A->nrows + 256 * RPL - 1) / (256 * RPL);
   csr_dc_kernel<0, false, EpiGemv, RPL, STAGE, MAXR><<<nt, 256, 0, s>>>(
      A->rowptr, A->didx, A->doff, A->dval, x, 0, A->nrows, e, nullptr, A->dc_n, A->danch);
}



template <int RPL>
static void launch_rp(hipStream_t s, const amg_mat *A, const double *x, double *y)
{
   EpiGemv e{nullptr, y, 0, 0, 1.0, 0.0};
   if (!A->rpat) return;
   const int nt = (A->nrows + 256 * RPL - 1) / (256 * RPL);
   csr_rp_kernel<0, false, EpiGemv, RPL><<<nt, 256, 0, s>>>(A->rpat, A->ptab, A->rp_n, A->doff, A->dval, x,
                                                            0, A->nrows, e, nullptr, A->dc_n, A->danch);
}

template <int RPL>
static void launch_rpp(hipStream_t s, const amg_mat *A, const double *x, double *y)
{
   EpiGemv e{nullptr, y, 0, 0, 1.0, 0.0};
   if (!A->ppat) return;
   const int nt = (A->nrows + 512 * RPL - 1) / (512 * RPL);
   csr_rpp_kernel<0, false, EpiGemv, RPL><<<nt, 256, A->pp_n * A->pp_stride * 4, s>>>(
      A->ppat, A->pptab, A->pp_n, A->doff, A->dval, x, 0, A->nrows, e, nullptr, A->dc_n, A->pp_stride, A->danch,
      A->pp_centre0, A->pbase, A->pdelta);
}

// Jacobi sweep y = x + w (x - A x)/a_ii through the paired kernel, OPT as
// csr_rpp_kernel (timing of the epilogue forms; f = x)
template <int OPT>
static void launch_rpp_jac(hipStream_t s, const amg_mat *A, const double *x, double *y)
{
   EpiJacobi e{x, x, y, 0.8};
   if (!A->ppat || A->nrows != A->ncols) return;
   const int nt = (A->nrows + 1023) / 1024;
   csr_rpp_kernel<1, true, EpiJacobi, 2, OPT><<<nt, 256, A->pp_n * A->pp_stride * 4, s>>>(
      A->ppat, A->pptab, A->pp_n, A->doff, A->dval, x, 0, A->nrows, e, nullptr, A->dc_n, A->pp_stride, A->danch,
      A->pp_centre0, A->pbase, A->pdelta);
}

// ablations of the row-pattern kernel on the 512^3 operator (timing only):
// MODE 1: offsets forced to 0 (same table work, x read once per row);
// MODE 2: matrix-free 7-pt stencil with offsets in registers (no tables);
// MODE 3: MODE 2 with interior rows only (no bounds tests)
template <int MODE, int RPL>
__global__ __launch_bounds__(256) void abl_rp_k(const unsigned char *__restrict__ rpat,
                                                const unsigned char *__restrict__ ptab_g, int np,
                                                const int *__restrict__ doff_g, const double *__restrict__ dval_g,
                                                const double *__restrict__ x, int n, double *__restrict__ y)
{
   constexpr int PS = AMG_RP_STRIDE;
   __shared__ int otab[256];
   __shared__ double vtab[256];
   __shared__ __attribute__((aligned(16))) unsigned char ptab[256 * PS];
   const int tid = (int)threadIdx.x;
   const int r0 = blockIdx.x * 256 * RPL;
   if (MODE == 1) {
      if (tid < 256) {
         otab[tid] = doff_g[tid];
         vtab[tid] = dval_g[tid];
      }
      const int nw = (np * PS) >> 2;
      for (int w = tid; w < nw; w += 256)
         reinterpret_cast<unsigned int *>(ptab)[w] = reinterpret_cast<const unsigned int *>(ptab_g)[w];
      __syncthreads();
   }
#pragma unroll
   for (int q = 0; q < RPL; q++) {
      const int row = r0 + q * 256 + tid;
      if (row >= n) continue;
      double acc = 0.0;
      if (MODE == 1) {
         const unsigned char *pp = ptab + rpat[row] * PS;
         const int len = pp[0];
         for (int j = 0; j < len; j++) {
            const int bb = pp[1 + j];
            acc += vtab[bb] * x[row + 0 * otab[bb]];
         }
      } else {
         const int off[7] = {0, -262144, -512, -1, 1, 512, 262144};
#pragma unroll
         for (int j = 0; j < 7; j++) {
            if (MODE == 4 && (j == 1 || j == 6)) continue; // no +-n^2
            if (MODE == 5 && (j == 2 || j == 5)) continue; // no +-n
            const int c = row + off[j];
            if (MODE >= 3 || (c >= 0 && c < n)) acc += (j == 0 ? 6.0 : -1.0) * x[MODE >= 3 ? min(max(c, 0), n - 1) : c];
         }
      }
      y[row] = acc;
   }
}

// copy ablations with the row-pattern kernel's lane -> row mapping
template <int MODE>
__global__ __launch_bounds__(256) void abl_copy_k(const double *__restrict__ x, int n, double *__restrict__ y)
{
   const int r0 = blockIdx.x * 1024;
#pragma unroll
   for (int q = 0; q < 4; q++) {
      const int row = r0 + q * 256 + (int)threadIdx.x;
      if (row >= n) continue;
      if (MODE == 0) y[row] = x[row];
      else y[row] = x[row] + x[min(row + 1, n - 1)] + x[max(row - 1, 0)];
   }
}

// paired-row ablations: lane owns V consecutive rows and reads each x offset
// with V/2 16-byte loads (8-byte aligned for odd offsets)
template <int MODE, int V>
__global__ __launch_bounds__(256) void abl_pair_k(const double *__restrict__ x, int n, double *__restrict__ y)
{
   const int r0 = blockIdx.x * 1024;
#pragma unroll
   for (int q = 0; q < 4 / V; q++) {
      const int row = r0 + (q * 256 + (int)threadIdx.x) * V;
      if (row >= n) continue;
      v2d acc[V / 2];
#pragma unroll
      for (int h = 0; h < V / 2; h++) acc[h] = v2d{0.0, 0.0};
      if (MODE == 0) {
#pragma unroll
         for (int h = 0; h < V / 2; h++) acc[h] = *reinterpret_cast<const v2d *>(x + row + 2 * h);
      } else {
         const int off[7] = {0, -262144, -512, -1, 1, 512, 262144};
#pragma unroll
         for (int j = 0; j < 7; j++) {
            const int c = min(max(row + off[j], 0), n - V);
#pragma unroll
            for (int h = 0; h < V / 2; h++) {
               const v2d xv = *reinterpret_cast<const v2du *>(x + c + 2 * h);
               const double w = j == 0 ? 6.0 : -1.0;
               acc[h].x += w * xv.x;
               acc[h].y += w * xv.y;
            }
         }
      }
#pragma unroll
      for (int h = 0; h < V / 2; h++) *reinterpret_cast<v2d *>(y + row + 2 * h) = acc[h];
   }
}

const char *tune_variant_name(int v)
{
   static const char *names[] = {"plain_base",   "vi_base",         "vi_strided",
                                 "vi_unr_skip_shfl", "vi_rpt2_ch4096", "vi_xcd",
                                 "vi_nt",        "vi_ch1024",       "plain_strided",
                                 "ABL_localgather", "ABL_noLDS",    "ABL_streamonly",
                                 "vi_gtab",      "vi_persist2048",  "vi_persist4096",
                                 "vi_w8",        "plain_w8",        "vi_w8_nt",     "vi_w8_ch4096",
                                 "dc_rpl1",      "dc_rpl2_m8",      "dc_rpl2",      "dc_rpl4_m8",
                                 "dc_rpl8_m8",   "rp_rpl1",         "rp_rpl2",      "rp_rpl4",
                                 "rp_rpl8",      "ABL_rp_off0",     "ABL_stencil",  "ABL_stencil_clamp",
                                 "ABL_st_nonn",  "ABL_st_non",      "ABL_copy",     "ABL_copy3",
                                 "long_t64_r64",  "long_t256_r8",   "long_t256_r16", "long_t256_r32",
                                 "long_t256_r64", "long_t128_r16", "long_t256_r256",
                                 "ABL_copy_v2", "ABL_pair_st_v2", "ABL_copy_v4", "ABL_pair_st_v4",
                                 "rpp_rpl1", "rpp_rpl2", "rpp_rpl4",
                                 "ABL_jac_o0", "ABL_jac_o1", "ABL_jac_o2", "ABL_jac_o3",
                                 "mp_bf_rpl2", "mp_br_rpl2", "mp_bf_rpl1", "mp_bf_rpl4",
                                 "ABL_mp_bf_res", "ABL_mp_br_res", "ABL_mp_bf_jac", "ABL_mp_br_jac",
                                 "mp_f2_rpl2", "ABL_mp_f2_res", "ABL_mp_br_res_nt", "ABL_mp_br_jac_nt",
                                 "ABL_mp_f2_res_nt", "ABL_mp_f2_jac", "mp_f3_rpl2", "ABL_mp_f3_res", "ABL_mp_f3_jac",
                                 "mp_f3_rpl4"};
   return (v >= 0 && v < 71) ? names[v] : "?";
}

void launch_tune_variant(hipStream_t s, int v, const amg_mat *A, const double *x, double *y)
{
   switch (v) {
   case 0: launch_matvec_cfg<TileCfg<1, 2048, false, false>>(s, A, x, y); break;
   case 1: launch_matvec_cfg<TileCfg<1, 2048, false, false>, true>(s, A, x, y); break;
   case 2: launch_matvec_cfg<TileCfg<1, 2048, false, false, false, false, false, true>, true>(s, A, x, y); break;
   case 3: launch_matvec_cfg<TileCfg<1, 2048, false, false, true, true, true>, true>(s, A, x, y); break;
   case 4: launch_matvec_cfg<TileCfg<2, 4096, false, false>, true>(s, A, x, y); break;
   case 5: launch_matvec_cfg<TileCfg<1, 2048, false, true>, true>(s, A, x, y); break;
   case 6: launch_matvec_cfg<TileCfg<1, 2048, true, false>, true>(s, A, x, y); break;
   case 7: launch_matvec_cfg<TileCfg<1, 1024, false, false>, true>(s, A, x, y); break;
   case 8: launch_matvec_cfg<TileCfg<1, 2048, false, false, false, false, false, true>>(s, A, x, y); break;
   case 9:
      ablation_kernel<1><<<(A->nrows + 255) / 256, 256, 0, s>>>(A->rowptr, A->col, A->val, x,
                                                               A->nrows, y);
      break;
   case 10:
      ablation_kernel<2><<<(A->nrows + 255) / 256, 256, 0, s>>>(A->rowptr, A->col, A->val, x,
                                                               A->nrows, y);
      break;
   case 11:
      ablation_kernel<3><<<(A->nrows + 255) / 256, 256, 0, s>>>(A->rowptr, A->col, A->val, x,
                                                                A->nrows, y);
      break;
   case 12: {
      EpiGemv e{nullptr, y, 0, 0, 1.0, 0.0};
      if (A->vidx)
         csr_tile_kernel<ProdCfg, 0, false, EpiGemv, true, true><<<cfg_blocks<ProdCfg>(0, A->nrows), 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, 0, A->nrows, e, nullptr, A->vidx, A->vtab);
      break;
   }
   case 13:
   case 14: {
      EpiGemv e{nullptr, y, 0, 0, 1.0, 0.0};
      const int nt = cfg_blocks<ProdCfg>(0, A->nrows);
      if (A->vidx)
         csr_ptile_kernel<ProdCfg, 0, false, EpiGemv, true><<<std::min(nt, v == 13 ? 2048 : 4096), 256, 0, s>>>(
            A->rowptr, A->col, A->val, x, 0, A->nrows, e, nullptr, A->vidx, A->vtab, nt);
      break;
   }
   case 15: launch_matvec_cfg<TileCfg<1, 2048, false, false, false, false, false, false, true>, true>(s, A, x, y); break;
   case 16: launch_matvec_cfg<TileCfg<1, 2048, false, false, false, false, false, false, true>>(s, A, x, y); break;
   case 17: launch_matvec_cfg<TileCfg<1, 2048, true, false, false, false, false, false, true>, true>(s, A, x, y); break;
   case 18: launch_matvec_cfg<TileCfg<1, 4096, false, false, false, false, false, false, true>, true>(s, A, x, y); break;
   case 19: launch_dc<1, true>(s, A, x, y); break;
   case 20: launch_dc<2, true, 8>(s, A, x, y); break;
   case 21: launch_dc<2, true>(s, A, x, y); break;
   case 22: launch_dc<4, true, 8>(s, A, x, y); break;
   case 23: launch_dc<8, true, 8>(s, A, x, y); break;
   case 24: launch_rp<1>(s, A, x, y); break;
   case 25: launch_rp<2>(s, A, x, y); break;
   case 26: launch_rp<4>(s, A, x, y); break;
   case 27: launch_rp<8>(s, A, x, y); break;
   case 28:
   case 29:
   case 30:
   case 31:
   case 32: {
      if (!A->rpat) break;
      const int nt = (A->nrows + 1023) / 1024;
      const unsigned char *rp = A->rpat, *pt = A->ptab;
      const int np = A->rp_n, n = A->nrows;
      if (v == 28) abl_rp_k<1, 4><<<nt, 256, 0, s>>>(rp, pt, np, A->doff, A->dval, x, n, y);
      if (v == 29) abl_rp_k<2, 4><<<nt, 256, 0, s>>>(rp, pt, np, A->doff, A->dval, x, n, y);
      if (v == 30) abl_rp_k<3, 4><<<nt, 256, 0, s>>>(rp, pt, np, A->doff, A->dval, x, n, y);
      if (v == 31) abl_rp_k<4, 4><<<nt, 256, 0, s>>>(rp, pt, np, A->doff, A->dval, x, n, y);
      if (v == 32) abl_rp_k<5, 4><<<nt, 256, 0, s>>>(rp, pt, np, A->doff, A->dval, x, n, y);
      break;
   }
   case 33: abl_copy_k<0><<<(A->nrows + 1023) / 1024, 256, 0, s>>>(x, A->nrows, y); break;
   case 34: abl_copy_k<2><<<(A->nrows + 1023) / 1024, 256, 0, s>>>(x, A->nrows, y); break;
   case 35: launch_long_cfg<0, false, 64, 64>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 36: launch_long_cfg<0, false, 256, 8>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 37: launch_long_cfg<0, false, 256, 16>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 38: launch_long_cfg<0, false, 256, 32>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 39: launch_long_cfg<0, false, 256, 64>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 40: launch_long_cfg<0, false, 128, 16>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 41: launch_long_cfg<0, false, 256, 256>(s, A, x, 0, A->nrows, EpiGemv{nullptr, y, 0, 0, 1.0, 0.0}); break;
   case 42: abl_pair_k<0, 2><<<(A->nrows + 1023) / 1024, 256, 0, s>>>(x, A->nrows, y); break;
   case 43: abl_pair_k<1, 2><<<(A->nrows + 1023) / 1024, 256, 0, s>>>(x, A->nrows, y); break;
   case 44: abl_pair_k<0, 4><<<(A->nrows + 1023) / 1024, 256, 0, s>>>(x, A->nrows, y); break;
   case 45: abl_pair_k<1, 4><<<(A->nrows + 1023) / 1024, 256, 0, s>>>(x, A->nrows, y); break;
   case 46: launch_rpp<1>(s, A, x, y); break;
   case 47: launch_rpp<2>(s, A, x, y); break;
   case 48: launch_rpp<4>(s, A, x, y); break;
   case 49: launch_rpp_jac<0>(s, A, x, y); break;
   case 50: launch_rpp_jac<1>(s, A, x, y); break;
   case 51: launch_rpp_jac<2>(s, A, x, y); break;
   case 52: launch_rpp_jac<3>(s, A, x, y); break;
   case 53: launch_mp_tune<0, 2, 0>(s, A, x, y); break;
   case 54: launch_mp_tune<1, 2, 0>(s, A, x, y); break;
   case 55: launch_mp_tune<0, 1, 0>(s, A, x, y); break;
   case 56: launch_mp_tune<0, 4, 0>(s, A, x, y); break;
   case 57: launch_mp_tune<0, 2, 1>(s, A, x, y); break;
   case 58: launch_mp_tune<1, 2, 1>(s, A, x, y); break;
   case 59: launch_mp_tune<0, 2, 2>(s, A, x, y); break;
   case 60: launch_mp_tune<1, 2, 2>(s, A, x, y); break;
   case 61: launch_mp_tune<2, 2, 0>(s, A, x, y); break;
   case 62: launch_mp_tune<2, 2, 1>(s, A, x, y); break;
   case 63: launch_mp_tune<1, 2, 1, 1>(s, A, x, y); break;
   case 64: launch_mp_tune<1, 2, 2, 1>(s, A, x, y); break;
   case 65: launch_mp_tune<2, 2, 1, 1>(s, A, x, y); break;
   case 66: launch_mp_tune<2, 2, 2>(s, A, x, y); break;
   case 67: launch_mp_tune<3, 2, 0>(s, A, x, y); break;
   case 68: launch_mp_tune<3, 2, 1>(s, A, x, y); break;
   case 69: launch_mp_tune<3, 2, 2>(s, A, x, y); break;
   case 70: launch_mp_tune<3, 4, 0>(s, A, x, y); break;
   default: break;
   }
}
#endif // AMG_DEV_TUNE

// ---------------------------------------------------------------------------
// PMC calibration streams (tools/pmc_traffic.py): known byte counts read or
// written with one access width per lane, to calibrate rocprofv3 FETCH_SIZE /
// WRITE_SIZE per access width on gfx950 (MI355X_MICROARCH.md, HBM section)
// ---------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void calib_read_k(const unsigned char *__restrict__ buf,
                                                   long long bytes, double *__restrict__ out)
{
   const long long n = bytes / W;
   const long long stride = (long long)gridDim.x * blockDim.x;
   double acc = 0.0;
   for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
      if (W == 16) {
         const v2d v = reinterpret_cast<const v2d *>(buf)[i];
         acc += v.x + v.y;
      } else if (W == 8) {
         acc += reinterpret_cast<const double *>(buf)[i];
      } else if (W == 4) {
         acc += (double)reinterpret_cast<const int *>(buf)[i];
      } else {
         acc += (double)buf[i];
      }
   }
   if (acc == 12345.678) out[0] = acc; // keep the loads
}

__global__ __launch_bounds__(256) void calib_write8_k(double *__restrict__ buf, long long n)
{
   const long long stride = (long long)gridDim.x * blockDim.x;
   for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
      buf[i] = (double)i;
}

// STREAM triad a = b + q c on 16-byte lanes, one double2 per thread (the
// practical HBM ceiling bench.py reports beside the 8 TB/s peak)
__global__ __launch_bounds__(256) void triad_k(v2d *__restrict__ a, const v2d *__restrict__ b,
                                               const v2d *__restrict__ c, double q, long long n2)
{
   const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
   if (i < n2) {
      const v2d x = b[i], y = c[i];
      v2d r;
      r.x = x.x + q * y.x;
      r.y = x.y + q * y.y;
      a[i] = r;
   }
}
void stream_triad(hipStream_t s, double *a, const double *b, const double *c, double q, long long n)
{
   const long long n2 = n / 2;
   const long long nb = (n2 + 255) / 256;
   if (nb > 0)
      triad_k<<<(unsigned)nb, 256, 0, s>>>(reinterpret_cast<v2d *>(a), reinterpret_cast<const v2d *>(b),
                                          reinterpret_cast<const v2d *>(c), q, n2);
}

void calib_stream(hipStream_t s, int mode, void *buf, long long bytes, double *out)
{
   const int nb = 8192;
   switch (mode) {
   case 0: calib_read_k<16><<<nb, 256, 0, s>>>((const unsigned char *)buf, bytes, out); break;
   case 1: calib_read_k<8><<<nb, 256, 0, s>>>((const unsigned char *)buf, bytes, out); break;
   case 2: calib_read_k<4><<<nb, 256, 0, s>>>((const unsigned char *)buf, bytes, out); break;
   case 3: calib_read_k<1><<<nb, 256, 0, s>>>((const unsigned char *)buf, bytes, out); break;
   case 4: calib_write8_k<<<nb, 256, 0, s>>>((double *)buf, bytes / 8); break;
   default: break;
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
// Injected delay (SMEM_Solve.cpp:137-145 usleep, DMEM_DelayProc
// DMEM_Misc.cpp:668-684) as a wait on the stream: one lane polls the device
// wall clock (bounded: every launch ends after `ticks`)
__global__ void delay_k(unsigned long long ticks)
{
   if (threadIdx.x != 0) return;
   const unsigned long long t0 = wall_clock64();
   while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

void delay(hipStream_t s, double usec, int wall_khz)
{
   if (!(usec > 0.0)) return;
   usec = std::min(usec, 1e7); // at most 10 s per delay
   delay_k<<<1, 64, 0, s>>>((unsigned long long)(usec * 1e-3 * wall_khz));
}

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
   // In-block operands (SMEM_Smooth.cpp:253-263, 290-300): a column the lane
   // has NOT updated yet this sweep holds its old value, which is u_prev's
   // copy (0 in the zero-guess sweep); the row updated just before (the
   // stencil's -1 / +1 neighbour) comes from a register; only older updated
   // rows are re-read from u, as relaxed agent-scope atomics (gfx950 stores
   // write through to L2 without refreshing the CU's L1).  Every operand is
   // the value the reference's sequential loop reads, so results are
   // bit-identical, and the row's loads no longer wait on the previous row.
   auto ld = [u](int k) { return __hip_atomic_load(u + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
   auto st = [u](int k, double v) {
      __hip_atomic_store(u + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   };
   const int b = blockIdx.x * blockDim.x + threadIdx.x;
   if (b >= nblk) return;
   const int ns = blk[b], ne = blk[b + 1];
   int last_i = -1;
   double last = 0.0;
   for (int c = 0; c < ne - ns; c++) {
      const int i = reverse ? ne - 1 - c : ns + c;
      const int rs = rowptr[i], rend = rowptr[i + 1];
      const double a = val[rs];
      const double old = zero ? 0.0 : u_prev[i];
      double v = old;
      if (a != 0.0) {
         const double d = ds ? ds[i] : a;
         double res = f[i];
         for (int jj = rs; jj < rend; jj++) {
            const int ii = col[jj];
            if (ii >= ns && ii < ne) {
               const bool done = reverse ? ii > i : ii < i;
               const double x = !done ? (zero ? 0.0 : u_prev[ii]) : (ii == last_i ? last : ld(ii));
               res -= val[jj] * x;
            } else if (!zero) {
               res -= val[jj] * u_prev[ii];
            }
         }
         v = zero ? weight * res / d : old + weight * res / d;
      }
      // a_ii == 0: the row keeps its value (0 after the zero-guess reset)
      if (a != 0.0 || zero) st(i, v);
      last_i = i;
      last = v;
   }
}

// asynchronous Gauss-Seidel (SMEM_Async_Parfor_GaussSeidel[T] SMEM_Smooth.cpp:164-220,
// SMEM_Async_GaussSeidel[T] :475-531; semi-async: one sweep per launch,
// SMEM_SemiAsync_* :135-162 / :445-473): one lane per block of rows, rows in
// order (reverse: backwards), every u access a relaxed agent-scope atomic,
// other blocks' rows read live -- the reference's racy in-place update.
// No zero-guess special case and no weight (u_i += res / a_ii), as the
// reference.  Blocks never wait for one another within a launch.
__global__ void async_gs_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                           const double *__restrict__ val, const double *__restrict__ f, double *u,
                           const int *__restrict__ blk, int nblk, int sweeps, int reverse)
{
   auto ld = [u](int k) { return __hip_atomic_load(u + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
   const int b = blockIdx.x * blockDim.x + threadIdx.x;
   if (b >= nblk) return;
   const int ns = blk[b], ne = blk[b + 1];
   for (int k = 0; k < sweeps; k++)
      for (int c = 0; c < ne - ns; c++) {
         const int i = reverse ? ne - 1 - c : ns + c;
         const int rs = rowptr[i], rend = rowptr[i + 1];
         const double a = val[rs];
         if (a == 0.0) continue;
         double res = f[i];
         for (int jj = rs; jj < rend; jj++) res -= val[jj] * ld(col[jj]);
         __hip_atomic_store(u + i, ld(i) + res / a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
}

void async_gs(hipStream_t s, const amg_mat *A, const double *f, double *u, const int *d_blk, int nblk,
              int sweeps, int semi, int reverse)
{
   if (nblk <= 0 || sweeps <= 0) return;
   const int tpb = 64, nb = (nblk + tpb - 1) / tpb;
   if (semi)
      for (int k = 0; k < sweeps; k++)
         async_gs_k<<<nb, tpb, 0, s>>>(A->rowptr, A->col, A->val, f, u, d_blk, nblk, 1, reverse);
   else
      async_gs_k<<<nb, tpb, 0, s>>>(A->rowptr, A->col, A->val, f, u, d_blk, nblk, sweeps, reverse);
}

// Hybrid Jacobi / Gauss-Seidel, one WAVE per block (SMEM_Smooth.cpp:265-304 /
// 548-585; the reference's thread-range block, here any block): the block's
// rows in chunks of 64, lane l owning the chunk's l-th row in sweep order.
// Every row's sum is res = f_i - sum a_ij x_j over its entries in CSR order,
// with x_j the operand the reference's sequential loop reads:
//   * a column outside the block: u_prev (skipped in the zero-guess sweep);
//   * an in-block column not updated yet this sweep: its old value u_prev
//     (0 in the zero-guess sweep);
//   * an in-block column updated in an EARLIER chunk: its new value (loaded,
//     agent-scope, after the chunk fence);
//   * an in-block column updated earlier in THIS chunk: a dependency.
// Phase 1 (all lanes at once, coalesced loads): each lane forms its rounded
// products and sums the prefix up to its first dependency.  Phase 2 (the
// chain): step s = 0 .. 63, lane s adds its tail -- the dependent products
// with the values broadcast (v_readlane) at the earlier steps, the other
// tail products as precomputed -- in CSR order, divides, and its new value is
// broadcast to every lane that depends on it.  The operations and their
// order are the sequential loop's: bit-identical.  Rows of at most RMAX
// entries (longer rows: hybrid_jgs_k).
// rows of older chunks were stored by THIS wave with write-through (sc1,
// agent-scope relaxed) stores and are re-read with L1-bypassing (sc1) loads:
// only the stores' completion is needed -- no cache write-back / invalidate
// (an agent-scope fence costs several microseconds per chunk)
__device__ __forceinline__ void wait_own_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double readlane_d(double v, int s)
{
   const unsigned long long b = (unsigned long long)__double_as_longlong(v);
   const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, s);
   const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), s);
   return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <int RMAX>
__global__ __launch_bounds__(256) void hybrid_jgs_wave_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                         const double *__restrict__ val, const double *__restrict__ f,
                                                         double *u, const double *__restrict__ u_prev,
                                                         const int *__restrict__ blk, int nblk,
                                                         const double *__restrict__ ds, double weight, int zero,
                                                         int reverse)
{
   const int lane = (int)threadIdx.x & 63;
   const int b = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
   if (b >= nblk) return; // whole waves
   const int ns = blk[b], ne = blk[b + 1];
   const int nb = ne - ns;
   for (int c0 = 0; c0 < nb; c0 += 64) {
      const int cnt = min(64, nb - c0);
      const bool act = lane < cnt;
      const int i = reverse ? ne - 1 - (c0 + lane) : ns + c0 + lane;
      double res = 0.0, a = 0.0, d = 1.0, old = 0.0;
      double pa[RMAX], xd[RMAX];
      int dl[RMAX];
      int len = 0, fd = RMAX;
#pragma unroll
      for (int k = 0; k < RMAX; k++) {
         pa[k] = 0.0;
         xd[k] = 0.0;
         dl[k] = -2;
      }
      if (act) {
         const int rs = rowptr[i];
         len = rowptr[i + 1] - rs;
         a = val[rs];
         d = ds ? ds[i] : a;
         old = zero ? 0.0 : u_prev[i];
         res = f[i];
         int jj[RMAX];
         double vv[RMAX], xx[RMAX];
#pragma unroll
         for (int k = 0; k < RMAX; k++) {
            jj[k] = 0;
            vv[k] = 0.0;
            if (k < len) {
               jj[k] = col[rs + k];
               vv[k] = val[rs + k];
            }
         }
         // operands (dl: -1 independent product, -2 nothing, >= 0 dependency lane)
#pragma unroll
         for (int k = 0; k < RMAX; k++) {
            xx[k] = 0.0;
            if (k >= len) continue;
            const int j = jj[k];
            if (j >= ns && j < ne) {
               const bool done = reverse ? j > i : j < i;
               if (!done) {
                  xx[k] = zero ? 0.0 : u_prev[j];
                  dl[k] = -1;
               } else {
                  const int pos = reverse ? ne - 1 - j : j - ns; // position in sweep order
                  if (pos >= c0) {
                     dl[k] = pos - c0;
                  } else {
                     xx[k] = __hip_atomic_load(u + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                     dl[k] = -1;
                  }
               }
            } else if (!zero) {
               xx[k] = u_prev[j];
               dl[k] = -1;
            }
         }
#pragma unroll
         for (int k = 0; k < RMAX; k++) {
            if (k >= len) break;
            if (dl[k] >= 0 && fd == RMAX) fd = k;
            if (dl[k] == -1) pa[k] = vv[k] * xx[k];
            else if (dl[k] >= 0) pa[k] = vv[k];
            if (fd == RMAX && dl[k] == -1) res = res - pa[k];
         }
      }
      auto finish = [&](double r) { return (a != 0.0) ? (zero ? weight * r / d : old + weight * r / d) : old; };
      double v = old;
      if (act && fd == RMAX) v = finish(res);
      for (int st = 0; st < cnt; st++) {
         if (lane == st && fd < RMAX) {
            double r = res;
#pragma unroll
            for (int k = 0; k < RMAX; k++) {
               if (k < fd || k >= len || dl[k] == -2) continue;
               r = r - (dl[k] >= 0 ? pa[k] * xd[k] : pa[k]);
            }
            v = finish(r);
         }
         const double vs = readlane_d(v, st);
#pragma unroll
         for (int k = 0; k < RMAX; k++)
            if (dl[k] == st) xd[k] = vs;
      }
      // a_ii == 0: the row keeps its value (0 after the zero-guess reset)
      if (act && (a != 0.0 || zero)) __hip_atomic_store(u + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the next chunk's loads of these rows see the stores
      if (c0 + 64 < nb) wait_own_stores();
   }
}

// Hybrid Jacobi / Gauss-Seidel with C lanes per block and 64 / C blocks per
// wave (one wave per workgroup): the blocks advance side by side, so every
// wave instruction of the dependency chain serves 64 / C rows.  A block runs
// in chunks of C rows; lane sl of a block's lane group owns the chunk's sl-th
// row in sweep order.  Phase 1 (all lanes, branch-free batches of 8 entries:
// every column / value load of a batch, then every operand load, in flight
// together): the row's operands as in hybrid_jgs_wave_k, its prefix up to the
// first in-chunk dependency, and its tail -- every entry from there on, in CSR
// order -- as (tag, value): a product, or a coefficient whose operand is the
// previous row (DPP row shift), an earlier row of this chunk (the group's LDS
// value row) or the previous chunk's last row (carried in a register).  Tails
// live in registers indexed by entry (RMAX <= 8) or in LDS.  Phase 2: step
// s = 0 .. C - 1, lane s of every group adds its tail and divides.  The
// operations and their order are the reference's sequential loop's:
// bit-identical.  Rows of older chunks are loaded (agent scope) after this
// wave's stores have completed.  VI: values through the value index.
constexpr int JG_NONE = -2, JG_PROD = -1, JG_PREV = -3, JG_CARRY = -4, JG_FAR = -5, JG_PLAIN = -6;

__device__ __forceinline__ double dpp_shr1(double v)
{
   // lane l <- lane l - 1 within each row of 16 lanes (row_shr:1)
   const unsigned long long b = (unsigned long long)__double_as_longlong(v);
   const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, 0x111, 0xf, 0xf, false);
   const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), 0x111, 0xf, 0xf, false);
   return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

template <int C, int RMAX, bool VI, bool UNR = false, int WPE = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1))) void hybrid_jgs_grp_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                       const double *__restrict__ val,
                                                       const unsigned char *__restrict__ vidx,
                                                       const double *__restrict__ vtab, const double *__restrict__ f,
                                                       double *u, const double *__restrict__ u_prev,
                                                       const int *__restrict__ blk, int nblk,
                                                       const double *__restrict__ ds, double weight, int zero,
                                                       int reverse, double *apply_u = nullptr,
                                                       double *__restrict__ apply_priv = nullptr,
                                                       unsigned long long *stamp = nullptr)
{
   stamp_begin(stamp);
   const RowRec rst = stamp_rows(stamp);
   static_assert(C == 8 || C == 16, "lane groups inside DPP rows");
   constexpr int B = 64 / C;
   // UNR (small levels, latency-bound): the whole row's loads in one batch and
   // every tail in LDS (occupancy does not matter there; the re-read of long
   // tails costs two dependent loads per entry at every step)
   constexpr int KB = UNR ? RMAX : 8;                // entries per batch
   constexpr bool REG = RMAX <= 8;                   // tails in registers
   constexpr int TL = REG ? 1 : UNR ? RMAX - 1 : 16; // LDS tail slots (longer tails: re-read at the step)
   __shared__ double tv[TL][64];
   __shared__ signed char tg[TL][64];
   __shared__ double cv[64]; // the chunk's values (generic in-chunk dependencies)
   const int lane = (int)threadIdx.x, q = lane / C, sl = lane % C;
   const int b = (int)blockIdx.x * B + q;
   const bool has = b < nblk;
   const int ns = has ? blk[b] : 0, ne = has ? blk[b + 1] : 0, nb = ne - ns;
   int nmax = nb; // the wave runs the longest block's chunks
   for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
   double carry = 0.0;
   volatile double *cvv = cv;
   // the row pointers run one chunk ahead (their latency hides behind a chunk)
   auto row_of = [&](int c) { return reverse ? ne - 1 - (c + sl) : ns + c + sl; };
   int rs_n = 0, re_n = 0;
   if (has && sl < nb) {
      rs_n = rowptr[row_of(0)];
      re_n = rowptr[row_of(0) + 1];
   }
   for (int c0 = 0; c0 < nmax; c0 += C) {
      const bool act = has && c0 + sl < nb;
      const int i = act ? row_of(c0) : 0;
      double res = 0.0, a = 0.0, d = 1.0, old = 0.0;
      const int rs = act ? rs_n : 0, len = act ? re_n - rs_n : 0;
      int tl = 0;
      if (act) {
         d = ds ? ds[i] : 0.0;
         old = zero ? 0.0 : u_prev[i];
         res = f[i];
      }
      if (has && c0 + C + sl < nb) {
         rs_n = rowptr[row_of(c0 + C)];
         re_n = rowptr[row_of(c0 + C) + 1];
      }
      // the operand of column j: JG_PLAIN (u_prev), JG_PROD (a ready product:
      // 0 in the zero sweep), JG_FAR (an older chunk's row, re-read), a
      // dependency (JG_PREV, JG_CARRY, >= 0: this chunk's row), JG_NONE
      auto kind = [&](int j) -> int {
         if (j >= ns && j < ne) {
            const bool done = reverse ? j > i : j < i;
            if (!done) return zero ? JG_PROD : JG_PLAIN; // not yet updated: u_prev (0 in the zero sweep)
            const int pos = reverse ? ne - 1 - j : j - ns;
            return pos >= c0 ? (pos - c0 == sl - 1 ? JG_PREV : pos - c0) : pos == c0 - 1 ? JG_CARRY : JG_FAR;
         }
         return zero ? JG_NONE : JG_PLAIN; // the zero sweep skips out-of-block columns
      };
      int kov = 0; // entry where the tail leaves the LDS slots
      double pa[REG ? RMAX : 1];
      int pt[REG ? RMAX : 1];
      bool dep = false;
#pragma unroll
      for (int k = 0; k < (REG ? RMAX : 1); k++) pt[k] = JG_NONE;
      for (int kb = 0; kb < RMAX; kb += KB) {
         if (!__any(kb < len)) break;
         int jk[KB], tk[KB];
         double vk[KB], xk[KB];
#pragma unroll
         for (int k = 0; k < KB; k++) { // column / value loads (clamped: always in range)
            const int e = rs + max(0, min(kb + k, len - 1));
            jk[k] = col[e];
            vk[k] = VI ? vtab[vidx[e]] : val[e];
         }
         if (kb == 0) a = vk[0];
         bool far = false;
#pragma unroll
         for (int k = 0; k < KB; k++) { // operand kinds
            const int t = (act && kb + k < len) ? kind(jk[k]) : JG_NONE;
            far = far || t == JG_FAR;
            tk[k] = t;
         }
#pragma unroll
         for (int k = 0; k < KB; k++) { // operand loads (own row when unused)
            const double xv = u_prev[tk[k] == JG_PLAIN ? jk[k] : i];
            xk[k] = tk[k] == JG_PLAIN ? xv : 0.0;
         }
         if (__any(far)) {
            wait_own_stores(); // older chunks' stores (this wave's) have reached memory
#pragma unroll
            for (int k = 0; k < KB; k++)
               if (tk[k] == JG_FAR) xk[k] = __hip_atomic_load(u + jk[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
         }
#pragma unroll
         for (int k = 0; k < KB; k++) { // CSR order: prefix, then tail
            int t = tk[k];
            if (t == JG_NONE) continue;
            const bool prod = t == JG_PLAIN || t == JG_PROD || t == JG_FAR;
            if (prod) t = JG_PROD;
            dep = dep || !prod;
            const double w = prod ? vk[k] * xk[k] : vk[k];
            if (!dep) {
               res = res - w;
            } else if (REG) {
               pa[kb + k < (REG ? RMAX : 1) ? kb + k : 0] = w;
               pt[kb + k < (REG ? RMAX : 1) ? kb + k : 0] = t;
               tl = 1;
            } else {
               if (tl < TL) {
                  tv[tl][lane] = w;
                  tg[tl][lane] = (signed char)t;
               } else if (tl == TL) {
                  kov = kb + k;
               }
               tl++;
            }
         }
      }
      if (!ds) d = a;
      auto finish = [&](double r) { return (a != 0.0) ? (zero ? weight * r / d : old + weight * r / d) : old; };
      double v = old;
      if (act && tl == 0) v = finish(res);
      double vprev = 0.0;
      for (int st = 0; st < C; st++) {
         if (act && sl == st && tl > 0) {
            double r = res;
            if (REG) {
#pragma unroll
               for (int k = 0; k < (REG ? RMAX : 1); k++) {
                  const int t = pt[k];
                  if (t == JG_NONE) continue;
                  const double cw = cvv[q * C + max(t, 0)];
                  const double x = t == JG_PREV ? vprev : t == JG_CARRY ? carry : cw;
                  r = r - (t == JG_PROD ? pa[k] : pa[k] * x);
               }
            } else {
               const int tn = min(tl, TL);
               for (int t0 = 0; t0 < tn; t0 += 4) {
                  int tt[4];
                  double ww[4], cw[4];
#pragma unroll
                  for (int m = 0; m < 4; m++) {
                     const int slot = min(t0 + m, TL - 1);
                     tt[m] = t0 + m < tn ? (int)tg[slot][lane] : JG_NONE;
                     ww[m] = tv[slot][lane];
                     cw[m] = cvv[q * C + max(tt[m], 0)];
                  }
#pragma unroll
                  for (int m = 0; m < 4; m++) {
                     const int t = tt[m];
                     if (t == JG_NONE) continue;
                     const double x = t == JG_PREV ? vprev : t == JG_CARRY ? carry : cw[m];
                     r = r - (t == JG_PROD ? ww[m] : ww[m] * x);
                  }
               }
               // the tail past the slots (long rows with an early dependency):
               // its entries again from memory, in CSR order
               for (int k = kov; tl > TL && k < len; k++) {
                  const int j = col[rs + k];
                  const double vk = VI ? vtab[vidx[rs + k]] : val[rs + k];
                  const int t = kind(j);
                  if (t == JG_NONE) continue;
                  if (t == JG_PLAIN || t == JG_PROD || t == JG_FAR) {
                     const double x = t == JG_PLAIN  ? u_prev[j]
                                      : t == JG_FAR ? __hip_atomic_load(u + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                    : 0.0;
                     r = r - vk * x;
                  } else {
                     const double x = t == JG_PREV ? vprev : t == JG_CARRY ? carry : cvv[q * C + t];
                     r = r - vk * x;
                  }
               }
            }
            v = finish(r);
         }
         if (sl == st) cvv[lane] = v;
         vprev = dpp_shr1(v);
      }
      carry = __shfl(v, q * C + C - 1, 64);
      // a_ii == 0: the row keeps its value (0 after the zero-guess reset)
      if (act && (a != 0.0 || zero)) __hip_atomic_store(u + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // apply_u: the FULL_ASYNC correction folded in (the reference's add, then
      // read, in the capture form: atomic_noret_mode)
      if (apply_u && act) {
         const double o = atomicAdd(apply_u + i, v);
         apply_priv[i] = o + v;
         stamp_row(rst, i, o, o + v);
      }
   }
   stamp_end(stamp);
}

// Hybrid Jacobi / Gauss-Seidel, LDS tile form (jgs_wave 3): a workgroup of
// 256 lanes owns NB consecutive blocks and walks them in passes of CH rows per
// block (in sweep order).  Phase 1 (all lanes, one lane per row, consecutive
// lanes on consecutive rows of a block: coalesced CH-row segments) forms each
// row's prefix -- f_i minus its products up to the first in-pass dependency,
// in CSR order -- and its tail as (tag, value) slots: a ready product, or the
// coefficient of an earlier row of this pass; rows of earlier passes are
// products of the values this workgroup stored (re-read at agent scope after
// the stores completed).  Phase 2 (one wave, lane q = block q): the CH steps
// of every block's chain side by side, operands from LDS ([step][block]
// layout: the lanes' reads are consecutive), each new value into the pass's
// value row.  Tails past TMAX slots are re-read from memory at the step.  The
// operations and their order are the reference's sequential loop's
// (SMEM_Smooth.cpp:265-304 / 548-585): bit-identical.  Any row length.
template <int NB, int CH, int TMAX, bool VI, bool SHORT = false, int NT = 256, int OCC = 1, bool NORET = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(OCC))) void hybrid_jgs_tile_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                         const double *__restrict__ val,
                                                         const unsigned char *__restrict__ vidx,
                                                         const double *__restrict__ vtab, const double *__restrict__ f,
                                                         double *u, const double *__restrict__ u_prev,
                                                         const int *__restrict__ blk, int nblk,
                                                         const double *__restrict__ ds, double weight, int zero,
                                                         int reverse, double *apply_u, double *__restrict__ apply_priv,
                                                         unsigned long long *stamp)
{
   constexpr bool noret = NORET;
   stamp_begin(stamp);
   const RowRec rst = stamp_rows(stamp);
   constexpr int SP = NB + 1, NS = CH * SP, RPT = NB * CH / NT;
   static_assert(NB == 64 && (NB * CH) % NT == 0, "one phase-2 wave, whole rows per lane");
   __shared__ double sP[NS], sOld[NS], sD[NS], sV[NS];
   __shared__ double sW[TMAX][NS];
   __shared__ signed char sT[TMAX][NS];
   __shared__ int sM[NS]; // bit 0: a_ii != 0, bits 1-15: tail length, bits 16-31: entry past the slots
   __shared__ int sBlk[NB + 1];
   const int t = (int)threadIdx.x;
   const int b0 = (int)blockIdx.x * NB;
   if (t <= NB) sBlk[t] = blk[min(b0 + t, nblk)];
   __syncthreads();
   int nmax = 0; // the longest block's passes (every wave computes it)
   {
      const int q = t & 63;
      nmax = sBlk[q + 1] - sBlk[q];
      for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
   }
   auto ld_u = [u](int k) { return __hip_atomic_load(u + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
   // operand kinds (as hybrid_jgs_grp_k): JG_PLAIN u_prev, JG_PROD a ready
   // product (0 in the zero sweep), JG_FAR an earlier pass's row (re-read),
   // >= 0 an earlier row of this pass, JG_NONE skipped
   auto kind = [&](int j, int i, int ns, int ne, int c0) -> int {
      if (j >= ns && j < ne) {
         const bool done = reverse ? j > i : j < i;
         if (!done) return zero ? JG_PROD : JG_PLAIN;
         const int pos = reverse ? ne - 1 - j : j - ns;
         return pos >= c0 ? pos - c0 : JG_FAR;
      }
      return zero ? JG_NONE : JG_PLAIN;
   };
   int rs_n[RPT], re_n[RPT]; // row pointers one pass ahead
#pragma unroll
   for (int it = 0; it < RPT; it++) {
      const int r = it * NT + t, q = r / CH, sl = r % CH;
      const int ns = sBlk[q], ne = sBlk[q + 1];
      rs_n[it] = re_n[it] = 0;
      if (sl < ne - ns) {
         const int i = reverse ? ne - 1 - sl : ns + sl;
         rs_n[it] = rowptr[i];
         re_n[it] = rowptr[i + 1];
      }
   }
   for (int c0 = 0; c0 < nmax; c0 += CH) {
      // phase 1
      if constexpr (SHORT) {
         // rows of at most 8 entries: every load of the lane's RPT rows in flight
         // together (columns / values, then operands), no per-row loop
         int iv[RPT], nsv[RPT], nev[RPT], lenv[RPT], slotv[RPT];
         double Pv[RPT], oldv[RPT], ddv[RPT], av[RPT];
         int jk[RPT][8];
         double vk[RPT][8], xk[RPT][8];
#pragma unroll
         for (int it = 0; it < RPT; it++) {
            const int r = it * NT + t, q = r / CH, sl = r % CH;
            slotv[it] = sl * SP + q;
            const int ns = sBlk[q], ne = sBlk[q + 1], pos = c0 + sl;
            nsv[it] = ns;
            nev[it] = ne;
            const bool act = pos < ne - ns;
            const int i = act ? (reverse ? ne - 1 - pos : ns + pos) : 0;
            iv[it] = i;
            const int rs = rs_n[it], len = act ? re_n[it] - rs_n[it] : 0;
            lenv[it] = act ? len : -1;
            if (pos + CH < ne - ns) {
               const int in = reverse ? ne - 1 - (pos + CH) : ns + pos + CH;
               rs_n[it] = rowptr[in];
               re_n[it] = rowptr[in + 1];
            }
            Pv[it] = act ? f[i] : 0.0;
            oldv[it] = (act && !zero) ? u_prev[i] : 0.0;
            ddv[it] = (act && ds) ? ds[i] : 1.0;
#pragma unroll
            for (int k = 0; k < 8; k++) { // clamped: an empty row reads its a_ii slot (the next row's first)
               const int e = rs + max(0, min(k, len - 1));
               jk[it][k] = col[e];
               vk[it][k] = VI ? vtab[vidx[e]] : val[e];
            }
            av[it] = act ? vk[it][0] : 0.0;
         }
         bool far = false;
#pragma unroll
         for (int it = 0; it < RPT; it++)
#pragma unroll
            for (int k = 0; k < 8; k++) { // operand loads (own row when unused)
               const int tg = k < lenv[it] ? kind(jk[it][k], iv[it], nsv[it], nev[it], c0) : JG_NONE;
               far = far || tg == JG_FAR;
               const double xv = u_prev[tg == JG_PLAIN ? jk[it][k] : iv[it]];
               xk[it][k] = tg == JG_PLAIN ? xv : 0.0;
            }
         if (far) {
#pragma unroll
            for (int it = 0; it < RPT; it++)
#pragma unroll
               for (int k = 0; k < 8; k++)
                  if (k < lenv[it] && kind(jk[it][k], iv[it], nsv[it], nev[it], c0) == JG_FAR)
                     xk[it][k] = ld_u(jk[it][k]);
         }
#pragma unroll
         for (int it = 0; it < RPT; it++) {
            const int slot = slotv[it];
            double P = Pv[it];
            int tl = 0;
            bool dep = false;
#pragma unroll
            for (int k = 0; k < 8; k++) { // CSR order: prefix, then tail
               const int tg = k < lenv[it] ? kind(jk[it][k], iv[it], nsv[it], nev[it], c0) : JG_NONE;
               if (tg == JG_NONE) continue;
               const bool prod = tg == JG_PLAIN || tg == JG_PROD || tg == JG_FAR;
               dep = dep || !prod;
               const double w = prod ? vk[it][k] * xk[it][k] : vk[it][k];
               if (!dep) {
                  P = P - w;
               } else {
                  if (tl < TMAX) {
                     sW[tl][slot] = w;
                     sT[tl][slot] = (signed char)(prod ? JG_PROD : tg);
                  }
                  tl++;
               }
            }
            // (tails past TMAX re-read from entry TMAX slots after the first dependency)
            int kov = 0;
            if (tl > TMAX) {
               int seen = 0;
#pragma unroll
               for (int k = 0; k < 8; k++) {
                  const int tg = k < lenv[it] ? kind(jk[it][k], iv[it], nsv[it], nev[it], c0) : JG_NONE;
                  if (tg == JG_NONE) continue;
                  const bool prod = tg == JG_PLAIN || tg == JG_PROD || tg == JG_FAR;
                  if (!prod || seen > 0) seen++;
                  if (seen == TMAX + 1 && kov == 0) kov = k;
               }
            }
            sP[slot] = P;
            sOld[slot] = oldv[it];
            sD[slot] = ds ? ddv[it] : av[it];
            sM[slot] = (av[it] != 0.0 ? 1 : 0) | (min(tl, 0x7fff) << 1) | (kov << 16);
         }
      } else {
#pragma unroll
         for (int it = 0; it < RPT; it++) {
            const int r = it * NT + t, q = r / CH, sl = r % CH, slot = sl * SP + q;
            const int ns = sBlk[q], ne = sBlk[q + 1], pos = c0 + sl;
            const bool act = pos < ne - ns;
            const int i = act ? (reverse ? ne - 1 - pos : ns + pos) : 0;
            const int rs = rs_n[it], len = act ? re_n[it] - rs_n[it] : 0;
            if (pos + CH < ne - ns) {
               const int in = reverse ? ne - 1 - (pos + CH) : ns + pos + CH;
               rs_n[it] = rowptr[in];
               re_n[it] = rowptr[in + 1];
            }
            double P = 0.0, old = 0.0, a = 0.0, dd = 1.0;
            int tl = 0, kov = 0;
            bool dep = false;
            if (act) {
               P = f[i];
               old = zero ? 0.0 : u_prev[i];
               if (ds) dd = ds[i];
               // a_ii = val[rowptr[i]] as the reference reads it: an empty row's is the
               // next row's first value (as hybrid_jgs_grp_k's clamped first load)
               if (len == 0) a = VI ? vtab[vidx[rs]] : val[rs];
            }
            for (int kb = 0; kb < len; kb += 8) {
               int jk[8], tk[8];
               double vk[8], xk[8];
   #pragma unroll
               for (int k = 0; k < 8; k++) { // column / value loads (clamped: always in range)
                  const int e = rs + min(kb + k, len - 1);
                  jk[k] = col[e];
                  vk[k] = VI ? vtab[vidx[e]] : val[e];
               }
               if (kb == 0) a = vk[0];
               bool far = false;
   #pragma unroll
               for (int k = 0; k < 8; k++) {
                  tk[k] = kb + k < len ? kind(jk[k], i, ns, ne, c0) : JG_NONE;
                  far = far || tk[k] == JG_FAR;
               }
   #pragma unroll
               for (int k = 0; k < 8; k++) { // operand loads (own row when unused)
                  const double xv = u_prev[tk[k] == JG_PLAIN ? jk[k] : i];
                  xk[k] = tk[k] == JG_PLAIN ? xv : 0.0;
               }
               if (far) {
   #pragma unroll
                  for (int k = 0; k < 8; k++)
                     if (tk[k] == JG_FAR) xk[k] = ld_u(jk[k]);
               }
   #pragma unroll
               for (int k = 0; k < 8; k++) { // CSR order: prefix, then tail
                  const int tg = tk[k];
                  if (tg == JG_NONE) continue;
                  const bool prod = tg == JG_PLAIN || tg == JG_PROD || tg == JG_FAR;
                  dep = dep || !prod;
                  const double w = prod ? vk[k] * xk[k] : vk[k];
                  if (!dep) {
                     P = P - w;
                  } else {
                     if (tl < TMAX) {
                        sW[tl][slot] = w;
                        sT[tl][slot] = (signed char)(prod ? JG_PROD : tg);
                     } else if (tl == TMAX) {
                        kov = kb + k;
                     }
                     tl++;
                  }
               }
            }
            if (!ds) dd = a;
            sP[slot] = P;
            sOld[slot] = old;
            sD[slot] = dd;
            sM[slot] = (a != 0.0 ? 1 : 0) | (min(tl, 0x7fff) << 1) | (kov << 16);
         }
      }
      __syncthreads();
      // phase 2: lane q walks block q's CH steps
      if (t < NB) {
         const int q = t, ns = sBlk[q], ne = sBlk[q + 1];
         const int cnt = min(CH, ne - ns - c0);
         for (int s = 0; s < cnt; s++) {
            const int slot = s * SP + q;
            const int m = sM[slot], tl = (m >> 1) & 0x7fff;
            double r = sP[slot];
            const int tn = min(tl, TMAX);
            for (int k = 0; k < tn; k++) {
               const int tg = sT[k][slot];
               const double w = sW[k][slot];
               r = r - (tg == JG_PROD ? w : w * sV[max(tg, 0) * SP + q]);
            }
            if (tl > TMAX) { // the tail past the slots, again from memory in CSR order
               const int pos = c0 + s, i = reverse ? ne - 1 - pos : ns + pos;
               const int rs = rowptr[i], len = rowptr[i + 1] - rs;
               for (int k = m >> 16; k < len; k++) {
                  const int j = col[rs + k];
                  const double vk = VI ? vtab[vidx[rs + k]] : val[rs + k];
                  const int tg = kind(j, i, ns, ne, c0);
                  if (tg == JG_NONE) continue;
                  const double x = tg == JG_PLAIN ? u_prev[j] : tg == JG_FAR ? ld_u(j) : tg == JG_PROD ? 0.0
                                                                                                       : sV[tg * SP + q];
                  r = r - vk * x;
               }
            }
            const double old = sOld[slot], d = sD[slot];
            sV[slot] = (m & 1) ? (zero ? weight * r / d : old + weight * r / d) : old;
         }
      }
      __syncthreads();
      // write-out (coalesced): a_ii == 0 keeps the row's value (0 after the zero-guess reset);
      // apply_u: the correction u_shared += v (atomic_correct_k's operations)
#pragma unroll
      for (int it = 0; it < RPT; it++) {
         const int r = it * NT + t, q = r / CH, sl = r % CH, slot = sl * SP + q;
         const int ns = sBlk[q], ne = sBlk[q + 1], pos = c0 + sl;
         if (pos < ne - ns) {
            const int i = reverse ? ne - 1 - pos : ns + pos;
            const double v = sV[slot];
            if ((sM[slot] & 1) || zero) __hip_atomic_store(u + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (apply_u && noret) {
               add_noret(apply_u + i, v);
            } else if (apply_u) {
               const double o = atomicAdd(apply_u + i, v);
               apply_priv[i] = o + v;
               stamp_row(rst, i, o, o + v);
            }
         }
      }
      if (apply_u && noret) { // the reference's read of u after its add
         wait_vm_all();
#pragma unroll
         for (int it = 0; it < RPT; it++) {
            const int r = it * NT + t, q = r / CH, sl = r % CH;
            const int ns = sBlk[q], ne = sBlk[q + 1], pos = c0 + sl;
            if (pos < ne - ns) {
               const int i = reverse ? ne - 1 - pos : ns + pos;
               apply_priv[i] = read_agent(apply_u + i);
               stamp_row(rst, i);
            }
         }
      }
      if (c0 + CH < nmax) {
         wait_own_stores(); // the next pass's loads of these rows see the stores
         __syncthreads();
      }
   }
   stamp_end(stamp);
}

__global__ void row_max_k(const int *__restrict__ rowptr, int n, int *__restrict__ out)
{
   int m = 0;
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
      m = max(m, rowptr[i + 1] - rowptr[i]);
   for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_down(m, o, 64));
   if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

void row_max(hipStream_t s, const amg_mat *A, int *d_out)
{
   const int n = A->nrows;
   if (n <= 0) return;
   row_max_k<<<std::max(1, std::min(1024, (n + 255) / 256)), 256, 0, s>>>(A->rowptr, n, d_out);
}

bool hybrid_jgs(hipStream_t s, const amg_mat *A, const double *f, double *u, const double *u_prev,
                const int *d_blk, int nblk, const double *diag_scale, double weight, int zero,
                int reverse, double *apply_u, double *apply_priv, unsigned long long *stamp)
{
   if (nblk <= 0) return false;
   int mode = A->ctx->jgs_wave;
   if (mode == 3) {
      // short rows: passes of 16 rows per block, 4 tail slots; longer rows
      // (27-pt, classical): passes of 4 rows, 16 slots
      const int nwg = (nblk + 63) / 64;
#define JGS_TILE(CH, TM, V, SH, OC)                                                                                  \
   hybrid_jgs_tile_k<64, CH, TM, V, SH, SH ? 512 : 256, OC><<<nwg, SH ? 512 : 256, 0, s>>>(A->rowptr, A->col, A->val, A->vidx, A->vtab, f, u, u_prev, \
                                                        d_blk, nblk, diag_scale, weight, zero, reverse, apply_u,  \
                                                        apply_priv, apply_u ? stamp : nullptr)
      const bool vi = A->vidx != nullptr;
      if (A->maxrow >= 0 && A->maxrow <= 8) {
         // AMG_JGS_TILE_OCC=4: registers capped for two workgroups per CU
         static const int occ = [] {
            const char *v = std::getenv("AMG_JGS_TILE_OCC");
            return v ? std::atoi(v) : 1;
         }();
         if (occ == 4) {
            if (vi) JGS_TILE(16, 4, true, true, 4);
            else JGS_TILE(16, 4, false, true, 4);
         } else {
            if (vi) JGS_TILE(16, 4, true, true, 1);
            else JGS_TILE(16, 4, false, true, 1);
         }
      } else {
         if (vi) JGS_TILE(4, 16, true, false, 1);
         else JGS_TILE(4, 16, false, false, 1);
      }
#undef JGS_TILE
      return apply_u != nullptr;
   }
   // small levels (fewer workgroups than CUs) are latency-bound: jgs_small 1
   // runs them one wave per block, 2 with the whole row's loads in one batch
   const int small_form = A->ctx->jgs_small;
   const bool small = (nblk + 7) / 8 < 1024 && A->maxrow > 8 && A->maxrow <= 32;
   if (mode == 1 && small && small_form == 1) mode = 2;
   if (mode == 1 && small && small_form == 2) {
      const int nwg = (nblk + 7) / 8;
      if (A->vidx)
         hybrid_jgs_grp_k<8, 32, true, true><<<nwg, 64, 0, s>>>(A->rowptr, A->col, A->val, A->vidx, A->vtab, f, u,
                                                                 u_prev, d_blk, nblk, diag_scale, weight, zero, reverse);
      else
         hybrid_jgs_grp_k<8, 32, false, true><<<nwg, 64, 0, s>>>(A->rowptr, A->col, A->val, A->vidx, A->vtab, f, u,
                                                                  u_prev, d_blk, nblk, diag_scale, weight, zero,
                                                                  reverse);
      return false;
   }
   if (mode == 1 && A->maxrow >= 1 && A->maxrow <= 32) {
      // 8 lanes per block, 8 blocks per wave
      const int nwg = (nblk + 7) / 8;
      const bool vi = A->vidx != nullptr;
#define JGS_GRP(R, V)                                                                                               \
   hybrid_jgs_grp_k<8, R, V><<<nwg, 64, 0, s>>>(A->rowptr, A->col, A->val, A->vidx, A->vtab, f, u, u_prev, d_blk, \
                                                nblk, diag_scale, weight, zero, reverse, apply_u, apply_priv,     \
                                                apply_u ? stamp : nullptr)
      // AMG_JGS_WPE=6 / 8: registers capped for 6 / 8 waves per SIMD (rows of <= 8 entries)
      static const int jwpe = [] {
         const char *v = std::getenv("AMG_JGS_WPE");
         return v ? std::atoi(v) : 0;
      }();
      if (A->maxrow <= 8 && vi && jwpe == 8) {
         hybrid_jgs_grp_k<8, 8, true, false, 8><<<nwg, 64, 0, s>>>(A->rowptr, A->col, A->val, A->vidx, A->vtab, f, u, u_prev,
                                                                  d_blk, nblk, diag_scale, weight, zero, reverse, apply_u,
                                                                  apply_priv, apply_u ? stamp : nullptr);
      } else if (A->maxrow <= 8 && vi && jwpe == 6) {
         hybrid_jgs_grp_k<8, 8, true, false, 6><<<nwg, 64, 0, s>>>(A->rowptr, A->col, A->val, A->vidx, A->vtab, f, u, u_prev,
                                                                  d_blk, nblk, diag_scale, weight, zero, reverse, apply_u,
                                                                  apply_priv, apply_u ? stamp : nullptr);
      } else if (A->maxrow <= 8) {
         if (vi) JGS_GRP(8, true);
         else JGS_GRP(8, false);
      } else {
         if (vi) JGS_GRP(32, true);
         else JGS_GRP(32, false);
      }
#undef JGS_GRP
      return apply_u != nullptr;
   }
   if (mode == 2 && A->maxrow >= 0 && A->maxrow <= 32) {
      const int nwg = (nblk + 3) / 4;
      if (A->maxrow <= 8)
         hybrid_jgs_wave_k<8><<<nwg, 256, 0, s>>>(A->rowptr, A->col, A->val, f, u, u_prev, d_blk, nblk, diag_scale,
                                                  weight, zero, reverse);
      else
         hybrid_jgs_wave_k<32><<<nwg, 256, 0, s>>>(A->rowptr, A->col, A->val, f, u, u_prev, d_blk, nblk,
                                                   diag_scale, weight, zero, reverse);
      return false;
   }
   const int tpb = 64;
   hybrid_jgs_k<<<(nblk + tpb - 1) / tpb, tpb, 0, s>>>(A->rowptr, A->col, A->val, f, u, u_prev,
                                                       d_blk, nblk, diag_scale, weight, zero,
                                                       reverse);
   return false;
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

// composed smoothed transfers (SmoothTransfer, SMEM_Setup.cpp:1173-1254, applied
// as R~ r = R (r - w A D^-1 r), P~ e = P e - w D^-1 A P e; the oracle's
// or_hier_set_composed_transfers order of operations)
__global__ void xfer_div_k(const double *__restrict__ diag, const double *__restrict__ x,
                           double *__restrict__ out, int rb, int re)
{
   EW_LOOP(i, rb, re) out[i] = x[i] / diag[i];
}
void xfer_div(hipStream_t s, const double *diag, const double *x, double *out, int rb, int re)
{
   if (re > rb) xfer_div_k<<<ew_blocks(re - rb), 256, 0, s>>>(diag, x, out, rb, re);
}
__global__ void xfer_sub_k(double mw, const double *__restrict__ r, const double *__restrict__ y,
                           double *__restrict__ z, int rb, int re)
{
   EW_LOOP(i, rb, re) z[i] = r[i] + mw * y[i];
}
void xfer_sub(hipStream_t s, double w, const double *r, const double *y, double *z, int rb, int re)
{
   if (re > rb) xfer_sub_k<<<ew_blocks(re - rb), 256, 0, s>>>(-w, r, y, z, rb, re);
}
__global__ void xfer_corr_k(double mw, const double *__restrict__ y, const double *__restrict__ diag,
                            double *__restrict__ e, int rb, int re)
{
   EW_LOOP(i, rb, re)
   {
      const double t = y[i] / diag[i];
      e[i] = e[i] + mw * t;
   }
}
void xfer_corr(hipStream_t s, double w, const double *y, const double *diag, double *e, int rb, int re)
{
   if (re > rb) xfer_corr_k<<<ew_blocks(re - rb), 256, 0, s>>>(-w, y, diag, e, rb, re);
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

__global__ void dmem_scale_k(const double *__restrict__ diag, const double *__restrict__ l1, double omega,
                             double *__restrict__ sc, double *__restrict__ nsc, int n)
{
   EW_LOOP(i, 0, n)
   {
      const double v = l1 ? l1[i] : (diag[i] == 0.0 ? 1.0 : diag[i] / omega);
      sc[i] = v;
      nsc[i] = -v;
   }
}
void dmem_scale(hipStream_t s, const double *diag, const double *l1, double omega, double *sc, double *nsc, int n)
{
   if (n > 0) dmem_scale_k<<<ew_blocks(n), 256, 0, s>>>(diag, l1, omega, sc, nsc, n);
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
   // a_ii := A_data[A_i[i]] for every row, as the reference reads it: an empty
   // row sees the next row's first value (the zero padding after the last row)
   EW_LOOP(i, 0, n) diag[i] = val[rowptr[i]];
}
void extract_diag(hipStream_t s, const amg_mat *A)
{
   if (A->nrows > 0)
      extract_diag_k<<<ew_blocks(A->nrows), 256, 0, s>>>(A->rowptr, A->val, A->diag, A->nrows);
}

// *flag = 1 when some diag[i] differs from diag[0] in its bits (the writers
// all store 1)
__global__ void diag_uniform_k(const double *__restrict__ diag, int n, int *flag)
{
   const long long d0 = __double_as_longlong(diag[0]);
   EW_LOOP(i, 1, n)
   if (__double_as_longlong(diag[i]) != d0) *flag = 1;
}
void diag_uniform(hipStream_t s, const amg_mat *A, int *d_flag)
{
   if (A->nrows > 1) diag_uniform_k<<<ew_blocks(A->nrows), 256, 0, s>>>(A->diag, A->nrows, d_flag);
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

// DMEM_Misc.cpp:612-666 DMEM_ChebyUpdate(d, u) after the first cycle:
//   branch 0 (MULT / sync)      d = (w-1) d + w delta u
//   branch 1 (async, cheby_grid) d' = (w-1) d + w delta u ; u = (w-1) d + w delta u
//   branch 2 (async, other grid) u = w delta u
// om1 = w - 1.0 and omd = w * delta are formed on the host, as the reference's
// left-to-right `(omega - 1.0) * d + omega * delta * u` rounds them.
__global__ void dmem_cheby_k(double *__restrict__ d, double *__restrict__ u, int n, int branch,
                             double om1, double omd)
{
   EW_LOOP(i, 0, n)
   {
      const double ui = u[i];
      if (branch == 2) {
         u[i] = omd * ui;
      } else {
         const double dp = d[i];
         d[i] = om1 * dp + omd * ui;
         if (branch == 1) u[i] = om1 * dp + omd * ui;
      }
   }
}
void dmem_cheby_update(hipStream_t s, double *d, double *u, int n, int branch, double om1, double omd)
{
   if (n > 0) dmem_cheby_k<<<ew_blocks(n), 256, 0, s>>>(d, u, n, branch, om1, omd);
}

// DMEM_Mult.cpp:46-55 with acceleration: x += e; ChebyUpdate(d, e) (copy on the
// first cycle); x += d -- one pass
__global__ void dmem_mult_accel_k(double *__restrict__ x, const double *__restrict__ e,
                                  double *__restrict__ d, int n, int first, double om1, double omd)
{
   EW_LOOP(i, 0, n)
   {
      const double ei = e[i];
      const double xi = x[i] + 1.0 * ei;
      const double di = first ? ei : om1 * d[i] + omd * ei;
      d[i] = di;
      x[i] = xi + 1.0 * di;
   }
}
void dmem_mult_accel(hipStream_t s, double *x, const double *e, double *d, int n, int first, double om1,
                     double omd)
{
   if (n > 0) dmem_mult_accel_k<<<ew_blocks(n), 256, 0, s>>>(x, e, d, n, first, om1, omd);
}

// SMEM_Async_AMG.cpp:296-299 (FULL_ASYNC): omp atomic u[i] += e[i]; u_k[i] = u[i]
template <bool NORET>
__global__ void atomic_correct_k(double *u, const double *__restrict__ e,
                                 double *__restrict__ u_priv, int n, unsigned long long *stamp)
{
   constexpr bool noret = NORET;
   stamp_begin(stamp);
   const RowRec rst = stamp_rows(stamp);
   EW_LOOP(i, 0, n)
   {
      const double ei = e[i];
      if (noret) {
         add_noret(u + i, ei);
         wait_vm_all();
         u_priv[i] = read_agent(u + i);
         stamp_row(rst, i);
      } else {
         const double old = atomicAdd(u + i, ei);
         u_priv[i] = old + ei;
         stamp_row(rst, i, old, old + ei);
      }
   }
   stamp_end(stamp);
}
void atomic_correct(hipStream_t s, double *u, const double *e, double *u_priv, int n, unsigned long long *stamp)
{
   if (n <= 0) return;
   if (atomic_noret_mode()) atomic_correct_k<true><<<ew_blocks(n), 256, 0, s>>>(u, e, u_priv, n, stamp);
   else atomic_correct_k<false><<<ew_blocks(n), 256, 0, s>>>(u, e, u_priv, n, stamp);
}

// the n 4-word correction records of AmgCorrTimes: window start (min'ed),
// window end (max'ed), no row arrays
__global__ void stamp_init_k(unsigned long long *st, int n)
{
   EW_LOOP(i, 0, n)
   {
      st[4 * i] = ~0ull;
      st[4 * i + 1] = 0ull;
      st[4 * i + 2] = 0ull;
      st[4 * i + 3] = 0ull;
   }
}
void stamp_init(hipStream_t s, unsigned long long *stamps, int n)
{
   if (n > 0) stamp_init_k<<<ew_blocks(n), 256, 0, s>>>(stamps, n);
}

// SEMI_ASYNC update (SMEM_Async_AMG.cpp:238-283, under the reference's lock;
// here the updates of all levels are serialised on one stream): u += e,
// u_priv = u -- plain read-modify-write, no other level touches u meanwhile
__global__ void semi_correct_k(double *__restrict__ u, const double *__restrict__ e,
                               double *__restrict__ u_priv, int n)
{
   EW_LOOP(i, 0, n)
   {
      const double v = u[i] + e[i];
      u[i] = v;
      if (u_priv) u_priv[i] = v;
   }
}
void semi_correct(hipStream_t s, double *u, const double *e, double *u_priv, int n)
{
   if (n > 0) semi_correct_k<<<ew_blocks(n), 256, 0, s>>>(u, e, u_priv, n);
}

// READ_RES residual update (SMEM_Async_AMG.cpp:288-295 / 270-275): the shared
// residual r -= y (y = A e of the level's correction), the level's private
// residual = the value after its update.  atomic: FULL_ASYNC (device-scope fp64
// atomics); otherwise the serialised SEMI_ASYNC form.
__global__ void res_update_k(double *r, const double *__restrict__ y, double *__restrict__ r_priv, int n,
                             int atomic, unsigned long long *stamp)
{
   stamp_begin(stamp);
   const RowRec rst = stamp_rows(stamp);
   EW_LOOP(i, 0, n)
   {
      const double yi = y[i];
      double v;
      double o;
      if (atomic) {
         o = atomicAdd(r + i, -yi);
         v = o - yi;
      } else {
         o = r[i];
         v = o - yi;
         r[i] = v;
      }
      r_priv[i] = v;
      stamp_row(rst, i, o, v);
   }
   stamp_end(stamp);
}
void res_update(hipStream_t s, double *r, const double *y, double *r_priv, int n, int atomic,
                unsigned long long *stamp)
{
   if (n > 0) res_update_k<<<ew_blocks(n), 256, 0, s>>>(r, y, r_priv, n, atomic, stamp);
}

// u[rb, re) += x[rb, re) with device-scope atomics (the GLOBAL residual
// phase's fine-grid smoothing correction, SMEM_Async_AMG.cpp:61-70)
__global__ void atomic_add_k(double *u, const double *__restrict__ x, int rb, int re)
{
   EW_LOOP(i, rb, re) atomicAdd(u + i, x[i]);
}
void atomic_add(hipStream_t s, double *u, const double *x, int rb, int re)
{
   if (re > rb) atomic_add_k<<<ew_blocks(re - rb), 256, 0, s>>>(u, x, rb, re);
}

// ---------------------------------------------------------------------------
// deterministic reductions: fixed grid, fixed per-lane order, fixed tree
// ---------------------------------------------------------------------------
static inline int red_blocks(int n) { return std::max(1, std::min(1024, (n + 2047) / 2048)); }

// MODE 0: sum x^2, 1: sum x y, 2: sum |x|
template <int MODE>
__global__ __launch_bounds__(256) void partials_k(const double *__restrict__ x,
                                                  const double *__restrict__ y, int n,
                                                  double *__restrict__ partials)
{
   __shared__ double red[4];
   double s = 0.0;
   for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
      s += MODE == 1 ? x[i] * y[i] : MODE == 2 ? fabs(x[i]) : x[i] * x[i];
   s = block_sum_256(s, red);
   if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

void sumsq_partials(hipStream_t s, const double *x, int n, double *partials, int *nparts)
{
   const int nb = red_blocks(n);
   partials_k<0><<<nb, 256, 0, s>>>(x, nullptr, n, partials);
   *nparts = nb;
}

void abssum_partials(hipStream_t s, const double *x, int n, double *partials, int *nparts)
{
   const int nb = red_blocks(n);
   partials_k<2><<<nb, 256, 0, s>>>(x, nullptr, n, partials);
   *nparts = nb;
}

void dot_partials(hipStream_t s, const double *x, const double *y, int n, double *partials,
                  int *nparts)
{
   const int nb = red_blocks(n);
   partials_k<1><<<nb, 256, 0, s>>>(x, y, n, partials);
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

// ---------------------------------------------------------------------------
// value-indexed CSR construction: the distinct values of val (by bit pattern)
// collected into a device hash set, then every entry encoded as a one-byte
// index into the sorted table of at most 256 values
// ---------------------------------------------------------------------------
constexpr unsigned long long VI_EMPTY = ~0ULL;

__device__ __forceinline__ unsigned int vi_hash(unsigned long long k)
{
   k ^= k >> 33;
   k *= 0xff51afd7ed558ccdULL;
   k ^= k >> 33;
   return (unsigned int)k;
}

__device__ __forceinline__ void vi_insert(unsigned long long key, unsigned long long *slots,
                                          int nslots, int *count)
{
   if (__atomic_load_n(count, __ATOMIC_RELAXED) > 256) return; // table already useless
   unsigned int h = vi_hash(key) & (nslots - 1);
   for (int probe = 0; probe < nslots; probe++) {
      const unsigned long long cur = __atomic_load_n(&slots[h], __ATOMIC_RELAXED);
      if (cur == key) return;
      if (cur == VI_EMPTY) {
         const unsigned long long prev = atomicCAS(&slots[h], VI_EMPTY, key);
         if (prev == VI_EMPTY) {
            atomicAdd(count, 1);
            return;
         }
         if (prev == key) return;
      }
      h = (h + 1) & (nslots - 1);
   }
}

// CSR-DC keys: (col - row) in the high 32 bits, the value-index byte low
__device__ __forceinline__ unsigned long long dc_key(int off, unsigned char b)
{
   return ((unsigned long long)(unsigned int)off << 8) | b;
}

// anchor of row i: its first column (the diagonal for diag-first square
// operators, the parent coarse point for interpolation rows)
__global__ void dc_collect_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                             const unsigned char *__restrict__ vidx, int n,
                             unsigned long long *slots, int nslots, int *count, int *maxlen)
{
   unsigned long long last0 = VI_EMPTY, last1 = VI_EMPTY;
   int ml = 0, offrow = 0;
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      const int rs = rowptr[i], re = rowptr[i + 1];
      ml = max(ml, re - rs);
      const int anc = rs < re ? col[rs] : i;
      offrow |= (anc != i);
      for (int k = rs; k < re; k++) {
         const unsigned long long key = dc_key(col[k] - anc, vidx[k]);
         if (key == last0 || key == last1) continue;
         last1 = last0;
         last0 = key;
         vi_insert(key, slots, nslots, count);
      }
   }
   atomicMax(maxlen, ml);
   if (offrow) atomicOr(maxlen + 1, 1); // some row's anchor is not its own index
}

__global__ void dc_encode_k(const int *__restrict__ rowptr, const int *__restrict__ col,
                            const unsigned char *__restrict__ vidx, int n,
                            const unsigned long long *__restrict__ keys, int T,
                            unsigned char *__restrict__ didx, int *__restrict__ anch)
{
   __shared__ unsigned long long tk[256];
   if (threadIdx.x < 256) tk[threadIdx.x] = threadIdx.x < T ? keys[threadIdx.x] : VI_EMPTY;
   __syncthreads();
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      const int rs = rowptr[i], re = rowptr[i + 1];
      const int anc = rs < re ? col[rs] : i;
      if (anch) anch[i] = anc;
      for (int k = rs; k < re; k++) {
         const unsigned long long key = dc_key(col[k] - anc, vidx[k]);
         int lo = 0, hi = T - 1;
         while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tk[mid] < key)
               lo = mid + 1;
            else
               hi = mid;
         }
         didx[k] = (unsigned char)lo;
      }
   }
}

// ---- row-pattern construction ------------------------------------------------
// key of row i's dictionary sequence: exact for <= 7 entries (length byte +
// the entries), else a 56-bit hash above the length byte (verified after
// encoding, so a collision only disables the format)
__device__ __forceinline__ unsigned long long rp_key(const unsigned char *__restrict__ didx, int rs, int len)
{
   if (len <= 7) {
      unsigned long long k = (unsigned long long)len;
      for (int j = 0; j < len; j++) k |= (unsigned long long)didx[rs + j] << (8 * (j + 1));
      return k;
   }
   unsigned long long h = 0xcbf29ce484222325ULL ^ (unsigned long long)len;
   for (int j = 0; j < len; j++) h = (h ^ didx[rs + j]) * 0x100000001b3ULL;
   h ^= h >> 29;
   h *= 0xbf58476d1ce4e5b9ULL;
   h ^= h >> 32;
   return (h << 8) | (unsigned long long)len;
}

// distinct row keys into slots (first row of each into rep), and the number of
// rows that cannot be coded (empty or longer than AMG_DC_MAXROW)
__global__ void rp_collect_k(const int *__restrict__ rowptr, const unsigned char *__restrict__ didx, int n,
                             unsigned long long *slots, int *rep, int nslots, int *count, int *bad)
{
   unsigned long long last = VI_EMPTY;
   int nbad = 0;
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      const int rs = rowptr[i], len = rowptr[i + 1] - rs;
      if (len < 1 || len > AMG_DC_MAXROW) {
         nbad++;
         continue;
      }
      const unsigned long long key = rp_key(didx, rs, len);
      if (key == last) continue;
      last = key;
      if (__atomic_load_n(count, __ATOMIC_RELAXED) > 256) continue; // too many patterns: only count bad rows
      unsigned int h = vi_hash(key) & (nslots - 1);
      for (int probe = 0; probe < nslots; probe++) {
         const unsigned long long cur = __atomic_load_n(&slots[h], __ATOMIC_RELAXED);
         if (cur == key) break;
         if (cur == VI_EMPTY) {
            const unsigned long long prev = atomicCAS(&slots[h], VI_EMPTY, key);
            if (prev == VI_EMPTY) {
               atomicAdd(count, 1);
               rep[h] = i;
               break;
            }
            if (prev == key) break;
         }
         h = (h + 1) & (nslots - 1);
      }
   }
   if (nbad) atomicAdd(bad, nbad);
}

// pattern table: entry t = [length, dictionary bytes of representative row rep[t]]
__global__ void rp_table_k(const int *__restrict__ rowptr, const unsigned char *__restrict__ didx,
                           const int *__restrict__ rep, int T, unsigned char *__restrict__ ptab)
{
   const int t = blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= T) return;
   const int rs = rowptr[rep[t]], len = rowptr[rep[t] + 1] - rs;
   unsigned char *pp = ptab + t * AMG_RP_STRIDE;
   pp[0] = (unsigned char)len;
   for (int j = 0; j < AMG_DC_MAXROW; j++) pp[1 + j] = j < len ? didx[rs + j] : 0;
}

// rpat[i] = index of row i's key among the T sorted keys; rows whose bytes
// differ from their pattern (a hash collision) are counted in bad
__global__ void rp_encode_k(const int *__restrict__ rowptr, const unsigned char *__restrict__ didx, int n,
                            const unsigned long long *__restrict__ keys, int T,
                            const unsigned char *__restrict__ ptab, unsigned char *__restrict__ rpat,
                            int *bad)
{
   __shared__ unsigned long long tk[256];
   if (threadIdx.x < 256) tk[threadIdx.x] = threadIdx.x < T ? keys[threadIdx.x] : VI_EMPTY;
   __syncthreads();
   int nbad = 0;
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      const int rs = rowptr[i], len = rowptr[i + 1] - rs;
      const unsigned long long key = rp_key(didx, rs, len);
      int lo = 0, hi = T - 1;
      while (lo < hi) {
         const int mid = (lo + hi) >> 1;
         if (tk[mid] < key)
            lo = mid + 1;
         else
            hi = mid;
      }
      rpat[i] = (unsigned char)lo;
      const unsigned char *pp = ptab + lo * AMG_RP_STRIDE;
      bool ok = tk[lo] == key && pp[0] == len;
      for (int j = 0; ok && j < len; j++) ok = pp[1 + j] == didx[rs + j];
      nbad += !ok;
   }
   if (nbad) atomicAdd(bad, nbad);
}

// row-pair keys p0 * 257 + p1 (p1 = 256 when row 2t+1 does not exist)
// pair key: (pattern of row 2t, of row 2t+1 or 256 if none, anchor delta
// da = anch[2t+1] - anch[2t] + AMG_PP_DA0 in [0, AMG_PP_NDA)); a delta out of
// range flags the matrix (flags[AMG_PP_NK])
__device__ __forceinline__ int pp_key(const unsigned char *__restrict__ rpat, const int *__restrict__ anch, int n,
                                      int t)
{
   const bool two = 2 * t + 1 < n;
   const int da = (two && anch) ? anch[2 * t + 1] - anch[2 * t] + AMG_PP_DA0 : AMG_PP_DA0;
   if (da < 0 || da >= AMG_PP_NDA) return -1;
   return (rpat[2 * t] * 257 + (two ? rpat[2 * t + 1] : 256)) * AMG_PP_NDA + da;
}

__global__ void pp_collect_k(const unsigned char *__restrict__ rpat, const int *__restrict__ anch, int n,
                             unsigned char *flags)
{
   const int np = (n + 1) / 2;
   for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < np; t += gridDim.x * blockDim.x) {
      int k = pp_key(rpat, anch, n, t);
      if (k < 0) k = AMG_PP_NK;
      if (!flags[k]) flags[k] = 1;
   }
}

// ppat[t] = the pair's table index; counts[p] += pairs of pattern p
__global__ __launch_bounds__(256) void pp_encode_k(const unsigned char *__restrict__ rpat,
                                                   const int *__restrict__ anch, int n,
                                                   const unsigned char *__restrict__ map,
                                                   unsigned char *__restrict__ ppat,
                                                   unsigned long long *__restrict__ counts)
{
   __shared__ unsigned int hist[256];
   hist[threadIdx.x] = 0;
   __syncthreads();
   const int np = (n + 1) / 2;
   for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < np; t += gridDim.x * blockDim.x) {
      const unsigned char p = map[pp_key(rpat, anch, n, t)];
      ppat[t] = p;
      atomicAdd(&hist[p], 1u);
   }
   __syncthreads();
   if (hist[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
}

void pp_collect(hipStream_t s, const amg_mat *A, unsigned char *flags)
{
   if (A->nrows <= 0) return;
   pp_collect_k<<<std::min(8192, (A->nrows + 511) / 512), 256, 0, s>>>(A->rpat, A->danch, A->nrows, flags);
}

// one workgroup per 512-row slab: least anchor of its even rows, then each
// pair's 16-bit delta from it
__global__ __launch_bounds__(256) void pp_anchor_k(const int *__restrict__ anch, int n, int *__restrict__ pbase,
                                                  unsigned short *__restrict__ pdelta, int *__restrict__ ok)
{
   __shared__ int red[2][256];
   const int slab = (int)blockIdx.x, tid = (int)threadIdx.x;
   const long long row = (long long)slab * 512 + 2 * tid;
   const int a = row < n ? anch[row] : INT_MAX;
   red[0][tid] = a;
   red[1][tid] = row < n ? a : INT_MIN;
   __syncthreads();
   for (int w = 128; w > 0; w >>= 1) {
      if (tid < w) {
         red[0][tid] = min(red[0][tid], red[0][tid + w]);
         red[1][tid] = max(red[1][tid], red[1][tid + w]);
      }
      __syncthreads();
   }
   const int lo = red[0][0], hi = red[1][0];
   if (tid == 0) {
      pbase[slab] = lo;
      if ((long long)hi - lo > 65535) *ok = 0;
   }
   if (row < n) pdelta[row >> 1] = (unsigned short)(a - lo);
}

void pp_anchor_compress(hipStream_t s, const amg_mat *A, int *pbase, unsigned short *pdelta, int *ok)
{
   const int ns = (A->nrows + 511) / 512;
   if (ns > 0) pp_anchor_k<<<ns, 256, 0, s>>>(A->danch, A->nrows, pbase, pdelta, ok);
}

void pp_encode(hipStream_t s, const amg_mat *A, const unsigned char *map, unsigned char *ppat,
               unsigned long long *counts)
{
   if (A->nrows <= 0) return;
   pp_encode_k<<<std::min(8192, (A->nrows + 511) / 512), 256, 0, s>>>(A->rpat, A->danch, A->nrows, map, ppat,
                                                                        counts);
}

void rp_collect(hipStream_t s, const amg_mat *A, unsigned long long *slots, int *rep, int nslots, int *count,
                int *bad)
{
   if (A->nrows <= 0) return;
   rp_collect_k<<<std::min(8192, (A->nrows + 255) / 256), 256, 0, s>>>(A->rowptr, A->didx, A->nrows, slots,
                                                                         rep, nslots, count, bad);
}

void rp_table(hipStream_t s, const amg_mat *A, const int *rep, int T, unsigned char *ptab)
{
   if (T > 0) rp_table_k<<<1, 256, 0, s>>>(A->rowptr, A->didx, rep, T, ptab);
}

void rp_encode(hipStream_t s, const amg_mat *A, const unsigned long long *keys, int T,
               const unsigned char *ptab, unsigned char *rpat, int *bad)
{
   if (A->nrows <= 0) return;
   rp_encode_k<<<std::min(8192, (A->nrows + 255) / 256), 256, 0, s>>>(A->rowptr, A->didx, A->nrows, keys, T,
                                                                        ptab, rpat, bad);
}

void dc_collect(hipStream_t s, const amg_mat *A, unsigned long long *slots, int nslots, int *count,
                int *maxlen)
{
   if (A->nrows <= 0) return;
   dc_collect_k<<<std::min(8192, (A->nrows + 255) / 256), 256, 0, s>>>(
      A->rowptr, A->col, A->vidx, A->nrows, slots, nslots, count, maxlen);
}

void dc_encode(hipStream_t s, const amg_mat *A, const unsigned long long *keys, int T,
               unsigned char *didx, int *anch)
{
   if (A->nrows <= 0) return;
   dc_encode_k<<<std::min(8192, (A->nrows + 255) / 256), 256, 0, s>>>(A->rowptr, A->col, A->vidx,
                                                                        A->nrows, keys, T, didx, anch);
}

__global__ void vi_collect_k(const double *__restrict__ val, long long nnz,
                             unsigned long long *slots, int nslots, int *count)
{
   unsigned long long last0 = VI_EMPTY, last1 = VI_EMPTY;
   const long long stride = (long long)gridDim.x * blockDim.x;
   for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nnz; i += stride) {
      const unsigned long long key = (unsigned long long)__double_as_longlong(val[i]);
      if (key == last0 || key == last1) continue;
      last1 = last0;
      last0 = key;
      if (key == VI_EMPTY) {
         atomicAdd(count, 1 << 20); // the sentinel pattern itself: give up on the table
         continue;
      }
      // more than 256 distinct values: the table is useless, stop probing
      // (a nearly full table would cost nslots probes per new value)
      if (__atomic_load_n(count, __ATOMIC_RELAXED) > 256) return;
      unsigned int h = vi_hash(key) & (nslots - 1);
      for (int probe = 0; probe < nslots; probe++) {
         const unsigned long long cur = __atomic_load_n(&slots[h], __ATOMIC_RELAXED);
         if (cur == key) break;
         if (cur == VI_EMPTY) {
            const unsigned long long prev = atomicCAS(&slots[h], VI_EMPTY, key);
            if (prev == VI_EMPTY) {
               atomicAdd(count, 1);
               break;
            }
            if (prev == key) break;
         }
         h = (h + 1) & (nslots - 1);
      }
   }
}

__global__ void vi_encode_k(const double *__restrict__ val, long long nnz,
                            const unsigned long long *__restrict__ keys, int T,
                            unsigned char *__restrict__ vidx)
{
   __shared__ unsigned long long tk[256];
   if (threadIdx.x < 256) tk[threadIdx.x] = threadIdx.x < T ? keys[threadIdx.x] : VI_EMPTY;
   __syncthreads();
   const long long stride = (long long)gridDim.x * blockDim.x;
   for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nnz; i += stride) {
      const unsigned long long key = (unsigned long long)__double_as_longlong(val[i]);
      int lo = 0, hi = T - 1;
      while (lo < hi) {
         const int mid = (lo + hi) >> 1;
         if (tk[mid] < key)
            lo = mid + 1;
         else
            hi = mid;
      }
      vidx[i] = (unsigned char)lo;
   }
}

void vi_collect(hipStream_t s, const double *val, long long nnz, unsigned long long *slots, int nslots,
                int *count)
{
   if (nnz <= 0) return;
   const long long nb = std::min<long long>(8192, (nnz + 255) / 256);
   vi_collect_k<<<(int)nb, 256, 0, s>>>(val, nnz, slots, nslots, count);
}

void vi_encode(hipStream_t s, const double *val, long long nnz, const unsigned long long *keys, int T,
               unsigned char *vidx)
{
   if (nnz <= 0) return;
   const long long nb = std::min<long long>(8192, (nnz + 255) / 256);
   vi_encode_k<<<(int)nb, 256, 0, s>>>(val, nnz, keys, T, vidx);
}

} // namespace amgk
