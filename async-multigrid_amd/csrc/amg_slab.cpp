// amg_slab.cpp -- z-slab hierarchies of the structured problem
// (amg_dist_hier_create_slab): config 4's multi-GPU path with the single-GPU
// kernels.
//
// Every rank owns planes [za, zb) of every distributed level's nx * ny * nz
// box (level-0 planes split evenly, coarse plane K with the owner of fine
// plane 2K + 1, amg_dist.cpp structured_planes).  Its operators are the
// EXTENDED slab operators: the rows of the owned planes with their global
// entries in their global order, plus up to two ghost planes on either side
// (diagonal-only rows of A, empty rows of P / R) -- square 7-pt / 27-pt box
// operators of zb - za + glo + ghi planes, so the compressed forms, the plane
// march (csr_mz_kernel / csr_mz27_kernel over the owned planes), the
// geometric transfers and the fused level-0 residual + restriction of one GPU
// run on them unchanged.  Every row sums its entries in its global CSR order:
// the iterate is bit-identical to one GPU's and to the oracle's.
//
// The ghost planes are contiguous: the exchange is two RCCL send / receive
// pairs of whole planes with the neighbouring ranks (no pack kernel), on the
// communication stream while the compute stream runs the planes that read no
// ghost (DMEM's finestIntra ghost exchange, DMEM_Comm.cpp:81-348 /
// CreateCommData_LocalRes DMEM_Setup.cpp:666-1265, and hypre's ParCSR halo
// inside hypre_ParCSRMatrixMatvec).  The cycle is SMEM_Sync_Parfor_Vcycle
// (SMEM_Sync_AMG.cpp:8-145) with SMEM_Solve's outer loop (SMEM_Solve.cpp:128-240).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "amg_dist_internal.h"

using namespace amgd;

int amg_gen_register_ext(amg_ctx *ctx, const amg_gen *g, int which, int level, int e0, int e1, int o0, int o1,
                         int ce0, int ce1, amg_mat **out);

namespace {

constexpr int SLAB_GHOST = 2; // ghost planes allocated on either side (the fused kernel reads two above)

SlabGeom geom_of(const amg_gen *g, int l, const std::vector<int> &zp, int r)
{
   SlabGeom s;
   amg_gen_dims(g, l, &s.nx, &s.ny, &s.nz);
   s.P = (long long)s.nx * s.ny;
   s.za = zp[r];
   s.zb = zp[r + 1];
   s.glo = std::min(SLAB_GHOST, s.za);
   s.ghi = std::min(SLAB_GHOST, s.nz - s.zb);
   return s;
}

// column planes read by the owned rows (planes [a, b)) of operator `which` of
// level l: the first and last planes' rows bound them (columns are monotone
// in the row plane for the box operators)
int col_planes(const amg_gen *g, int which, int l, int a, int b, int &cmin, int &cmax)
{
   const int cl = which == AMG_GEN_P ? l + 1 : l;
   int cx, cy, cz;
   amg_gen_dims(g, cl, &cx, &cy, &cz);
   const long long cP = (long long)cx * cy;
   cmin = 1 << 30;
   cmax = -1;
   for (int z : {a, b - 1}) {
      const long long nnz = amg_gen_nnz(g, which, l, z, z + 1);
      AMG_ARG(nnz >= 0, "amg_dist_hier_create_slab: %s", amg_last_error());
      int rx, ry, rz;
      amg_gen_dims(g, which == AMG_GEN_R ? l + 1 : l, &rx, &ry, &rz);
      std::vector<int> rp((size_t)rx * ry + 1), cj(std::max(1LL, nnz));
      std::vector<double> cv(std::max(1LL, nnz));
      AMG_TRY(amg_gen_fill(g, which, l, z, z + 1, rp.data(), cj.data(), cv.data(), 0));
      for (long long k = 0; k < nnz; k++) {
         cmin = std::min(cmin, (int)(cj[k] / cP));
         cmax = std::max(cmax, (int)(cj[k] / cP));
      }
   }
   return AMG_OK;
}

// ghost planes per rank of operator `which` at level l: rows on planes zr[l'],
// columns owned zc[l'']
int op_needs(const amg_gen *g, int which, int l, const std::vector<int> &zr, const std::vector<int> &zc,
             std::vector<int> &nlo, std::vector<int> &nhi)
{
   const int R = (int)zr.size() - 1;
   nlo.assign(R, 0);
   nhi.assign(R, 0);
   for (int r = 0; r < R; r++) {
      if (zr[r + 1] <= zr[r]) continue;
      int cmin, cmax;
      AMG_TRY(col_planes(g, which, l, zr[r], zr[r + 1], cmin, cmax));
      nlo[r] = std::max(0, zc[r] - cmin);
      nhi[r] = std::max(0, cmax + 1 - zc[r + 1]);
   }
   return AMG_OK;
}

// a slab operator: rows = planes of rg (extended unless rows_owned_only),
// columns = the extended planes of cg, or the whole column box (cfull)
int slab_mat(amg_dist_hier *D, const amg_gen *g, int which, int l, const SlabGeom &rg, bool rows_owned_only,
             const SlabGeom &cg, bool cfull, DistMat &M)
{
   const int re0 = rows_owned_only ? rg.za : rg.e0();
   const int re1 = rows_owned_only ? rg.zb : rg.zb + rg.ghi;
   const int ce0 = cfull ? 0 : cg.e0();
   const int ce1 = cfull ? cg.nz : cg.zb + cg.ghi;
   AMG_TRY(amg_gen_register_ext(D->ctx, g, which, l, re0, re1, rg.za, rg.zb, ce0, ce1, &M.A));
   M.slab = true;
   M.row0 = (long long)rg.za * rg.P;
   M.nrows = (int)((long long)rg.nzl() * rg.P);
   M.sro = rows_owned_only ? 0 : rg.off();
   M.sco = cfull ? 0 : cg.off();
   M.cP = cg.P;
   M.ncol_own = (int)(cfull ? (long long)cg.nz * cg.P : (long long)cg.nzl() * cg.P);
   M.replicated_cols = cfull;
   M.b0 = 0;
   M.b1 = M.nrows;
   return AMG_OK;
}

// weights of the geometric transfers of level l (R's row at coarse (1, 1, 1))
int geo_weights(const amg_gen *g, int l, amgk::GeoT &t, bool *ok)
{
   *ok = false;
   int nx, ny, nz;
   amg_gen_dims(g, l, &nx, &ny, &nz);
   if ((nx | ny | nz) & 1 || nx < 6 || ny < 6 || nz < 6) return AMG_OK;
   int cx, cy, cz;
   amg_gen_dims(g, l + 1, &cx, &cy, &cz);
   if (cx * 2 != nx || cy * 2 != ny || cz * 2 != nz) return AMG_OK;
   const long long nnz = amg_gen_nnz(g, AMG_GEN_R, l, 1, 2);
   AMG_ARG(nnz >= 0, "amg_dist_hier_create_slab: %s", amg_last_error());
   std::vector<int> rp((size_t)cx * cy + 1), cj(std::max(1LL, nnz));
   std::vector<double> cv(std::max(1LL, nnz));
   AMG_TRY(amg_gen_fill(g, AMG_GEN_R, l, 1, 2, rp.data(), cj.data(), cv.data(), 0));
   const int row = 1 * cx + 1;
   if (rp[row + 1] - rp[row] != 27) return AMG_OK;
   for (int k = 0; k < 27; k++) t.w[k] = cv[rp[row] + k];
   t.nx = nx;
   t.ny = ny;
   t.nz = nz;
   *ok = true;
   return AMG_OK;
}

long long tiles(long long n) { return (n + 255) / 256; }

} // namespace

// ---------------------------------------------------------------------------
// exchange and slab operator launches
// ---------------------------------------------------------------------------
int amgd::slab_xchg(amg_ctx *c, hipStream_t s, double *x, long long n_own, long long cP, const std::vector<int> &nlo,
                    const std::vector<int> &nhi)
{
   const int me = c->xport->rank, R = c->xport->nranks;
   int peers[2];
   void *sp[2], *rp[2];
   long long sb[2], rb[2];
   int np = 0;
   if (me > 0) {
      // my lowest planes -> the upper ghosts of rank me - 1; my lower ghosts <- its top planes
      peers[np] = me - 1;
      sp[np] = x;
      sb[np] = (long long)nhi[me - 1] * cP * 8;
      rp[np] = x - (long long)nlo[me] * cP;
      rb[np] = (long long)nlo[me] * cP * 8;
      if (sb[np] || rb[np]) np++;
   }
   if (me < R - 1) {
      peers[np] = me + 1;
      sp[np] = x + n_own - (long long)nlo[me + 1] * cP;
      sb[np] = (long long)nlo[me + 1] * cP * 8;
      rp[np] = x + n_own;
      rb[np] = (long long)nhi[me] * cP * 8;
      if (sb[np] || rb[np]) np++;
   }
   return xp_p2p(c, s, np, peers, sp, sb, rp, rb);
}

void amgd::slab_spgemv(hipStream_t s, const DistMat &M, const double *x, const double *b, const amgk::Gemv &g,
                       double *y, long long rb, long long re, double *partials)
{
   amgk::spgemv(s, M.A, x - M.sco, b ? b - M.sro : nullptr, g, y - M.sro, (int)(M.sro + rb),
                (int)(M.sro + re), partials);
}

void amgd::slab_jacobi(hipStream_t s, const DistMat &M, const double *f, const double *x, const double *l1,
                       double omega, double *out, long long rb, long long re)
{
   amgk::jacobi_sweep(s, M.A, f - M.sro, x - M.sco, l1 ? l1 - M.sro : nullptr, omega, out - M.sro,
                      (int)(M.sro + rb), (int)(M.sro + re));
}

const double *amgd::slab_diag(const DistMat &M) { return M.A->diag + M.sro; }

namespace {

// RCCL exchange of x's ghost planes on the communication stream, ordered
// after everything the compute stream issued before (no pack kernel: the
// planes are contiguous); the caller waits on D->ev_comm
int xchg_begin(amg_dist_hier *D, double *x, const DistMat &M)
{
   amg_ctx *c = D->ctx;
   AMG_HIP(hipEventRecord(D->ev_pack, c->stream));
   AMG_HIP(hipStreamWaitEvent(c->comm_stream, D->ev_pack, 0));
   AMG_TRY(slab_xchg(c, c->comm_stream, x, M.ncol_own, M.cP, M.nlo, M.nhi));
   AMG_HIP(hipEventRecord(D->ev_comm, c->comm_stream));
   return AMG_OK;
}

// a square slab operator (reach one plane): the owned planes that read no
// ghost first, overlapping the exchange, then the one or two boundary planes.
// launch(rb, re, partial offset) on owned rows; the norm partials of the
// segments are laid out bottom plane, interior, top plane (*nparts in total)
template <class F>
int split_A(amg_dist_hier *D, const DistMat &M, double *x, F launch, long long *nparts = nullptr)
{
   const int me = D->ctx->xport->rank;
   const long long P = M.cP, n = M.nrows;
   const bool lo = M.nlo[me] > 0, hi = M.nhi[me] > 0;
   if (!lo && !hi) {
      launch(0LL, n, 0LL);
      if (nparts) *nparts = tiles(n);
      return AMG_OK;
   }
   AMG_TRY(xchg_begin(D, x, M));
   const long long i0 = lo ? P : 0, i1 = hi ? n - P : n;
   const long long t_lo = lo ? tiles(P) : 0, t_in = i1 > i0 ? tiles(i1 - i0) : 0;
   if (i1 > i0) launch(i0, i1, t_lo);
   AMG_HIP(hipStreamWaitEvent(D->ctx->stream, D->ev_comm, 0));
   if (lo) launch(0LL, P, 0LL);
   if (hi) launch(n - P, n, t_lo + t_in);
   if (nparts) *nparts = t_lo + t_in + (hi ? tiles(P) : 0);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

struct SProf {
   amg_dist_hier *D;
   int cat;
   bool on;
   hipEvent_t a = nullptr, b = nullptr;
   SProf(amg_dist_hier *D_, int cat_, bool en) : D(D_), cat(cat_), on(en && D_->o.profile)
   {
      if (on) {
         hipEventCreate(&a);
         hipEventCreate(&b);
         hipEventRecord(a, D->ctx->stream);
      }
   }
   ~SProf()
   {
      if (on) {
         hipEventRecord(b, D->ctx->stream);
         D->pend[cat].push_back({a, b});
      }
   }
};

bool s_reuse(const amg_dist_hier *D)
{
   return D->o.reuse_outer_residual && D->o.num_pre_smooth_sweeps > 0 && !dist_mult_accel(D);
}

// the slab levels' zero-guess sweeps folded into their restrictions (as the
// single-GPU V-cycle does; AMG_ZG_FOLD_SLAB=0 turns it off)
bool zg_fold_on()
{
   static const bool on = [] {
      const char *e = std::getenv("AMG_ZG_FOLD_SLAB");
      return e ? std::atoi(e) != 0 : true;
   }();
   return on;
}

int s_smooth(amg_dist_hier *D, int l, const double *f, int sweeps, bool allow_reuse)
{
   DLevel &v = D->lv[l];
   hipStream_t s = D->ctx->stream;
   const bool l1 = D->o.smoother == AMG_L1_JACOBI;
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && v.zero_flag == 1) {
         if (v.zero_done)
            v.zero_done = false; // folded into the restriction that produced f (same bits)
         else
            amgk::jacobi_zero(s, slab_diag(v.A), f, l1 ? v.l1 : nullptr, D->o.smooth_weight, v.u, 0, v.n, 0);
      } else if (k == 0 && allow_reuse && D->pre_ready) {
         std::swap(v.u, v.u_alt);
         D->pre_ready = false;
      } else {
         SProf pr(D, 1, l == 0);
         double *x = v.u, *out = v.u_alt;
         AMG_TRY(split_A(D, v.A, x, [&](long long rb, long long re, long long) {
            slab_jacobi(s, v.A, f, x, l1 ? v.l1 : nullptr, D->o.smooth_weight, out, rb, re);
         }));
         std::swap(v.u, v.u_alt);
      }
   }
   return AMG_OK;
}

// coarse planes of level 1 whose fused residual + restriction reads only owned
// u / f planes of level 0 (fine planes 2K - 1 .. 2K + 3 within the box)
void rr_interior(const amg_dist_hier *D, int &k0, int &k1)
{
   const DLevel &v = D->lv[0];
   const int za = v.sg.za, zb = v.sg.zb, nz = v.sg.nz;
   k0 = v.Ka;
   k1 = v.Kb;
   while (k0 < k1 && std::max(0, 2 * k0 - 1) < za) k0++;
   while (k1 > k0 && std::min(nz - 1, 2 * (k1 - 1) + 3) >= zb) k1--;
}

// fused level-0 residual + restriction f_1 = R_0 (f - A_0 u) on the owned
// coarse planes (dst: level 1's owned rows, or the allgather slot; dcz0 its
// first coarse plane), overlapping u's exchange with the interior planes
int s_res_restrict(amg_dist_hier *D, const double *f, double *u, double *dst, int dcz0,
                   amgk::ZeroGuess zg = amgk::ZeroGuess())
{
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   DLevel &v = D->lv[0];
   const int me = c->xport->rank;
   const SlabGeom &sg = v.sg;
   auto run = [&](int K0, int K1) {
      if (K1 > K0)
         amgk::mz_residual_restrict(s, v.A.A, f - sg.off(), u - sg.off(), v.g, v.d_geo_w, dst, K0, K1, sg.e0(),
                                    dcz0, zg);
   };
   if (D->rr_ulo[me] == 0 && D->rr_uhi[me] == 0 && c->xport->nranks == 1) {
      run(v.Ka, v.Kb);
      return AMG_OK;
   }
   static const int no_overlap = std::getenv("AMG_SLAB_NO_OVERLAP") ? std::atoi(std::getenv("AMG_SLAB_NO_OVERLAP")) : 0;
   if (no_overlap) {
      AMG_TRY(slab_xchg(c, s, u, v.n, sg.P, D->rr_ulo, D->rr_uhi));
      if (no_overlap == 2) AMG_TRY(slab_xchg(c, s, const_cast<double *>(f), v.n, sg.P, D->rr_flo, D->rr_fhi));
      run(v.Ka, v.Kb);
      return AMG_OK;
   }
   AMG_HIP(hipEventRecord(D->ev_pack, s));
   AMG_HIP(hipStreamWaitEvent(c->comm_stream, D->ev_pack, 0));
   AMG_TRY(slab_xchg(c, c->comm_stream, u, v.n, sg.P, D->rr_ulo, D->rr_uhi));
   AMG_HIP(hipEventRecord(D->ev_comm, c->comm_stream));
   int k0, k1;
   rr_interior(D, k0, k1);
   run(k0, k1);
   AMG_HIP(hipStreamWaitEvent(s, D->ev_comm, 0));
   if (k1 > k0) {
      run(v.Ka, k0);
      run(k1, v.Kb);
   } else {
      run(v.Ka, v.Kb);
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

// restricted residual at the first replicated level: every rank's owned
// coarse rows (slot) allgathered and scattered into the full vector f_rep
int s_gather(amg_dist_hier *D, hipStream_t s, double *slot, double *gath, double *full)
{
   amg_ctx *c = D->ctx;
   const int R = c->xport->nranks;
   AMG_TRY(xp_allgather(c, s, slot, gath, (long long)D->gath_blk * 8));
   launch_scatter_blocks(s, gath, D->gath_blk, D->d_gcnt, D->d_gdsp, R, full);
   return AMG_OK;
}

} // namespace

// ---------------------------------------------------------------------------
// transfers (sync and async paths)
// ---------------------------------------------------------------------------
int amgd::slab_restrict(amg_dist_hier *D, hipStream_t s, int l, double *r, double *dst, const XchgFn &xchg,
                        amgk::ZeroGuess zg)
{
   DLevel &v = D->lv[l];
   DistMat &M = v.R;
   const bool to_rep = l + 1 >= D->Ld;
   if (!M.replicated_cols) AMG_TRY(xchg(r, M.ncol_own, M.cP, M.nlo, M.nhi));
   if (v.geo) {
      const long long coff = to_rep ? 0 : D->lv[l + 1].sg.off();
      const int cz0 = to_rep ? v.Ka : D->lv[l + 1].sg.e0();
      if (zg.u) { // the ZeroGuess vectors are indexed like dst (level l + 1's owned rows)
         zg.d -= coff;
         zg.u -= coff;
         zg.lo += coff;
         if (zg.hi >= 0) zg.hi += coff;
      }
      amgk::geo_restrict(s, v.g, v.d_geo_w, r - v.sg.off(), dst - coff, v.Ka, v.Kb, v.sg.e0(), cz0, zg);
   } else {
      slab_spgemv(s, M, r, nullptr, amgk::gemv_mode(1.0, 0.0), dst, 0, M.nrows, nullptr);
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int amgd::slab_prolong(amg_dist_hier *D, hipStream_t s, int l, double *x, double *out, bool add,
                       const XchgFn &xchg)
{
   DLevel &v = D->lv[l];
   DistMat &M = v.P;
   const bool from_rep = l + 1 >= D->Ld;
   if (!M.replicated_cols) AMG_TRY(xchg(x, M.ncol_own, M.cP, M.nlo, M.nhi));
   if (v.geo) {
      if (!add) amgk::vset(s, out, 0.0, 0, v.n);
      const long long coff = from_rep ? 0 : D->lv[l + 1].sg.off();
      const int cz0 = from_rep ? 0 : D->lv[l + 1].sg.e0();
      amgk::geo_prolong(s, v.g, v.d_geo_w, x - coff, out - v.sg.off(), v.sg.za, v.sg.zb, v.sg.e0(), cz0);
   } else {
      slab_spgemv(s, M, x, add ? out : nullptr, amgk::gemv_mode(1.0, add ? 1.0 : 0.0), out, 0, M.nrows, nullptr);
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// synchronous cycle
// ---------------------------------------------------------------------------
int amgd::slab_vcycle(amg_dist_hier *D, bool precond)
{
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   const int L = D->L, Ld = D->Ld;
   const amgk::Gemv res_mode = amgk::gemv_mode(-1.0, 1.0);
   XchgFn xchg = [&](double *x, long long n, long long cP, const std::vector<int> &lo,
                     const std::vector<int> &hi) { return slab_xchg(c, s, x, n, cP, lo, hi); };
   const int R = c->xport->nranks;
   double *slot = D->gath_buf ? D->gath_buf + (size_t)D->gath_blk * R : nullptr;
   // a fold flag set by an earlier cycle that returned early (an error between
   // the restriction and the level's smoothing) must not skip this cycle's sweep
   for (auto &lv : D->lv) lv.zero_done = false;
   for (int l = 0; l < Ld && l < L - 1; l++) {
      DLevel &v = D->lv[l];
      double *fl = (l == 0 && precond) ? D->r0 : v.f;
      v.zero_flag = (l == 0 && !precond) ? 0 : 1;
      AMG_TRY(s_smooth(D, l, fl, D->o.num_pre_smooth_sweeps, l == 0 && s_reuse(D)));
      const bool to_rep = l + 1 == Ld;
      double *dst = to_rep ? slot : D->lv[l + 1].f;
      // a slab level l + 1 (not the coarsest) starts its pre-smoothing with the
      // zero-guess sweep u = w f / a: a geometric restriction writes it with f
      // (as the single-GPU V-cycle does, amg_solver.cpp vcycle)
      amgk::ZeroGuess zg;
      if (!to_rep && l + 1 < L - 1 && D->o.smoother == AMG_JACOBI && D->o.num_pre_smooth_sweeps >= 1 &&
          zg_fold_on()) {
         // the fold writes u_{l+1} / reads a_ii on the coarse rows both
         // restrictions write: owned coarse planes [Ka, Kb) of level l + 1,
         // indexed from its first owned row -- the level's own rows exactly
         const DLevel &nx = D->lv[l + 1];
         AMG_ARG(nx.sg.za == v.Ka && nx.sg.zb == v.Kb && (long long)nx.n == (long long)(v.Kb - v.Ka) * nx.sg.P &&
                    nx.A.sro >= 0 && nx.A.sro + nx.n <= (long long)nx.A.A->nrows,
                 "slab zero-guess fold: level %d owns planes [%d, %d) (%d rows, diag rows [%lld, +%d) of %d), "
                 "the restriction writes [%d, %d)",
                 l + 1, nx.sg.za, nx.sg.zb, nx.n, nx.A.sro, nx.n, nx.A.A->nrows, v.Ka, v.Kb);
         zg.d = slab_diag(nx.A);
         zg.w = D->o.smooth_weight;
         zg.u = nx.u;
         zg.hi = nx.n;
         zg.err = c->d_err;
      }
      if (l == 0 && D->geo0) {
         SProf pr(D, 0, true);
         // the right-hand side's ghost planes: f's were exchanged at the solve's
         // start; the outer residual (preconditioner mode) changes every cycle
         if (precond) AMG_TRY(slab_xchg(c, s, fl, v.n, v.sg.P, D->rr_flo, D->rr_fhi));
         AMG_TRY(s_res_restrict(D, fl, v.u, dst, v.Ka, zg)); // dst: coarse plane Ka first
         // level l + 1 is a slab level only below Ld (to_rep: the replicated
         // tail, which has no DLevel -- D->lv holds Ld entries)
         if (!to_rep) D->lv[l + 1].zero_done = zg.u != nullptr;
      } else {
         {
            SProf pr(D, 0, l == 0);
            AMG_TRY(split_A(D, v.A, v.u, [&](long long rb, long long re, long long) {
               slab_spgemv(s, v.A, v.u, fl, res_mode, v.r_fine, rb, re, nullptr);
            }));
         }
         SProf pr(D, 2, l == 0);
         AMG_TRY(slab_restrict(D, s, l, v.r_fine, dst, xchg, v.geo ? zg : amgk::ZeroGuess()));
         if (!to_rep) D->lv[l + 1].zero_done = v.geo && zg.u != nullptr;
      }
      if (to_rep) AMG_TRY(s_gather(D, s, slot, D->gath_buf, D->f_rep));
   }
   const double *u_rep = nullptr;
   if (Ld < L) {
      AMG_TRY(amg_hier_subcycle(D->coarse, s, D->f_rep, &u_rep));
   } else {
      DLevel &v = D->lv[L - 1];
      const double *fl = (L == 1 && precond) ? D->r0 : v.f;
      AMG_TRY(s_smooth(D, L - 1, fl, D->o.num_pre_smooth_sweeps + D->o.num_post_smooth_sweeps, false));
   }
   for (int l = std::min(Ld, L - 1) - 1; l >= 0; l--) {
      DLevel &v = D->lv[l];
      v.zero_flag = 0;
      {
         SProf pr(D, 3, l == 0);
         double *xc = (l + 1 < Ld) ? D->lv[l + 1].u : const_cast<double *>(u_rep);
         AMG_TRY(slab_prolong(D, s, l, xc, v.u, true, xchg));
      }
      AMG_TRY(s_smooth(D, l, (l == 0 && precond) ? D->r0 : v.f, D->o.num_post_smooth_sweeps, false));
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int amgd::slab_outer_residual(amg_dist_hier *D, int slot)
{
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   DLevel &v = D->lv[0];
   long long np = 0;
   double *p;
   AMG_TRY(amg_ctx_partials(c, (size_t)tiles(v.n) + 8, &p));
   {
      SProf pr(D, 4, true);
      if (s_reuse(D) && D->L > 1) {
         const bool l1 = D->o.smoother == AMG_L1_JACOBI;
         double *r0 = (D->o.reuse_outer_residual >= 2 && D->o.solver == AMG_MULT) ? nullptr : D->r0;
         double *x = v.u, *un = v.u_alt;
         AMG_TRY(split_A(D, v.A, x, [&](long long rb, long long re, long long poff) {
            const DistMat &M = v.A;
            amgk::residual_jacobi(s, M.A, v.f - M.sro, x - M.sco, l1 ? v.l1 - M.sro : nullptr,
                                  D->o.smooth_weight, r0 ? r0 - M.sro : nullptr, un - M.sro,
                                  (int)(M.sro + rb), (int)(M.sro + re), p + poff);
         }, &np));
         D->pre_ready = true;
      } else {
         double *x = dist_iterate(D);
         AMG_TRY(split_A(D, v.A, x, [&](long long rb, long long re, long long poff) {
            slab_spgemv(s, v.A, x, v.f, amgk::gemv_mode(-1.0, 1.0), D->r0, rb, re, p + poff);
         }, &np));
         D->pre_ready = false;
      }
   }
   double *sum = D->d_hist + slot;
   amgk::reduce_partials(s, p, (int)np, sum, 0, c->d_scalars + 4096);
   AMG_TRY(xp_allreduce(c, s, sum, 1));
   launch_sqrt(s, sum, sum);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int amgd::slab_solve_begin(amg_dist_hier *D, const double *f_local)
{
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   for (auto &v : D->lv) {
      for (double *p : {v.f, v.u, v.u_alt, v.r_fine})
         amgk::vset(s, p - v.sg.off(), 0.0, 0, (int)v.sg.ext_rows());
      v.zero_flag = 0;
   }
   DLevel &v0 = D->lv[0];
   amgk::vset(s, D->r0 - v0.sg.off(), 0.0, 0, (int)v0.sg.ext_rows());
   AMG_TRY(h2d(s, v0.f, f_local, (size_t)v0.n * sizeof(double)));
   if (D->geo0) AMG_TRY(slab_xchg(c, s, v0.f, v0.n, v0.sg.P, D->rr_flo, D->rr_fhi));
   if (D->coarse) AMG_TRY(amg_hier_reset(D->coarse));
   if (D->x_acc) {
      amgk::vset(s, D->x_acc - v0.sg.off(), 0.0, 0, (int)v0.sg.ext_rows());
      amgk::vset(s, D->d_acc, 0.0, 0, std::max(1, v0.n));
   }
   D->acc.reset(D->o);
   D->iter = 0;
   AMG_TRY(slab_outer_residual(D, 0));
   AMG_TRY(d2h(s, c->h_pinned, D->d_hist, sizeof(double)));
   D->r0norm = c->h_pinned[0];
   D->have_state = true;
   return AMG_OK;
}

int amgd::slab_fine_spmv(amg_dist_hier *D, int reps, double *ms)
{
   amg_ctx *c = D->ctx;
   DLevel &v = D->lv[0];
   hipStream_t s = c->stream;
   hipEvent_t a, b;
   AMG_HIP(hipEventCreate(&a));
   AMG_HIP(hipEventCreate(&b));
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   AMG_HIP(hipEventRecord(a, s));
   for (int r = 0; r < reps; r++)
      AMG_TRY(split_A(D, v.A, v.u, [&](long long rb, long long re, long long) {
         slab_spgemv(s, v.A, v.u, nullptr, mv, v.r_fine, rb, re, nullptr);
      }));
   AMG_HIP(hipEventRecord(b, s));
   AMG_HIP(hipEventSynchronize(b));
   float t = 0.f;
   AMG_HIP(hipEventElapsedTime(&t, a, b));
   hipEventDestroy(a);
   hipEventDestroy(b);
   *ms = (double)t / reps;
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// construction
// ---------------------------------------------------------------------------
extern "C" int amg_dist_hier_create_slab(amg_ctx *c, const amg_gen *g, const amg_opts *opts, amg_dist_hier **out)
{
   AMG_ARG(c && c->xport && g && opts && out, "amg_dist_hier_create_slab: bad argument");
   AMG_TRY(dist_check_opts(opts));
   const int R = c->xport->nranks, me = c->xport->rank;
   const int L = amg_gen_num_levels(g);
   std::vector<std::vector<int>> zp;
   structured_planes(g, R, zp);
   auto D = std::make_unique<amg_dist_hier>();
   D->ctx = c;
   D->o = *opts;
   D->L = L;
   D->slab = true;
   D->part.rs.resize(L);
   for (int l = 0; l < L; l++) {
      int nx, ny, nz;
      amg_gen_dims(g, l, &nx, &ny, &nz);
      D->part.rs[l].resize(R + 1);
      for (int r = 0; r <= R; r++) D->part.rs[l][r] = (long long)zp[l][r] * nx * ny;
   }
   // distributed levels: every rank owns >= 2 planes (the fused kernel's two
   // ghost planes above come from one neighbour) and the level is not below
   // the replication threshold; at least level 0, at most L - 1 (the
   // coarsest is replicated)
   int Ld = L;
   for (int l = 0; l < L; l++) {
      bool ok = D->part.total(l) >= c->replicate_rows || l == 0;
      for (int r = 0; r < R && ok; r++) ok = zp[l][r + 1] - zp[l][r] >= 2;
      if (!ok) {
         Ld = l;
         break;
      }
   }
   AMG_ARG(Ld >= 1, "amg_dist_hier_create_slab: every rank needs at least 2 planes of level 0 (%d ranks, %lld planes)",
           R, (long long)(zp[0][R] - zp[0][0]));
   if (L > 1) Ld = std::min(Ld, L - 1);
   D->Ld = Ld;
   D->lv.resize(Ld);
   AMG_HIP(hipEventCreateWithFlags(&D->ev_pack, hipEventDisableTiming));
   AMG_HIP(hipEventCreateWithFlags(&D->ev_comm, hipEventDisableTiming));
   for (int l = 0; l < Ld; l++) {
      DLevel &v = D->lv[l];
      v.sg = geom_of(g, l, zp[l], me);
      v.row0 = (long long)v.sg.za * v.sg.P;
      v.n = (int)((long long)v.sg.nzl() * v.sg.P);
   }
   if (Ld < L) D->sg_rep = geom_of(g, Ld, zp[Ld], me);
   for (int l = 0; l < Ld; l++) {
      DLevel &v = D->lv[l];
      AMG_TRY(slab_mat(D.get(), g, AMG_GEN_A, l, v.sg, false, v.sg, false, v.A));
      AMG_TRY(op_needs(g, AMG_GEN_A, l, zp[l], zp[l], v.A.nlo, v.A.nhi));
      for (int r = 0; r < R; r++)
         AMG_ARG(v.A.nlo[r] <= 1 && v.A.nhi[r] <= 1, "amg_dist_hier_create_slab: A_%d reaches beyond one plane", l);
      if (l < L - 1) {
         const bool rep = l + 1 >= Ld;
         const SlabGeom &cg = rep ? D->sg_rep : D->lv[l + 1].sg;
         AMG_TRY(slab_mat(D.get(), g, AMG_GEN_P, l, v.sg, false, cg, rep, v.P));
         if (!rep) AMG_TRY(op_needs(g, AMG_GEN_P, l, zp[l], zp[l + 1], v.P.nlo, v.P.nhi));
         AMG_TRY(slab_mat(D.get(), g, AMG_GEN_R, l, cg, rep, v.sg, false, v.R));
         AMG_TRY(op_needs(g, AMG_GEN_R, l, zp[l + 1], zp[l], v.R.nlo, v.R.nhi));
         v.Ka = cg.za;
         v.Kb = cg.zb;
      }
      // ghost planes come from the neighbouring ranks' owned planes only
      for (int which = 0; which < 3; which++) {
         const DistMat &M = which == 0 ? v.A : which == 1 ? v.P : v.R;
         if (!M.A || M.replicated_cols) continue;
         const std::vector<int> &zc = zp[which == 1 ? l + 1 : l];
         for (int r = 0; r < R; r++) {
            const int below = r > 0 ? zc[r] - zc[r - 1] : 0, above = r < R - 1 ? zc[r + 2] - zc[r + 1] : 0;
            AMG_ARG(M.nlo[r] <= std::min(SLAB_GHOST, below) && M.nhi[r] <= std::min(SLAB_GHOST, above),
                    "amg_dist_hier_create_slab: level %d operator %d of rank %d reads %d / %d ghost planes", l,
                    which, r, M.nlo[r], M.nhi[r]);
         }
      }
      AMG_TRY(lvec(D.get(), l, &v.f));
      AMG_TRY(lvec(D.get(), l, &v.u));
      AMG_TRY(lvec(D.get(), l, &v.u_alt));
      AMG_TRY(lvec(D.get(), l, &v.r_fine));
      AMG_TRY(lvec(D.get(), l, &v.l1));
      amgk::l1_norms(c->stream, v.A.A, v.l1 - v.sg.off());
      v.cap = v.n;
   }
   // geometric transfers: R_l / P_l checked entry for entry against the box
   // form on every rank's rows (all ranks agree through a sum of the flags)
   {
      int *bad = nullptr;
      AMG_HIP(hipMalloc(&bad, sizeof(int) * std::max(1, Ld)));
      AMG_HIP(hipMemsetAsync(bad, 0, sizeof(int) * std::max(1, Ld), c->stream));
      std::vector<char> cand(Ld, 0);
      for (int l = 0; l < Ld && l < L - 1; l++) {
         DLevel &v = D->lv[l];
         bool ok = false;
         AMG_TRY(geo_weights(g, l, v.g, &ok));
         if (!ok || !c->fuse_transfer) continue;
         cand[l] = 1;
         const bool rep = l + 1 >= Ld;
         const SlabGeom &cg = rep ? D->sg_rep : D->lv[l + 1].sg;
         const long long cbase = rep ? 0 : (long long)cg.e0() * cg.P;
         amgk::geo_check(c->stream, v.P.A, 1, v.g, bad + l, (int)v.P.sro, (int)(v.P.sro + v.P.nrows),
                         (long long)v.sg.e0() * v.sg.P, cbase);
         amgk::geo_check(c->stream, v.R.A, 0, v.g, bad + l, (int)v.R.sro, (int)(v.R.sro + v.R.nrows),
                         (long long)(rep ? cg.za : cg.e0()) * cg.P, (long long)v.sg.e0() * v.sg.P);
      }
      std::vector<int> hb(std::max(1, Ld));
      AMG_HIP(hipMemcpyAsync(hb.data(), bad, sizeof(int) * hb.size(), hipMemcpyDeviceToHost, c->stream));
      AMG_HIP(hipStreamSynchronize(c->stream));
      hipFree(bad);
      std::vector<double> flags(std::max(1, Ld));
      for (int l = 0; l < Ld; l++) flags[l] = cand[l] && !hb[l] ? 0.0 : 1.0;
      AMG_TRY(amg_dist_allreduce_sum(c, flags.data(), (int)flags.size()));
      for (int l = 0; l < Ld && l < L - 1; l++) {
         DLevel &v = D->lv[l];
         v.geo = flags[l] == 0.0;
         if (v.geo) {
            AMG_TRY(dvec(D.get(), 27, &v.d_geo_w));
            AMG_TRY(h2d(c->stream, v.d_geo_w, v.g.w, sizeof(v.g.w)));
         }
      }
   }
   // fused level-0 residual + restriction (the single-GPU conditions)
   if (Ld >= 1 && L > 1 && D->lv[0].geo) {
      DLevel &v = D->lv[0];
      const amg_mat *A = v.A.A;
      const amgk::GeoT &gg = v.g;
      D->geo0 = A->mz_P && !A->mz27 && A->mz_S == gg.nx && gg.nx >= 64 && gg.nx <= 512 && 512 % gg.nx == 0 &&
                (gg.ny / 2) % (512 / gg.nx) == 0;
      if (D->geo0) {
         // u planes 2K - 1 .. 2K + 3 and f planes 2K .. 2K + 2 of the owned
         // coarse planes K (within the box), per rank
         D->rr_ulo.assign(R, 0);
         D->rr_uhi.assign(R, 0);
         D->rr_flo.assign(R, 0);
         D->rr_fhi.assign(R, 0);
         const int nz = gg.nz;
         for (int r = 0; r < R; r++) {
            const int za = zp[0][r], zb = zp[0][r + 1], Ka = zp[1][r], Kb = zp[1][r + 1];
            if (Kb <= Ka) continue;
            const int u0 = std::max(0, 2 * Ka - 1), u1 = std::min(nz - 1, 2 * (Kb - 1) + 3);
            const int f0 = 2 * Ka, f1 = std::min(nz - 1, 2 * (Kb - 1) + 2);
            D->rr_ulo[r] = std::max(0, za - u0);
            D->rr_uhi[r] = std::max(0, u1 + 1 - zb);
            D->rr_flo[r] = std::max(0, za - f0);
            D->rr_fhi[r] = std::max(0, f1 + 1 - zb);
            const int below = r > 0 ? zp[0][r] - zp[0][r - 1] : 0, above = r < R - 1 ? zp[0][r + 2] - zp[0][r + 1] : 0;
            if (D->rr_ulo[r] > std::min(SLAB_GHOST, below) || D->rr_uhi[r] > std::min(SLAB_GHOST, above))
               D->geo0 = false;
         }
      }
      // the fused composed prolongation reads P e on fine planes za - 1 .. zb
      // (the 7-pt stencil around the owned planes): coarse planes of level 1
      // from the first candidate of za - 1 to the last of zb
      D->xfp0 = D->geo0;
      if (D->xfp0 && Ld >= 2) {
         D->xp_lo.assign(R, 0);
         D->xp_hi.assign(R, 0);
         const int nz = gg.nz, ncz = nz / 2;
         for (int r = 0; r < R; r++) {
            const int za = zp[0][r], zb = zp[0][r + 1], Ka = zp[1][r], Kb = zp[1][r + 1];
            if (zb <= za) continue;
            int cmin = ncz, cmax = -1;
            for (int p = std::max(0, za - 1); p <= std::min(nz - 1, zb); p++) {
               if (p & 1) {
                  cmin = std::min(cmin, (p - 1) / 2), cmax = std::max(cmax, (p - 1) / 2);
               } else {
                  if (p >= 2) cmin = std::min(cmin, p / 2 - 1), cmax = std::max(cmax, p / 2 - 1);
                  if (p / 2 < ncz) cmin = std::min(cmin, p / 2), cmax = std::max(cmax, p / 2);
               }
            }
            if (cmax < 0) continue;
            D->xp_lo[r] = std::max(0, Ka - cmin);
            D->xp_hi[r] = std::max(0, cmax + 1 - Kb);
            const int below = r > 0 ? zp[1][r] - zp[1][r - 1] : 0, above = r < R - 1 ? zp[1][r + 2] - zp[1][r + 1] : 0;
            if (D->xp_lo[r] > std::min(SLAB_GHOST, below) || D->xp_hi[r] > std::min(SLAB_GHOST, above))
               D->xfp0 = false;
         }
      }
   }
   // replicated coarse levels
   if (Ld < L) {
      AMG_TRY(dist_build_replicated(D.get(), [&](int which, int level, amg_mat **m) {
         int nx, ny, nz;
         amg_gen_dims(g, which == AMG_GEN_R ? level + 1 : level, &nx, &ny, &nz);
         return amg_gen_register(c, g, which, level, 0, nz, m);
      }));
   }
   AMG_TRY(lvec(D.get(), 0, &D->r0));
   AMG_TRY(dvec(D.get(), D->hist_cap, &D->d_hist));
   if (D->o.solver == AMG_MULT && D->o.accel_type != AMG_NO_ACCEL) {
      AMG_TRY(lvec(D.get(), 0, &D->x_acc));
      AMG_TRY(dvec(D.get(), std::max(1, D->lv[0].n), &D->d_acc));
   }
   AMG_HIP(hipStreamSynchronize(c->stream));
   *out = D.release();
   return AMG_OK;
}

extern "C" int amg_dist_hier_slab_info(const amg_dist_hier *D, int *distributed_levels, int *geometric, int *fused)
{
   AMG_ARG(D, "amg_dist_hier_slab_info: null hierarchy");
   if (distributed_levels) *distributed_levels = D->slab ? D->Ld : 0;
   int m = 0;
   if (D->slab)
      for (int l = 0; l < D->Ld; l++)
         if (D->lv[l].geo) m |= 1 << l;
   if (geometric) *geometric = m;
   if (fused) *fused = D->slab && D->geo0 ? 1 : 0;
   return AMG_OK;
}
