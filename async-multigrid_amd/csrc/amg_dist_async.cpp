// amg_dist_async.cpp -- asynchronous additive AMG across GPUs.
//
// Reference: the DMEM asynchronous additive solver (DMEM_Add.cpp:20-178 driver,
// AddCycle :180-329, DMEM_AddCorrect_LocalRes :391-458, DMEM_AddCheckComm
// :460-528, DMEM_AddResidual_LocalRes :530-556; message engine DMEM_Comm.cpp)
// and its shared-memory form SMEM_Async_Add_AMG (SMEM_Async_AMG.cpp:7-437).
//
// MI355X mapping.  The reference gives every level ("grid k") its own group of
// MPI ranks holding a full copy of the fine problem and ships whole-vector
// corrections between the groups.  Here every GPU owns a z-slab of every level
// and every level k runs as its own HIP stream on every GPU:
//   * level k restricts its private residual down to level k, smooths there
//     (SMEM smoother semantics: zero-guess symmetric / L1 / weighted Jacobi),
//     prolongs back and adds the correction into the shared slab of u with
//     device-scope fp64 atomics -- the GPU-resident equivalent of the
//     gridjToGridk correction messages, without moving vectors between GPUs;
//   * it then recomputes its private residual f - A u_k from the value of u it
//     observed at its own update (LOCAL residual, SMEM_Async_AMG.cpp:284-301);
//   * every operator application of level k exchanges its ghost rows with the
//     neighbouring ranks through level k's OWN device-resident channels
//     (amg_link.cpp: the sender's copy kernel writes the ghost rows straight
//     into a slot of the receiver's memory, sequence words in host memory,
//     polled by the receiving level's host thread -- the MPI_Test analogue of
//     DMEM_Comm.cpp:81-348), and each level group runs its correction loop on
//     its own host thread: level k on rank r waits only for level k on the
//     ranks it exchanges with, as each DMEM grid does within its own
//     communicator, never for another level (no shared comm stream, no
//     head-of-line coupling; DMEM_Smooth.cpp:165-269 likewise moves ghost data
//     independently of the other message classes);
//   * levels below the replication threshold are computed redundantly on every
//     rank after an allgather of the restricted residual, also over level k's
//     channels.
// ASYNC_MULTADD may use the reference's smoothed transfers (smooth_transfer:
// P~ = (I - w D^-1 A) P, R~ = P~^T, SmoothTransfer SMEM_Setup.cpp:1173-1254),
// composed on the fly from the slab operators (R~ r = R (r - w A D^-1 r)).
// Termination: each level performs num_cycles corrections (LOCAL convergence,
// fixed count), then the threads join and the outer residual is formed.  A
// deterministic schedule (async_schedule) runs the level corrections on one
// host thread and one stream, in the oracle's order (bit-identical to
// or_async_add under or_set_async_schedule).
#include <algorithm>
#include <cmath>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "amg_dist_internal.h"

using namespace amgd;

namespace {

bool multadd_of(const amg_opts &o) { return o.solver == AMG_ASYNC_MULTADD || o.solver == AMG_MULTADD; }

int level_n(const amg_dist_hier *D, int l)
{
   return l < D->Ld ? D->lv[l].n : D->cA[l - D->Ld]->nrows;
}

int level_cap(const amg_dist_hier *D, int l)
{
   return l < D->Ld ? D->lv[l].cap : D->cA[l - D->Ld]->nrows;
}

// the level stream's exchange of a slab vector's ghost planes, through the
// comm stream (XchgFn of slab_restrict / slab_prolong)
XchgFn level_xchg(amg_dist_hier *D, AsyncLevel &a);

// hand the level stream's work to the comm stream (and back): the RCCL
// operation runs on c->comm_stream after everything level k issued before it
int to_comm(amg_dist_hier *D, AsyncLevel &a)
{
   AMG_HIP(hipEventRecord(a.ev_ready, a.s));
   AMG_HIP(hipStreamWaitEvent(D->ctx->comm_stream, a.ev_ready, 0));
   return AMG_OK;
}

int from_comm(amg_dist_hier *D, AsyncLevel &a)
{
   AMG_HIP(hipEventRecord(a.ev_done, D->ctx->comm_stream));
   AMG_HIP(hipStreamWaitEvent(a.s, a.ev_done, 0));
   return AMG_OK;
}

// ghost exchange of x for M: packed on the level stream; through the level's
// device-resident channels (D->links, the asynchronous solve) or, for the
// level-grouped solve's grid, sent / received on the comm stream
int a_halo(amg_dist_hier *D, AsyncLevel &a, DistMat &M, double *x)
{
   if (M.slab) {
      if (M.replicated_cols || D->ctx->xport->nranks == 1) return AMG_OK;
      return level_xchg(D, a)(x, M.ncol_own, M.cP, M.nlo, M.nhi);
   }
   if (M.replicated_cols || M.peers.empty()) return AMG_OK;
   double *&sb = a.sbuf[&M];
   if (!sb) {
      // the level groups' buffers are made by setup_async (a level thread must
      // not allocate: dvec appends to the hierarchy's list and zeroes on the
      // main stream); the grid's on first use, ordered before this stream
      AMG_ARG(a.k < 0, "a_halo: level %d has no send buffer for this operator", a.k);
      AMG_TRY(dvec(D, std::max<long long>(1, M.nsend), &sb));
      AMG_HIP(hipStreamSynchronize(D->ctx->stream));
   }
   launch_gather(a.s, x, M.d_send_idx, sb, (int)M.nsend);
   const int np = (int)M.peers.size();
   if (D->links && a.k >= 0) {
      for (int i = 0; i < np; i++)
         if (M.scnt[i] > 0) AMG_TRY(link_send(D->links, a.k, M.peers[i], sb + M.soff[i], M.scnt[i], a.s));
      for (int i = 0; i < np; i++)
         if (M.rcnt[i] > 0)
            AMG_TRY(link_recv(D->links, a.k, M.peers[i], x + M.ncol_own + M.roff[i], M.rcnt[i], a.s));
      return AMG_OK;
   }
   std::vector<void *> sp(np), rp(np);
   std::vector<long long> sbytes(np), rbytes(np);
   for (int i = 0; i < np; i++) {
      sp[i] = sb + M.soff[i];
      sbytes[i] = M.scnt[i] * 8;
      rp[i] = x + M.ncol_own + M.roff[i];
      rbytes[i] = M.rcnt[i] * 8;
   }
   AMG_TRY(to_comm(D, a));
   AMG_TRY(xp_p2p(D->ctx, D->ctx->comm_stream, np, M.peers.data(), sp.data(), sbytes.data(), rp.data(),
                  rbytes.data()));
   return from_comm(D, a);
}

int a_spgemv(amg_dist_hier *D, AsyncLevel &a, DistMat &M, double *x, const double *b,
             const amgk::Gemv &g, double *y)
{
   AMG_TRY(a_halo(D, a, M, x));
   if (M.slab)
      slab_spgemv(a.s, M, x, b, g, y, 0, M.nrows, nullptr);
   else
      amgk::spgemv(a.s, M.A, x, b, g, y, 0, M.nrows, nullptr);
   return AMG_OK;
}

XchgFn level_xchg(amg_dist_hier *D, AsyncLevel &a)
{
   return [D, &a](double *x, long long n, long long cP, const std::vector<int> &lo, const std::vector<int> &hi) {
      // one rank: no neighbour, nothing to exchange -- and no hop through the
      // shared comm stream, which would serialise the level streams
      if (D->ctx->xport->nranks == 1) return (int)AMG_OK;
      if (D->links && a.k >= 0) return link_xchg_planes(D->links, a.k, a.s, x, n, cP, lo, hi);
      AMG_TRY(to_comm(D, a));
      AMG_TRY(slab_xchg(D->ctx, D->ctx->comm_stream, x, n, cP, lo, hi));
      return from_comm(D, a);
   };
}

// y = A_l x (+ b per g) on level l
int apply_A(amg_dist_hier *D, AsyncLevel &a, int l, double *x, const double *b, const amgk::Gemv &g,
            double *y)
{
   if (l < D->Ld) return a_spgemv(D, a, D->lv[l].A, x, b, g, y);
   amgk::spgemv(a.s, D->cA[l - D->Ld], x, b, g, y, 0, level_n(D, l), nullptr);
   return AMG_OK;
}

const double *diag_of(const amg_dist_hier *D, int l)
{
   if (l < D->Ld) return D->slab ? slab_diag(D->lv[l].A) : D->lv[l].A.A->diag;
   return D->cA[l - D->Ld]->diag;
}

const double *l1_of(const amg_dist_hier *D, int l)
{
   return l < D->Ld ? D->lv[l].l1 : D->cl1[l - D->Ld];
}

// the MULTADD transfers are the smoothed ones, composed (smooth_transfer)
// (P~ only with post-smoothing, R~ only with pre-smoothing: SmoothTransfer,
// SMEM_Setup.cpp:1176-1180,1245-1250)
bool composed(const amg_dist_hier *D)
{
   return D->o.smooth_transfer == 1 && (D->o.solver == AMG_ASYNC_MULTADD || D->o.solver == AMG_MULTADD) &&
          (D->o.num_pre_smooth_sweeps > 0 || D->o.num_post_smooth_sweeps > 0);
}
static bool composed_r(const amg_dist_hier *D) { return composed(D) && D->o.num_pre_smooth_sweeps > 0; }
static bool composed_p(const amg_dist_hier *D) { return composed(D) && D->o.num_post_smooth_sweeps > 0; }

// the level-0 composed restriction as one fused pass: slab hierarchies whose
// level 0 runs the fused residual + restriction (geo0) with uniform values
bool fused_xfer0(const amg_dist_hier *D)
{
   return composed_r(D) && D->slab && D->geo0 && D->ctx->fuse_xfer && D->lv[0].A.A && D->lv[0].A.A->mp_uni;
}

// the level-0 composed prolongation as one fused pass (and, when asked, the
// FULL_ASYNC atomic correction with it): slab hierarchies whose level 0 runs
// the fused kernels and whose level-1 ghost needs fit (xfp0)
bool fused_xfp0(const amg_dist_hier *D)
{
   return composed_p(D) && D->slab && D->xfp0 && D->ctx->fuse_xfer && D->ctx->fuse_xfp_slab && D->lv[0].A.A;
}

// every rank's restricted rows (slot) into the replicated level's full vector
int gather_restricted(amg_dist_hier *D, AsyncLevel &a, double *slot, double *full)
{
   const int R = D->ctx->xport->nranks;
   if (R == 1 && a.k >= 0) {
      // one rank: the allgather is a copy (no transport: the level threads
      // must not share the communicator)
      amgk::vcopy(a.s, slot, a.gath, 0, D->gath_blk);
   } else if (D->links && a.k >= 0) {
      AMG_TRY(link_allgather(D->links, a.k, a.s, slot, a.gath, D->gath_blk));
   } else {
      AMG_TRY(to_comm(D, a));
      AMG_TRY(xp_allgather(D->ctx, D->ctx->comm_stream, slot, a.gath, (long long)D->gath_blk * 8));
      AMG_TRY(from_comm(D, a));
   }
   launch_scatter_blocks(a.s, a.gath, D->gath_blk, D->d_gcnt, D->d_gdsp, R, full);
   return AMG_OK;
}

// r[l+1] = R_l r[l] (SMEM_Sync_Parfor_Restrict / hypre MatvecT in AddCycle); with
// composed smoothed transfers R~_l r = R_l (r - w A_l D_l^-1 r): t = r ./ a;
// y = A t; t = r + (-w) y (the oracle's or_hier_set_composed_transfers order)
int restrict_to(amg_dist_hier *D, AsyncLevel &a, int l)
{
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   const int Ld = D->Ld;
   double *r = a.r[l];
   const int R = D->ctx->xport->nranks;
   double *slot = (l + 1 == Ld) ? a.gath + (size_t)D->gath_blk * R : nullptr;
   if (fused_xfer0(D) && l == 0) {
      // the composed restriction of the slab's level 0 in one pass (the fused
      // residual + restriction kernel's composed mode): r's ghost planes as
      // that kernel reads them, then coarse planes [Ka, Kb)
      DLevel &v = D->lv[0];
      if (R > 1) AMG_TRY(level_xchg(D, a)(r, v.n, v.sg.P, D->rr_ulo, D->rr_uhi));
      amgk::mz_xfer_restrict(a.s, v.A.A, r - v.sg.off(), v.g, v.d_geo_w, D->o.smooth_weight,
                             l + 1 < Ld ? a.r[1] : slot, v.Ka, v.Kb, v.sg.e0(), v.Ka);
      if (l + 1 < Ld) return AMG_OK;
      return gather_restricted(D, a, slot, a.r[l + 1]);
   }
   if (composed_r(D)) {
      const int n = level_n(D, l);
      amgk::xfer_div(a.s, diag_of(D, l), r, a.xt, 0, n);
      AMG_TRY(apply_A(D, a, l, a.xt, nullptr, mv, a.xy));
      amgk::xfer_sub(a.s, D->o.smooth_weight, r, a.xy, a.xt, 0, n);
      r = a.xt;
   }
   if (D->slab && l + 1 < Ld) return slab_restrict(D, a.s, l, r, a.r[l + 1], level_xchg(D, a));
   if (l + 1 < Ld) return a_spgemv(D, a, D->lv[l].R, r, nullptr, mv, a.r[l + 1]);
   if (l + 1 == Ld) {
      if (D->slab)
         AMG_TRY(slab_restrict(D, a.s, l, r, slot, level_xchg(D, a)));
      else
         AMG_TRY(a_spgemv(D, a, D->lv[l].R, r, nullptr, mv, slot));
      return gather_restricted(D, a, slot, a.r[l + 1]);
   }
   amgk::spgemv(a.s, D->cR[l - Ld], r, nullptr, mv, a.r[l + 1], 0, level_n(D, l + 1), nullptr);
   return AMG_OK;
}

// out = P_l x (x on level l+1, out on level l); composed smoothed transfers:
// out = P x;  y = A out;  out = out + (-w) (y ./ a)
int prolong_to(amg_dist_hier *D, AsyncLevel &a, int l, double *x, double *out, int apply = 0,
               double *u = nullptr, double *u_priv = nullptr, unsigned long long *stamp = nullptr)
{
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   if (l == 0 && fused_xfp0(D)) {
      // P~ e = P e - w (A P e) ./ a over the owned fine planes in one march
      // (mz_xfer_prolong): the coarse ghost planes it reads, then the kernel;
      // apply 1: the atomic correction of u (u_priv = the value after it)
      DLevel &v = D->lv[0];
      const bool from_rep = D->Ld < 2;
      long long coff = 0;
      int cz0 = 0;
      if (!from_rep) {
         const DLevel &c1 = D->lv[1];
         coff = c1.sg.off();
         cz0 = c1.sg.e0();
         if (D->ctx->xport->nranks > 1)
            AMG_TRY(level_xchg(D, a)(x, c1.n, c1.sg.P, D->xp_lo, D->xp_hi));
      }
      const long long off = v.sg.off();
      if (apply == 1)
         amgk::mz_xfer_prolong(a.s, v.A.A, x - coff, v.g, v.d_geo_w, D->o.smooth_weight, 1, u - off, u_priv - off,
                               v.sg.za, v.sg.zb, v.sg.e0(), cz0, stamp);
      else
         amgk::mz_xfer_prolong(a.s, v.A.A, x - coff, v.g, v.d_geo_w, D->o.smooth_weight, 0, out - off, nullptr,
                               v.sg.za, v.sg.zb, v.sg.e0(), cz0);
      return AMG_OK;
   }
   if (D->slab && l < D->Ld)
      AMG_TRY(slab_prolong(D, a.s, l, x, out, false, level_xchg(D, a)));
   else if (l < D->Ld)
      AMG_TRY(a_spgemv(D, a, D->lv[l].P, x, nullptr, mv, out));
   else
      amgk::spgemv(a.s, D->cP[l - D->Ld], x, nullptr, mv, out, 0, level_n(D, l), nullptr);
   if (composed_p(D)) {
      AMG_TRY(apply_A(D, a, l, out, nullptr, mv, a.xy));
      amgk::xfer_corr(a.s, D->o.smooth_weight, a.xy, diag_of(D, l), out, 0, level_n(D, l));
   }
   return AMG_OK;
}

// smooth_all_levels (amg_solver.cpp) on level l, zero initial guess (the add
// cycle sets zero_flags[k] = 1): symmetric Jacobi for MULTADD with pre and
// post sweeps (SMEM_Sync_Symmetric[L1]Jacobi, SMEM_Smooth.cpp:643-762, the
// DMEM_AddSmooth 2-step form DMEM_Smooth.cpp:574-638), else L1 / weighted
// Jacobi (SMEM_Sync_[L1]Jacobi :365-443).  u_prev / sy / sr: scratch with ghost room.
int a_smooth(amg_dist_hier *D, AsyncLevel &a, int l, const double *f, double *u, int sweeps)
{
   const amg_opts &o = D->o;
   hipStream_t s = a.s;
   const int n = level_n(D, l);
   const bool l1 = o.smoother == AMG_L1_JACOBI;
   const double omega = l1 ? 1.0 : o.smooth_weight;
   const double *l1v = l1 ? l1_of(D, l) : nullptr;
   const double *dg = diag_of(D, l);
   const bool sym = multadd_of(o) && o.num_post_smooth_sweeps > 0 && o.num_pre_smooth_sweeps > 0;
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   if (sweeps <= 0) return AMG_OK;
   if (sym) {
      // amg_sym_jacobi_dev with zero_first = 1, variant 0 (SMEM)
      amgk::vcopy(s, f, a.sr, 0, n);
      for (int k = 0;;) {
         amgk::sym_scale(s, dg, l1v, omega, a.sr, 0, n, 0);
         AMG_TRY(apply_A(D, a, l, a.sr, nullptr, mv, a.sy));
         amgk::sym_update(s, dg, l1v, omega, a.sr, a.sy, u, 0, n, 0, 1);
         if (++k == sweeps) break;
         AMG_TRY(apply_A(D, a, l, u, nullptr, mv, a.sy));
         amgk::vsub(s, f, a.sy, a.sr, 0, n);
      }
      return AMG_OK;
   }
   for (int k = 0; k < sweeps; k++) {
      if (k == 0) {
         amgk::jacobi_zero(s, dg, f, l1v, omega, u, 0, n, 0);
      } else {
         amgk::vcopy(s, u, a.u_prev, 0, n);
         if (l < D->Ld) {
            DistMat &M = D->lv[l].A;
            AMG_TRY(a_halo(D, a, M, a.u_prev));
            if (M.slab)
               slab_jacobi(s, M, f, a.u_prev, l1v, omega, u, 0, n);
            else
               amgk::jacobi_sweep(s, M.A, f, a.u_prev, l1v, omega, u, 0, n);
         } else {
            amgk::jacobi_sweep(s, D->cA[l - D->Ld], f, a.u_prev, l1v, omega, u, 0, n);
         }
      }
   }
   return AMG_OK;
}

// DMEM_Setup.cpp:1911-1913: cheby_grid is clamped to the last grid
int cheby_grid_of(const amg_dist_hier *D)
{
   return std::min(D->o.cheby_grid, (int)D->al.size() - 1);
}

// one correction of level k (SMEM_Async_Add_AMG inner body / DMEM AddCycle)
// j >= 0 (free race): record the correction's update point -- the atomic add
// into the shared slab, where it reads and writes the shared iterate -- as
// its end event (amg_dist_async_correction_ms)
int level_correction(amg_dist_hier *D, int k, int j = -1)
{
   AsyncLevel &a = D->al[k];
   const amg_opts &o = D->o;
   const int L = D->L;
   hipStream_t s = a.s;
   const bool multadd = multadd_of(o);
   const int coarsest = multadd ? k : k + 1;
   for (int l = 0; l < coarsest && l < L - 1; l++) AMG_TRY(restrict_to(D, a, l));
   if (multadd) {
      amgk::vset(s, a.e[k], 0.0, 0, level_n(D, k));
      AMG_TRY(a_smooth(D, a, k, a.r[k], a.e[k], o.num_fine_smooth_sweeps));
   } else {
      // AFACx (SMEM_Sync_AMG.cpp:296-406 per level): coarse smooth, prolong,
      // fine residual, fine smooth
      const int fg = k, cg = k + 1;
      const int nf = level_n(D, fg), nc = level_n(D, cg);
      amgk::vset(s, a.uf, 0.0, 0, nf);
      amgk::vset(s, a.uc, 0.0, 0, nc);
      AMG_TRY(a_smooth(D, a, cg, a.r[cg], a.uc, o.num_coarse_smooth_sweeps));
      AMG_TRY(prolong_to(D, a, fg, a.uc, a.e[fg]));
      AMG_TRY(apply_A(D, a, fg, a.e[fg], nullptr, amgk::gemv_mode(1.0, 0.0), a.sy));
      amgk::vsub(s, a.r[fg], a.sy, a.rf, 0, nf);
      AMG_TRY(a_smooth(D, a, fg, a.rf, a.uf, o.num_fine_smooth_sweeps));
      amgk::vcopy(s, a.uf, a.e[k], 0, nf);
   }
   // the atomic correction rides on the fused level-0 prolongation where it
   // can (no acceleration step between them)
   const bool fuse_corr = k > 0 && o.accel_type == AMG_NO_ACCEL && fused_xfp0(D);
   // (the fused prolongation + atomic correction: its whole launch is the window)
   if (j >= 0 && fuse_corr && D->corr.record_start(k, j, s))
      return amg_set_error(AMG_ERR_HIP, "level %d: correction event", k);
   unsigned long long *stp = j >= 0 ? D->corr.stamp(k, j) : nullptr;
   for (int l = k - 1; l >= 0; l--)
      AMG_TRY(prolong_to(D, a, l, a.e[l + 1], a.e[l], (l == 0 && fuse_corr) ? 1 : 0, D->lv[0].u, a.u_priv,
                         (l == 0 && fuse_corr) ? stp : nullptr));
   const int n0 = D->lv[0].n;
   if (o.accel_type != AMG_NO_ACCEL) {
      // DMEM_Add.cpp:319-324: ChebyUpdate(gridk.d, U_array[0]) on the level's
      // fine correction, async branch (DMEM_Misc.cpp:650-663): the cheby_grid
      // level carries d, the others scale by w*delta; first cycle: d = u
      const bool mine = k == cheby_grid_of(D);
      double om1 = 0.0, omd = 0.0;
      if (a.acc.next(o, &om1, &omd))
         amgk::dmem_cheby_update(s, a.d_acc, a.e[0], n0, mine ? 1 : 2, om1, omd);
      else if (mine)
         amgk::vcopy(s, a.e[0], a.d_acc, 0, n0);
   }
   // correction into the shared slab; u_priv = the value each row saw
   if (j >= 0 && !fuse_corr && D->corr.record_start(k, j, s))
      return amg_set_error(AMG_ERR_HIP, "level %d: correction event", k);
   if (!fuse_corr) amgk::atomic_correct(s, D->lv[0].u, a.e[0], a.u_priv, n0, stp);
   if (j >= 0 && D->corr.record(k, j, s)) return amg_set_error(AMG_ERR_HIP, "level %d: correction event", k);
   // private residual r_k = f - A u_k  (SMEM_Residual on u_k)
   AMG_TRY(a_spgemv(D, a, D->lv[0].A, a.u_priv, nullptr, amgk::gemv_mode(1.0, 0.0), a.y));
   amgk::vsub(s, D->lv[0].f, a.y, a.r[0], 0, n0);
   return AMG_OK;
}

int setup_async(amg_dist_hier *D)
{
   if (!D->al.empty()) return AMG_OK;
   amg_ctx *c = D->ctx;
   amg_transport *t = c->xport;
   const int L = D->L, Ld = D->Ld;
   const int active = std::max(1, L - 1);
   AMG_ARG((int)c->level_streams.size() >= active,
           "amg_dist_async_solve: context has %d level streams, need %d (amg_init nstreams)",
           (int)c->level_streams.size(), active);
   // l1 norms of the replicated levels
   for (int l = Ld; l < L; l++) {
      double *p;
      AMG_TRY(dvec(D, std::max(1, level_n(D, l)), &p));
      amgk::l1_norms(c->stream, D->cA[l - Ld], p);
      D->cl1.push_back(p);
   }
   const bool multadd = multadd_of(D->o);
   D->al.resize(active);
   for (int k = 0; k < active; k++) {
      AsyncLevel &a = D->al[k];
      a.s = c->level_streams[k];
      AMG_HIP(hipEventCreateWithFlags(&a.ev_ready, hipEventDisableTiming));
      AMG_HIP(hipEventCreateWithFlags(&a.ev_done, hipEventDisableTiming));
      const int coarsest = std::min(L - 1, multadd ? k : k + 1);
      a.r.assign(coarsest + 1, nullptr);
      a.e.assign(k + 1, nullptr);
      for (int l = 0; l <= coarsest; l++) AMG_TRY(lvec(D, l, &a.r[l]));
      for (int l = 0; l <= k; l++) AMG_TRY(lvec(D, l, &a.e[l]));
      const int k1 = std::min(L - 1, k + 1);
      AMG_TRY(lvec(D, 0, &a.u_priv));
      AMG_TRY(lvec2(D, 0, k1, &a.y));
      AMG_TRY(lvec2(D, k, k1, &a.u_prev));
      AMG_TRY(lvec2(D, k, k1, &a.sy));
      AMG_TRY(lvec2(D, k, k1, &a.sr));
      if (!multadd) {
         AMG_TRY(lvec(D, k, &a.uf));
         AMG_TRY(lvec(D, k1, &a.uc));
         AMG_TRY(lvec(D, k, &a.rf));
      }
      if (Ld < L) AMG_TRY(dvec(D, (size_t)D->gath_blk * (t->nranks + 1), &a.gath));
      // the row form's packed send buffers, one per operator with peers
      for (int l = 0; l < Ld; l++)
         for (DistMat *M : {&D->lv[l].A, &D->lv[l].P, &D->lv[l].R}) {
            if (!M->A || M->slab || M->replicated_cols || M->peers.empty()) continue;
            double *&sb = a.sbuf[M];
            if (!sb) AMG_TRY(dvec(D, std::max<long long>(1, M->nsend), &sb));
         }
      a.k = k;
   }
   if (D->o.accel_type != AMG_NO_ACCEL)
      AMG_TRY(dvec(D, std::max(1, D->lv[0].n), &D->al[cheby_grid_of(D)].d_acc));
   AMG_HIP(hipStreamSynchronize(c->stream));
   // the level groups' channels (amg_link.cpp): the largest message a peer
   // sends me in any exchange of a level correction -- the ghost rows of every
   // distributed operator, and the allgather block into the replicated levels
   if (t->nranks > 1) {
      const int R = t->nranks, me = t->rank;
      std::vector<long long> cap1(R, 0);
      for (int l = 0; l < Ld; l++)
         for (const DistMat *M : {&D->lv[l].A, &D->lv[l].P, &D->lv[l].R}) {
            if (!M->A || M->replicated_cols) continue;
            if (M->slab) {
               if (me > 0) cap1[me - 1] = std::max(cap1[me - 1], (long long)M->nlo[me] * M->cP);
               if (me < R - 1) cap1[me + 1] = std::max(cap1[me + 1], (long long)M->nhi[me] * M->cP);
            } else {
               for (size_t i = 0; i < M->peers.size(); i++)
                  cap1[M->peers[i]] = std::max(cap1[M->peers[i]], M->rcnt[i]);
            }
         }
      if (fused_xfp0(D) && Ld >= 2) {
         const long long P1 = D->lv[1].sg.P;
         if (me > 0) cap1[me - 1] = std::max(cap1[me - 1], (long long)D->xp_lo[me] * P1);
         if (me < R - 1) cap1[me + 1] = std::max(cap1[me + 1], (long long)D->xp_hi[me] * P1);
      }
      if (fused_xfer0(D)) {
         const long long P0 = D->lv[0].sg.P;
         if (me > 0) cap1[me - 1] = std::max(cap1[me - 1], (long long)D->rr_ulo[me] * P0);
         if (me < R - 1) cap1[me + 1] = std::max(cap1[me + 1], (long long)D->rr_uhi[me] * P0);
      }
      if (Ld < L)
         for (int p = 0; p < R; p++)
            if (p != me) cap1[p] = std::max(cap1[p], (long long)D->gath_blk);
      std::vector<long long> caps((size_t)active * R, 0);
      for (int k = 0; k < active; k++)
         for (int p = 0; p < R; p++) caps[(size_t)k * R + p] = cap1[p];
      // ranks on several nodes: the transport's send / recv (D->links stays null)
      bool one = false;
      AMG_TRY(link_single_node(D, &one));
      if (one) AMG_TRY(link_create(D, active, caps, &D->links));
   }
   return AMG_OK;
}

// the composed smoothed transfers' scratch (first solve that asks for them)
int setup_composed(amg_dist_hier *D)
{
   if (!composed(D)) return AMG_OK;
   for (auto &a : D->al)
      if (!a.xt) {
         AMG_TRY(lvec(D, 0, &a.xt));
         AMG_TRY(lvec(D, 0, &a.xy));
      }
   return AMG_OK;
}

} // namespace

// ---- level-grouped corrections (grid k of the DMEM add solver) ----------------
// AddCycle (DMEM_Add.cpp:180-329, NUMLEVELS_INTERPOLANTS): the grid's residual
// F[0] restricted level by level to level k, DMEM_AddSmooth there
// (DMEM_Smooth.cpp:574-638: u = f ./ s; v = A u; u = 2u + v ./ (-s), s = a_ii / w
// (1 where a_ii = 0, DMEM_Setup.cpp:471-482) or the L1 row norm) -- or
// hypre_GaussElimSolve on the coarsest grid, an exact dense solve here --
// then prolonged back to level 0 (MatvecOutOfPlace(P, U_c, 0, Vtemp, U_f)).
int amgd::grid_prepare(amg_dist_hier *D, int k)
{
   const int L = D->L, Ld = D->Ld;
   AMG_ARG(k >= 0 && k < L, "amg_grid_add: grid %d outside [0, %d)", k, L);
   AMG_ARG(!D->slab, "amg_grid_add: use a row-partitioned hierarchy (amg_dist_hier_create[_structured]), "
                     "not a z-slab one");
   GridState &g = D->grid;
   if (g.ready && g.k == k) return AMG_OK;
   AMG_ARG(!g.ready, "amg_grid_add: the hierarchy already serves grid %d", g.k);
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   g.k = k;
   // the replicated levels' L1 norms (as setup_async)
   if (D->cl1.empty())
      for (int l = Ld; l < L; l++) {
         double *p;
         AMG_TRY(dvec(D, std::max(1, level_n(D, l)), &p));
         amgk::l1_norms(s, D->cA[l - Ld], p);
         D->cl1.push_back(p);
      }
   // the grid's own level vectors F[l], U[l] (l <= k) and smoother scratch
   AsyncLevel &a = g.al;
   a.s = s;
   AMG_HIP(hipEventCreateWithFlags(&a.ev_ready, hipEventDisableTiming));
   AMG_HIP(hipEventCreateWithFlags(&a.ev_done, hipEventDisableTiming));
   a.r.assign(k + 1, nullptr);
   a.e.assign(k + 1, nullptr);
   for (int l = 0; l <= k; l++) {
      AMG_TRY(dvec(D, std::max(1, level_cap(D, l)), &a.r[l]));
      AMG_TRY(dvec(D, std::max(1, level_cap(D, l)), &a.e[l]));
   }
   const int ck = std::max(1, level_cap(D, k));
   AMG_TRY(dvec(D, ck, &a.sy));
   AMG_TRY(dvec(D, ck, &a.sr));
   AMG_TRY(dvec(D, ck, &a.u_prev));
   if (Ld < L) AMG_TRY(dvec(D, (size_t)D->gath_blk * (c->xport->nranks + 1), &a.gath));
   if (k == L - 1) {
      // hypre_GaussElimSetup: the coarsest operator gathered and factorised
      AMG_ARG(k >= Ld, "amg_grid_add: the coarsest level must be replicated "
                       "(amg_dist_hier_set_replicate_rows)");
      const amg_mat *Ac = D->cA[k - Ld];
      const int n = Ac->nrows;
      AMG_ARG(n <= 4096, "amg_grid_add: coarsest level of %d rows too large for the dense solve", n);
      std::vector<int> rp(n + 1), cj(std::max<long long>(1, Ac->nnz));
      std::vector<double> cv(std::max<long long>(1, Ac->nnz));
      AMG_TRY(amg_mat_download(c, Ac, rp.data(), cj.data(), cv.data()));
      g.n_c = n;
      g.lu.assign((size_t)n * n, 0.0);
      g.piv.assign(n, 0);
      for (int i = 0; i < n; i++)
         for (int q = rp[i]; q < rp[i + 1]; q++) g.lu[(size_t)i * n + cj[q]] += cv[q];
      for (int cc = 0; cc < n; cc++) {
         int p = cc;
         for (int i = cc + 1; i < n; i++)
            if (std::fabs(g.lu[(size_t)i * n + cc]) > std::fabs(g.lu[(size_t)p * n + cc])) p = i;
         g.piv[cc] = p;
         if (p != cc)
            for (int j = 0; j < n; j++) std::swap(g.lu[(size_t)cc * n + j], g.lu[(size_t)p * n + j]);
         const double d = g.lu[(size_t)cc * n + cc];
         if (d == 0.0) continue; // singular pivot: that unknown stays 0
         for (int i = cc + 1; i < n; i++) {
            const double m = (g.lu[(size_t)i * n + cc] /= d);
            for (int j = cc + 1; j < n; j++) g.lu[(size_t)i * n + j] -= m * g.lu[(size_t)cc * n + j];
         }
      }
      g.fh.assign(n, 0.0);
   } else {
      const int n = level_n(D, k);
      AMG_TRY(dvec(D, std::max(1, n), &g.sc));
      AMG_TRY(dvec(D, std::max(1, n), &g.nsc));
      const bool l1 = D->o.smoother == AMG_L1_JACOBI;
      amgk::dmem_scale(s, diag_of(D, k), l1 ? l1_of(D, k) : nullptr, D->o.smooth_weight, g.sc, g.nsc, n);
   }
   AMG_HIP(hipStreamSynchronize(s));
   g.ready = true;
   return AMG_OK;
}

int amgd::grid_cycle(amg_dist_hier *D, const double *r0, double **u0)
{
   GridState &g = D->grid;
   const int k = g.k, L = D->L;
   AsyncLevel &a = g.al;
   hipStream_t s = a.s;
   amgk::vcopy(s, r0, a.r[0], 0, D->lv[0].n);
   for (int l = 0; l < k; l++) AMG_TRY(restrict_to(D, a, l));
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   if (k == L - 1) {
      // hypre_GaussElimSolve: A_c u = f_c on the gathered coarsest level
      const int n = g.n_c;
      std::vector<double> &x = g.fh;
      AMG_TRY(d2h(s, x.data(), a.r[k], (size_t)n * 8));
      for (int cc = 0; cc < n; cc++)
         if (g.piv[cc] != cc) std::swap(x[cc], x[g.piv[cc]]);
      for (int i = 0; i < n; i++)
         for (int j = 0; j < i; j++) x[i] -= g.lu[(size_t)i * n + j] * x[j];
      for (int i = n - 1; i >= 0; i--) {
         for (int j = i + 1; j < n; j++) x[i] -= g.lu[(size_t)i * n + j] * x[j];
         const double d = g.lu[(size_t)i * n + i];
         x[i] = d != 0.0 ? x[i] / d : 0.0;
      }
      AMG_TRY(h2d(s, a.e[k], x.data(), (size_t)n * 8));
   } else {
      // DMEM_AddSmooth with simple_jacobi_flag = -1 (DMEM_Main.cpp:122)
      const int n = level_n(D, k);
      amgk::vset(s, a.e[k], 0.0, 0, n);
      amgk::vivaxpy(s, a.r[k], g.sc, a.e[k], 0, n);
      AMG_TRY(apply_A(D, a, k, a.e[k], nullptr, mv, a.sy));
      amgk::vscale(s, 2.0, a.e[k], 0, n);
      amgk::vivaxpy(s, a.sy, g.nsc, a.e[k], 0, n);
   }
   for (int l = k - 1; l >= 0; l--) AMG_TRY(prolong_to(D, a, l, a.e[l + 1], a.e[l]));
   *u0 = a.e[0];
   return AMG_OK;
}

// r = b - A x on the grid's fine level (halo exchange inside the grid)
int amgd::grid_residual(amg_dist_hier *D, double *x, const double *b, double *r)
{
   return a_spgemv(D, D->grid.al, D->lv[0].A, x, b, amgk::gemv_mode(-1.0, 1.0), r);
}

extern "C" int amg_dist_async_solve(amg_dist_hier *D, const double *f_local, int *level_corrections,
                                    double *relres)
{
   AMG_ARG(D && f_local, "amg_dist_async_solve: null argument");
   AMG_ARG(D->o.solver == AMG_ASYNC_MULTADD || D->o.solver == AMG_ASYNC_AFACX,
           "amg_dist_async_solve: ASYNC_MULTADD / ASYNC_AFACX hierarchies only");
   AMG_ARG(D->o.async_type == AMG_FULL_ASYNC, "amg_dist_async_solve: SEMI_ASYNC not supported");
   AMG_ARG(D->L >= 2, "amg_dist_async_solve: needs at least two levels");
   const int sched = D->o.async_schedule;
   AMG_ARG(sched >= AMG_SCHED_FREE && sched <= AMG_SCHED_TIMED, "amg_dist_async_solve: async_schedule %d", sched);
   AMG_ARG(sched != AMG_SCHED_TIMED || ((int)D->async_dur.size() >= D->L && (int)D->async_t.size() >= D->L),
           "amg_dist_async_solve: AMG_SCHED_TIMED needs amg_dist_hier_set_async_durations / _times");
   amg_ctx *c = D->ctx;
   AMG_TRY(setup_async(D));
   AMG_TRY(setup_composed(D));
   AMG_TRY(dist_solve_begin(D, f_local));
   if (D->links) AMG_TRY(link_reset(D->links, sched != AMG_SCHED_FREE));
   const int active = (int)D->al.size();
   const int n0 = D->lv[0].n;
   // a deterministic schedule runs every level on one stream and one host
   // thread, in the schedule's order; free: a stream and a host thread per level
   for (int k = 0; k < active; k++) D->al[k].s = c->level_streams[sched != AMG_SCHED_FREE ? 0 : k];
   // the free race's update windows on the device clock (amg_dist_async_update_windows)
   // and every row's update time (amg_dist_async_update_rows); the fused
   // level-0 prolongation + correction indexes the slab vector from its ghost
   // planes' start
   if (sched == AMG_SCHED_FREE) {
      std::vector<long long> koff(D->L, 0);
      for (int k = 1; k < active; k++)
         if (D->o.accel_type == AMG_NO_ACCEL && fused_xfp0(D)) koff[k] = D->lv[0].sg.off();
      if (D->corr.stamps_begin(c->stream, D->L, std::max(1, D->o.num_cycles), n0, koff))
         return amg_set_error(AMG_ERR_OOM, "amg_dist_async_solve: update-window stamps");
   }
   hipEvent_t ready, t_start;
   std::vector<hipEvent_t> t_end(active);
   AMG_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
   AMG_HIP(hipEventCreate(&t_start));
   for (auto &e : t_end) AMG_HIP(hipEventCreate(&e));
   AMG_HIP(hipEventRecord(ready, c->stream));
   AMG_HIP(hipEventRecord(t_start, c->stream));
   D->corr.reset(D->L);
   for (int k = 0; k < active; k++) {
      AMG_HIP(hipStreamWaitEvent(D->al[k].s, ready, 0));
      // level_vector[k].r[0] = vector.r[0] (SMEM_Async_AMG.cpp:10-15)
      amgk::vcopy(D->al[k].s, D->r0, D->al[k].r[0], 0, n0);
      D->al[k].acc.reset(D->o);
   }
   // one correction of level k (DMEM_DelayProc before AddCycle, DMEM_Add.cpp:106)
   auto correct = [&](int k, int j = -1) -> int {
      if (D->o.delay_level < 0 || D->o.delay_level == k) dist_delay(D, D->al[k].s);
      return level_correction(D, k, j);
   };
   const int N = D->o.num_cycles;
   std::vector<int> st(active, AMG_OK);
   std::vector<std::string> msg(active);
   if (sched == AMG_SCHED_FREE) {
      // every level group on its own host thread: it blocks only on its own
      // channels (the MPI_Test loop of amg_link.cpp)
      std::vector<std::thread> th;
      for (int k = 0; k < active; k++)
         th.emplace_back([&, k] {
            hipSetDevice(c->device);
            for (int cyc = 0; cyc < N && st[k] == AMG_OK; cyc++) st[k] = correct(k, cyc);
            // the level's finish: its stream reaches this marker after its last
            // correction (recorded here, not after the join, so a level that is
            // done early is not stamped with the slowest level's time)
            if (st[k] == AMG_OK && hipEventRecord(t_end[k], D->al[k].s) != hipSuccess)
               st[k] = amg_set_error(AMG_ERR_HIP, "level %d: hipEventRecord", k);
            if (st[k] == AMG_OK && D->links) st[k] = link_drain(D->links, k);
            if (st[k] != AMG_OK) {
               msg[k] = amg_last_error(); // thread-local: handed to the caller's thread
               if (D->links) link_abort(D->links);
            }
         });
      for (auto &t : th) t.join();
   } else {
      // the oracle's or_set_async_schedule order: 1 / 2 level after level, 3
      // cycle-major round robin, 4 timed (end times (j+1) dur[k], ties to the
      // finer level); every rank issues the same sequence
      std::vector<int> done_k(active, 0);
      for (int q = 0; q < active * N && st[0] == AMG_OK; q++) {
         int k;
         if (sched == AMG_SCHED_ROUND_ROBIN) {
            k = q % active;
         } else if (sched == AMG_SCHED_TIMED) {
            k = -1;
            double tb = 0.0;
            for (int j = 0; j < active; j++) {
               if (done_k[j] >= N) continue;
               const double t = amg_timed_end(D->async_t[j], D->async_dur[j], done_k[j]);
               if (k < 0 || t < tb) k = j, tb = t;
            }
         } else {
            k = sched == AMG_SCHED_FINEST_FIRST ? q / N : active - 1 - q / N;
         }
         st[0] = correct(k);
         const bool last = ++done_k[k] == N;
         if (st[0] == AMG_OK && last && hipEventRecord(t_end[k], D->al[k].s) != hipSuccess)
            st[0] = amg_set_error(AMG_ERR_HIP, "level %d: hipEventRecord", k);
      }
      for (int k = 0; k < active && st[0] == AMG_OK && D->links; k++) st[0] = link_drain(D->links, k);
      if (st[0] != AMG_OK && D->links) link_abort(D->links);
   }
   for (int k = 0; k < active; k++) {
      if (st[k] == AMG_OK && N <= 0) AMG_HIP(hipEventRecord(t_end[k], D->al[k].s));
      hipEvent_t done;
      AMG_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
      AMG_HIP(hipEventRecord(done, D->al[k].s)); // everything level k issued (drains included)
      AMG_HIP(hipStreamWaitEvent(c->stream, done, 0));
      AMG_HIP(hipEventDestroy(done));
   }
   AMG_HIP(hipEventDestroy(ready));
   for (int k = 0; k < active; k++)
      if (st[k] != AMG_OK) {
         for (auto &e : t_end) hipEventDestroy(e);
         hipEventDestroy(t_start);
         for (auto &a : D->al) hipStreamSynchronize(a.s);
         if (sched == AMG_SCHED_FREE) return amg_set_error(st[k], "level %d: %s", k, msg[k].c_str());
         return st[k];
      }
   D->pre_ready = false;
   AMG_TRY(dist_outer_residual(D, 1));
   D->iter = 1;
   AMG_TRY(d2h(c->stream, c->h_pinned, D->d_hist + 1, sizeof(double)));
   if (relres) *relres = c->h_pinned[0] / D->r0norm;
   if (level_corrections)
      for (int k = 0; k < D->L; k++) level_corrections[k] = k < active ? N : 0;
   if (sched == AMG_SCHED_FREE) {
      std::vector<int> cnt(D->L, 0);
      for (int k = 0; k < active; k++) cnt[k] = N;
      if (D->corr.collect(t_start, cnt)) return amg_set_error(AMG_ERR_HIP, "amg_dist_async_solve: correction times");
      if (D->corr.stamps_collect(cnt, c->wall_khz))
         return amg_set_error(AMG_ERR_HIP, "amg_dist_async_solve: update-window stamps");
   }
   D->level_ms.assign(D->L, 0.0);
   for (int k = 0; k < active; k++) {
      float ms = 0.f;
      AMG_HIP(hipEventElapsedTime(&ms, t_start, t_end[k]));
      D->level_ms[k] = ms;
      AMG_HIP(hipEventDestroy(t_end[k]));
   }
   AMG_HIP(hipEventDestroy(t_start));
   return AMG_OK;
}

extern "C" int amg_dist_hier_set_async_durations(amg_dist_hier *D, const double *ms, int n)
{
   AMG_ARG(D && ms && n >= D->L, "amg_dist_hier_set_async_durations: need %d levels", D ? D->L : 0);
   for (int k = 0; k < D->L; k++)
      AMG_ARG(ms[k] > 0.0, "amg_dist_hier_set_async_durations: level %d: %g", k, ms[k]);
   D->async_dur.assign(ms, ms + D->L);
   D->async_t.assign(D->L, {});
   return AMG_OK;
}

extern "C" int amg_dist_hier_set_async_times(amg_dist_hier *D, const double *t, const int *n, int nlev)
{
   AMG_ARG(D && t && n && nlev >= D->L, "amg_dist_hier_set_async_times: need %d levels", D ? D->L : 0);
   D->async_t.assign(D->L, {});
   D->async_dur.assign(D->L, 1.0);
   for (int k = 0, off = 0; k < D->L; off += n[k], k++) {
      AMG_ARG(n[k] >= 0, "amg_dist_hier_set_async_times: level %d: %d entries", k, n[k]);
      D->async_t[k].assign(t + off, t + off + n[k]);
   }
   return AMG_OK;
}

extern "C" int amg_dist_async_update_windows(const amg_dist_hier *D, int level, double *ms, int cap, int *count)
{
   AMG_ARG(D && count && level >= 0 && level < D->L, "amg_dist_async_update_windows: bad argument");
   const bool start = cap < 0;
   if (start) cap = -cap;
   const auto &vv = start ? D->corr.w0 : D->corr.w1;
   const auto &v = level < (int)vv.size() ? vv[level] : std::vector<double>();
   *count = (int)v.size();
   for (int j = 0; j < (int)v.size() && j < cap && ms; j++) ms[j] = v[j];
   return AMG_OK;
}

extern "C" int amg_dist_async_update_rows(const amg_dist_hier *D, int level, int corr, double *ms, int cap,
                                          int *count)
{
   AMG_ARG(D && count && level >= 0 && level < D->L && corr >= 0,
           "amg_dist_async_update_rows: bad argument");
   *count = D->corr.rows_of(level, corr, ms, cap < 0 ? -cap : cap, cap < 0);
   return AMG_OK;
}

extern "C" int amg_dist_async_correction_ms(const amg_dist_hier *D, int level, double *ms, int cap, int *count)
{
   AMG_ARG(D && count && level >= 0 && level < D->L, "amg_dist_async_correction_ms: bad argument");
   const bool start = cap < 0; // cap < 0: the update windows' start times, -cap entries
   if (start) cap = -cap;
   const auto &vv = start ? D->corr.ms0 : D->corr.ms;
   const auto &v = level < (int)vv.size() ? vv[level] : std::vector<double>();
   *count = (int)v.size();
   for (int j = 0; j < (int)v.size() && j < cap && ms; j++) ms[j] = v[j];
   return AMG_OK;
}

extern "C" int amg_dist_async_level_ms(const amg_dist_hier *D, double *ms)
{
   AMG_ARG(D && ms, "amg_dist_async_level_ms: null argument");
   AMG_ARG(!D->level_ms.empty(), "amg_dist_async_level_ms: no asynchronous solve yet");
   for (int k = 0; k < D->L; k++) ms[k] = D->level_ms[k];
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// DMEM_AsyncSmooth (DMEM_Smooth.cpp:16-313), ASYNC_JACOBI / ASYNC_L1_JACOBI on
// the fine grid: Jacobi in residual-update form with asynchronous ghost
// deltas.  Per relaxation k:
//    u = r ./ s   (s = a_ii / omega, 1 if a_ii == 0; or l1_i)
//    [accel_type: DMEM_ChebyUpdate(d, u), async branch -- the fine grid is grid 0]
//    e = u;  x += e;  r -= A_diag e                    (owned columns only)
//    send e's boundary values to the neighbours       (finestIntra_outsideSend, ACCUMULATE)
//    r -= A_offd g for every ghost delta g that HAS arrived  (finestIntra_outsideRecv)
// The exchange runs on the communication stream, double-buffered over NBUF
// slots; deltas that have not arrived are applied in a later relaxation, so a
// rank never waits for its neighbours except when a slot must be reused.  At
// the end every delta is drained and the true residual ||f - A x|| formed.
// A_diag / A_offd are the [owned | ghost] column split of the slab CSR: the
// products run through the tile kernel with the other region zeroed.
// ---------------------------------------------------------------------------
namespace {

// one relaxation's local update (DMEM_Smooth.cpp:100-112, 171-183, 229):
//   u = 0 + r ./ s;  [ChebyUpdate(d, u), async branch of cheby_grid];
//   e = 0 + u;  x += e
// acc: 0 none, 1 first cycle (d = u), 2 recurrence with om1 = w - 1, omd = w delta
// (this grid is cheby_grid), 3 recurrence on another grid (u = omd u)
// gate (SPS): the device flag of this sweep; 0 = no relaxation (e = 0, x kept)
__global__ void ajac_update_k(const double *__restrict__ r, const double *__restrict__ sc,
                              double *__restrict__ e, double *__restrict__ x, double *__restrict__ d,
                              int n, int acc, double om1, double omd, const int *__restrict__ gate)
{
   if (gate && *gate == 0) {
      for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) e[i] = 0.0;
      return;
   }
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      double u = 0.0 + r[i] / sc[i];
      if (acc == 1) {
         d[i] = u;
      } else if (acc == 2) {
         const double dp = d[i];
         d[i] = om1 * dp + omd * u;
         u = om1 * dp + omd * u;
      } else if (acc == 3) {
         u = omd * u;
      }
      const double ei = 0.0 + 1.0 * u;
      e[i] = ei;
      x[i] += 1.0 * ei;
   }
}

// wJacobi_scale_gridk (DMEM_Setup.cpp:474-480): a_ii / omega, 1 where a_ii == 0;
// L1: L1_row_norm_gridk
__global__ void ajac_scale_k(const double *__restrict__ diag, const double *__restrict__ l1,
                             double omega, double *__restrict__ sc, int n)
{
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      if (l1)
         sc[i] = l1[i];
      else
         sc[i] = diag[i] == 0.0 ? 1.0 : diag[i] / omega;
   }
}

constexpr int AJ_NBUF = 4;

// SPS messages carry the sender's residual norm after each peer's deltas
// (data[vec_len + 1], DMEM_Comm.cpp:216-220): peer i's segment of the slot is
// [scnt[i] deltas | norm] at soff[i] + i.  One thread per slot entry.
__device__ __forceinline__ int seg_of(const long long *__restrict__ off, int np, long long p)
{
   int lo = 0, hi = np - 1; // last segment with off[seg] <= p
   while (lo < hi) {
      const int mid = (lo + hi + 1) / 2;
      if (off[mid] <= p) lo = mid;
      else hi = mid - 1;
   }
   return lo;
}

__global__ void sps_pack_k(const double *__restrict__ e, const int *__restrict__ idx, long long nsend,
                           const long long *__restrict__ soff, int np, const double *__restrict__ norm,
                           double *__restrict__ out)
{
   const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
   if (p < nsend) out[p + seg_of(soff, np, p)] = e[idx[p]];
   if (p < np) out[soff[p + 1] + p] = norm[0];
}

__global__ void sps_unpack_k(const double *__restrict__ in, long long ng, const long long *__restrict__ roff, int np,
                             double *__restrict__ g, double *__restrict__ rnorm)
{
   const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
   if (p < ng) g[p] = in[p + seg_of(roff, np, p)];
   if (p < np) rnorm[p] = in[roff[p + 1] + p];
}

// StochasticParallelSouthwellUpdateProbability (DMEM_Smooth.cpp:548-572) and the
// draw that follows it (:286-290), for sweep k >= 1 (sweep 0 always relaxes,
// update_flag = 1 at :70): x = the neighbours whose latest norm exceeds mine
// (not counted for RANDOM); p = (1/x)(1/alpha), exp(-x alpha) or alpha; relax
// when draws[k-1] < p.  One lane; count = the sweeps relaxed in.
__global__ void sps_decide_k(const double *__restrict__ mynorm, const double *__restrict__ rnorm, int np,
                             int type, double alpha, const double *__restrict__ draws, int k,
                             int *__restrict__ gate, long long *__restrict__ count)
{
   if (threadIdx.x != 0 || blockIdx.x != 0) return;
   int up = 1;
   if (k > 0) {
      double x = 0.0;
      if (type != AMG_SPS_RANDOM)
         for (int i = 0; i < np; i++)
            if (mynorm[0] < rnorm[i]) x++;
      double p;
      if (type == AMG_SPS_INVERSE)
         p = (1.0 / x) * (1.0 / alpha);
      else if (type == AMG_SPS_EXPONENTIAL)
         p = exp(-x * alpha);
      else
         p = alpha;
      up = draws[k - 1] < p ? 1 : 0;
   }
   gate[0] = up;
   count[0] += up;
}

// glibc random_r TYPE_3 (the default state of rand(), degree 31, separation 3):
// seeded by the Lehmer generator 16807 r mod (2^31 - 1), 310 outputs discarded,
// then r_i = r_{i-31} + r_{i-3} (mod 2^32), output r_i >> 1
std::vector<double> rand_double_stream(unsigned seed, int n, double low, double high)
{
   std::vector<unsigned> r(344 + (size_t)std::max(n, 0));
   int32_t w = seed == 0 ? 1 : (int32_t)seed;
   r[0] = (unsigned)w;
   for (int i = 1; i < 31; i++) {
      const int32_t hi = w / 127773, lo = w % 127773;
      w = 16807 * lo - 2836 * hi;
      if (w < 0) w += 2147483647;
      r[i] = (unsigned)w;
   }
   for (int i = 31; i < 34; i++) r[i] = r[i - 31];
   for (size_t i = 34; i < r.size(); i++) r[i] = r[i - 31] + r[i - 3];
   std::vector<double> out(std::max(n, 0));
   for (int k = 0; k < n; k++) out[k] = low + (high - low) * ((double)(r[344 + k] >> 1) / 2147483647.0);
   return out;
}

int async_jacobi_run(amg_dist_hier *D, const double *f_local, int sweeps, int l1, bool sps, double *relres,
                     long long *relaxations);

} // namespace

extern "C" int amg_rand_double_stream(unsigned seed, int n, double low, double high, double *out)
{
   AMG_ARG(n >= 0 && (n == 0 || out), "amg_rand_double_stream: bad argument");
   const std::vector<double> v = rand_double_stream(seed, n, low, high);
   std::copy(v.begin(), v.end(), out);
   return AMG_OK;
}

extern "C" int amg_dist_async_jacobi(amg_dist_hier *D, const double *f_local, int sweeps, int l1,
                                     double *relres)
{
   return async_jacobi_run(D, f_local, sweeps, l1, false, relres, nullptr);
}

extern "C" int amg_dist_async_jacobi_log(const amg_dist_hier *D, double *events, int cap, int *count)
{
   AMG_ARG(D && count && cap >= 0, "amg_dist_async_jacobi_log: bad argument");
   *count = (int)(D->ajac_log.size() / 5);
   for (int i = 0; i < (int)D->ajac_log.size() && i < 5 * cap && events; i++) events[i] = D->ajac_log[i];
   return AMG_OK;
}

extern "C" int amg_dist_async_jacobi_stats(const amg_dist_hier *D, double *stats, int n)
{
   AMG_ARG(D && stats && n >= 0, "amg_dist_async_jacobi_stats: bad argument");
   AMG_ARG(!D->ajac_stats.empty(), "amg_dist_async_jacobi_stats: no asynchronous Jacobi run yet");
   for (int i = 0; i < n && i < (int)D->ajac_stats.size(); i++) stats[i] = D->ajac_stats[i];
   return AMG_OK;
}

extern "C" int amg_dist_async_sps(amg_dist_hier *D, const double *f_local, int sweeps, double *relres,
                                  long long *relaxations)
{
   return async_jacobi_run(D, f_local, sweeps, 0, true, relres, relaxations);
}

namespace {

int async_jacobi_run(amg_dist_hier *D, const double *f_local, int sweeps, int l1, bool sps, double *relres,
                     long long *relaxations)
{
   AMG_ARG(D && f_local && sweeps >= 0, "amg_dist_async_jacobi: bad argument");
   AMG_ARG(!D->slab, "amg_dist_async_jacobi / _sps: use a row-partitioned hierarchy "
                     "(amg_dist_hier_create[_structured]), not a z-slab one");
   AMG_ARG(!sps || D->o.accel_type == AMG_NO_ACCEL, "amg_dist_async_sps: no accel_type with SPS gating");
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream, cs = c->comm_stream;
   DLevel &v = D->lv[0];
   DistMat &M = v.A;
   const int n = v.n, ng = M.nghost, no = M.ncol_own;
   const int np = (int)M.peers.size();
   AMG_ARG(no == n, "amg_dist_async_jacobi: square fine operator expected");
   // state: x (= u of level 0), r, e_ext = [e | 0], g_ext = [0 | g], w
   double *x = dist_iterate(D), *r = v.r_fine, *eext = v.u_alt, *gext = v.f, *w = v.l1;
   std::vector<double *> dtmp;
   auto tmp = [&](size_t cnt) -> double * {
      double *p = nullptr;
      if (hipMalloc(&p, std::max<size_t>(1, cnt) * sizeof(double)) != hipSuccess) return nullptr;
      dtmp.push_back(p);
      return p;
   };
   // slot sizes: SPS appends the sender's norm to every peer's deltas
   const long long SS = std::max<long long>(1, M.nsend + (sps ? np : 0)), RS = std::max<long long>(1, ng + (sps ? np : 0));
   double *wv = tmp(n), *f = tmp(n), *sbuf = tmp((size_t)SS * AJ_NBUF), *rbuf = tmp((size_t)RS * AJ_NBUF),
          *dacc = tmp(n);
   AccelState acc;
   acc.reset(D->o);
   const bool accel = D->o.accel_type != AMG_NO_ACCEL;
   (void)w;
   int st = AMG_OK;
   auto fail = [&](int code) {
      hipStreamSynchronize(s);
      hipStreamSynchronize(cs);
      for (double *p : dtmp) hipFree(p);
      return code;
   };
   if (!wv || !f || !sbuf || !rbuf || !dacc) return fail(amg_set_error(AMG_ERR_OOM, "amg_dist_async_jacobi: workspace"));
   // SPS: [my norm per slot (NBUF) | latest neighbour norms (np) | draws
   // (sweeps)], gate flag, relaxation count, the segment offsets soff / roff
   double *part = nullptr, sps_alpha = D->o.sps_alpha;
   double *snorm = nullptr, *lnorm = nullptr, *draws = nullptr;
   int *gate = nullptr;
   long long *count = nullptr, *d_soff = nullptr, *d_roff = nullptr;
   if (sps) {
      double *ws = tmp((size_t)AJ_NBUF + np + sweeps + 2 + 2 * (np + 1));
      if (!ws) return fail(amg_set_error(AMG_ERR_OOM, "amg_dist_async_sps: workspace"));
      // the reference's RandDouble stream: one draw per sweep after the first
      const std::vector<double> dr = rand_double_stream(0, sweeps, 0.0, 1.0);
      double *pp = nullptr;
      if ((st = amg_ctx_partials(c, 65536, &pp)) != AMG_OK) return fail(st);
      part = pp;
      snorm = ws;
      lnorm = snorm + AJ_NBUF;
      draws = lnorm + np;
      gate = reinterpret_cast<int *>(draws + sweeps);
      count = reinterpret_cast<long long *>(draws + sweeps + 1);
      d_soff = reinterpret_cast<long long *>(draws + sweeps + 2);
      d_roff = d_soff + np + 1;
      amgk::vset(s, ws, 0.0, 0, (long long)AJ_NBUF + np + sweeps + 2);
      if (sweeps > 0 && (st = h2d(s, draws, dr.data(), (size_t)sweeps * sizeof(double))) != AMG_OK)
         return fail(st);
      std::vector<long long> so(M.soff), ro(M.roff);
      so.resize(np + 1);
      ro.resize(np + 1);
      so[np] = M.nsend;
      ro[np] = ng;
      if (np > 0 && ((st = h2d(s, d_soff, so.data(), (size_t)(np + 1) * 8)) != AMG_OK ||
                     (st = h2d(s, d_roff, ro.data(), (size_t)(np + 1) * 8)) != AMG_OK))
         return fail(st);
      // sps_min_prob > 0: alpha = -log(min_prob) / num_sends (DMEM_Setup.cpp:1168-1169)
      if (D->o.sps_min_prob > 0 && np > 0) sps_alpha = -std::log(D->o.sps_min_prob) / (double)np;
   }
   if ((st = h2d(s, f, f_local, (size_t)n * sizeof(double))) != AMG_OK) return fail(st);
   const int nb = std::max(1, std::min(65536, (n + 255) / 256));
   ajac_scale_k<<<nb, 256, 0, s>>>(M.A->diag, l1 ? v.l1 : nullptr, D->o.smooth_weight, wv, n);
   amgk::vset(s, x, 0.0, 0, v.cap);
   amgk::vcopy(s, f, r, 0, n); // x = 0: r = b
   amgk::vset(s, eext, 0.0, 0, v.cap);
   amgk::vset(s, gext, 0.0, 0, v.cap);
   const amgk::Gemv upd = amgk::gemv_mode(-1.0, 1.0); // r = r - A z
   hipEvent_t packed[AJ_NBUF], sent[AJ_NBUF], arrived[AJ_NBUF];
   for (int q = 0; q < AJ_NBUF; q++) {
      hipEventCreateWithFlags(&packed[q], hipEventDisableTiming);
      hipEventCreateWithFlags(&sent[q], hipEventDisableTiming);
      hipEventCreateWithFlags(&arrived[q], hipEventDisableTiming);
   }
   // the overlap record: per sweep the exchange window on the comm stream and
   // the interior product's window on the compute stream (timing events)
   std::vector<hipEvent_t> tev((size_t)sweeps * 4, nullptr);
   for (auto &e : tev) hipEventCreate(&e);
   auto tx0 = [&](int k) { return tev[(size_t)k * 4]; };
   auto tx1 = [&](int k) { return tev[(size_t)k * 4 + 1]; };
   auto ti0 = [&](int k) { return tev[(size_t)k * 4 + 2]; };
   auto ti1 = [&](int k) { return tev[(size_t)k * 4 + 3]; };
   // the deltas through device-resident channels (amg_link.cpp) where the
   // ranks share a node: a send is a copy kernel on the comm stream straight
   // into the neighbour's slot (overlapping the interior product on the
   // compute stream), a receive an MPI_Test-like poll; SPS (norms ride with
   // the deltas) and AMG_AJAC_LINKS=0 keep the transport's grouped send/recv
   static const bool links_env = [] {
      const char *e = std::getenv("AMG_AJAC_LINKS");
      return e ? std::atoi(e) != 0 : true;
   }();
   bool use_links = !sps && links_env && c->xport->nranks > 1;
   if (use_links && !D->ajac_links) {
      // ranks on several nodes: the transport's grouped send / recv
      bool one = false;
      if ((st = link_single_node(D, &one)) != AMG_OK) return fail(st);
      use_links = one;
   }
   if (use_links && !D->ajac_links) {
      // channels carry both directions (link_create maps a peer's slots only
      // where caps > 0): a peer I only send to (a pattern-nonsymmetric
      // operator: scnt > 0, rcnt = 0) needs its channel too
      std::vector<long long> caps(c->xport->nranks, 0);
      for (int i = 0; i < np; i++) caps[M.peers[i]] = std::max(M.rcnt[i], M.scnt[i]);
      // 8 slots per channel: a sender runs up to 8 sweeps ahead of a peer's receipts
      if ((st = link_create(D, 1, caps, &D->ajac_links, 8)) != AMG_OK) return fail(st);
   }
   if (use_links && (st = link_reset(D->ajac_links, true)) != AMG_OK) return fail(st);
   std::vector<long long> got_cnt(np, 0);
   D->ajac_log.clear();
   auto logev = [&](int type, double a, double b = 0.0, double c = 0.0, double d = 0.0) {
      if (sps) return;
      for (double v : {(double)type, a, b, c, d}) D->ajac_log.push_back(v);
   };
   long long on_time = 0, late = 0;
   double send_wait_ms = 0.0; // host time a send waited for its slot (flow control)
   // r -= A_offd g on the rows that have ghost columns (outside the interior [b0, b1))
   auto apply_offd = [&]() {
      amgk::spgemv(s, M.A, gext, r, upd, r, 0, M.b0, nullptr);
      amgk::spgemv(s, M.A, gext, r, upd, r, M.b1, n, nullptr);
   };
   // every delta that has arrived from peer i, each applied on its own, then
   // the ghost region cleared (so no delta is applied twice)
   auto poll_links = [&](int k, bool block) -> int {
      for (int i = 0; i < np; i++) {
         if (M.rcnt[i] <= 0) continue;
         for (;;) {
            int got = 0;
            double *dst = gext + no + M.roff[i];
            if (block) {
               if (got_cnt[i] >= sweeps) break;
               AMG_TRY(link_recv(D->ajac_links, 0, M.peers[i], dst, M.rcnt[i], s));
               got = 1;
            } else {
               AMG_TRY(link_try_recv(D->ajac_links, 0, M.peers[i], dst, M.rcnt[i], s, &got));
            }
            if (!got) break;
            if (got_cnt[i] == k) on_time++;
            else late++;
            logev(3, M.peers[i], (double)got_cnt[i]);
            got_cnt[i]++;
            apply_offd();
            amgk::vset(s, gext + no + M.roff[i], 0.0, 0, M.rcnt[i]);
         }
      }
      return AMG_OK;
   };
   std::vector<int> pending; // relaxations whose ghost deltas are not applied yet
   auto apply = [&](int k) -> int {
      const int q = k % AJ_NBUF;
      AMG_HIP(hipStreamWaitEvent(s, arrived[q], 0));
      if (sps) { // the deltas, and the neighbours' norms that came with them
         const long long m = std::max<long long>(ng, np);
         sps_unpack_k<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(rbuf + (size_t)q * RS, ng, d_roff, np, gext + no,
                                                                   lnorm);
      } else {
         AMG_HIP(hipMemcpyAsync(gext + no, rbuf + (size_t)q * RS, (size_t)ng * sizeof(double),
                                hipMemcpyDeviceToDevice, s));
      }
      amgk::spgemv(s, M.A, gext, r, upd, r, 0, n, nullptr); // r -= A_offd g
      logev(4, k);
      return AMG_OK;
   };
   // the sweeps, the drain and the final checks; every failure after this point
   // (a send timeout, an aborted peer, a HIP error) leaves through one path:
   // the peers are told (link_abort), the events destroyed, the workspace freed
   auto sweep_all = [&]() -> int {
      for (int k = 0; k < sweeps && st == AMG_OK; k++) {
         const int q = k % AJ_NBUF;
         // the slot's previous delta must be applied and its send finished
         for (size_t i = 0; i < pending.size();) {
            if (pending[i] <= k - AJ_NBUF) {
               if ((st = apply(pending[i])) != AMG_OK) break;
               pending.erase(pending.begin() + i);
            } else {
               i++;
            }
         }
         if (st != AMG_OK) break;
         AMG_HIP(hipStreamWaitEvent(s, sent[q], 0));
         double om1 = 0.0, omd = 0.0;
         const int am = !accel ? 0 : !acc.next(D->o, &om1, &omd) ? 1 : D->o.cheby_grid == 0 ? 2 : 3;
         if (sps) {
            // my residual L1 norm (DMEM_Smooth.cpp:258-268), sent with this sweep's
            // deltas; then this sweep's update decision
            int parts = 0;
            amgk::abssum_partials(s, r, n, part, &parts);
            amgk::reduce_partials(s, part, parts, snorm + q, 0, c->d_scalars + 4096);
            sps_decide_k<<<1, 64, 0, s>>>(snorm + q, lnorm, np, D->o.sps_probability_type, sps_alpha, draws, k, gate,
                                          count);
         }
         ajac_update_k<<<nb, 256, 0, s>>>(r, wv, eext, x, dacc, n, am, om1, omd, gate);
         logev(1, k, am, om1, omd);
         if (use_links) {
            if (np > 0) {
               launch_gather(s, eext, M.d_send_idx, sbuf + (size_t)q * SS, (int)M.nsend);
               AMG_HIP(hipEventRecord(packed[q], s));
               AMG_HIP(hipStreamWaitEvent(cs, packed[q], 0));
            }
            bool first = true;
            for (int i = 0; i < np && st == AMG_OK; i++) {
               if (M.scnt[i] <= 0) continue;
               // a full slot ring: keep receiving (and acknowledging) while waiting,
               // or two ranks that both wait to send would wait on each other
               const auto t0 = std::chrono::steady_clock::now();
               for (;;) {
                  int ok = 0;
                  if ((st = link_can_send(D->ajac_links, 0, M.peers[i], &ok)) != AMG_OK || ok) break;
                  if ((st = poll_links(k, false)) != AMG_OK) break;
                  if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > link_timeout_s()) {
                     st = amg_set_error(AMG_ERR_RCCL, "amg_dist_async_jacobi: send to rank %d timed out", M.peers[i]);
                     break;
                  }
                  std::this_thread::yield();
               }
               send_wait_ms += 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
               // the exchange window: from the first copy's issue (after any wait)
               if (st == AMG_OK && first && hipEventRecord(tx0(k), cs) != hipSuccess)
                  st = amg_set_error(AMG_ERR_HIP, "amg_dist_async_jacobi: event");
               first = false;
               if (st == AMG_OK)
                  st = link_send(D->ajac_links, 0, M.peers[i], sbuf + (size_t)q * SS + M.soff[i], M.scnt[i], cs);
            }
            if (st == AMG_OK && first) AMG_HIP(hipEventRecord(tx0(k), cs));
            if (st != AMG_OK) break;
            AMG_HIP(hipEventRecord(tx1(k), cs));
            AMG_HIP(hipEventRecord(sent[q], cs));
            // r -= A_diag e (ghost region of e_ext stays zero), overlapping the sends
            AMG_HIP(hipEventRecord(ti0(k), s));
            amgk::spgemv(s, M.A, eext, r, upd, r, 0, n, nullptr);
            logev(2, k);
            AMG_HIP(hipEventRecord(ti1(k), s));
            if ((st = poll_links(k, false)) != AMG_OK) break;
            D->iter = k + 1;
            continue;
         }
         if (np > 0) {
            if (sps) { // the norm travels with the deltas (data[vec_len + 1], DMEM_Comm.cpp:216-220)
               const long long m = std::max<long long>(M.nsend, np);
               sps_pack_k<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(eext, M.d_send_idx, M.nsend, d_soff, np, snorm + q,
                                                                       sbuf + (size_t)q * SS);
            } else {
               launch_gather(s, eext, M.d_send_idx, sbuf + (size_t)q * SS, (int)M.nsend);
            }
            AMG_HIP(hipEventRecord(packed[q], s));
            AMG_HIP(hipStreamWaitEvent(cs, packed[q], 0));
            AMG_HIP(hipEventRecord(tx0(k), cs));
            std::vector<void *> sp(np), rp(np);
            std::vector<long long> sb(np), rb(np);
            const int g = sps ? 1 : 0;
            for (int i = 0; i < np; i++) {
               sp[i] = sbuf + (size_t)q * SS + M.soff[i] + g * i;
               sb[i] = (M.scnt[i] + g) * 8;
               rp[i] = rbuf + (size_t)q * RS + M.roff[i] + g * i;
               rb[i] = (M.rcnt[i] + g) * 8;
            }
            if ((st = xp_p2p(c, cs, np, M.peers.data(), sp.data(), sb.data(), rp.data(), rb.data())) != AMG_OK)
               break;
            AMG_HIP(hipEventRecord(sent[q], cs));
            AMG_HIP(hipEventRecord(arrived[q], cs));
            pending.push_back(k);
         }
         AMG_HIP(hipEventRecord(tx1(k), cs));
         // r -= A_diag e (ghost region of e_ext stays zero), overlapping the exchange
         AMG_HIP(hipEventRecord(ti0(k), s));
         amgk::spgemv(s, M.A, eext, r, upd, r, 0, n, nullptr);
         logev(2, k);
         AMG_HIP(hipEventRecord(ti1(k), s));
         // deltas that have already arrived (host poll: never blocks)
         for (size_t i = 0; i < pending.size();) {
            if (hipEventQuery(arrived[pending[i] % AJ_NBUF]) == hipSuccess) {
               if ((st = apply(pending[i])) != AMG_OK) break;
               pending.erase(pending.begin() + i);
            } else {
               break; // in order: later slots cannot have arrived first
            }
         }
         D->iter = k + 1;
      }
      for (size_t i = 0; st == AMG_OK && i < pending.size(); i++) st = apply(pending[i]); // drain
      if (use_links && st == AMG_OK) {
         st = poll_links(sweeps, true); // the deltas still in flight, each applied once
         if (st == AMG_OK) st = link_drain(D->ajac_links, 0);
         for (int i = 0; i < np && st == AMG_OK; i++)
            if (M.rcnt[i] > 0 && got_cnt[i] != sweeps)
               st = amg_set_error(AMG_ERR_RCCL, "amg_dist_async_jacobi: %lld deltas from rank %d, expected %d",
                                  got_cnt[i], M.peers[i], sweeps);
      }
      return st;
   };
   st = sweep_all();
   if (st != AMG_OK && use_links) link_abort(D->ajac_links);
   for (int q = 0; q < AJ_NBUF; q++) {
      hipEventDestroy(packed[q]);
      hipEventDestroy(sent[q]);
      hipEventDestroy(arrived[q]);
   }
   if (st != AMG_OK) {
      for (auto e : tev) hipEventDestroy(e);
      return fail(st);
   }
   // the overlap record: the fraction of each sweep's exchange window that the
   // interior product covers, the windows' lengths
   {
      AMG_HIP(hipStreamSynchronize(cs));
      AMG_HIP(hipStreamSynchronize(s));
      double hid = 0.0, xs = 0.0, is = 0.0;
      int cntk = 0;
      for (int k = 0; k < sweeps && np > 0; k++) {
         float a0 = 0.f, a1 = 0.f, b0 = 0.f, b1 = 0.f;
         if (hipEventElapsedTime(&a0, tx0(0), tx0(k)) != hipSuccess ||
             hipEventElapsedTime(&a1, tx0(0), tx1(k)) != hipSuccess ||
             hipEventElapsedTime(&b0, tx0(0), ti0(k)) != hipSuccess ||
             hipEventElapsedTime(&b1, tx0(0), ti1(k)) != hipSuccess) {
            (void)hipGetLastError();
            continue;
         }
         const double xd = a1 - a0, ov = std::max(0.0, (double)std::min(a1, b1) - (double)std::max(a0, b0));
         hid += xd > 0 ? std::min(1.0, ov / xd) : 1.0;
         xs += xd;
         is += b1 - b0;
         cntk++;
      }
      long long nrecv = 0;
      for (int i = 0; i < np; i++) nrecv += M.rcnt[i] > 0 ? 1 : 0;
      D->ajac_stats.assign(9, 0.0);
      D->ajac_stats[8] = sweeps > 0 ? send_wait_ms / sweeps : 0.0; // host flow-control wait per sweep
      D->ajac_stats[0] = cntk ? hid / cntk : 0.0;  // hidden fraction of the exchange
      D->ajac_stats[1] = cntk ? xs / cntk : 0.0;   // exchange window, ms per sweep
      D->ajac_stats[2] = cntk ? is / cntk : 0.0;   // interior product, ms per sweep
      D->ajac_stats[3] = use_links && nrecv * sweeps > 0 ? (double)on_time / (double)(nrecv * sweeps) : -1.0;
      D->ajac_stats[4] = use_links ? (double)late : -1.0;
      D->ajac_stats[7] = use_links ? 1.0 : 0.0;
   }
   for (auto e : tev) hipEventDestroy(e);
   // every delta applied once <=> the incrementally kept r equals f - A x (to
   // rounding): its global norm, beside the true residual's below
   {
      double *pp;
      if ((st = amg_ctx_partials(c, 65536, &pp)) != AMG_OK) return fail(st);
      int parts = 0;
      amgk::sumsq_partials(s, r, n, pp, &parts);
      amgk::reduce_partials(s, pp, parts, D->d_hist + 3, 0, c->d_scalars + 4096);
      if ((st = xp_allreduce(c, s, D->d_hist + 3, 1)) != AMG_OK) return fail(st);
      launch_sqrt(s, D->d_hist + 3, D->d_hist + 3);
      double rn = 0.0;
      if ((st = d2h(s, &rn, D->d_hist + 3, sizeof(double))) != AMG_OK) return fail(st);
      D->ajac_stats[5] = rn;
   }
   if (relaxations) {
      *relaxations = sps ? 0 : sweeps;
      if (sps && (st = d2h(s, relaxations, count, sizeof(long long))) != AMG_OK) return fail(st);
   }
   // true residual f - A x with a synchronous exchange, and its global norm
   amgk::vcopy(s, f, v.f, 0, n);
   if ((st = dist_outer_residual(D, 1)) != AMG_OK) return fail(st);
   D->pre_ready = false;
   double hn[2] = {0, 0};
   if ((st = d2h(s, hn, D->d_hist + 1, sizeof(double))) != AMG_OK) return fail(st);
   // ||f|| (x0 = 0): the initial residual norm
   double *p;
   if ((st = amg_ctx_partials(c, 65536, &p)) != AMG_OK) return fail(st);
   int parts = 0;
   amgk::sumsq_partials(s, f, n, p, &parts);
   amgk::reduce_partials(s, p, parts, D->d_hist + 2, 0, c->d_scalars + 4096);
   if ((st = xp_allreduce(c, s, D->d_hist + 2, 1)) != AMG_OK) return fail(st);
   launch_sqrt(s, D->d_hist + 2, D->d_hist + 2);
   if ((st = d2h(s, hn + 1, D->d_hist + 2, sizeof(double))) != AMG_OK) return fail(st);
   D->r0norm = hn[1];
   D->have_state = true;
   D->ajac_stats[6] = hn[0]; // the true residual norm
   if (relres) *relres = hn[1] > 0 ? hn[0] / hn[1] : 0.0;
   for (double *q : dtmp) hipFree(q);
   return AMG_OK;
}

} // namespace
