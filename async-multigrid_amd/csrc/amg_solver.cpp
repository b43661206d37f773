// amg_solver.cpp -- host-side orchestration on the device: the level
// hierarchy (AllData analogue), the synchronous multiplicative V-cycle
// (SMEM_Sync_Parfor_Vcycle), the synchronous additive cycle
// (SMEM_Sync_Add_Vcycle), the SMEM_Solve outer loop with the Chebyshev
// update, and the asynchronous additive solver (SMEM_Async_Add_AMG) with one
// HIP stream per level.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <utility>
#include <thread>
#include <vector>

#include "amg_internal.h"

int amg_reduce_to_host(amg_ctx *c, const double *partials, int np, int do_sqrt, double *out);
int amg_hybrid_jgs_dev(amg_ctx *c, hipStream_t s, const amg_mat *A, const double *f, double *u,
                       double *u_prev, int n_vec, const int *d_blk, int nblk, int blk_lo,
                       int blk_hi, const double *ds, double weight, int sweeps, int zero_first,
                       int reverse, double *apply_u = nullptr, double *apply_priv = nullptr,
                       bool *applied = nullptr, unsigned long long *stamp = nullptr);
int amg_sym_jacobi_dev(hipStream_t s, const amg_mat *A, const double *f, double *u, double *y,
                       double *r, double omega, const double *l1, int sweeps, int zero_first,
                       int rb, int re, int variant);

namespace {

enum ProfCat { PROF_FINE_SPMV = 0, PROF_FINE_SMOOTH = 1, PROF_RESTRICT0 = 2, PROF_PROLONG0 = 3,
               PROF_OUTER = 4,
               PROF_NCAT = 5 };

struct Level {
   amg_mat *A = nullptr, *P = nullptr, *R = nullptr;
   int n = 0;
   double *f = nullptr, *u = nullptr, *u_alt = nullptr, *u_prev = nullptr, *y = nullptr,
          *r_fine = nullptr;
   double *l1 = nullptr, *adiag = nullptr;
   std::vector<int> blk;
   int *d_blk = nullptr;
   int zero_flag = 0;
   bool zero_done = false; // the zero-guess sweep already written by the restriction into this level
};

// per-level private vectors of the additive cycles (level_vector[k], SMEM_Setup.cpp:292-341)
struct AddLevel {
   std::vector<double *> r, e; // r[l], e[l] for l <= min(k+1, L-1)
   double *u_prev = nullptr, *y = nullptr, *u_priv = nullptr, *y_fine = nullptr, *scratch = nullptr;
   double *u_fine = nullptr, *u_coarse = nullptr, *u_coarse_prev = nullptr, *u_fine_prev = nullptr,
          *r_fine = nullptr;
   // asynchronous options: READ_RES private correction sum (level_vector[k].f[0]),
   // GLOBAL residual phase's fine smoothing correction and scratch (n0 each)
   double *f_acc = nullptr, *g_u = nullptr, *g_prev = nullptr, *g_y = nullptr, *g_r = nullptr;
   hipEvent_t ev_a = nullptr, ev_b = nullptr; // level stream <-> update stream (SEMI_ASYNC)
   double *xt = nullptr, *xy = nullptr;       // composed smoothed transfers' scratch (n0 each)
};

} // namespace

struct amg_hier {
   amg_ctx *ctx = nullptr;
   int L = 0;
   amg_opts o{};
   std::vector<Level> lv;
   std::vector<AddLevel> al;
   double *r0 = nullptr; // vector.r[0]: the outer residual
   double *e0 = nullptr, *e0_alt = nullptr; // BPX: vector.e[0] (+ ping-pong partner)
   double *u_outer = nullptr, *y_outer = nullptr;
   double *d_hist = nullptr; // device residual-norm history
   int hist_cap = 0;
   double r0norm = 0.0;
   double cheby_omega = 2.0;
   int iter = 0;
   bool have_state = false;
   bool pre_ready = false; // lv[0].u_alt holds u + w r0 / a_ii for the current u
   bool r0_stale = false;  // reuse_outer_residual 2: r0 not written for the current u
   // geometric transfers (detect_geo): geo[l] when R_l / P_l equal the box
   // transfers of level l (dims gl[l], weights d_geo_w[l] on the device);
   // geo0: level 0 is also plane-marched and runs the fused residual + restriction
   std::vector<char> geo;
   std::vector<amgk::GeoT> gl;
   std::vector<double *> d_geo_w;
   bool geo0 = false;
   // psw[l]: level l's prolongation + correction runs fused into its first
   // post-smoothing sweep (geometric P_l, 7-pt marched A_l of the same box)
   std::vector<char> psw;
   // xfr[l] / xfp[l]: level l's composed smoothed restriction / prolongation
   // runs as one fused pass (mz_xfer_restrict / mz_xfer_prolong: geometric
   // R_l / P_l, marched 7-pt A_l; the restriction needs uniform values)
   std::vector<char> xfr, xfp;
   // hipGraphs of launch-bound loops (ctx->graphs): the synchronous additive
   // cycle (g_add, on ctx->stream) and each asynchronous level's correction
   // (g_lev[k] on stream g_lev_s[k]); captured after one eager run (lazy
   // allocations), dropped when the options or blocks change
   unsigned g_gen = 0; // ctx->knob_gen the cached graphs were captured under
   hipGraphExec_t g_add = nullptr;
   bool g_add_warm = false;
   std::vector<hipGraphExec_t> g_lev;
   std::vector<hipStream_t> g_lev_s;
   std::vector<char> g_lev_warm;
   // fused level-0 last post sweep + outer residual (ctx->fuse_outer): the
   // V-cycle left its last post sweep to outer_residual; u2: u'' buffer;
   // store_u1: write u' (always in mode 1; mode 2: the last step of a batch)
   bool post_deferred = false;
   bool store_u1 = true;
   double *u2 = nullptr;
   // fuse_outer 3 without a stored u': u' of one z-slab (slab_planes + 2 planes)
   double *slab_scr = nullptr;
   long long slab_cap = 0;
   // AMG_SCHED_TIMED: per-level correction time (amg_hier_set_async_durations)
   // or recorded end times (amg_hier_set_async_times)
   std::vector<double> async_dur;
   std::vector<std::vector<double>> async_t;
   // per-correction end times of the last free race (amg_async_correction_ms)
   AmgCorrTimes corr;
   // the correction whose update-window start a fused update kernel records
   // (mark_update_start; -1: none)
   int mark_k = -1, mark_j = 0;
   unsigned long long *mark_stamp = nullptr; // its execution-window stamp
   // per level of the last amg_async_solve: ms from its start to the level's
   // last correction (amg_async_level_ms)
   std::vector<double> level_ms;
   // delay / fault injection: one generator per reference thread (srand(tid),
   // SMEM_Solve.cpp:113), reset by every solve
   std::vector<unsigned long long> delay_rng;
   std::vector<void *> allocs;
   // profiling
   std::vector<std::pair<hipEvent_t, hipEvent_t>> pend[PROF_NCAT];
   double prof_ms[PROF_NCAT] = {0, 0, 0, 0, 0};
   long long prof_n[PROF_NCAT] = {0, 0, 0, 0, 0};
};

static int dalloc(amg_hier *H, size_t n, double **p)
{
   hipError_t e = hipMalloc(p, std::max<size_t>(n, 1) * sizeof(double));
   if (e != hipSuccess)
      return amg_set_error(AMG_ERR_OOM, "amg_hier: allocation of %zu doubles: %s", n,
                           hipGetErrorString(e));
   H->allocs.push_back(*p);
   e = hipMemsetAsync(*p, 0, std::max<size_t>(n, 1) * sizeof(double), H->ctx->stream);
   if (e != hipSuccess) return amg_set_error(AMG_ERR_HIP, "memset: %s", hipGetErrorString(e));
   return AMG_OK;
}

// SMEM_Main.cpp:641-649: MULT and BPX run ONE_LEVEL (every thread on every
// level), the additive solvers ALL_LEVELS (thread groups per level)
static bool is_all_levels(const amg_opts &o)
{
   return !(o.solver == AMG_MULT || o.solver == AMG_BPX);
}

static bool is_multadd(const amg_opts &o)
{
   return o.solver == AMG_MULTADD || o.solver == AMG_ASYNC_MULTADD;
}

// ---- profiling helpers -----------------------------------------------------
struct ProfScope {
   amg_hier *H;
   int cat;
   hipStream_t s;
   hipEvent_t a = nullptr, b = nullptr;
   bool on;
   ProfScope(amg_hier *H_, int cat_, hipStream_t s_, bool enabled = true)
      : H(H_), cat(cat_), s(s_), on(enabled && H_->o.profile)
   {
      if (on) {
         hipEventCreate(&a);
         hipEventCreate(&b);
         hipEventRecord(a, s);
      }
   }
   ~ProfScope()
   {
      if (on) {
         hipEventRecord(b, s);
         H->pend[cat].push_back({a, b});
      }
   }
};

static void prof_drain(amg_hier *H)
{
   for (int c = 0; c < PROF_NCAT; c++) {
      for (auto &p : H->pend[c]) {
         float ms = 0.f;
         hipEventSynchronize(p.second);
         if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
            H->prof_ms[c] += ms;
            H->prof_n[c] += 1;
         }
         hipEventDestroy(p.first);
         hipEventDestroy(p.second);
      }
      H->pend[c].clear();
   }
}

extern "C" int amg_hier_profile_read(amg_hier *H, double *ms, long long *launches, int reset)
{
   AMG_ARG(H, "amg_hier_profile_read: null hierarchy");
   AMG_HIP(hipStreamSynchronize(H->ctx->stream));
   prof_drain(H);
   for (int c = 0; c < PROF_NCAT; c++) {
      if (ms) ms[c] = H->prof_ms[c];
      if (launches) launches[c] = H->prof_n[c];
      if (reset) {
         H->prof_ms[c] = 0;
         H->prof_n[c] = 0;
      }
   }
   return AMG_OK;
}

// ---- block partitions --------------------------------------------------------
static void partition_equal(int n, int T, std::vector<int> &blk)
{
   // SMEM_Setup.cpp:1018-1030
   blk.assign(T + 1, 0);
   int size = n / T, rest = n - size * T;
   for (int t = 0; t < T; t++) blk[t] = (t < rest) ? t * size + t : t * size + rest;
   blk[T] = n;
}

static int upload_blocks(amg_hier *H, Level &l)
{
   if (l.d_blk) {
      hipFree(l.d_blk);
      l.d_blk = nullptr;
   }
   AMG_HIP(hipMalloc(&l.d_blk, l.blk.size() * sizeof(int)));
   AMG_HIP(hipMemcpyAsync(l.d_blk, l.blk.data(), l.blk.size() * sizeof(int), hipMemcpyHostToDevice,
                          H->ctx->stream));
   AMG_HIP(hipStreamSynchronize(H->ctx->stream));
   return AMG_OK;
}

static int default_blocks(amg_hier *H, Level &l)
{
   if (H->o.num_threads > 0) {
      partition_equal(l.n, H->o.num_threads, l.blk);
   } else {
      const int B = std::max(1, H->o.jgs_block_rows);
      const int nb = std::max(1, (l.n + B - 1) / B);
      l.blk.resize(nb + 1);
      for (int b = 0; b <= nb; b++) l.blk[b] = std::min(l.n, b * B);
   }
   return upload_blocks(H, l);
}

static void graphs_reset(amg_hier *H);

extern "C" int amg_hier_set_blocks(amg_hier *H, int level, const int *blk, int nblk)
{
   AMG_ARG(H && blk && level >= 0 && level < H->L && nblk > 0, "amg_hier_set_blocks: bad argument");
   Level &l = H->lv[level];
   AMG_ARG(blk[0] == 0 && blk[nblk] == l.n, "amg_hier_set_blocks: blocks must cover [0,%d)", l.n);
   for (int b = 0; b < nblk; b++) AMG_ARG(blk[b] <= blk[b + 1], "amg_hier_set_blocks: unsorted");
   l.blk.assign(blk, blk + nblk + 1);
   graphs_reset(H);
   return upload_blocks(H, l);
}

// ---- creation ----------------------------------------------------------------
static int hier_prepare_smoother_arrays(amg_hier *H)
{
   hipStream_t s = H->ctx->stream;
   for (int l = 0; l < H->L; l++) {
      Level &v = H->lv[l];
      amgk::l1_norms(s, v.A, v.l1);
      amgk::a_diag(s, v.A->diag, H->o.smooth_weight, v.adiag, v.n);
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

// Geometric transfers: level 0's box comes from a plane-marched A_0 (7-pt on
// nx * ny * nz: S = nx, P = nx ny); level l + 1's box is level l's halved
// while every level above it was geometric.  R_l / P_l qualify when they equal,
// entry for entry (checked on the device), coarse K <-> fine 2K + {0,1,2}^3
// with one weight per offset (read from coarse row (1, 1, 1) of R_l).  Such
// levels restrict / prolong with the geometric kernels; level 0 additionally
// fuses its residual into the restriction when the box fits that kernel.
static int check_geo_level(amg_hier *H, int l, int nx, int ny, int nz, bool *ok)
{
   *ok = false;
   const amg_mat *A = H->lv[l].A, *R = H->lv[l].R, *P = H->lv[l].P;
   if ((nx | ny | nz) & 1 || nx < 6 || ny < 6 || nz < 6) return AMG_OK;
   if ((long long)nx * ny * nz != A->nrows) return AMG_OK;
   const int ncx = nx / 2, ncy = ny / 2;
   const long long nc = (long long)A->nrows / 8;
   if (R->nrows != nc || R->ncols != A->nrows || P->nrows != A->nrows || P->ncols != nc) return AMG_OK;
   hipStream_t s = H->ctx->stream;
   const int K = (1 * ncy + 1) * ncx + 1;
   int rp[2];
   AMG_HIP(hipMemcpyAsync(rp, R->rowptr + K, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   if (rp[1] - rp[0] != 27) return AMG_OK;
   amgk::GeoT g{};
   AMG_HIP(hipMemcpyAsync(g.w, R->val + rp[0], sizeof(g.w), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   g.nx = nx;
   g.ny = ny;
   g.nz = nz;
   int *bad = nullptr;
   AMG_HIP(hipMalloc(&bad, sizeof(int)));
   AMG_HIP(hipMemsetAsync(bad, 0, sizeof(int), s));
   amgk::geo_check(s, R, 0, g, bad);
   amgk::geo_check(s, P, 1, g, bad);
   int hbad = 1;
   hipError_t e = hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, s);
   if (e == hipSuccess) e = hipStreamSynchronize(s);
   hipFree(bad);
   if (e != hipSuccess) return amg_set_error(AMG_ERR_HIP, "check_geo_level: %s", hipGetErrorString(e));
   if (hbad) return AMG_OK;
   AMG_TRY(dalloc(H, 27, &H->d_geo_w[l]));
   AMG_HIP(hipMemcpyAsync(H->d_geo_w[l], g.w, sizeof(g.w), hipMemcpyHostToDevice, s));
   H->gl[l] = g;
   *ok = true;
   return AMG_OK;
}

static int detect_geo(amg_hier *H)
{
   H->geo.assign(H->L, 0);
   H->gl.assign(H->L, amgk::GeoT{});
   H->d_geo_w.assign(H->L, nullptr);
   H->geo0 = false;
   H->psw.assign(H->L, 0);
   H->xfr.assign(H->L, 0);
   H->xfp.assign(H->L, 0);
   if (H->L < 2 || !H->ctx->fuse_transfer) return AMG_OK;
   const amg_mat *A = H->lv[0].A;
   if (!A->mz_P || A->mz_P % A->mz_S) return AMG_OK;
   int nx = A->mz_S, ny = A->mz_P / A->mz_S, nz = A->nrows / A->mz_P;
   for (int l = 0; l < H->L - 1; l++) {
      bool ok = false;
      AMG_TRY(check_geo_level(H, l, nx, ny, nz, &ok));
      if (!ok) break;
      H->geo[l] = 1;
      nx /= 2;
      ny /= 2;
      nz /= 2;
   }
   const amgk::GeoT &g = H->gl[0];
   for (int l = 0; l < H->L - 1; l++) {
      const amg_mat *Al = H->lv[l].A;
      const amgk::GeoT &gg = H->gl[l];
      const bool box7 = H->geo[l] && Al->mz_P && !Al->mz27 && Al->mz_S == gg.nx &&
                        (long long)Al->mz_P == (long long)gg.nx * gg.ny && Al->nrows / Al->mz_P == gg.nz;
      // the LDS-ring forms (4 / 5) fuse only the levels they tile (lines of
      // 512k points, 2 / 4 lines per workgroup); the others stay unfused
      const int fp = H->ctx->fuse_prolong;
      H->psw[l] = box7 && fp && (fp < 4 || (gg.nx % 512 == 0 && gg.ny % (fp == 4 ? 2 : 4) == 0));
      H->xfp[l] = box7 && H->ctx->fuse_xfer;
      H->xfr[l] = box7 && H->ctx->fuse_xfer && Al->mp_uni && gg.nx >= 64 && gg.nx <= 512 && 512 % gg.nx == 0 &&
                  (gg.ny / 2) % (512 / gg.nx) == 0;
   }
   H->geo0 = H->geo[0] && !A->mz27 && g.nx >= 64 && g.nx <= 512 && 512 % g.nx == 0 && (g.ny / 2) % (512 / g.nx) == 0;
   return AMG_OK;
}

extern "C" int amg_hier_fused(const amg_hier *H)
{
   if (!H) return 0;
   int m = H->geo0 ? 1 : 0;
   for (int l = 0; l < H->L; l++)
      if (H->geo[l]) m |= 2 << l;
   return m;
}

extern "C" int amg_hier_fused_prolong(const amg_hier *H)
{
   if (!H) return 0;
   int m = 0;
   for (int l = 0; l < (int)H->psw.size(); l++)
      if (H->psw[l]) m |= 1 << l;
   return m;
}

extern "C" int amg_hier_create(amg_ctx *c, int L, amg_mat *const *A, amg_mat *const *P,
                               amg_mat *const *R, const amg_opts *opts, amg_hier **out)
{
   AMG_ARG(c && A && out && L >= 1 && opts, "amg_hier_create: bad argument");
   AMG_ARG(L == 1 || (P && R), "amg_hier_create: P and R required for L > 1");
   for (int l = 0; l < L; l++) {
      AMG_ARG(A[l] && A[l]->nrows == A[l]->ncols, "amg_hier_create: A[%d] must be square", l);
      if (l < L - 1) {
         AMG_ARG(P[l] && R[l], "amg_hier_create: P/R[%d] missing", l);
         AMG_ARG(P[l]->nrows == A[l]->nrows && P[l]->ncols == A[l + 1]->nrows,
                 "amg_hier_create: P[%d] is %dx%d, expected %dx%d", l, P[l]->nrows, P[l]->ncols,
                 A[l]->nrows, A[l + 1]->nrows);
         AMG_ARG(R[l]->nrows == A[l + 1]->nrows && R[l]->ncols == A[l]->nrows,
                 "amg_hier_create: R[%d] is %dx%d", l, R[l]->nrows, R[l]->ncols);
      }
   }
   amg_hier *H = new amg_hier();
   H->ctx = c;
   H->L = L;
   H->o = *opts;
   H->lv.resize(L);
   for (int l = 0; l < L; l++) {
      Level &v = H->lv[l];
      v.A = A[l];
      v.P = (l < L - 1) ? P[l] : nullptr;
      v.R = (l < L - 1) ? R[l] : nullptr;
      v.n = A[l]->nrows;
      AMG_TRY(dalloc(H, v.n, &v.f));
      AMG_TRY(dalloc(H, v.n, &v.u));
      AMG_TRY(dalloc(H, v.n, &v.u_alt));
      AMG_TRY(dalloc(H, v.n, &v.u_prev));
      AMG_TRY(dalloc(H, v.n, &v.y));
      AMG_TRY(dalloc(H, v.n, &v.r_fine));
      AMG_TRY(dalloc(H, v.n, &v.l1));
      AMG_TRY(dalloc(H, v.n, &v.adiag));
      AMG_TRY(default_blocks(H, v));
   }
   AMG_TRY(dalloc(H, H->lv[0].n, &H->r0));
   if (H->o.solver == AMG_BPX) {
      AMG_TRY(dalloc(H, H->lv[0].n, &H->e0));
      AMG_TRY(dalloc(H, H->lv[0].n, &H->e0_alt));
   }
   AMG_TRY(dalloc(H, H->lv[0].n, &H->u_outer));
   AMG_TRY(dalloc(H, H->lv[0].n, &H->y_outer));
   H->hist_cap = 1 << 16;
   AMG_TRY(dalloc(H, H->hist_cap, &H->d_hist));
   if (is_all_levels(H->o)) {
      H->al.resize(L);
      const int n0 = H->lv[0].n;
      for (int k = 0; k < L; k++) {
         AddLevel &a = H->al[k];
         const int top = std::min(k + 1, L - 1);
         a.r.assign(L, nullptr);
         a.e.assign(L, nullptr);
         for (int l = 0; l <= top; l++) {
            if (l > 0) AMG_TRY(dalloc(H, H->lv[l].n, &a.r[l])); // r[0]: the caller's fine residual
            AMG_TRY(dalloc(H, H->lv[l].n, &a.e[l]));
         }
         const int nk = H->lv[k].n;
         AMG_TRY(dalloc(H, std::max(nk, n0), &a.u_prev));
         AMG_TRY(dalloc(H, std::max(nk, n0), &a.y));
         AMG_TRY(dalloc(H, n0, &a.u_priv));
         AMG_TRY(dalloc(H, n0, &a.y_fine));
         AMG_TRY(dalloc(H, std::max(nk, n0), &a.scratch));
         AMG_TRY(dalloc(H, nk, &a.u_fine));
         AMG_TRY(dalloc(H, nk, &a.u_fine_prev));
         AMG_TRY(dalloc(H, nk, &a.r_fine));
         const int nc = H->lv[top].n;
         AMG_TRY(dalloc(H, nc, &a.u_coarse));
         AMG_TRY(dalloc(H, nc, &a.u_coarse_prev));
      }
   }
   AMG_TRY(hier_prepare_smoother_arrays(H));
   AMG_TRY(detect_geo(H));
   AMG_HIP(hipStreamSynchronize(c->stream));
   *out = H;
   return AMG_OK;
}

static void graphs_reset(amg_hier *H)
{
   if (H->g_add) hipGraphExecDestroy(H->g_add);
   H->g_add = nullptr;
   H->g_add_warm = false;
   for (auto &g : H->g_lev)
      if (g) hipGraphExecDestroy(g);
   H->g_lev.assign(H->L, nullptr);
   H->g_lev_s.assign(H->L, nullptr);
   H->g_lev_warm.assign(H->L, 0);
}

// a context knob changed since the cached graphs were captured: drop them
// (kernel knobs are read at launch, so a replayed graph keeps the old setting)
static void graphs_check(amg_hier *H)
{
   if (H->g_gen != H->ctx->knob_gen) {
      graphs_reset(H);
      H->g_gen = H->ctx->knob_gen;
   }
}

// issue `body` on stream s through a cached graph: the first call runs it
// eagerly (allocations, scratch growth), the second captures and instantiates,
// every call from then on launches the graph
template <class F>
static int graph_issue(hipGraphExec_t &gx, bool &warm, hipStream_t s, F body)
{
   if (!warm) {
      warm = true;
      AMG_TRY(body());
      AMG_HIP(hipGetLastError());
      return AMG_OK;
   }
   if (!gx) {
      AMG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const int st = body();
      hipGraph_t g = nullptr;
      const hipError_t e = hipStreamEndCapture(s, &g);
      if (st != AMG_OK) {
         if (g) hipGraphDestroy(g);
         return st;
      }
      if (e != hipSuccess) {
         if (g) hipGraphDestroy(g);
         return amg_set_error(AMG_ERR_HIP, "graph capture: %s", hipGetErrorString(e));
      }
      const hipError_t ei = hipGraphInstantiate(&gx, g, nullptr, nullptr, 0);
      hipGraphDestroy(g);
      if (ei != hipSuccess) {
         gx = nullptr;
         return amg_set_error(AMG_ERR_HIP, "graph instantiate: %s", hipGetErrorString(ei));
      }
   }
   AMG_HIP(hipGraphLaunch(gx, s));
   return AMG_OK;
}

extern "C" int amg_hier_free(amg_hier *H)
{
   if (!H) return AMG_OK;
   std::lock_guard<std::recursive_mutex> td(amg_teardown_mutex());
   hipStreamSynchronize(H->ctx->stream);
   for (auto s : H->ctx->level_streams) hipStreamSynchronize(s);
   prof_drain(H);
   graphs_reset(H);
   for (auto &a : H->al) {
      if (a.ev_a) hipEventDestroy(a.ev_a);
      if (a.ev_b) hipEventDestroy(a.ev_b);
   }
   for (void *p : H->allocs) hipFree(p);
   for (auto &l : H->lv) hipFree(l.d_blk);
   delete H;
   return AMG_OK;
}

extern "C" int amg_hier_set_opts(amg_hier *H, const amg_opts *opts)
{
   AMG_ARG(H && opts, "amg_hier_set_opts: null argument");
   AMG_ARG(is_all_levels(*opts) == is_all_levels(H->o),
           "amg_hier_set_opts: cannot switch between ONE_LEVEL and ALL_LEVELS solvers");
   const bool w = opts->smooth_weight != H->o.smooth_weight;
   const bool t = opts->num_threads != H->o.num_threads || opts->jgs_block_rows != H->o.jgs_block_rows;
   H->o = *opts;
   graphs_reset(H);
   if (w) AMG_TRY(hier_prepare_smoother_arrays(H));
   if (t)
      for (auto &l : H->lv) AMG_TRY(default_blocks(H, l));
   return AMG_OK;
}

extern "C" int amg_hier_vec(amg_hier *H, int which, int level, amg_vec **out)
{
   AMG_ARG(H && out && level >= 0 && level < H->L, "amg_hier_vec: bad argument");
   amg_vec *v = new amg_vec();
   v->ctx = H->ctx;
   v->n = H->lv[level].n;
   v->owns = false;
   switch (which) {
   case AMG_VEC_F: v->d = H->lv[level].f; break;
   case AMG_VEC_U: v->d = H->lv[level].u; break;
   case AMG_VEC_R:
      if (level == 0 && H->r0_stale) {
         // the outer residual of the current iterate, in the order of the
         // fused kernel that skipped it (reuse_outer_residual 2)
         Level &l0 = H->lv[0];
         amgk::spgemv(H->ctx->stream, l0.A, l0.u, l0.f, amgk::gemv_mode(-1.0, 1.0), H->r0, 0, l0.n,
                      nullptr);
         AMG_HIP(hipStreamSynchronize(H->ctx->stream));
         H->r0_stale = false;
      }
      v->d = level == 0 ? H->r0 : H->lv[level].r_fine;
      break;
   default: delete v; return amg_set_error(AMG_ERR_ARG, "amg_hier_vec: unknown vector %d", which);
   }
   *out = v;
   return AMG_OK;
}

// ---- smoothing (SMEM_Smooth dispatcher, SMEM_Solve.cpp:264-377) --------------
// ONE_LEVEL (MULT) smoothing of level l's f/u; may swap u <-> u_alt.
static void smooth_one_level(amg_hier *H, hipStream_t s, int l, const double *f, int sweeps,
                             bool from_outer_residual)
{
   Level &v = H->lv[l];
   const amg_opts &o = H->o;
   const int zf = v.zero_flag;
   const bool prof = (l == 0);
   if (o.smoother == AMG_HYBRID_JACOBI_GAUSS_SEIDEL ||
       o.smoother == AMG_L1_HYBRID_JACOBI_GAUSS_SEIDEL) {
      const double *ds = (o.smoother == AMG_L1_HYBRID_JACOBI_GAUSS_SEIDEL) ? v.l1 : v.adiag;
      ProfScope ps(H, PROF_FINE_SMOOTH, s, prof);
      amg_hybrid_jgs_dev(H->ctx, s, v.A, f, v.u, v.u_prev, v.n, v.d_blk, (int)v.blk.size() - 1, 0,
                         v.n, ds, 1.0, sweeps, zf, 0);
      return;
   }
   if (o.smoother == AMG_ASYNC_GAUSS_SEIDEL || o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL) {
      // SMEM_Async_Parfor_GaussSeidel / SMEM_SemiAsync_Parfor_GaussSeidel
      // (SMEM_Solve.cpp:342-347): in place, no zero-guess special case
      ProfScope ps(H, PROF_FINE_SMOOTH, s, prof);
      amgk::async_gs(s, v.A, f, v.u, v.d_blk, (int)v.blk.size() - 1, sweeps,
                     o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL, 0);
      return;
   }
   const bool l1 = (o.smoother == AMG_L1_JACOBI);
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zf == 1) {
         if (v.zero_done)
            v.zero_done = false; // folded into the restriction that produced f (same bits)
         else
            amgk::jacobi_zero(s, v.A->diag, f, l1 ? v.l1 : nullptr, o.smooth_weight, v.u, 0, v.n, 0);
      } else if (k == 0 && from_outer_residual && H->pre_ready) {
         // the outer-residual kernel already produced u + w r / a_ii from this
         // very u and r = f - A u (same summation order): take it
         std::swap(v.u, v.u_alt);
         H->pre_ready = false;
      } else if (k == 0 && from_outer_residual) {
         // r0 = f - A u was computed by the outer loop on this very u with the
         // same summation order; the sweep is u += w r / a (bit-identical)
         amgk::jacobi_from_residual(s, v.A->diag, H->r0, l1 ? v.l1 : nullptr, o.smooth_weight,
                                    v.u, 0, v.n);
      } else {
         {
            ProfScope ps(H, PROF_FINE_SMOOTH, s, prof);
            amgk::jacobi_sweep(s, v.A, f, v.u, l1 ? v.l1 : nullptr, o.smooth_weight, v.u_alt, 0, v.n);
         }
         std::swap(v.u, v.u_alt);
      }
   }
}

// the free race's update-window start of the correction in H->mark_k, right
// before the kernel that adds it into the shared iterate
static void mark_update_start(amg_hier *H, hipStream_t s)
{
   if (H->mark_k < 0) return;
   H->corr.record_start(H->mark_k, H->mark_j, s);
   H->mark_k = -1;
}

// ALL_LEVELS smoothing of A[Alevel] with f -> u (row range version of the
// smoothers), zero flag of `flag_level`.  apply_u (hybrid JGS, the LDS tile
// form): the FULL_ASYNC correction apply_u += u, apply_priv = the value after
// it, folded into the last sweep; returns whether it was
static bool smooth_all_levels(amg_hier *H, hipStream_t s, int Alevel, const double *f, double *u,
                              double *u_prev, double *y, double *r, int sweeps, int flag_level,
                              double *apply_u = nullptr, double *apply_priv = nullptr)
{
   Level &v = H->lv[Alevel];
   const amg_opts &o = H->o;
   const int zf = H->lv[flag_level].zero_flag;
   const bool sym = is_multadd(o) && o.num_post_smooth_sweeps > 0 && o.num_pre_smooth_sweeps > 0;
   if (o.smoother == AMG_HYBRID_JACOBI_GAUSS_SEIDEL) {
      const int nb = (int)v.blk.size() - 1;
      if (!apply_u || sweeps <= 0) {
         amg_hybrid_jgs_dev(H->ctx, s, v.A, f, u, u_prev, v.n, v.d_blk, nb, 0, v.n, nullptr, 1.0, sweeps, zf, 0);
         return false;
      }
      if (sweeps > 1)
         amg_hybrid_jgs_dev(H->ctx, s, v.A, f, u, u_prev, v.n, v.d_blk, nb, 0, v.n, nullptr, 1.0, sweeps - 1, zf, 0);
      mark_update_start(H, s);
      bool applied = false;
      amg_hybrid_jgs_dev(H->ctx, s, v.A, f, u, u_prev, v.n, v.d_blk, nb, 0, v.n, nullptr, 1.0, 1,
                         sweeps > 1 ? 0 : zf, 0, apply_u, apply_priv, &applied, H->mark_stamp);
      return applied;
   } else if (o.smoother == AMG_ASYNC_GAUSS_SEIDEL || o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL) {
      // SMEM_Async_GaussSeidel / SMEM_SemiAsync_GaussSeidel (SMEM_Solve.cpp:281-286)
      amgk::async_gs(s, v.A, f, u, v.d_blk, (int)v.blk.size() - 1, sweeps,
                     o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL, 0);
   } else if (o.smoother == AMG_L1_JACOBI) {
      if (sym) {
         amg_sym_jacobi_dev(s, v.A, f, u, y, r, 1.0, v.l1, sweeps, zf, 0, v.n, 0);
      } else {
         for (int k = 0; k < sweeps; k++) {
            if (k == 0 && zf == 1) {
               amgk::jacobi_zero(s, v.A->diag, f, v.l1, 1.0, u, 0, v.n, 0);
            } else {
               amgk::vcopy(s, u, u_prev, 0, v.n);
               amgk::jacobi_sweep(s, v.A, f, u_prev, v.l1, 1.0, u, 0, v.n);
            }
         }
      }
   } else {
      if (sym) {
         amg_sym_jacobi_dev(s, v.A, f, u, y, r, o.smooth_weight, nullptr, sweeps, zf, 0, v.n, 0);
      } else {
         for (int k = 0; k < sweeps; k++) {
            if (k == 0 && zf == 1) {
               amgk::jacobi_zero(s, v.A->diag, f, nullptr, o.smooth_weight, u, 0, v.n, 0);
            } else {
               amgk::vcopy(s, u, u_prev, 0, v.n);
               amgk::jacobi_sweep(s, v.A, f, u_prev, nullptr, o.smooth_weight, u, 0, v.n);
            }
         }
      }
   }
   return false;
}

// ---- SMEM_Sync_Parfor_Vcycle (SMEM_Sync_AMG.cpp:8-145) -------------------------
// defer_post: leave level 0's last post-smoothing sweep to outer_residual,
// which runs it fused with the outer residual (mz_sweep_outer)
static void vcycle(amg_hier *H, bool precond, bool reuse_r0, bool defer_post = false)
{
   hipStream_t s = H->ctx->stream;
   const amg_opts &o = H->o;
   const int L = H->L;
   const amgk::Gemv res_mode = amgk::gemv_mode(-1.0, 1.0);
   const amgk::Gemv mv_mode = amgk::gemv_mode(1.0, 0.0);
   const amgk::Gemv pro_mode = amgk::gemv_mode(1.0, 1.0);
   static const bool zg_fold = [] {
      const char *e = std::getenv("AMG_ZG_FOLD");
      return e ? std::atoi(e) != 0 : true;
   }();
   for (auto &lv : H->lv) lv.zero_done = false;
   for (int l = 0; l < L - 1; l++) {
      Level &v = H->lv[l];
      v.zero_flag = 1;
      if (l == 0 && !precond) v.zero_flag = 0;
      const double *f_fine = (l == 0 && precond) ? H->r0 : v.f;
      smooth_one_level(H, s, l, f_fine, o.num_pre_smooth_sweeps, l == 0 && reuse_r0);
      // level l + 1 (not the coarsest) starts its pre-smoothing with the
      // zero-guess Jacobi sweep u = w f / a: a geometric restriction writes it
      // together with f (one pass over the coarse level fewer)
      Level &nx = H->lv[l + 1];
      amgk::ZeroGuess zg;
      if (zg_fold && l + 1 < L - 1 && o.smoother == AMG_JACOBI && o.num_pre_smooth_sweeps >= 1) {
         zg.d = nx.A->diag;
         zg.w = o.smooth_weight;
         zg.u = nx.u;
         zg.hi = nx.n;
         zg.err = H->ctx->d_err;
      }
      if (l == 0 && H->geo0) {
         // level-0 residual and restriction in one pass (no r_fine vector)
         ProfScope ps(H, PROF_FINE_SPMV, s);
         amgk::mz_residual_restrict(s, v.A, f_fine, v.u, H->gl[0], H->d_geo_w[0], nx.f, 0, -1, 0, 0, zg);
         nx.zero_done = zg.u != nullptr;
         continue;
      }
      {
         ProfScope ps(H, PROF_FINE_SPMV, s, l == 0);
         amgk::spgemv(s, v.A, v.u, f_fine, res_mode, v.r_fine, 0, v.n, nullptr);
      }
      {
         ProfScope ps(H, PROF_RESTRICT0, s, l == 0);
         if (H->geo[l]) {
            amgk::geo_restrict(s, H->gl[l], H->d_geo_w[l], v.r_fine, nx.f, 0, -1, 0, 0, zg);
            nx.zero_done = zg.u != nullptr;
         }
         else
            amgk::spgemv(s, v.R, v.r_fine, nullptr, mv_mode, H->lv[l + 1].f, 0, H->lv[l + 1].n,
                         nullptr);
      }
   }
   Level &c = H->lv[L - 1];
   smooth_one_level(H, s, L - 1, c.f, o.num_pre_smooth_sweeps + o.num_post_smooth_sweeps, false);
   for (int l = L - 2; l >= 0; l--) {
      Level &v = H->lv[l];
      v.zero_flag = 0;
      const double *f_fine = (l == 0 && precond) ? H->r0 : v.f;
      const bool l1 = o.smoother == AMG_L1_JACOBI;
      if (H->psw[l] && o.num_post_smooth_sweeps >= 1 && (l1 || o.smoother == AMG_JACOBI)) {
         // u += P e fused into the first post sweep (the corrected u is never
         // stored; the sweep's output is the same bits)
         {
            ProfScope ps(H, PROF_FINE_SMOOTH, s, l == 0);
            amgk::mz_prolong_sweep(s, v.A, f_fine, v.u, H->lv[l + 1].u, H->gl[l], H->d_geo_w[l],
                                   l1 ? v.l1 : nullptr, o.smooth_weight, v.u_alt);
         }
         std::swap(v.u, v.u_alt);
         smooth_one_level(H, s, l, f_fine, o.num_post_smooth_sweeps - 1, false);
         continue;
      }
      {
         ProfScope ps(H, PROF_PROLONG0, s, l == 0);
         if (H->geo[l])
            amgk::geo_prolong(s, H->gl[l], H->d_geo_w[l], H->lv[l + 1].u, v.u);
         else
            amgk::spgemv(s, v.P, H->lv[l + 1].u, v.u, pro_mode, v.u, 0, v.n, nullptr);
      }
      if (l == 0 && defer_post) {
         smooth_one_level(H, s, l, f_fine, o.num_post_smooth_sweeps - 1, false);
         H->post_deferred = true;
         continue;
      }
      smooth_one_level(H, s, l, f_fine, o.num_post_smooth_sweeps, false);
   }
}

// ---- SMEM_Sync_Parfor_BPXcycle (SMEM_Sync_AMG.cpp:147-294), solver BPX ----------
// r[0] (the outer residual) restricted to every level; every level (the
// coarsest too) smoothed from a zero guess with num_pre sweeps into its
// correction e[l]; e_fine += P e_coarse upwards; u += e[0] (u = e[0] in
// preconditioner mode).  e[l] = lv[l].u and r[l] = lv[l].f for l > 0 (the
// cycle uses neither for anything else); e[0] has its own pair.
static void bpx_cycle(amg_hier *H, bool precond)
{
   hipStream_t s = H->ctx->stream;
   const amg_opts &o = H->o;
   const int L = H->L;
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   const amgk::Gemv pro_mode = amgk::gemv_mode(1.0, 1.0);
   for (int l = 0; l < L - 1; l++) {
      ProfScope ps(H, PROF_RESTRICT0, s, l == 0);
      amgk::spgemv(s, H->lv[l].R, l == 0 ? H->r0 : H->lv[l].f, nullptr, mv, H->lv[l + 1].f, 0,
                   H->lv[l + 1].n, nullptr);
   }
   Level &v0 = H->lv[0];
   for (int l = 0; l < L; l++) {
      H->lv[l].zero_flag = 1;
      if (l == 0) {
         std::swap(v0.u, H->e0);
         std::swap(v0.u_alt, H->e0_alt);
      }
      smooth_one_level(H, s, l, l == 0 ? H->r0 : H->lv[l].f, o.num_pre_smooth_sweeps, false);
      if (l == 0) {
         std::swap(v0.u, H->e0);
         std::swap(v0.u_alt, H->e0_alt);
      }
   }
   for (int l = L - 2; l >= 0; l--) {
      double *ef = (l == 0) ? H->e0 : H->lv[l].u;
      ProfScope ps(H, PROF_PROLONG0, s, l == 0);
      amgk::spgemv(s, H->lv[l].P, H->lv[l + 1].u, ef, pro_mode, ef, 0, H->lv[l].n, nullptr);
   }
   if (precond)
      amgk::vcopy(s, H->e0, v0.u, 0, v0.n);
   else
      amgk::vaxpy(s, 1.0, H->e0, v0.u, 0, v0.n);
}

// ---- SMEM_Sync_Add_Vcycle (SMEM_Sync_AMG.cpp:408-621), res_compute LOCAL ------
// The level corrections are accumulated into u in level order.
// MULTADD with smooth_transfer: the reference's smoothed transfers
// (SmoothTransfer, SMEM_Setup.cpp:1173-1254) composed from the plain P, R, A
// forms P~ only with post-smoothing and R~ only with pre-smoothing (SMEM_Setup.cpp:1176-1180,1245-1250)
static bool composed_transfers(const amg_hier *H)
{
   return H->o.smooth_transfer == 1 && is_multadd(H->o) &&
          (H->o.num_pre_smooth_sweeps > 0 || H->o.num_post_smooth_sweeps > 0);
}
static bool composed_r(const amg_hier *H) { return composed_transfers(H) && H->o.num_pre_smooth_sweeps > 0; }
static bool composed_p(const amg_hier *H) { return composed_transfers(H) && H->o.num_post_smooth_sweeps > 0; }

// rc = R~_l r (composed) or R_l r; t / y: scratch of level l's size
static void xfer_restrict(amg_hier *H, hipStream_t s, int l, const double *r, double *rc, double *t, double *y)
{
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   const Level &v = H->lv[l];
   if (composed_r(H) && H->xfr[l]) {
      amgk::mz_xfer_restrict(s, v.A, r, H->gl[l], H->d_geo_w[l], H->o.smooth_weight, rc);
      return;
   }
   if (composed_r(H)) {
      // t = r ./ a;  y = A t;  t = r + (-w) y;  rc = R t
      amgk::xfer_div(s, v.A->diag, r, t, 0, v.n);
      amgk::spgemv(s, v.A, t, nullptr, mv, y, 0, v.n, nullptr);
      amgk::xfer_sub(s, H->o.smooth_weight, r, y, t, 0, v.n);
      r = t;
   }
   if (H->geo[l]) // the checked geometric R (bit-identical to its SpMV)
      amgk::geo_restrict(s, H->gl[l], H->d_geo_w[l], r, rc);
   else
      amgk::spgemv(s, v.R, r, nullptr, mv, rc, 0, H->lv[l + 1].n, nullptr);
}

// ef = P~_l ec (composed) or P_l ec; y: scratch of level l's size.  apply
// (level 0, composed, fused form only): 1 = the FULL_ASYNC atomic correction
// u += ef, u_priv = u after it; 2 = u += ef -- ef itself is then not stored;
// returns whether the correction was applied
static bool xfer_prolong(amg_hier *H, hipStream_t s, int l, const double *ec, double *ef, double *y, int apply = 0,
                         double *u = nullptr, double *u_priv = nullptr)
{
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   const Level &v = H->lv[l];
   if (composed_p(H) && H->xfp[l]) {
      if (apply) mark_update_start(H, s);
      if (apply)
         amgk::mz_xfer_prolong(s, v.A, ec, H->gl[l], H->d_geo_w[l], H->o.smooth_weight, apply, u, u_priv, 0, -1, 0,
                               0, H->mark_stamp);
      else
         amgk::mz_xfer_prolong(s, v.A, ec, H->gl[l], H->d_geo_w[l], H->o.smooth_weight, 0, ef, nullptr);
      return apply != 0;
   }
   if (H->geo[l]) // u = P e from 0.0 (the SpMV's alpha 1, beta 0 start)
      amgk::geo_prolong(s, H->gl[l], H->d_geo_w[l], ec, ef, 0, -1, 0, 0, 1);
   else
      amgk::spgemv(s, v.P, ec, nullptr, mv, ef, 0, v.n, nullptr);
   if (composed_p(H)) {
      // y = A ef;  ef = ef + (-w) (y ./ a)
      amgk::spgemv(s, v.A, ef, nullptr, mv, y, 0, v.n, nullptr);
      amgk::xfer_corr(s, H->o.smooth_weight, y, v.A->diag, ef, 0, v.n);
   }
   return false;
}

static int ensure_xfer_scratch(amg_hier *H, AddLevel &a)
{
   if (!composed_transfers(H) || a.xt) return AMG_OK;
   AMG_TRY(dalloc(H, H->lv[0].n, &a.xt));
   AMG_TRY(dalloc(H, H->lv[0].n, &a.xy));
   return AMG_OK;
}

// apply / u / u_priv: the level-0 correction fused into the last prolongation
// where it can be (xfer_prolong); returns whether it was (e[0] not written)
static bool add_level_correction(amg_hier *H, hipStream_t s, int k, const double *r_fine0, int apply = 0,
                                 double *u = nullptr, double *u_priv = nullptr)
{
   const int L = H->L;
   const amg_opts &o = H->o;
   const bool multadd = is_multadd(o);
   AddLevel &a = H->al[k];
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   H->lv[k].zero_flag = 1;
   const int coarsest = multadd ? k : k + 1;
   // r[0] = the fine residual (level_vector[k].r[0], SMEM_Sync_AMG.cpp:418-421):
   // only ever read, so the caller's vector stands in for the copy
   auto rl = [&](int l) -> const double * { return l == 0 ? r_fine0 : a.r[l]; };
   for (int l = 0; l < coarsest; l++)
      if (l < L - 1) xfer_restrict(H, s, l, rl(l), a.r[l + 1], a.xt, a.xy);
   if (k == L - 1) {
      // hypre_GaussElimSolve writes hypre's U_array, never read back by the
      // reference's cycle: the coarsest correction e[k] keeps its zero value
   } else if (multadd) {
      amgk::vset(s, a.e[k], 0.0, 0, H->lv[k].n);
      // level 0's correction is its own smoothing: the FULL_ASYNC update
      // folded into the last sweep where the smoother's kernel allows it
      const bool ap = k == 0 && apply == 1 && H->ctx->jgs_fold;
      if (smooth_all_levels(H, s, k, rl(k), a.e[k], a.u_prev, a.y, a.scratch, o.num_fine_smooth_sweeps, k,
                            ap ? u : nullptr, ap ? u_priv : nullptr))
         return true;
   } else {
      const int fg = k, cg = k + 1;
      amgk::vset(s, a.u_fine, 0.0, 0, H->lv[fg].n);
      amgk::vset(s, a.u_coarse, 0.0, 0, H->lv[cg].n);
      smooth_all_levels(H, s, cg, rl(cg), a.u_coarse, a.u_coarse_prev, a.y, a.scratch,
                        o.num_coarse_smooth_sweeps, k);
      amgk::spgemv(s, H->lv[fg].P, a.u_coarse, nullptr, mv, a.e[fg], 0, H->lv[fg].n, nullptr);
      // SMEM_Residual: y = A e; r_fine = r - y
      amgk::spgemv(s, H->lv[fg].A, a.e[fg], nullptr, mv, a.y, 0, H->lv[fg].n, nullptr);
      amgk::vsub(s, rl(fg), a.y, a.r_fine, 0, H->lv[fg].n);
      smooth_all_levels(H, s, fg, a.r_fine, a.u_fine, a.u_fine_prev, a.y, a.scratch,
                        o.num_fine_smooth_sweeps, k);
      amgk::vcopy(s, a.u_fine, a.e[k], 0, H->lv[k].n);
   }
   bool applied = false;
   for (int l = k - 1; l >= 0; l--)
      applied = xfer_prolong(H, s, l, a.e[l + 1], a.e[l], a.xy, l == 0 ? apply : 0, u, u_priv);
   return applied;
}

static void sync_add_vcycle(amg_hier *H)
{
   hipStream_t s = H->ctx->stream;
   for (int k = 0; k < H->L; k++) {
      const bool done = add_level_correction(H, s, k, H->r0, k < H->L - 1 ? 2 : 0, H->lv[0].u);
      if (k < H->L - 1 && !done) amgk::vaxpy(s, 1.0, H->al[k].e[0], H->lv[0].u, 0, H->lv[0].n);
   }
}

// ---- SMEM_Solve (SMEM_Solve.cpp:11-262, synchronous branch) --------------------
// Can the next cycle's first level-0 sweep come from the outer residual?
// (MULT, no preconditioner mode, Jacobi / L1 Jacobi, pre-smoothing on)
static bool reuse_applies(const amg_hier *H)
{
   const amg_opts &o = H->o;
   return o.solver == AMG_MULT && o.cheby_flag != 1 && o.reuse_outer_residual &&
          (o.smoother == AMG_JACOBI || o.smoother == AMG_SYMM_JACOBI ||
           o.smoother == AMG_L1_JACOBI) &&
          o.num_pre_smooth_sweeps > 0 && H->L > 1;
}

// can level 0's last post sweep run fused with the outer residual
// (mz_sweep_outer: plain weighted Jacobi, the 7-pt master form with S = 512)?
static bool fused_outer_applies(const amg_hier *H)
{
   const amg_opts &o = H->o;
   if (H->ctx->fuse_outer == 3) {
      // the slab form: any plane-marched level 0 whose planes are whole
      // 256-row norm tiles, Jacobi or L1 Jacobi
      const amg_mat *A = H->lv[0].A;
      return reuse_applies(H) && o.num_post_smooth_sweeps >= 1 && (H->psw.empty() || !H->psw[0]) && A->mz_P &&
             A->didx && A->mz_P % 256 == 0 && H->lv[0].n % A->mz_P == 0;
   }
   return H->ctx->fuse_outer && reuse_applies(H) && o.smoother == AMG_JACOBI && o.num_post_smooth_sweeps >= 1 &&
          (H->psw.empty() || !H->psw[0]) && amgk::mz_sweep_outer_ok(H->lv[0].A);
}

// fuse_outer 3: level 0's deferred last post sweep and the outer residual
// (+ the next cycle's first sweep) slab by slab over z.  Slab [s0, s1):
// sweep 1 u' = u + w (f - A u) ./ a over planes [s0-1, s1+1) (the z halo the
// residual's +-P operands need), then the residual sweep r = f - A u',
// u'' = u' + w r ./ a over [s0, s1), which reads u' and f back from the
// Infinity Cache instead of HBM.  Both are the ordinary marched kernels over
// plane ranges (the same per-row operand order), and the norm partials land
// at their global tiles: u', u'', r and every partial are bit-identical to the
// two full sweeps.  Without a stored u' the slab's u' lives in a (Z + 2)-plane
// scratch re-used by every slab (its dirty lines are overwritten in the cache,
// not written back).
static void outer_slabs(amg_hier *H, double *p, bool skip_r)
{
   hipStream_t s = H->ctx->stream;
   Level &v = H->lv[0];
   const amg_mat *A = v.A;
   const long long P = A->mz_P;
   const int nz = (int)(v.n / P), Z = std::min(H->ctx->outer_slab, nz);
   const double *l1 = H->o.smoother == AMG_L1_JACOBI ? v.l1 : nullptr;
   const double w = H->o.smooth_weight;
   for (int s0 = 0; s0 < nz; s0 += Z) {
      const int s1 = std::min(nz, s0 + Z);
      const int a = std::max(0, s0 - 1), b = std::min(nz, s1 + 1);
      // plane k of u' at xs + k P (the scratch holds planes s0-1 .. s1)
      double *xs = H->store_u1 ? v.u_alt : H->slab_scr + P * (1 - (long long)s0);
      amgk::jacobi_sweep(s, A, v.f, v.u, l1, w, xs, (int)(a * P), (int)(b * P));
      amgk::residual_jacobi(s, A, v.f, xs, l1, w, skip_r ? nullptr : H->r0, H->u2, (int)(s0 * P), (int)(s1 * P),
                            p + s0 * P / 256);
   }
}

extern "C" int amg_hier_fused_outer(const amg_hier *H)
{
   return (H && fused_outer_applies(H)) ? H->ctx->fuse_outer : 0;
}

// r = f - A u and ||r|| into d_hist[slot].  With reuse, the same kernel also
// emits the next cycle's first Jacobi sweep u_alt = u + w r / a_ii.  After a
// V-cycle that deferred level 0's last post sweep (post_deferred), that sweep
// runs in the same march (mz_sweep_outer): u' = u + w (f - A u) ./ a into
// u_alt (swapped in as u), r = f - A u', and u'' = u' + w r ./ a into u2
// (swapped in as u_alt, the next cycle's first sweep) -- the same bits as the
// sweep followed by the fused outer residual.
static int outer_residual(amg_hier *H, int slot)
{
   amg_ctx *c = H->ctx;
   Level &v = H->lv[0];
   double *p;
   const int nb = amgk::tile_blocks(0, v.n);
   AMG_TRY(amg_ctx_partials(c, nb, &p));
   if (H->post_deferred) {
      if (!H->u2) AMG_TRY(dalloc(H, v.n, &H->u2));
      const bool skip_r = H->o.reuse_outer_residual >= 2;
      if (c->fuse_outer == 3 && !H->store_u1) {
         const long long need = (long long)(std::min(c->outer_slab, v.n / v.A->mz_P) + 2) * v.A->mz_P;
         if (H->slab_cap < need) {
            AMG_TRY(dalloc(H, need, &H->slab_scr));
            H->slab_cap = need;
         }
      }
      {
         ProfScope ps(H, PROF_OUTER, c->stream);
         if (c->fuse_outer == 3)
            outer_slabs(H, p, skip_r);
         else
            amgk::mz_sweep_outer(c->stream, v.A, v.f, v.u, H->store_u1 ? v.u_alt : nullptr,
                                 skip_r ? nullptr : H->r0, H->u2, H->o.smooth_weight, p);
      }
      std::swap(v.u, v.u_alt);  // u = u' (when stored)
      std::swap(v.u_alt, H->u2); // u_alt = u''
      H->post_deferred = false;
      H->pre_ready = true;
      H->r0_stale = skip_r;
      amgk::reduce_partials(c->stream, p, nb, H->d_hist + slot, 1, c->d_scalars + 4096);
      AMG_HIP(hipGetLastError());
      return AMG_OK;
   }
   {
      ProfScope ps(H, PROF_OUTER, c->stream);
      if (reuse_applies(H)) {
         const bool l1 = (H->o.smoother == AMG_L1_JACOBI);
         const bool skip_r = H->o.reuse_outer_residual >= 2;
         amgk::residual_jacobi(c->stream, v.A, v.f, v.u, l1 ? v.l1 : nullptr, H->o.smooth_weight,
                               skip_r ? nullptr : H->r0, v.u_alt, 0, v.n, p);
         H->pre_ready = true;
         H->r0_stale = skip_r;
      } else {
         amgk::spgemv(c->stream, v.A, v.u, v.f, amgk::gemv_mode(-1.0, 1.0), H->r0, 0, v.n, p);
         H->pre_ready = false;
         H->r0_stale = false;
      }
   }
   amgk::reduce_partials(c->stream, p, nb, H->d_hist + slot, 1, c->d_scalars + 4096);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

static void init_vectors(amg_hier *H)
{
   // Misc.cpp:565-692 InitVectors / InitSolve
   hipStream_t s = H->ctx->stream;
   for (int l = 0; l < H->L; l++) {
      Level &v = H->lv[l];
      if (l > 0) amgk::vset(s, v.f, 0.0, 0, v.n);
      amgk::vset(s, v.u, 0.0, 0, v.n);
      amgk::vset(s, v.u_alt, 0.0, 0, v.n);
      amgk::vset(s, v.u_prev, 0.0, 0, v.n);
      amgk::vset(s, v.y, 0.0, 0, v.n);
      amgk::vset(s, v.r_fine, 0.0, 0, v.n);
      v.zero_flag = 0;
   }
   for (auto &a : H->al) {
      for (size_t l = 0; l < a.r.size(); l++) {
         if (a.r[l]) amgk::vset(s, a.r[l], 0.0, 0, H->lv[l].n);
         if (a.e[l]) amgk::vset(s, a.e[l], 0.0, 0, H->lv[l].n);
      }
   }
   amgk::vset(s, H->u_outer, 0.0, 0, H->lv[0].n);
   amgk::vset(s, H->y_outer, 0.0, 0, H->lv[0].n);
   if (H->e0) {
      amgk::vset(s, H->e0, 0.0, 0, H->lv[0].n);
      amgk::vset(s, H->e0_alt, 0.0, 0, H->lv[0].n);
   }
}

// ---- delay / fault injection (SMEM_Solve.cpp:33-43, 112-146) ------------------
// threads T-1 (DELAY_ONE / FAIL_ONE) or the last ceil(T delay_frac) (DELAY_SOME,
// DELAY_ALL: frac 1) sleep; in cycle k a sleeping thread sleeps RandDouble(0,
// 2 delay_usec) microseconds (the per-thread usec_vec draw of :41 is
// overwritten at :139 and never used).  rand() after srand(tid) is shared,
// unsynchronised glibc state in the reference; here every thread has its own
// splitmix64 stream seeded with its id -- the delays only move time.
static int delay_threads(const amg_opts &o)
{
   return std::max(1, o.num_threads);
}

static bool thread_sleeps(const amg_opts &o, int t, int k)
{
   const int T = delay_threads(o);
   switch (o.delay_type) {
   case AMG_DELAY_ONE: return t == T - 1;
   case AMG_FAIL_ONE: return t == T - 1 && k == o.fail_iter;
   case AMG_DELAY_SOME: return t >= T - (int)std::ceil((double)T * o.delay_frac);
   case AMG_DELAY_ALL: return true;
   default: return false;
   }
}

static double rand_double(unsigned long long &st, double lo, double hi)
{
   unsigned long long z = (st += 0x9E3779B97F4A7C15ULL);
   z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
   z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
   z ^= z >> 31;
   return lo + (hi - lo) * (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// the longest sleep of threads [t0, t1) in cycle k (0: none sleeps)
static double delay_usec(amg_hier *H, int t0, int t1, int k)
{
   const amg_opts &o = H->o;
   if (o.delay_type == AMG_DELAY_NONE || o.delay_usec <= 0) return 0.0;
   double d = 0.0;
   for (int t = t0; t < t1; t++)
      if (thread_sleeps(o, t, k)) d = std::max(d, (double)(int)rand_double(H->delay_rng[t], 0.0, 2.0 * o.delay_usec));
   return d;
}

static void delay_reset(amg_hier *H)
{
   const int T = delay_threads(H->o);
   H->delay_rng.assign(T, 0);
   for (int t = 0; t < T; t++) H->delay_rng[t] = 0x5DEECE66DULL * (unsigned long long)(t + 1);
}

static int solve_begin(amg_hier *H, const amg_vec *f, const amg_vec *u)
{
   amg_ctx *c = H->ctx;
   Level &v = H->lv[0];
   AMG_ARG(f->n == v.n && u->n == v.n, "amg_solve: vector size %d/%d vs %d", f->n, u->n, v.n);
   for (auto &a : H->al) AMG_TRY(ensure_xfer_scratch(H, a));
   init_vectors(H);
   amgk::vcopy(c->stream, f->d, v.f, 0, v.n);
   amgk::vcopy(c->stream, u->d, v.u, 0, v.n);
   AMG_TRY(outer_residual(H, 0));
   AMG_HIP(hipMemcpyAsync(c->h_pinned, H->d_hist, sizeof(double), hipMemcpyDeviceToHost, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   H->r0norm = c->h_pinned[0];
   H->cheby_omega = 2.0;
   H->iter = 0;
   H->have_state = true;
   delay_reset(H);
   return AMG_OK;
}

// one outer iteration: cycle, Chebyshev update, outer residual + norm (no sync)
static int solve_step(amg_hier *H)
{
   amg_ctx *c = H->ctx;
   const amg_opts &o = H->o;
   const bool precond = o.cheby_flag == 1;
   const bool one_level = !is_all_levels(o);
   const bool reuse = reuse_applies(H);
   // the cycle starts when its slowest thread has slept (SMEM_Solve.cpp:137-145)
   amgk::delay(c->stream, delay_usec(H, 0, delay_threads(o), H->iter + 1), c->wall_khz);
   if (o.solver == AMG_BPX)
      bpx_cycle(H, precond); // SMEM_Solve.cpp:161-163
   else if (one_level)
      vcycle(H, precond, reuse, fused_outer_applies(H));
   else if (c->graphs && !H->o.profile && (graphs_check(H), true))
      AMG_TRY(graph_issue(H->g_add, H->g_add_warm, c->stream, [&] {
         sync_add_vcycle(H);
         return (int)AMG_OK;
      }));
   else
      sync_add_vcycle(H);
   if (o.cheby_flag == 1) {
      const double mu24 = 4.0 * std::pow(o.cheby_mu, 2.0);
      amgk::cheby_update(c->stream, H->lv[0].u, H->u_outer, H->y_outer, H->cheby_omega,
                         o.cheby_delta, H->lv[0].n);
      H->cheby_omega = 1.0 / (1.0 - H->cheby_omega / mu24);
   }
   H->iter++;
   const int slot = H->iter % (H->hist_cap - 1);
   return outer_residual(H, slot);
}

extern "C" int amg_solve(amg_hier *H, const amg_vec *f, amg_vec *u, double *reshist, int *cycles)
{
   AMG_ARG(H && f && u, "amg_solve: null argument");
   amg_ctx *c = H->ctx;
   AMG_TRY(solve_begin(H, f, u));
   if (reshist) reshist[0] = H->r0norm;
   int done = 0;
   for (int k = 1; k <= H->o.num_cycles; k++) {
      AMG_TRY(solve_step(H));
      done = k;
      if (H->o.check_resnorm == 1) {
         AMG_HIP(hipMemcpyAsync(c->h_pinned, H->d_hist + (H->iter % (H->hist_cap - 1)),
                                sizeof(double), hipMemcpyDeviceToHost, c->stream));
         AMG_HIP(hipStreamSynchronize(c->stream));
         const double rn = c->h_pinned[0];
         if (reshist) reshist[k] = rn;
         if (rn / H->r0norm < H->o.tol) break;
      }
   }
   amgk::vcopy(c->stream, H->lv[0].u, u->d, 0, u->n);
   AMG_HIP(hipStreamSynchronize(c->stream));
   if (cycles) *cycles = done;
   return AMG_OK;
}

extern "C" int amg_solve_iterate(amg_hier *H, int k)
{
   AMG_ARG(H && H->have_state, "amg_solve_iterate: call amg_solve (or amg_solve_start) first");
   for (int i = 0; i < k; i++) {
      // fuse_outer 2: the fused post sweep writes u' only in the batch's last
      // step (the iterate the caller can observe); the steps before consume it
      // in registers
      H->store_u1 = H->ctx->fuse_outer < 2 || i == k - 1;
      const int st = solve_step(H);
      H->store_u1 = true;
      AMG_TRY(st);
   }
   return AMG_OK;
}

extern "C" int amg_solve_start(amg_hier *H, const amg_vec *f, const amg_vec *u, double *r0norm)
{
   AMG_ARG(H && f && u, "amg_solve_start: null argument");
   AMG_TRY(solve_begin(H, f, u));
   if (r0norm) *r0norm = H->r0norm;
   return AMG_OK;
}

extern "C" int amg_solve_resnorm(amg_hier *H, double *out)
{
   AMG_ARG(H && out && H->have_state, "amg_solve_resnorm: no solve state");
   amg_ctx *c = H->ctx;
   AMG_HIP(hipMemcpyAsync(c->h_pinned, H->d_hist + (H->iter % (H->hist_cap - 1)), sizeof(double),
                          hipMemcpyDeviceToHost, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   *out = c->h_pinned[0];
   return AMG_OK;
}

extern "C" int amg_solve_get_u(amg_hier *H, amg_vec *u)
{
   AMG_ARG(H && u && u->n == H->lv[0].n, "amg_solve_get_u: bad argument");
   amgk::vcopy(H->ctx->stream, H->lv[0].u, u->d, 0, u->n);
   AMG_HIP(hipStreamSynchronize(H->ctx->stream));
   return AMG_OK;
}

int amg_hier_subcycle(amg_hier *H, hipStream_t, const double *f_dev, const double **u_dev)
{
   // level 0 of H is an inner level of a larger cycle: zero-guess pre-sweep
   // (zero_flags = 1 for l > 0, SMEM_Sync_AMG.cpp:29-32) on the restricted
   // residual, which precond mode reads from r0 -- except a one-level H, whose
   // only level is the coarsest and smooths its own f
   amgk::vcopy(H->ctx->stream, f_dev, H->L == 1 ? H->lv[0].f : H->r0, 0, H->lv[0].n);
   H->pre_ready = false;
   H->r0_stale = false;
   vcycle(H, true, false);
   *u_dev = H->lv[0].u;
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int amg_hier_reset(amg_hier *H)
{
   init_vectors(H);
   H->pre_ready = false;
   H->have_state = false;
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_vcycle(amg_hier *H)
{
   AMG_ARG(H, "amg_vcycle: null hierarchy");
   for (auto &a : H->al) AMG_TRY(ensure_xfer_scratch(H, a));
   H->pre_ready = false;
   if (is_all_levels(H->o))
      sync_add_vcycle(H);
   else
      if (H->o.solver == AMG_BPX)
         bpx_cycle(H, H->o.cheby_flag == 1);
      else
         vcycle(H, H->o.cheby_flag == 1, false);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

// ---- EigsPower (SMEM_Cheby.cpp:410-518) ------------------------------------------
// M^{-1} f = one preconditioner-mode V-cycle from a zero state (the reference
// uses HYPRE_BoomerAMGSolve here).
static int precond_apply(amg_hier *H, const double *fin, double *out)
{
   hipStream_t s = H->ctx->stream;
   H->pre_ready = false;
   for (int l = 0; l < H->L; l++) {
      amgk::vset(s, H->lv[l].u, 0.0, 0, H->lv[l].n);
      H->lv[l].zero_flag = 0;
   }
   amgk::vcopy(s, fin, H->r0, 0, H->lv[0].n);
   H->r0_stale = false;
   vcycle(H, true, false);
   amgk::vcopy(s, H->lv[0].u, out, 0, H->lv[0].n);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_eigs_power(amg_hier *H, int iters, double *eig_max, double *eig_min)
{
   AMG_ARG(H && eig_max && eig_min && iters >= 1, "amg_eigs_power: bad argument");
   AMG_ARG(!is_all_levels(H->o), "amg_eigs_power: MULT hierarchies only");
   amg_ctx *c = H->ctx;
   const int n = H->lv[0].n;
   amg_vec U{c, n, nullptr, false}, E{c, n, nullptr, false}, Fv{c, n, nullptr, false},
      V{c, n, nullptr, false};
   double *tmp;
   AMG_TRY(dalloc(H, 4 * (size_t)n, &tmp));
   U.d = tmp;
   E.d = tmp + n;
   Fv.d = tmp + 2 * (size_t)n;
   V.d = tmp + 3 * (size_t)n;
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   double dd;
   for (int pass = 0; pass < 2; pass++) {
      amgk::vset(c->stream, U.d, 1.0, 0, n);
      int it = 0;
      while (true) {
         AMG_TRY(amg_vec_dot(c, &U, &U, &dd));
         amgk::vscale(c->stream, 1.0 / std::sqrt(dd), U.d, 0, n);
         amgk::vcopy(c->stream, U.d, E.d, 0, n);
         amgk::spgemv(c->stream, H->lv[0].A, U.d, nullptr, mv, Fv.d, 0, n, nullptr);
         AMG_TRY(precond_apply(H, Fv.d, U.d));
         if (pass == 1) amgk::vcopy(c->stream, E.d, V.d, 0, n);
         it++;
         if (it == iters) break;
         if (pass == 1) amgk::vaxpy(c->stream, -(*eig_max), V.d, U.d, 0, n);
      }
      if (pass == 0) {
         amgk::vcopy(c->stream, E.d, V.d, 0, n);
         AMG_TRY(amg_vec_dot(c, &V, &U, eig_max));
      } else {
         AMG_TRY(amg_vec_dot(c, &V, &U, eig_min));
      }
   }
   AMG_HIP(hipStreamSynchronize(c->stream));
   return AMG_OK;
}

// ---- SMEM_Async_Add_AMG (SMEM_Async_AMG.cpp:7-437) ---------------------------------
// FULL_ASYNC, read_type READ_SOL, res_compute LOCAL, converge LOCAL: every
// level runs num_cycles corrections on its own stream with no inter-level
// synchronisation.  Corrections land in u through device-scope fp64 atomics
// and each level recomputes its private residual f - A u_k from the value of
// u it observed at its own update (SMEM_Async_AMG.cpp:284-301, 338-351).
// SMEM_Smooth over rows [blk[b0], blk[b1]) of the fine grid from a zero guess:
// the GLOBAL residual phase's fine smoothing of level k's A_ns_global slice
// (SMEM_Async_AMG.cpp:46-59), with level k's residual r.  Block-aligned slices
// (the hybrid / asynchronous GS smoothers work on whole blocks).
// Slice rows [rb, re); the block smoothers take blocks [b0, b1) (rb = blk[b0],
// re = blk[b1]).
static void smooth_fine_slice(amg_hier *H, hipStream_t s, int k, const double *r, int b0, int b1, int rb,
                              int re)
{
   Level &v = H->lv[0];
   AddLevel &a = H->al[k];
   const amg_opts &o = H->o;
   const int sweeps = o.num_fine_smooth_sweeps;
   if (re <= rb || sweeps <= 0) return;
   const bool sym = is_multadd(o) && o.num_post_smooth_sweeps > 0 && o.num_pre_smooth_sweeps > 0;
   if (o.smoother == AMG_HYBRID_JACOBI_GAUSS_SEIDEL || o.smoother == AMG_L1_HYBRID_JACOBI_GAUSS_SEIDEL) {
      amg_hybrid_jgs_dev(H->ctx, s, v.A, r, a.g_u, a.g_prev, v.n, v.d_blk + b0, b1 - b0, rb, re,
                         o.smoother == AMG_L1_HYBRID_JACOBI_GAUSS_SEIDEL ? v.l1 : nullptr, 1.0, sweeps, 1, 0);
   } else if (o.smoother == AMG_ASYNC_GAUSS_SEIDEL || o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL) {
      amgk::vset(s, a.g_u, 0.0, rb, re);
      amgk::async_gs(s, v.A, r, a.g_u, v.d_blk + b0, b1 - b0, sweeps, o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL, 0);
   } else {
      const bool l1 = o.smoother == AMG_L1_JACOBI;
      const double w = l1 ? 1.0 : o.smooth_weight;
      if (sym) {
         amg_sym_jacobi_dev(s, v.A, r, a.g_u, a.g_y, a.g_r, w, l1 ? v.l1 : nullptr, sweeps, 1, rb, re, 0);
      } else {
         for (int q = 0; q < sweeps; q++) {
            if (q == 0) {
               amgk::jacobi_zero(s, v.A->diag, r, l1 ? v.l1 : nullptr, w, a.g_u, rb, re, 0);
            } else {
               amgk::vcopy(s, a.g_u, a.g_prev, 0, v.n);
               amgk::jacobi_sweep(s, v.A, r, a.g_prev, l1 ? v.l1 : nullptr, w, a.g_u, rb, re);
            }
         }
      }
   }
}

// SMEM_Async_Add_AMG (SMEM_Async_AMG.cpp:7-437): every level k (its
// correction is nonzero for k <= L-2) runs its correction loop on its own HIP
// stream.  Options:
//   async_type FULL_ASYNC: corrections enter the shared u (READ_SOL) or the
//     shared residual (READ_RES) with device-scope fp64 atomics, racing like the
//     reference's `omp atomic` updates;
//   async_type SEMI_ASYNC: each level's whole update (u += e, u_k = u; or
//     r -= A e, r_k = r) is exclusive -- the reference takes a lock
//     (:238-283); here the updates of all levels run, in issue order, on one
//     update stream (the context's comm stream), so no two levels' updates
//     interleave;
//   read_type READ_SOL: the level recomputes r_k = f - A u_k from the u it saw
//     (:338-348); READ_RES (LOCAL residuals): it applies y = A e to the shared
//     residual and reads that back (:227-236, 288-295), accumulating its
//     corrections privately, added into u at the end (:416-426; SEMI_ASYNC
//     updates u directly, :268-279);
//   res_compute_type GLOBAL (ASYNC_MULTADD): each iteration first smooths the
//     level's slice of the fine grid from its residual and adds that into u
//     (:35-77), and ends with the level computing its slice of the global
//     residual f - A u into the shared r and reading the whole shared r back
//     (:356-414); slices = equal splits of the fine grid's blocks;
//   converge_test_type LOCAL: every level stops after num_cycles corrections;
//     GLOBAL: levels keep correcting until EVERY level has done num_cycles
//     (CheckConverge's all-levels count, Misc.cpp:418-441; the reference's
//     GLOBAL and ALL_LEVELS share the value 1) -- the host keeps up to two
//     corrections in flight per level stream and polls their completion.
// level_corrections[k] returns the corrections level k performed.
extern "C" int amg_async_solve(amg_hier *H, const amg_vec *f, amg_vec *u, int *level_corrections,
                               double *relres)
{
   AMG_ARG(H && f && u, "amg_async_solve: null argument");
   AMG_ARG(is_all_levels(H->o), "amg_async_solve: ASYNC_MULTADD / ASYNC_AFACX hierarchies only");
   const amg_opts &o = H->o;
   AMG_ARG(o.async_type == AMG_FULL_ASYNC || o.async_type == AMG_SEMI_ASYNC, "amg_async_solve: async_type %d",
           o.async_type);
   amg_ctx *c = H->ctx;
   const int L = H->L;
   AMG_ARG((int)c->level_streams.size() >= L, "amg_async_solve: context has %d level streams, need %d",
           (int)c->level_streams.size(), L);
   const bool semi = o.async_type == AMG_SEMI_ASYNC;
   // SMEM_Main.cpp:650-660: GLOBAL residuals only for ASYNC_MULTADD
   const bool global_res = o.res_compute_type == AMG_GLOBAL && o.solver == AMG_ASYNC_MULTADD;
   const bool read_res = o.read_type == AMG_READ_RES && !global_res;
   const bool conv_global = o.converge_test_type == AMG_GLOBAL;
   const int sched = o.async_schedule;
   AMG_ARG(sched >= AMG_SCHED_FREE && sched <= AMG_SCHED_TIMED, "amg_async_solve: async_schedule %d", sched);
   AMG_ARG(!conv_global || sched == AMG_SCHED_FREE || sched == AMG_SCHED_ROUND_ROBIN || sched == AMG_SCHED_TIMED,
           "amg_async_solve: a sequential schedule needs converge_test_type LOCAL");
   AMG_ARG(sched != AMG_SCHED_TIMED || ((int)H->async_dur.size() >= L && (int)H->async_t.size() >= L),
           "amg_async_solve: AMG_SCHED_TIMED needs amg_hier_set_async_durations / _times");
   AMG_TRY(solve_begin(H, f, u));
   Level &v0 = H->lv[0];
   const int n0 = v0.n;
   // levels with a correction loop: [k_lo, k_hi).  The finest level whose
   // correction is nonzero is L-2 (see add_level_correction); with GLOBAL
   // residuals no group runs level 0 -- the sliced fine-grid smoothing takes
   // its place (PartitionLevels' finest_level = 1, SMEM_Setup.cpp:609-615) --
   // and the coarsest level's group runs too: its correction is zero, but it
   // smooths its slice of the fine grid and forms its slice of the residual
   const int k_lo = global_res ? 1 : 0;
   const int k_hi = global_res ? L : std::max(k_lo + 1, L - 1);
   const int ngrp = k_hi - k_lo;
   // global slices (A_ns_global, SMEM_Setup.cpp:924-936): equal row splits of
   // the fine grid over the groups; the block smoothers split level 0's blocks
   // instead (no GS block straddles two slices)
   const bool blk_smoother = o.smoother == AMG_HYBRID_JACOBI_GAUSS_SEIDEL ||
                             o.smoother == AMG_L1_HYBRID_JACOBI_GAUSS_SEIDEL ||
                             o.smoother == AMG_ASYNC_GAUSS_SEIDEL || o.smoother == AMG_SEMI_ASYNC_GAUSS_SEIDEL;
   std::vector<int> gb(L + 1, 0), gr(L + 1, 0);
   {
      const int nb = (int)v0.blk.size() - 1;
      const int size = n0 / ngrp, rest = n0 - size * ngrp;
      for (int q = 0; q <= ngrp; q++) {
         gb[k_lo + q] = (int)((long long)nb * q / ngrp);
         gr[k_lo + q] = blk_smoother ? v0.blk[gb[k_lo + q]] : q * size + std::min(q, rest);
      }
   }
   // a deterministic schedule runs every level on one stream in the
   // schedule's order (the oracle's or_set_async_schedule 1 / 2 / 3)
   auto lstream = [&](int k) { return sched != AMG_SCHED_FREE ? c->level_streams[k_lo] : c->level_streams[k]; };
   for (int k = k_lo; k < k_hi; k++) {
      AddLevel &a = H->al[k];
      if (read_res && !a.f_acc) AMG_TRY(dalloc(H, n0, &a.f_acc));
      if (global_res && !a.g_u) {
         AMG_TRY(dalloc(H, n0, &a.g_u));
         AMG_TRY(dalloc(H, n0, &a.g_prev));
         AMG_TRY(dalloc(H, n0, &a.g_y));
         AMG_TRY(dalloc(H, n0, &a.g_r));
      }
      if (!a.ev_a) {
         AMG_HIP(hipEventCreateWithFlags(&a.ev_a, hipEventDisableTiming));
         AMG_HIP(hipEventCreateWithFlags(&a.ev_b, hipEventDisableTiming));
      }
   }
   hipEvent_t ready, t_start;
   AMG_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
   AMG_HIP(hipEventCreate(&t_start));
   H->corr.reset(L);
   // the free race's update windows on the device clock (amg_async_update_windows)
   const bool rec0 = sched == AMG_SCHED_FREE && !(c->graphs && !semi && !read_res && !global_res && !H->o.profile &&
                                                   (o.delay_type == AMG_DELAY_NONE || o.delay_usec <= 0));
   if (rec0 && H->corr.stamps_begin(c->stream, L, std::max(1, o.num_cycles) * (conv_global ? 16 : 1) + 1, n0))
      return amg_set_error(AMG_ERR_OOM, "amg_async_solve: update-window stamps");
   AMG_HIP(hipEventRecord(ready, c->stream));
   AMG_HIP(hipEventRecord(t_start, c->stream));
   for (int k = k_lo; k < k_hi; k++) {
      hipStream_t s = lstream(k);
      AMG_HIP(hipStreamWaitEvent(s, ready, 0));
      // level_vector[k].r[0] = vector.r[0] (SMEM_Async_AMG.cpp:10-15)
      amgk::vcopy(s, H->r0, H->al[k].y_fine, 0, n0);
      if (read_res) amgk::vset(s, H->al[k].f_acc, 0.0, 0, n0);
      if (global_res) {
         amgk::vset(s, H->al[k].g_u, 0.0, 0, n0);
         amgk::vset(s, H->al[k].g_prev, 0.0, 0, n0);
      }
   }
   AMG_HIP(hipStreamWaitEvent(c->comm_stream, ready, 0));
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   // SEMI_ASYNC update stream (the lock of :238-283)
   hipStream_t us = sched != AMG_SCHED_FREE ? lstream(k_lo) : c->comm_stream;
   std::vector<int> issued(L, 0);
   // converge GLOBAL under round robin: the correction about to run is the
   // group's last (it sees the converge flag at its barrier)
   bool rr_last = false;
   // graphs of the level corrections (ctx->graphs): the FULL_ASYNC / READ_SOL /
   // LOCAL-residual correction issues the same kernels with the same
   // arguments every time (no delays, no profiling events), so each level's
   // is captured once per stream and replayed
   const bool graphs = c->graphs && !semi && !read_res && !global_res && !H->o.profile &&
                       (o.delay_type == AMG_DELAY_NONE || o.delay_usec <= 0);
   // free race without graphs: record each correction's update point (the
   // atomic add / the exclusive update of the shared vectors) as its end event
   const bool rec = sched == AMG_SCHED_FREE && !graphs;
   // one correction of level k, issued on its stream
   auto correction = [&](int k) -> int {
      hipStream_t s = lstream(k);
      AddLevel &a = H->al[k];
      auto to_update = [&]() -> int {
         AMG_HIP(hipEventRecord(a.ev_a, s));
         AMG_HIP(hipStreamWaitEvent(us, a.ev_a, 0));
         return AMG_OK;
      };
      auto from_update = [&]() -> int {
         AMG_HIP(hipEventRecord(a.ev_b, us));
         AMG_HIP(hipStreamWaitEvent(s, a.ev_b, 0));
         return AMG_OK;
      };
      const int grb = gr[k], gre = gr[k + 1];
      unsigned long long *stp = rec ? H->corr.stamp(k, issued[k]) : nullptr;
      {
         // injected delay of the threads this level group stands for
         const int T = delay_threads(o), g = k - k_lo;
         const int t0 = (int)((long long)T * g / ngrp), t1 = std::max(t0 + 1, (int)((long long)T * (g + 1) / ngrp));
         amgk::delay(s, delay_usec(H, t0, std::min(t1, T), issued[k] + 1), c->wall_khz);
      }
      if (global_res) {
         smooth_fine_slice(H, s, k, a.y_fine, gb[k], gb[k + 1], grb, gre);
         if (!semi) amgk::atomic_add(s, v0.u, a.g_u, grb, gre);
      }
      // FULL_ASYNC / READ_SOL: the atomic correction fused into the level-0
      // prolongation (or level 0's last smoothing sweep) where the kernels
      // allow it; that kernel records the update-window start
      if (rec && !read_res && !semi) {
         H->mark_k = k;
         H->mark_j = issued[k];
         H->mark_stamp = stp;
      }
      const bool fused = add_level_correction(H, s, k, a.y_fine, (!read_res && !semi) ? 1 : 0, v0.u, a.u_priv);
      H->mark_k = -1;
      H->mark_stamp = nullptr;
      if (read_res) {
         amgk::spgemv(s, v0.A, a.e[0], nullptr, mv, a.y, 0, n0, nullptr);
         if (semi) {
            AMG_TRY(to_update());
            amgk::semi_correct(us, v0.u, a.e[0], nullptr, n0);
            amgk::res_update(us, H->r0, a.y, a.y_fine, n0, 0);
            AMG_TRY(from_update());
         } else {
            if (rec && H->corr.record_start(k, issued[k], s)) return amg_set_error(AMG_ERR_HIP, "correction event");
            amgk::vaxpy(s, 1.0, a.e[0], a.f_acc, 0, n0);
            amgk::res_update(s, H->r0, a.y, a.y_fine, n0, 1, stp);
         }
         if (rec && H->corr.record(k, issued[k], s)) return amg_set_error(AMG_ERR_HIP, "correction event");
      } else {
         if (semi) {
            AMG_TRY(to_update());
            if (global_res) amgk::semi_correct(us, v0.u, a.g_u, nullptr, n0); // :258-265 (g_u is 0 off the slice)
            amgk::semi_correct(us, v0.u, a.e[0], a.u_priv, n0);
            AMG_TRY(from_update());
         } else if (!fused) {
            if (rec && H->corr.record_start(k, issued[k], s)) return amg_set_error(AMG_ERR_HIP, "correction event");
            amgk::atomic_correct(s, v0.u, a.e[0], a.u_priv, n0, stp);
         }
         if (rec && H->corr.record(k, issued[k], s)) return amg_set_error(AMG_ERR_HIP, "correction event");
         if (!global_res) {
            // SMEM_Residual(A0, f, u_k, y, r_k): y = A u_k; r = f - y (one pass, y unused)
            amgk::residual_fsub(s, v0.A, a.u_priv, v0.f, a.y, a.y_fine, n0);
         }
      }
      // the reference leaves its loop after the converged correction BEFORE the
      // GLOBAL residual update (SMEM_Async_AMG.cpp:353-356): converge LOCAL's
      // N-th correction does not touch the shared residual
      // (converge GLOBAL: the correction whose barrier sees the flag, known
      // only under the round-robin schedule)
      const bool last = conv_global ? rr_last : issued[k] + 1 >= o.num_cycles;
      if (global_res && !last) {
         // :356-414: u_k = u; the level's slice of r = f - A u_k (SMEM_Residual:
         // y = A u_k, then r = f - y) into the shared r; then r_k = r (under the
         // update stream for SEMI_ASYNC)
         amgk::vcopy(s, v0.u, a.u_priv, 0, n0);
         amgk::spgemv(s, v0.A, a.u_priv, nullptr, mv, a.y, grb, gre, nullptr);
         if (semi) AMG_TRY(to_update());
         hipStream_t ws = semi ? us : s;
         amgk::vsub(ws, v0.f, a.y, H->r0, grb, gre);
         amgk::vcopy(ws, H->r0, a.y_fine, 0, n0);
         if (semi) AMG_TRY(from_update());
      }
      AMG_HIP(hipGetLastError());
      return AMG_OK;
   };
   if (graphs) graphs_check(H);
   if (graphs && (int)H->g_lev.size() != L) graphs_reset(H);
   auto run = [&](int k) -> int {
      if (!graphs) return correction(k);
      hipStream_t s = lstream(k);
      if (H->g_lev_s[k] != s) {
         if (H->g_lev[k]) hipGraphExecDestroy(H->g_lev[k]);
         H->g_lev[k] = nullptr;
         H->g_lev_s[k] = s;
      }
      bool warm = H->g_lev_warm[k] != 0;
      const int st = graph_issue(H->g_lev[k], warm, s, [&] { return correction(k); });
      H->g_lev_warm[k] = warm ? 1 : 0;
      return st;
   };
   if (sched == AMG_SCHED_FINEST_FIRST || sched == AMG_SCHED_COARSEST_FIRST) {
      // the level groups one after another (or_set_async_schedule 1 / 2)
      for (int q = 0; q < ngrp; q++) {
         const int k = sched == AMG_SCHED_FINEST_FIRST ? k_lo + q : k_hi - 1 - q;
         for (int cyc = 0; cyc < o.num_cycles; cyc++) {
            AMG_TRY(run(k));
            issued[k]++;
         }
      }
   } else if (sched == AMG_SCHED_ROUND_ROBIN && conv_global) {
      // round robin under converge GLOBAL (or_set_async_schedule 3): the
      // finest group's root raises the converge flag after its update once
      // every group (the idle coarsest group of the reference too, which
      // keeps the same count) has num_cycles corrections; a group stops at
      // the first of its own updates that sees the flag (Misc.cpp:418-441)
      std::vector<int> stopped(L, 0);
      bool flag = false;
      for (int left = ngrp; left > 0;)
         for (int k = k_lo; k < k_hi; k++) {
            if (stopped[k]) continue;
            // k_lo raises the flag after its update (counted with this
            // correction); the correction that sees it is the group's last
            bool raise = false;
            if (k == k_lo && !flag) {
               bool all = true;
               for (int l = k_lo; l < k_hi; l++)
                  if (issued[l] + (l == k ? 1 : 0) < o.num_cycles) all = false;
               // the reference's idle coarsest group runs its turn after the
               // last correcting level, so in round r it has r - 1 when k_lo checks
               if (k_hi < L && issued[k_lo] < o.num_cycles) all = false;
               raise = all;
            }
            rr_last = flag || raise;
            AMG_TRY(run(k));
            rr_last = false;
            issued[k]++;
            if (raise) flag = true;
            if (flag) {
               stopped[k] = 1;
               left--;
            }
         }
   } else if (sched == AMG_SCHED_TIMED) {
      // the race at fixed level speeds (or_set_async_schedule 4): level k's
      // j-th correction ends at j * dur[k]; whole corrections in the order of
      // their end times, ties to the finer level.  The reference's idle
      // coarsest group (LOCAL residuals: its correction is zero) takes its
      // turns too, as a group that issues nothing -- under converge GLOBAL its
      // count is part of the flag (the oracle's group L - 1).  Converge LOCAL:
      // a group stops after num_cycles; GLOBAL: k_lo raises the flag after an
      // update once every group has num_cycles, and each group stops at the
      // first of its corrections that sees the flag (as under round robin)
      const int kv = std::max(k_hi, L); // groups [k_lo, kv); k >= k_hi: idle
      std::vector<int> cnt(kv, 0), stopped(kv, 0);
      bool flag = false;
      for (;;) {
         int best = -1;
         double tb = 0.0;
         for (int k = k_lo; k < kv; k++) {
            if (stopped[k]) continue;
            const double t = amg_timed_end(H->async_t[k], H->async_dur[k], cnt[k]);
            if (best < 0 || t < tb) best = k, tb = t;
         }
         if (best < 0) break;
         bool raise = false;
         if (conv_global && best == k_lo && !flag) {
            raise = true;
            for (int l = k_lo; l < kv; l++)
               if (cnt[l] + (l == best ? 1 : 0) < o.num_cycles) raise = false;
         }
         if (best < k_hi) {
            rr_last = flag || raise;
            AMG_TRY(run(best));
            rr_last = false;
            issued[best]++;
         }
         cnt[best]++;
         if (raise) flag = true;
         if (conv_global ? flag : cnt[best] >= o.num_cycles) stopped[best] = 1;
      }
   } else if (!conv_global) {
      // free race, or round robin under converge LOCAL (one stream: the
      // cycle-major, level-minor issue order is the turn order)
      for (int cyc = 0; cyc < o.num_cycles; cyc++)
         for (int k = k_lo; k < k_hi; k++) {
            AMG_TRY(run(k));
            issued[k]++;
         }
   } else {
      // run until every level has completed num_cycles corrections; faster
      // levels keep correcting meanwhile (at most 2 in flight per level)
      constexpr int DEPTH = 2;
      std::vector<std::vector<hipEvent_t>> done(L, std::vector<hipEvent_t>(DEPTH));
      for (auto &d : done)
         for (auto &e : d) AMG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      std::vector<int> completed(L, 0);
      const long long cap = 1000LL * std::max(1, o.num_cycles);
      int st = AMG_OK;
      for (;;) {
         bool all = true;
         for (int k = k_lo; k < k_hi && st == AMG_OK; k++) {
            while (completed[k] < issued[k]) {
               // not ready: still pending; any other status is a device error
               const hipError_t q = hipEventQuery(done[k][completed[k] % DEPTH]);
               if (q == hipErrorNotReady) break;
               if (q != hipSuccess) {
                  st = amg_set_error(AMG_ERR_HIP, "amg_async_solve: level %d correction: %s", k,
                                     hipGetErrorString(q));
                  break;
               }
               completed[k]++;
            }
            if (completed[k] < o.num_cycles) all = false;
         }
         if (st != AMG_OK || all) break;
         bool progressed = false;
         for (int k = k_lo; k < k_hi && st == AMG_OK; k++) {
            if (issued[k] - completed[k] < DEPTH && issued[k] < cap) {
               if ((st = run(k)) != AMG_OK) break;
               const hipError_t er = hipEventRecord(done[k][issued[k] % DEPTH], c->level_streams[k]);
               if (er != hipSuccess) {
                  st = amg_set_error(AMG_ERR_HIP, "amg_async_solve: hipEventRecord: %s", hipGetErrorString(er));
                  break;
               }
               issued[k]++;
               progressed = true;
            }
         }
         if (st != AMG_OK) break;
         if (!progressed) std::this_thread::yield();
      }
      for (int k = k_lo; k < k_hi; k++) hipStreamSynchronize(c->level_streams[k]);
      for (auto &d : done)
         for (auto &e : d) hipEventDestroy(e);
      if (st != AMG_OK) return st;
   }
   // each level's finish (its stream after its last correction)
   std::vector<hipEvent_t> t_end(L, nullptr);
   for (int k = k_lo; k < k_hi; k++) {
      AMG_HIP(hipEventCreate(&t_end[k]));
      AMG_HIP(hipEventRecord(t_end[k], c->level_streams[k]));
      AMG_HIP(hipStreamWaitEvent(c->stream, t_end[k], 0));
   }
   AMG_HIP(hipEventRecord(ready, us));
   AMG_HIP(hipStreamWaitEvent(c->stream, ready, 0));
   if (read_res && !semi)
      for (int k = k_lo; k < k_hi; k++) amgk::vaxpy(c->stream, 1.0, H->al[k].f_acc, v0.u, 0, n0); // :416-426
   AMG_HIP(hipEventDestroy(ready));
   AMG_TRY(outer_residual(H, 1));
   AMG_HIP(hipMemcpyAsync(c->h_pinned, H->d_hist + 1, sizeof(double), hipMemcpyDeviceToHost, c->stream));
   amgk::vcopy(c->stream, v0.u, u->d, 0, n0);
   AMG_HIP(hipStreamSynchronize(c->stream));
   if (relres) *relres = c->h_pinned[0] / H->r0norm;
   if (level_corrections)
      for (int k = 0; k < L; k++) level_corrections[k] = issued[k];
   if (sched == AMG_SCHED_FREE && H->corr.collect(t_start, issued))
      return amg_set_error(AMG_ERR_HIP, "amg_async_solve: correction times");
   if (rec0 && H->corr.stamps_collect(issued, c->wall_khz))
      return amg_set_error(AMG_ERR_HIP, "amg_async_solve: update-window stamps");
   H->level_ms.assign(L, 0.0);
   for (int k = k_lo; k < k_hi; k++) {
      float ms = 0.f;
      // one stream under a deterministic schedule: a level's last correction
      // is not its stream's last work, so only the free race is timed
      if (sched == AMG_SCHED_FREE) AMG_HIP(hipEventElapsedTime(&ms, t_start, t_end[k]));
      H->level_ms[k] = ms;
      AMG_HIP(hipEventDestroy(t_end[k]));
   }
   AMG_HIP(hipEventDestroy(t_start));
   return AMG_OK;
}

extern "C" int amg_hier_set_async_durations(amg_hier *H, const double *ms, int n)
{
   AMG_ARG(H && ms && n >= H->L, "amg_hier_set_async_durations: need %d levels", H ? H->L : 0);
   for (int k = 0; k < H->L; k++) AMG_ARG(ms[k] > 0.0, "amg_hier_set_async_durations: level %d: %g", k, ms[k]);
   H->async_dur.assign(ms, ms + H->L);
   H->async_t.assign(H->L, {});
   return AMG_OK;
}

extern "C" int amg_hier_set_async_times(amg_hier *H, const double *t, const int *n, int nlev)
{
   AMG_ARG(H && t && n && nlev >= H->L, "amg_hier_set_async_times: need %d levels", H ? H->L : 0);
   H->async_t.assign(H->L, {});
   H->async_dur.assign(H->L, 1.0);
   for (int k = 0, off = 0; k < H->L; off += n[k], k++) {
      AMG_ARG(n[k] >= 0, "amg_hier_set_async_times: level %d: %d entries", k, n[k]);
      H->async_t[k].assign(t + off, t + off + n[k]);
   }
   return AMG_OK;
}

extern "C" int amg_async_correction_ms(const amg_hier *H, int level, double *ms, int cap, int *count)
{
   AMG_ARG(H && count && level >= 0 && level < H->L, "amg_async_correction_ms: bad argument");
   const bool start = cap < 0; // cap < 0: the update windows' start times, -cap entries
   if (start) cap = -cap;
   const auto &vv = start ? H->corr.ms0 : H->corr.ms;
   const auto &v = level < (int)vv.size() ? vv[level] : std::vector<double>();
   *count = (int)v.size();
   for (int j = 0; j < (int)v.size() && j < cap && ms; j++) ms[j] = v[j];
   return AMG_OK;
}

extern "C" int amg_async_update_windows(const amg_hier *H, int level, double *ms, int cap, int *count)
{
   AMG_ARG(H && count && level >= 0 && level < H->L, "amg_async_update_windows: bad argument");
   const bool start = cap < 0; // cap < 0: the windows' starts, -cap entries
   if (start) cap = -cap;
   const auto &vv = start ? H->corr.w0 : H->corr.w1;
   const auto &v = level < (int)vv.size() ? vv[level] : std::vector<double>();
   *count = (int)v.size();
   for (int j = 0; j < (int)v.size() && j < cap && ms; j++) ms[j] = v[j];
   return AMG_OK;
}

extern "C" int amg_async_update_rows(const amg_hier *H, int level, int corr, double *ms, int cap, int *count)
{
   AMG_ARG(H && count && level >= 0 && level < H->L && corr >= 0,
           "amg_async_update_rows: bad argument");
   *count = H->corr.rows_of(level, corr, ms, cap < 0 ? -cap : cap, cap < 0);
   return AMG_OK;
}

extern "C" int amg_async_level_ms(const amg_hier *H, double *ms)
{
   AMG_ARG(H && ms, "amg_async_level_ms: null argument");
   AMG_ARG(!H->level_ms.empty(), "amg_async_level_ms: no asynchronous solve yet");
   for (int k = 0; k < H->L; k++) ms[k] = H->level_ms[k];
   return AMG_OK;
}
