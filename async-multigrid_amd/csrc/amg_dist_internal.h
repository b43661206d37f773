// amg_dist_internal.h -- shared internals of the multi-GPU solve phase
// (amg_dist.cpp: transport, plans, synchronous cycle; amg_dist_async.cpp:
// asynchronous additive cycle).  Not part of the C-ABI.
#pragma once

#include <rccl/rccl.h>

#include <functional>
#include <map>
#include <vector>

#include "amg_internal.h"

struct amg_transport {
   int nranks = 1, rank = 0;
   ncclComm_t comm = nullptr;
   amg_host_xchg_fn fn = nullptr; // test transport through host memory
   void *user = nullptr;
   bool host() const { return fn != nullptr; }
};

#define AMG_NCCL(call)                                                                     \
   do {                                                                                    \
      ncclResult_t _r = (call);                                                            \
      if (_r != ncclSuccess)                                                               \
         return amg_set_error(AMG_ERR_RCCL, "%s:%d %s -> %s", __FILE__, __LINE__, #call,  \
                              ncclGetErrorString(_r));                                     \
   } while (0)

namespace amgd {


struct Partition {
   // per level: first global row of every rank (size nranks + 1)
   std::vector<std::vector<long long>> rs;
   long long rows_begin(int l, int r) const { return rs[l][r]; }
   long long rows_end(int l, int r) const { return rs[l][r + 1]; }
   long long total(int l) const { return rs[l].back(); }
};

// z-slab form of a distributed level of the structured problem
// (amg_dist_hier_create_slab): the rank owns planes [za, zb) of the level's
// nx * ny * nz box; its vectors hold glo / ghi ghost planes below / above the
// owned rows (the pointers the cycle passes around point at the first owned
// row, so the ghost planes sit at negative offsets and past the end)
struct SlabGeom {
   int nx = 0, ny = 0, nz = 0;
   long long P = 0; // rows per plane
   int za = 0, zb = 0;
   int glo = 0, ghi = 0;
   long long off() const { return glo * P; }
   long long ext_rows() const { return (long long)(zb - za + glo + ghi) * P; }
   int e0() const { return za - glo; } // global plane of the extended base
   int nzl() const { return zb - za; }
};

struct DistMat {
   amg_mat *A = nullptr;        // local rows, remapped columns
   long long row0 = 0;          // first global row
   int nrows = 0;
   int ncol_own = 0;            // owned columns (x region [0, ncol_own))
   int nghost = 0;              // ghost region [ncol_own, ncol_own + nghost)
   bool replicated_cols = false; // columns index a full replicated vector
   int b0 = 0, b1 = 0;          // interior rows [b0, b1): no ghost column
   std::vector<int> peers;      // union of send/recv peers
   std::vector<long long> scnt, rcnt; // doubles per peer
   std::vector<long long> soff, roff; // offsets into sendbuf / ghost region
   int *d_send_idx = nullptr;   // owned-column index list of all sends
   long long nsend = 0;
   double *sendbuf = nullptr;
   // slab form: A is the extended operator (rows / columns of the ghost planes
   // around the owned ones, amg_gen_register_ext); the owned rows are its rows
   // [sro, sro + nrows), the column vector's extended base is x - sco.
   // nlo[r] / nhi[r]: column planes below / above rank r's owned column planes
   // that rank r's rows read (its ghost planes, received from r -+ 1); cP:
   // column rows per plane
   bool slab = false;
   long long sro = 0, sco = 0, cP = 0;
   std::vector<int> nlo, nhi;
};

struct DLevel {
   int n = 0;                  // owned rows
   long long row0 = 0;
   int cap = 0;                // vector capacity (owned + max ghosts)
   DistMat A, P, R;            // P: level l -> l+1 (rows = level l), R: rows = level l+1
   double *f = nullptr, *u = nullptr, *u_alt = nullptr, *r_fine = nullptr, *l1 = nullptr;
   int zero_flag = 0;
   bool zero_done = false; // slab V-cycle: the zero-guess sweep already written by the restriction
   // slab form
   SlabGeom sg;
   bool geo = false;   // R_l / P_l are the box's geometric transfers (checked)
   amgk::GeoT g{};
   double *d_geo_w = nullptr;
   int Ka = 0, Kb = 0; // owned planes of level l + 1
};


// DMEM_ChebyUpdate scalars (DMEM_Setup.cpp:1905-1912, DMEM_Misc.cpp:624-642):
// c / c_prev of the recurrence and the cycle counter it tests (iter.cycle)
struct AccelState {
   double c = 0.0, c_prev = 1.0;
   int cycle = 0;
   void reset(const amg_opts &o)
   {
      c = o.cheby_mu;
      c_prev = 1.0;
      cycle = 0;
   }
   // this cycle's update: false on the first cycle (d = u copy), else the
   // factors om1 = w - 1 and omd = w * delta; advances the cycle counter
   bool next(const amg_opts &o, double *om1, double *omd);
};

// per-stream exchange state of the asynchronous additive cycle (one per level)
struct AsyncLevel {
   hipStream_t s = nullptr;
   hipEvent_t ev_ready = nullptr; // level stream -> comm stream: send data packed
   hipEvent_t ev_done = nullptr;  // comm stream -> level stream: exchange complete
   std::map<const DistMat *, double *> sbuf; // pack buffers of this stream
   std::vector<double *> r, e;               // r[l], e[l]: level-l residual / correction
   double *u_priv = nullptr, *y = nullptr, *y_fine = nullptr;
   double *u_prev = nullptr, *sy = nullptr, *sr = nullptr; // smoother scratch (level k)
   double *uf = nullptr, *uc = nullptr, *rf = nullptr; // AFACx fine / coarse iterates, fine residual
   double *gath = nullptr;                   // allgather staging at the replication level
   double *d_acc = nullptr;                  // ChebyUpdate d of the cheby_grid level
   double *xt = nullptr, *xy = nullptr;      // composed smoothed transfers' scratch (level-0 room)
   int k = -1;                               // the level group (its link channels)
   AccelState acc;
};

// per-level device-resident mailboxes of the asynchronous distributed solve
// (amg_link.cpp).  caps[k * R + src]: largest message (doubles) src sends me
// in level group k, 0 = no channel (the sets are symmetric by construction)
struct LinkSet;
int link_create(amg_dist_hier *D, int K, const std::vector<long long> &caps, LinkSet **out, int nslots = 2);
int link_single_node(amg_dist_hier *D, bool *one);
double link_timeout_s(); // AMG_LINK_TIMEOUT_S, default 300
// collective: sequence numbers back to 0 before a solve; one_thread: every
// level group driven by the calling thread (a deterministic schedule)
int link_reset(LinkSet *L, bool one_thread);
int link_send(LinkSet *L, int k, int peer, const double *src, long long n, hipStream_t s);
int link_recv(LinkSet *L, int k, int peer, double *dst, long long n, hipStream_t s);
// MPI_Test + receive: if the next message from peer has arrived, launch its
// unpack on s and set *got = 1; else *got = 0 and return at once
int link_try_recv(LinkSet *L, int k, int peer, double *dst, long long n, hipStream_t s, int *got);
// would link_send to peer go through without waiting (its slot acknowledged)?
// (publishes this thread's completed copies first); *ok
int link_can_send(LinkSet *L, int k, int peer, int *ok);
int link_drain(LinkSet *L, int k); // publish everything level group k has in flight
void link_abort(LinkSet *L);       // tell every peer to give up waiting on this rank
void link_free(LinkSet *L);
int link_xchg_planes(LinkSet *L, int k, hipStream_t s, double *x, long long n_own, long long cP,
                     const std::vector<int> &nlo, const std::vector<int> &nhi);
int link_allgather(LinkSet *L, int k, hipStream_t s, const double *mine, double *gath, long long blk);

// host <-> device copies ordered on stream s and complete on return
int h2d(hipStream_t s, void *dst, const void *src, size_t bytes);
int d2h(hipStream_t s, void *dst, const void *src, size_t bytes);
// transport operations on stream s over communicator comm (nullptr: the main one)
int xp_p2p(amg_ctx *c, hipStream_t s, int np, const int *peers, void *const *send,
           const long long *sbytes, void *const *recv, const long long *rbytes,
           ncclComm_t comm = nullptr);
int xp_allreduce(amg_ctx *c, hipStream_t s, double *dev, int n, ncclComm_t comm = nullptr);
int xp_allgather(amg_ctx *c, hipStream_t s, const void *send, void *recv, long long bytes,
                 ncclComm_t comm = nullptr);
void launch_gather(hipStream_t s, const double *x, const int *idx, double *out, int n);
void launch_scatter_blocks(hipStream_t s, const double *src, int blk, const int *cnt,
                           const int *dsp, int nranks, double *dst);
void launch_sqrt(hipStream_t s, const double *in, double *out);

} // namespace amgd

// one grid of the level-grouped add solver (amg_grid.cpp): level k's
// restriction / smoothing / prolongation buffers, the DMEM_AddSmooth scale
// vectors, the coarsest grid's dense LU
struct GridState {
   bool ready = false;
   int k = -1;
   amgd::AsyncLevel al;
   double *sc = nullptr, *nsc = nullptr; // s and -s of DMEM_AddSmooth
   int n_c = 0;
   std::vector<double> lu, fh;
   std::vector<int> piv;
};

struct amg_dist_hier {
   amg_ctx *ctx = nullptr;
   amg_opts o{};
   // z-slab hierarchy (amg_dist_hier_create_slab): slab-form distributed
   // levels, geometric transfers, fused level-0 residual + restriction (geo0)
   // reading rr_u* / rr_f* ghost planes of u / f (per rank, below / above)
   bool slab = false;
   bool geo0 = false;
   std::vector<int> rr_ulo, rr_uhi, rr_flo, rr_fhi;
   // the fused composed prolongation of level 0 (mz_xfer_prolong over the
   // owned fine planes): level-1 ghost planes it reads per rank, and whether
   // they fit the ghost room (xfp0)
   std::vector<int> xp_lo, xp_hi;
   bool xfp0 = false;
   amgd::SlabGeom sg_rep; // owned planes of the first replicated level (the allgather blocks)
   int L = 0, Ld = 0; // levels [0, Ld) distributed, [Ld, L) replicated
   amgd::Partition part;
   std::vector<amgd::DLevel> lv;
   // replicated coarse part
   amg_hier *coarse = nullptr;
   std::vector<amg_mat *> coarse_mats;
   double *f_rep = nullptr;   // full level-Ld vector (allgathered restriction)
   double *gath_buf = nullptr;
   int gath_blk = 0;
   int *d_gcnt = nullptr, *d_gdsp = nullptr;
   // outer loop state
   double *r0 = nullptr;
   double *d_hist = nullptr;
   int hist_cap = 1 << 16;
   double r0norm = 0;
   int iter = 0;
   bool pre_ready = false, have_state = false;
   hipEvent_t ev_pack = nullptr, ev_comm = nullptr;
   std::vector<void *> allocs;
   // profiling: [0] fine residual, [1] fine smoother, [2] R0, [3] P0, [4] outer residual
   std::vector<std::pair<hipEvent_t, hipEvent_t>> pend[5];
   // asynchronous additive cycle (built on first use): per-level state and
   // the per-level device-resident channels between ranks
   std::vector<amgd::AsyncLevel> al;
   amgd::LinkSet *links = nullptr;
   amgd::LinkSet *ajac_links = nullptr; // DMEM_AsyncSmooth's delta channels (one group)
   // amg_dist_async_jacobi_stats: the last asynchronous Jacobi run's overlap
   // and delta accounting
   std::vector<double> ajac_stats;
   // the last DMEM_AsyncSmooth run's schedule, 5 doubles per event in the
   // order its work entered the compute stream: {1, sweep, accel mode, om1,
   // omd} the relaxation update, {2, sweep} the interior product, {3, peer,
   // delta index} one peer's ghost delta applied, {4, sweep} every peer's
   // deltas of that sweep applied (the transport path); empty under SPS
   // (its gate is decided on the device)
   std::vector<double> ajac_log;
   std::vector<amg_mat *> cA, cP, cR; // replicated levels' operators (level Ld + i)
   std::vector<double *> cl1;         // and their l1 norms
   // DMEM_Mult with acceleration (accel_type != 0): x (the iterate; lv[0].u
   // then carries the cycle's correction e) and the ChebyUpdate direction d
   double *x_acc = nullptr, *d_acc = nullptr;
   amgd::AccelState acc;
   GridState grid;
   std::vector<double> level_ms; // amg_dist_async_level_ms
   std::vector<double> async_dur; // AMG_SCHED_TIMED: per-level correction time
   std::vector<std::vector<double>> async_t; // AMG_SCHED_TIMED: recorded end times (replay)
   AmgCorrTimes corr;             // per-correction end times of the last free race
   double prof_ms[5] = {0, 0, 0, 0, 0};
   long long prof_n[5] = {0, 0, 0, 0, 0};
};

namespace amgd {
int dalloc(amg_dist_hier *D, size_t bytes, void **p);
int dvec(amg_dist_hier *D, size_t n, double **p);
// a level vector: slab levels get their ghost planes around the owned rows
// (the pointer is the first owned row); lvec2: room for the ghost planes of
// both levels la and lb (scratch used on either)
int lvec(amg_dist_hier *D, int l, double **p);
int lvec2(amg_dist_hier *D, int la, int lb, double **p);
// ---- slab hierarchies (amg_slab.cpp) ----
// plane exchange of x's ghost planes for an operator with per-rank needs
// nlo / nhi (planes of cP rows below / above each rank's n_own owned rows)
int slab_xchg(amg_ctx *c, hipStream_t s, double *x, long long n_own, long long cP, const std::vector<int> &nlo,
              const std::vector<int> &nhi);
// y = alpha A x + beta b on owned rows [rb, re) of a slab operator (no exchange)
void slab_spgemv(hipStream_t s, const DistMat &M, const double *x, const double *b, const amgk::Gemv &g,
                 double *y, long long rb, long long re, double *partials);
void slab_jacobi(hipStream_t s, const DistMat &M, const double *f, const double *x, const double *l1,
                 double omega, double *out, long long rb, long long re);
// the diagonal of the owned rows
const double *slab_diag(const DistMat &M);
// level-l transfers of a slab hierarchy on stream s, ghost planes exchanged
// by xchg(x, M-like needs); restrict: dst = level l+1 owned rows (or the
// allgather slot when l + 1 is replicated); prolong: out = P_l x (add = false)
// or u += P_l x (add = true)
using XchgFn = std::function<int(double *x, long long n_own, long long cP, const std::vector<int> &nlo,
                                 const std::vector<int> &nhi)>;
int slab_restrict(amg_dist_hier *D, hipStream_t s, int l, double *r, double *dst, const XchgFn &xchg,
                  amgk::ZeroGuess zg = amgk::ZeroGuess());
int slab_prolong(amg_dist_hier *D, hipStream_t s, int l, double *x, double *out, bool add, const XchgFn &xchg);
// sync cycle pieces of slab hierarchies (amg_dist.cpp dispatches to them)
int slab_vcycle(amg_dist_hier *D, bool precond);
int slab_outer_residual(amg_dist_hier *D, int slot);
int slab_solve_begin(amg_dist_hier *D, const double *f_local);
int slab_fine_spmv(amg_dist_hier *D, int reps, double *ms);
// shared construction pieces (amg_dist.cpp)
int dist_check_opts(const amg_opts *o);
void structured_planes(const amg_gen *g, int R, std::vector<std::vector<int>> &z0);
// the replicated coarse levels [Ld, L): full(which, level, &mat) registers
// every row of an operator; builds D->coarse and the allgather buffers
int dist_build_replicated(amg_dist_hier *D, const std::function<int(int, int, amg_mat **)> &full);
// InitVectors + initial outer residual r0 = f - A u (u = 0) and its norm
int dist_solve_begin(amg_dist_hier *D, const double *f_local);
// r0 = f - A x, ||r0|| into d_hist[slot] (all ranks); x = dist_iterate(D)
int dist_outer_residual(amg_dist_hier *D, int slot);
// the level-0 iterate: x_acc for accelerated MULT (DMEM_Mult), else lv[0].u
bool dist_mult_accel(const amg_dist_hier *D);
double *dist_iterate(amg_dist_hier *D);
// DMEM_DelayProc: the injected per-cycle wait of this rank on stream s
void dist_delay(amg_dist_hier *D, hipStream_t s);
// grid k of the level-grouped add solver (amg_dist_async.cpp): buffers,
// AddCycle from the residual r0 (*u0: U[0], on D->ctx->stream), F[0] = b - A x
int grid_prepare(amg_dist_hier *D, int k);
int grid_cycle(amg_dist_hier *D, const double *r0, double **u0);
int grid_residual(amg_dist_hier *D, double *x, const double *b, double *r);
} // namespace amgd
