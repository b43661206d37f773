// amg_dist.cpp -- multi-GPU solve phase: one process per GPU, z-slab
// partition of every level, RCCL point-to-point ghost exchange over xGMI on a
// communication stream overlapped with the slab-interior SpMV on the compute
// stream, replicated coarse levels, RCCL allreduce for the residual norm.
//
// Reference counterparts: the DMEM message engine (DMEM_Comm.cpp:81-382
// SendRecv / CheckInFlight / CompleteRecv), the ParCSR halo exchange hypre
// performs inside hypre_ParCSRMatrixMatvec (called from DMEM_Add.cpp:230-308,
// DMEM_Mult.cpp:95-261), the comm-plan construction CreateCommData_LocalRes
// (DMEM_Setup.cpp:666-1265) and InnerProdFlag's MPI_Allreduce
// (DMEM_Misc.cpp:414-433).  The cycle itself is SMEM_Sync_Parfor_Vcycle
// (SMEM_Sync_AMG.cpp:8-145) with SMEM_Solve's outer loop (SMEM_Solve.cpp:128-240):
// the same kernels as the single-GPU path on slab-local CSR whose column ids
// were remapped to [owned | ghost] without reordering any row, so every row
// sum keeps its order and the iterates are bit-identical to one GPU.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <vector>

#include "amg_dist_internal.h"

using namespace amgd;

// ---------------------------------------------------------------------------
// transport
// ---------------------------------------------------------------------------


extern "C" int amg_dist_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int amg_dist_get_unique_id(char *id)
{
   AMG_ARG(id, "amg_dist_get_unique_id: null buffer");
   ncclUniqueId u;
   AMG_NCCL(ncclGetUniqueId(&u));
   std::memcpy(id, &u, sizeof(u));
   return AMG_OK;
}

extern "C" int amg_dist_init(amg_ctx *c, int nranks, int rank, const char *id)
{
   AMG_ARG(c && id && nranks >= 1 && rank >= 0 && rank < nranks, "amg_dist_init: bad argument");
   AMG_ARG(!c->xport, "amg_dist_init: already initialised");
   ncclUniqueId u;
   std::memcpy(&u, id, sizeof(u));
   AMG_HIP(hipSetDevice(c->device));
   auto *t = new amg_transport();
   t->nranks = nranks;
   t->rank = rank;
   ncclResult_t r = ncclCommInitRank(&t->comm, nranks, u, rank);
   if (r != ncclSuccess) {
      delete t;
      return amg_set_error(AMG_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
   }
   c->xport = t;
   return AMG_OK;
}

extern "C" int amg_dist_init_host(amg_ctx *c, int nranks, int rank, amg_host_xchg_fn fn, void *user)
{
   AMG_ARG(c && fn && nranks >= 1 && rank >= 0 && rank < nranks, "amg_dist_init_host: bad argument");
   AMG_ARG(!c->xport, "amg_dist_init_host: already initialised");
   auto *t = new amg_transport();
   t->nranks = nranks;
   t->rank = rank;
   t->fn = fn;
   t->user = user;
   c->xport = t;
   return AMG_OK;
}

extern "C" int amg_dist_finalize(amg_ctx *c)
{
   if (!c || !c->xport) return AMG_OK;
   std::lock_guard<std::recursive_mutex> td(amg_teardown_mutex());
   // nothing may be in flight on any stream when the communicator goes
   // (an async solve that returned early can leave level-stream work queued)
   hipStreamSynchronize(c->stream);
   hipStreamSynchronize(c->comm_stream);
   for (auto s : c->level_streams) hipStreamSynchronize(s);
   if (c->xport->comm) ncclCommDestroy(c->xport->comm);
   delete c->xport;
   c->xport = nullptr;
   return AMG_OK;
}

// host -> device copy ordered on stream s and complete on return (a pageable
// hipMemcpy on the null stream is not ordered against the non-blocking
// context streams, e.g. a pending hipMemsetAsync of the same buffer)
int amgd::h2d(hipStream_t s, void *dst, const void *src, size_t bytes)
{
   if (bytes == 0) return AMG_OK;
   AMG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
   AMG_HIP(hipStreamSynchronize(s));
   return AMG_OK;
}

int amgd::d2h(hipStream_t s, void *dst, const void *src, size_t bytes)
{
   if (bytes == 0) return AMG_OK;
   AMG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   return AMG_OK;
}

// point-to-point byte exchange with peers[i] (device buffers), on stream s
int amgd::xp_p2p(amg_ctx *c, hipStream_t s, int np, const int *peers, void *const *send,
                 const long long *sbytes, void *const *recv, const long long *rbytes,
                 ncclComm_t comm)
{
   amg_transport *t = c->xport;
   if (np == 0) return AMG_OK;
   if (!comm) comm = t->comm;
   if (!t->host()) {
      AMG_NCCL(ncclGroupStart());
      for (int i = 0; i < np; i++) {
         if (sbytes[i] > 0) AMG_NCCL(ncclSend(send[i], (size_t)sbytes[i], ncclChar, peers[i], comm, s));
         if (rbytes[i] > 0) AMG_NCCL(ncclRecv(recv[i], (size_t)rbytes[i], ncclChar, peers[i], comm, s));
      }
      AMG_NCCL(ncclGroupEnd());
      return AMG_OK;
   }
   AMG_HIP(hipStreamSynchronize(s));
   std::vector<std::vector<char>> hs(np), hr(np);
   std::vector<const void *> sp(np);
   std::vector<void *> rp(np);
   for (int i = 0; i < np; i++) {
      hs[i].resize(std::max(1LL, sbytes[i]));
      hr[i].resize(std::max(1LL, rbytes[i]));
      if (sbytes[i] > 0) AMG_TRY(d2h(s, hs[i].data(), send[i], sbytes[i]));
      sp[i] = hs[i].data();
      rp[i] = hr[i].data();
   }
   int st = t->fn(t->user, 0, np, peers, sp.data(), sbytes, rp.data(), rbytes);
   if (st != 0) return amg_set_error(AMG_ERR_RCCL, "host transport p2p failed (%d)", st);
   for (int i = 0; i < np; i++)
      if (rbytes[i] > 0) AMG_TRY(h2d(s, recv[i], hr[i].data(), rbytes[i]));
   return AMG_OK;
}

// in-place sum of n doubles (device) across ranks, on stream s
int amgd::xp_allreduce(amg_ctx *c, hipStream_t s, double *dev, int n, ncclComm_t comm)
{
   amg_transport *t = c->xport;
   if (t->nranks == 1) return AMG_OK;
   if (!comm) comm = t->comm;
   if (!t->host()) {
      AMG_NCCL(ncclAllReduce(dev, dev, (size_t)n, ncclDouble, ncclSum, comm, s));
      return AMG_OK;
   }
   AMG_HIP(hipStreamSynchronize(s));
   std::vector<double> h(n);
   AMG_TRY(d2h(s, h.data(), dev, n * sizeof(double)));
   void *rp[1] = {h.data()};
   long long b[1] = {(long long)n * 8};
   int st = t->fn(t->user, 1, 0, nullptr, nullptr, nullptr, rp, b);
   if (st != 0) return amg_set_error(AMG_ERR_RCCL, "host transport allreduce failed (%d)", st);
   AMG_TRY(h2d(s, dev, h.data(), n * sizeof(double)));
   return AMG_OK;
}

// allgather of equal-size byte blocks: recv = [rank0 block | rank1 block | ...]
int amgd::xp_allgather(amg_ctx *c, hipStream_t s, const void *send, void *recv, long long bytes,
                       ncclComm_t comm)
{
   amg_transport *t = c->xport;
   if (!comm) comm = t->comm;
   if (!t->host()) {
      AMG_NCCL(ncclAllGather(send, recv, (size_t)bytes, ncclChar, comm, s));
      return AMG_OK;
   }
   AMG_HIP(hipStreamSynchronize(s));
   std::vector<char> hs(std::max(1LL, bytes)), hr(std::max(1LL, bytes * t->nranks));
   if (bytes > 0) AMG_TRY(d2h(s, hs.data(), send, bytes));
   const void *sp[1] = {hs.data()};
   void *rp[1] = {hr.data()};
   long long sb[1] = {bytes}, rb[1] = {bytes * t->nranks};
   int st = t->fn(t->user, 2, 0, nullptr, sp, sb, rp, rb);
   if (st != 0) return amg_set_error(AMG_ERR_RCCL, "host transport allgather failed (%d)", st);
   if (bytes > 0)
      AMG_TRY(h2d(s, recv, hr.data(), bytes * t->nranks));
   return AMG_OK;
}

extern "C" int amg_dist_allreduce_sum(amg_ctx *c, double *h, int n)
{
   AMG_ARG(c && c->xport && h && n >= 0, "amg_dist_allreduce_sum: not initialised");
   double *d = c->d_scalars + 2048;
   AMG_ARG(n <= 1024, "amg_dist_allreduce_sum: at most 1024 values");
   AMG_HIP(hipMemcpyAsync(d, h, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
   AMG_TRY(xp_allreduce(c, c->stream, d, n));
   AMG_HIP(hipMemcpyAsync(h, d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   return AMG_OK;
}

extern "C" int amg_dist_barrier(amg_ctx *c)
{
   double z = 0;
   return amg_dist_allreduce_sum(c, &z, 1);
}

extern "C" int amg_dist_hier_set_replicate_rows(amg_ctx *c, long long rows)
{
   AMG_ARG(c && rows >= 0, "amg_dist_hier_set_replicate_rows: bad argument");
   c->replicate_rows = rows;
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__global__ void gather_k(const double *__restrict__ x, const int *__restrict__ idx,
                         double *__restrict__ out, int n)
{
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
      out[i] = x[idx[i]];
}

__global__ void scatter_blocks_k(const double *__restrict__ src, int blk, const int *__restrict__ cnt,
                                 const int *__restrict__ dsp, int nranks, double *__restrict__ dst)
{
   // src = [rank q block of blk doubles], keep the first cnt[q] of each at dsp[q]
   const int total = blk * nranks;
   for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
      const int q = i / blk, k = i - q * blk;
      if (k < cnt[q]) dst[dsp[q] + k] = src[i];
   }
}

__global__ void sqrt_to_k(const double *__restrict__ in, double *__restrict__ out)
{
   out[0] = sqrt(in[0]);
}

void amgd::launch_gather(hipStream_t s, const double *x, const int *idx, double *out, int n)
{
   if (n <= 0) return;
   gather_k<<<std::min(4096, (n + 255) / 256), 256, 0, s>>>(x, idx, out, n);
}

void amgd::launch_scatter_blocks(hipStream_t s, const double *src, int blk, const int *cnt,
                                 const int *dsp, int nranks, double *dst)
{
   const int total = blk * nranks;
   if (total <= 0) return;
   scatter_blocks_k<<<std::min(4096, (total + 255) / 256), 256, 0, s>>>(src, blk, cnt, dsp, nranks, dst);
}

void amgd::launch_sqrt(hipStream_t s, const double *in, double *out) { sqrt_to_k<<<1, 1, 0, s>>>(in, out); }

// ---------------------------------------------------------------------------
// distributed matrix: slab-local rows, columns remapped to [owned | ghost]
// ---------------------------------------------------------------------------


namespace {

} // namespace

int amgd::dalloc(amg_dist_hier *D, size_t bytes, void **p)
{
   hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 8));
   if (e != hipSuccess)
      return amg_set_error(AMG_ERR_OOM, "amg_dist: allocation of %zu bytes: %s", bytes,
                           hipGetErrorString(e));
   D->allocs.push_back(*p);
   AMG_HIP(hipMemsetAsync(*p, 0, std::max<size_t>(bytes, 8), D->ctx->stream));
   return AMG_OK;
}

int amgd::dvec(amg_dist_hier *D, size_t n, double **p)
{
   return dalloc(D, n * sizeof(double), (void **)p);
}

int amgd::lvec(amg_dist_hier *D, int l, double **p) { return lvec2(D, l, l, p); }

int amgd::lvec2(amg_dist_hier *D, int la, int lb, double **p)
{
   long long off = 0, tail = 1;
   for (int l : {la, lb}) {
      if (l < D->Ld) {
         const DLevel &v = D->lv[l];
         if (D->slab) {
            off = std::max(off, v.sg.off());
            tail = std::max(tail, v.sg.ext_rows() - v.sg.off());
         } else {
            tail = std::max(tail, (long long)std::max(v.cap, v.n));
         }
      } else if (l - D->Ld < (int)D->cA.size()) {
         tail = std::max(tail, (long long)D->cA[l - D->Ld]->nrows);
      }
   }
   double *b = nullptr;
   AMG_TRY(dvec(D, (size_t)(off + tail), &b));
   *p = b + off;
   return AMG_OK;
}

int amgd::dist_check_opts(const amg_opts *o)
{
   AMG_ARG(o->cheby_flag == 0 && (o->smoother == AMG_JACOBI || o->smoother == AMG_L1_JACOBI ||
                                   o->smoother == AMG_SYMM_JACOBI),
           "amg_dist: the distributed cycles support the Jacobi / L1 Jacobi / symmetric Jacobi "
           "smoothers without the SMEM Chebyshev (use accel_type, DMEM_ChebyUpdate)");
   AMG_ARG(o->accel_type == AMG_NO_ACCEL || o->accel_type == AMG_RICHARD_ACCEL ||
              o->accel_type == AMG_CHEBY_RECUR_ACCEL,
           "amg_dist: accel_type %d (AMG_NO_ACCEL / AMG_RICHARD_ACCEL / AMG_CHEBY_RECUR_ACCEL)",
           o->accel_type);
   AMG_ARG(o->cheby_grid >= 0, "amg_dist: cheby_grid %d < 0", o->cheby_grid);
   AMG_ARG(o->solver == AMG_MULT || o->solver == AMG_ASYNC_MULTADD || o->solver == AMG_ASYNC_AFACX,
           "amg_dist: solver must be MULT (amg_dist_solve_*) or ASYNC_MULTADD / ASYNC_AFACX "
           "(amg_dist_async_solve)");
   return AMG_OK;
}

namespace {

// owner of global column g of a level's column space: the rank r with
// rs[r] <= g < rs[r+1] (empty ranges are skipped)
int owner_of(const Partition &pt, int level, long long g)
{
   const auto &z = pt.rs[level];
   return (int)(std::upper_bound(z.begin(), z.end(), g) - z.begin()) - 1;
}

// Build a DistMat from host CSR rows (global columns) of column level `cl`.
int build_distmat(amg_dist_hier *D, DistMat &M, long long row0, int nrows, std::vector<int> &rp,
                  std::vector<int> &cj, std::vector<double> &cv, int cl, bool replicated_cols)
{
   amg_ctx *c = D->ctx;
   amg_transport *t = c->xport;
   const int R = t->nranks, me = t->rank;
   M.row0 = row0;
   M.nrows = nrows;
   M.replicated_cols = replicated_cols;
   const long long nnz = rp[nrows];
   int ncols_dev = 0;
   std::vector<long long> ghosts;
   if (replicated_cols) {
      // columns index the full replicated level-cl vector
      const long long full = D->part.total(cl);
      M.ncol_own = (int)full;
      M.nghost = 0;
      ncols_dev = (int)full;
      M.b0 = 0;
      M.b1 = nrows;
   } else {
      const long long c0 = D->part.rows_begin(cl, me), c1 = D->part.rows_end(cl, me);
      M.ncol_own = (int)(c1 - c0);
      for (long long k = 0; k < nnz; k++) {
         const long long g = cj[k];
         if (g < c0 || g >= c1) ghosts.push_back(g);
      }
      std::sort(ghosts.begin(), ghosts.end());
      ghosts.erase(std::unique(ghosts.begin(), ghosts.end()), ghosts.end());
      M.nghost = (int)ghosts.size();
      // remap; rows keep their entry order
      std::vector<char> has_ghost(nrows, 0);
      for (int i = 0; i < nrows; i++)
         for (int k = rp[i]; k < rp[i + 1]; k++) {
            const long long g = cj[k];
            if (g >= c0 && g < c1) {
               cj[k] = (int)(g - c0);
            } else {
               const long long gi = std::lower_bound(ghosts.begin(), ghosts.end(), g) - ghosts.begin();
               cj[k] = (int)(M.ncol_own + gi);
               has_ghost[i] = 1;
            }
         }
      // interior: the longest run of rows without ghost columns
      int best0 = 0, best1 = 0, cur0 = 0;
      for (int i = 0; i <= nrows; i++) {
         if (i == nrows || has_ghost[i]) {
            if (i - cur0 > best1 - best0) {
               best0 = cur0;
               best1 = i;
            }
            cur0 = i + 1;
         }
      }
      M.b0 = best0;
      M.b1 = best1;
      ncols_dev = M.ncol_own + M.nghost;
   }
   // device CSR
   AMG_TRY(amg_mat_create_device(c, nrows, std::max(1, ncols_dev), nnz, &M.A));
   AMG_TRY(h2d(c->stream, M.A->rowptr, rp.data(), ((size_t)nrows + 1) * sizeof(int)));
   if (nnz) {
      AMG_TRY(h2d(c->stream, M.A->col, cj.data(), nnz * sizeof(int)));
      AMG_TRY(h2d(c->stream, M.A->val, cv.data(), nnz * sizeof(double)));
   }
   AMG_TRY(amg_mat_finish(M.A));
   AMG_HIP(hipStreamSynchronize(c->stream));
   if (replicated_cols) return AMG_OK;

   // ---- communication plan (CreateCommData_LocalRes analogue) ----
   // requests per owner
   std::vector<long long> need(R, 0);
   std::vector<int> gown(M.nghost);
   for (int i = 0; i < M.nghost; i++) {
      gown[i] = owner_of(D->part, cl, ghosts[i]);
      need[gown[i]]++;
   }
   // everybody learns how much every rank needs from it
   long long *d_need = nullptr, *d_all = nullptr;
   AMG_HIP(hipMalloc(&d_need, R * sizeof(long long)));
   AMG_HIP(hipMalloc(&d_all, (size_t)R * R * sizeof(long long)));
   AMG_TRY(h2d(c->stream, d_need, need.data(), R * sizeof(long long)));
   AMG_TRY(xp_allgather(c, c->stream, d_need, d_all, R * sizeof(long long)));
   std::vector<long long> all((size_t)R * R);
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_TRY(d2h(c->stream, all.data(), d_all, (size_t)R * R * sizeof(long long)));
   hipFree(d_need);
   hipFree(d_all);
   // peers: ranks I receive from or send to
   for (int q = 0; q < R; q++) {
      if (q == me) continue;
      const long long rc = need[q], sc = all[(size_t)q * R + me];
      if (rc > 0 || sc > 0) {
         M.peers.push_back(q);
         M.rcnt.push_back(rc);
         M.scnt.push_back(sc);
      }
   }
   const int np = (int)M.peers.size();
   M.roff.assign(np, 0);
   M.soff.assign(np, 0);
   {
      long long ro = 0, so = 0;
      for (int i = 0; i < np; i++) {
         M.roff[i] = ro;
         ro += M.rcnt[i];
         M.soff[i] = so;
         so += M.scnt[i];
      }
      M.nsend = so;
   }
   // exchange the request lists (global ids) and turn them into send index lists
   std::vector<long long> req_host(M.nghost);
   for (int i = 0; i < M.nghost; i++) req_host[i] = ghosts[i]; // already grouped by owner
   long long *d_req = nullptr, *d_inc = nullptr;
   AMG_HIP(hipMalloc(&d_req, std::max<long long>(1, M.nghost) * sizeof(long long)));
   AMG_HIP(hipMalloc(&d_inc, std::max<long long>(1, M.nsend) * sizeof(long long)));
   if (M.nghost)
      AMG_TRY(h2d(c->stream, d_req, req_host.data(), M.nghost * sizeof(long long)));
   {
      std::vector<void *> sp(np), rq(np);
      std::vector<long long> sb(np), rb(np);
      for (int i = 0; i < np; i++) {
         // my requests to peer i live where its ghosts start in the sorted list
         const long long first =
            std::lower_bound(gown.begin(), gown.end(), M.peers[i]) - gown.begin();
         sp[i] = d_req + first;
         sb[i] = M.rcnt[i] * (long long)sizeof(long long);
         rq[i] = d_inc + M.soff[i];
         rb[i] = M.scnt[i] * (long long)sizeof(long long);
         // the ghost region for this peer starts at the same sorted position
         M.roff[i] = first;
      }
      AMG_TRY(xp_p2p(c, c->stream, np, M.peers.data(), sp.data(), sb.data(), rq.data(), rb.data()));
   }
   AMG_HIP(hipStreamSynchronize(c->stream));
   std::vector<long long> inc(std::max<long long>(1, M.nsend));
   if (M.nsend) AMG_TRY(d2h(c->stream, inc.data(), d_inc, M.nsend * sizeof(long long)));
   hipFree(d_req);
   hipFree(d_inc);
   const long long c0 = D->part.rows_begin(cl, me);
   std::vector<int> sidx(std::max<long long>(1, M.nsend));
   for (long long k = 0; k < M.nsend; k++) {
      const long long li = inc[k] - c0;
      AMG_ARG(li >= 0 && li < M.ncol_own, "amg_dist: request %lld outside owned columns", inc[k]);
      sidx[k] = (int)li;
   }
   AMG_TRY(dalloc(D, std::max<long long>(1, M.nsend) * sizeof(int), (void **)&M.d_send_idx));
   if (M.nsend)
      AMG_TRY(h2d(c->stream, M.d_send_idx, sidx.data(), M.nsend * sizeof(int)));
   AMG_TRY(dvec(D, std::max<long long>(1, M.nsend), &M.sendbuf));
   return AMG_OK;
}

// ghost exchange of x (owned region filled) for M: pack on the compute stream,
// RCCL send/recv on the comm stream; the caller waits on ev_comm before the
// boundary rows
int halo_begin(amg_dist_hier *D, DistMat &M, double *x)
{
   amg_ctx *c = D->ctx;
   if (M.replicated_cols || M.peers.empty()) return AMG_OK;
   if (M.nsend > 0) {
      const int nb = (int)std::min<long long>(4096, (M.nsend + 255) / 256);
      gather_k<<<nb, 256, 0, c->stream>>>(x, M.d_send_idx, M.sendbuf, (int)M.nsend);
   }
   AMG_HIP(hipEventRecord(D->ev_pack, c->stream));
   AMG_HIP(hipStreamWaitEvent(c->comm_stream, D->ev_pack, 0));
   const int np = (int)M.peers.size();
   std::vector<void *> sp(np), rp(np);
   std::vector<long long> sb(np), rb(np);
   for (int i = 0; i < np; i++) {
      sp[i] = M.sendbuf + M.soff[i];
      sb[i] = M.scnt[i] * 8;
      rp[i] = x + M.ncol_own + M.roff[i];
      rb[i] = M.rcnt[i] * 8;
   }
   AMG_TRY(xp_p2p(c, c->comm_stream, np, M.peers.data(), sp.data(), sb.data(), rp.data(), rb.data()));
   AMG_HIP(hipEventRecord(D->ev_comm, c->comm_stream));
   return AMG_OK;
}

int halo_end(amg_dist_hier *D, DistMat &M)
{
   if (M.replicated_cols || M.peers.empty()) return AMG_OK;
   AMG_HIP(hipStreamWaitEvent(D->ctx->stream, D->ev_comm, 0));
   return AMG_OK;
}

struct DProf {
   amg_dist_hier *D;
   int cat;
   bool on;
   hipEvent_t a = nullptr, b = nullptr;
   DProf(amg_dist_hier *D_, int cat_, bool en) : D(D_), cat(cat_), on(en && D_->o.profile)
   {
      if (on) {
         hipEventCreate(&a);
         hipEventCreate(&b);
         hipEventRecord(a, D->ctx->stream);
      }
   }
   ~DProf()
   {
      if (on) {
         hipEventRecord(b, D->ctx->stream);
         D->pend[cat].push_back({a, b});
      }
   }
};

// interior rows first (overlapping the exchange), boundary rows after it
template <class F>
int split_launch(amg_dist_hier *D, DistMat &M, double *x, F launch)
{
   AMG_TRY(halo_begin(D, M, x));
   launch(M.b0, M.b1, 0);
   AMG_TRY(halo_end(D, M));
   const int t0 = amgk::tile_blocks(M.b0, M.b1);
   launch(0, M.b0, t0);
   launch(M.b1, M.nrows, t0 + amgk::tile_blocks(0, M.b0));
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int nparts(const DistMat &M)
{
   return amgk::tile_blocks(M.b0, M.b1) + amgk::tile_blocks(0, M.b0) +
          amgk::tile_blocks(M.b1, M.nrows);
}

} // namespace

// ---------------------------------------------------------------------------
// construction
// ---------------------------------------------------------------------------
namespace {

// host CSR rows with global column ids
struct HostRows {
   std::vector<int> rp, cj;
   std::vector<double> cv;
};
// local rows of operator `which` (AMG_GEN_A/P/R) of level l on this rank
using LocalFn = std::function<int(int which, int level, HostRows &out)>;
// every row of operator `which` of level l (replicated levels), registered on the device
using FullFn = std::function<int(int which, int level, amg_mat **out)>;

int check_opts(const amg_opts *o) { return dist_check_opts(o); }

// levels [0, Ld) distributed, [Ld, L) replicated: the first level with fewer
// rows than replicate_rows, at least level 1, at most L-1 (coarsest replicated)
int split_level(const Partition &pt, int L, long long replicate_rows)
{
   if (L == 1) return 1;
   int Ld = L;
   for (int l = 0; l < L; l++)
      if (pt.total(l) < replicate_rows) {
         Ld = l;
         break;
      }
   return std::min(std::max(Ld, 1), L - 1);
}

int build_hier(amg_ctx *c, int L, Partition part, const amg_opts *opts, const LocalFn &local,
               const FullFn &full, amg_dist_hier **out)
{
   amg_transport *t = c->xport;
   const int me = t->rank;
   auto D = std::make_unique<amg_dist_hier>();
   D->ctx = c;
   D->o = *opts;
   D->L = L;
   D->part = std::move(part);
   D->Ld = split_level(D->part, L, c->replicate_rows);
   const int Ld = D->Ld;
   D->lv.resize(Ld);
   AMG_HIP(hipEventCreateWithFlags(&D->ev_pack, hipEventDisableTiming));
   AMG_HIP(hipEventCreateWithFlags(&D->ev_comm, hipEventDisableTiming));
   HostRows h;
   for (int l = 0; l < Ld; l++) {
      DLevel &v = D->lv[l];
      v.row0 = D->part.rows_begin(l, me);
      v.n = (int)(D->part.rows_end(l, me) - v.row0);
      AMG_TRY(local(AMG_GEN_A, l, h));
      AMG_ARG((int)h.rp.size() == v.n + 1, "amg_dist: level %d A has %zu rows, partition says %d",
              l, h.rp.size() - 1, v.n);
      AMG_TRY(build_distmat(D.get(), v.A, v.row0, v.n, h.rp, h.cj, h.cv, l, false));
      if (l < L - 1) {
         AMG_TRY(local(AMG_GEN_P, l, h));
         AMG_ARG((int)h.rp.size() == v.n + 1, "amg_dist: level %d P row count", l);
         AMG_TRY(build_distmat(D.get(), v.P, v.row0, v.n, h.rp, h.cj, h.cv, l + 1, l + 1 >= Ld));
         const long long c0 = D->part.rows_begin(l + 1, me), c1 = D->part.rows_end(l + 1, me);
         AMG_TRY(local(AMG_GEN_R, l, h));
         AMG_ARG((long long)h.rp.size() == c1 - c0 + 1, "amg_dist: level %d R row count", l);
         AMG_TRY(build_distmat(D.get(), v.R, c0, (int)(c1 - c0), h.rp, h.cj, h.cv, l, false));
      }
   }
   // vector capacities: owned + the largest ghost region of any matrix reading them
   for (int l = 0; l < Ld; l++) {
      DLevel &v = D->lv[l];
      int g_max = v.A.nghost;
      if (l < L - 1) g_max = std::max(g_max, v.R.nghost);
      if (l > 0) g_max = std::max(g_max, D->lv[l - 1].P.nghost);
      v.cap = v.n + g_max;
      AMG_TRY(dvec(D.get(), v.cap, &v.f));
      AMG_TRY(dvec(D.get(), v.cap, &v.u));
      AMG_TRY(dvec(D.get(), v.cap, &v.u_alt));
      AMG_TRY(dvec(D.get(), v.cap, &v.r_fine));
      AMG_TRY(dvec(D.get(), std::max(1, v.n), &v.l1));
      amgk::l1_norms(c->stream, v.A.A, v.l1);
   }
   AMG_TRY(dvec(D.get(), D->lv[0].cap, &D->r0));
   AMG_TRY(dvec(D.get(), D->hist_cap, &D->d_hist));
   if (D->o.solver == AMG_MULT && D->o.accel_type != AMG_NO_ACCEL) {
      AMG_TRY(dvec(D.get(), D->lv[0].cap, &D->x_acc));
      AMG_TRY(dvec(D.get(), std::max(1, D->lv[0].n), &D->d_acc));
   }
   // replicated coarse hierarchy (identical on every rank, no communication)
   if (Ld < L) AMG_TRY(dist_build_replicated(D.get(), full));
   AMG_HIP(hipStreamSynchronize(c->stream));
   *out = D.release();
   return AMG_OK;
}

// allgather of variable-size host byte blobs through the transport (setup only)
int host_allgatherv(amg_ctx *c, const void *mine, long long bytes, std::vector<char> &all,
                    std::vector<long long> &sizes)
{
   const int R = c->xport->nranks;
   long long *d = nullptr;
   AMG_HIP(hipMalloc(&d, (size_t)(R + 1) * sizeof(long long)));
   AMG_TRY(h2d(c->stream, d + R, &bytes, sizeof(long long)));
   AMG_TRY(xp_allgather(c, c->stream, d + R, d, sizeof(long long)));
   sizes.resize(R);
   AMG_TRY(d2h(c->stream, sizes.data(), d, R * sizeof(long long)));
   hipFree(d);
   long long mx = 1;
   for (long long v : sizes) mx = std::max(mx, v);
   char *db = nullptr;
   AMG_HIP(hipMalloc(&db, (size_t)mx * (R + 1)));
   char *mine_d = db + (size_t)mx * R;
   AMG_TRY(h2d(c->stream, mine_d, mine, bytes));
   AMG_TRY(xp_allgather(c, c->stream, mine_d, db, mx));
   std::vector<char> padded((size_t)mx * R);
   AMG_TRY(d2h(c->stream, padded.data(), db, (size_t)mx * R));
   hipFree(db);
   all.clear();
   for (int r = 0; r < R; r++)
      all.insert(all.end(), padded.begin() + (size_t)mx * r, padded.begin() + (size_t)mx * r + sizes[r]);
   return AMG_OK;
}

} // namespace

// the replicated coarse levels [Ld, L): the same sub-hierarchy on every rank
// (no communication), fed by one allgather of the restricted residual
int amgd::dist_build_replicated(amg_dist_hier *D, const std::function<int(int, int, amg_mat **)> &full)
{
   amg_ctx *c = D->ctx;
   const int R = c->xport->nranks, L = D->L, Ld = D->Ld;
   const amg_opts *opts = &D->o;
   const int Lc = L - Ld;
   std::vector<amg_mat *> As(Lc), Ps(std::max(1, Lc - 1)), Rs(std::max(1, Lc - 1));
   for (int l = Ld; l < L; l++) {
      AMG_TRY(full(AMG_GEN_A, l, &As[l - Ld]));
      D->coarse_mats.push_back(As[l - Ld]);
      if (l < L - 1) {
         AMG_TRY(full(AMG_GEN_P, l, &Ps[l - Ld]));
         D->coarse_mats.push_back(Ps[l - Ld]);
         AMG_TRY(full(AMG_GEN_R, l, &Rs[l - Ld]));
         D->coarse_mats.push_back(Rs[l - Ld]);
      }
   }
   D->cA.assign(As.begin(), As.end());
   D->cP.assign(Ps.begin(), Ps.begin() + (Lc - 1));
   D->cR.assign(Rs.begin(), Rs.begin() + (Lc - 1));
   amg_opts co = *opts;
   co.solver = AMG_MULT; // the replicated levels run the multiplicative sub-cycle
   co.profile = 0;
   co.reuse_outer_residual = 0;
   AMG_TRY(amg_hier_create(c, Lc, As.data(), Ps.data(), Rs.data(), &co, &D->coarse));
   AMG_TRY(dvec(D, D->part.total(Ld), &D->f_rep));
   // allgather blocks padded to the largest owned row count at level Ld
   int blk = 0;
   std::vector<int> cnt(R), dsp(R);
   for (int r = 0; r < R; r++) {
      cnt[r] = (int)(D->part.rows_end(Ld, r) - D->part.rows_begin(Ld, r));
      dsp[r] = (int)D->part.rows_begin(Ld, r);
      blk = std::max(blk, cnt[r]);
   }
   D->gath_blk = blk;
   AMG_TRY(dvec(D, (size_t)blk * (R + 1), &D->gath_buf));
   AMG_TRY(dalloc(D, R * sizeof(int), (void **)&D->d_gcnt));
   AMG_TRY(dalloc(D, R * sizeof(int), (void **)&D->d_gdsp));
   AMG_TRY(h2d(c->stream, D->d_gcnt, cnt.data(), R * sizeof(int)));
   AMG_TRY(h2d(c->stream, D->d_gdsp, dsp.data(), R * sizeof(int)));
   return AMG_OK;
}

// z-plane slabs of the structured problem: level-0 planes split evenly; coarse
// plane k follows the owner of the fine plane it is injected from (2k+1 under
// linear interpolation, the aggregate's second plane under aggregation), so
// restriction and prolongation only touch neighbouring slabs
void amgd::structured_planes(const amg_gen *g, int R, std::vector<std::vector<int>> &z0)
{
   const int L = amg_gen_num_levels(g);
   std::vector<int> nz(L);
   for (int l = 0; l < L; l++) {
      int a, b;
      amg_gen_dims(g, l, &a, &b, &nz[l]);
   }
   z0.assign(L, std::vector<int>(R + 1));
   for (int r = 0; r <= R; r++) z0[0][r] = (int)((long long)nz[0] * r / R);
   for (int l = 1; l < L; l++) {
      std::vector<int> own(nz[l]);
      for (int k = 0; k < nz[l]; k++) {
         const int fz = std::min(nz[l - 1] - 1, 2 * k + 1);
         own[k] = (int)(std::upper_bound(z0[l - 1].begin(), z0[l - 1].end(), fz) - z0[l - 1].begin()) - 1;
      }
      // z0[l][r] = first coarse plane owned by a rank >= r (own[] is monotone)
      for (int r = 0; r <= R; r++)
         z0[l][r] = (int)(std::lower_bound(own.begin(), own.end(), r) - own.begin());
   }
}

extern "C" int amg_dist_structured_row_starts(const amg_gen *g, int nranks, long long *row_starts)
{
   AMG_ARG(g && nranks >= 1 && row_starts, "amg_dist_structured_row_starts: bad argument");
   std::vector<std::vector<int>> z0;
   structured_planes(g, nranks, z0);
   for (size_t l = 0; l < z0.size(); l++) {
      int a, b, c;
      amg_gen_dims(g, (int)l, &a, &b, &c);
      for (int r = 0; r <= nranks; r++)
         row_starts[l * (nranks + 1) + r] = (long long)z0[l][r] * a * b;
   }
   return AMG_OK;
}

extern "C" int amg_dist_hier_create_structured(amg_ctx *c, const amg_gen *g, const amg_opts *opts,
                                               amg_dist_hier **out)
{
   AMG_ARG(c && c->xport && g && opts && out, "amg_dist_hier_create_structured: bad argument");
   AMG_TRY(check_opts(opts));
   const int R = c->xport->nranks, me = c->xport->rank;
   const int L = amg_gen_num_levels(g);
   std::vector<std::array<int, 3>> dims(L);
   for (int l = 0; l < L; l++) amg_gen_dims(g, l, &dims[l][0], &dims[l][1], &dims[l][2]);
   std::vector<std::vector<int>> z0;
   structured_planes(g, R, z0);
   Partition part;
   part.rs.resize(L);
   for (int l = 0; l < L; l++) {
      part.rs[l].resize(R + 1);
      for (int r = 0; r <= R; r++) part.rs[l][r] = (long long)z0[l][r] * dims[l][0] * dims[l][1];
   }
   auto local = [&](int which, int level, HostRows &h) -> int {
      const int pl = (which == AMG_GEN_R) ? level + 1 : level;
      const int a = z0[pl][me], b = z0[pl][me + 1];
      const long long nnz = amg_gen_nnz(g, which, level, a, b);
      AMG_ARG(nnz >= 0, "amg_dist: generator: %s", amg_last_error());
      const long long nr = (long long)dims[pl][0] * dims[pl][1] * (b - a);
      h.rp.assign(nr + 1, 0);
      h.cj.assign(std::max(1LL, nnz), 0);
      h.cv.assign(std::max(1LL, nnz), 0.0);
      if (nr > 0) AMG_TRY(amg_gen_fill(g, which, level, a, b, h.rp.data(), h.cj.data(), h.cv.data(), 0));
      return AMG_OK;
   };
   auto full = [&](int which, int level, amg_mat **m) -> int {
      const int pl = (which == AMG_GEN_R) ? level + 1 : level;
      return amg_gen_register(c, g, which, level, 0, dims[pl][2], m);
   };
   return build_hier(c, L, std::move(part), opts, local, full, out);
}

extern "C" int amg_dist_hier_create(amg_ctx *c, int L, const long long *row_starts,
                                    const amg_csr_part *A, const amg_csr_part *P,
                                    const amg_csr_part *Rm, const amg_opts *opts, amg_dist_hier **out)
{
   AMG_ARG(c && c->xport && L >= 1 && row_starts && A && opts && out && (L == 1 || (P && Rm)),
           "amg_dist_hier_create: bad argument");
   AMG_TRY(check_opts(opts));
   const int R = c->xport->nranks, me = c->xport->rank;
   Partition part;
   part.rs.resize(L);
   for (int l = 0; l < L; l++) {
      part.rs[l].assign(row_starts + (size_t)l * (R + 1), row_starts + (size_t)(l + 1) * (R + 1));
      AMG_ARG(part.rs[l][0] == 0, "amg_dist_hier_create: row_starts of level %d must start at 0", l);
      for (int r = 0; r < R; r++)
         AMG_ARG(part.rs[l][r] <= part.rs[l][r + 1], "amg_dist_hier_create: level %d row_starts not monotone", l);
      AMG_ARG(part.rs[l][R] < (1LL << 31), "amg_dist_hier_create: level %d exceeds int32 rows", l);
   }
   auto pick = [&](int which, int level) -> const amg_csr_part & {
      return which == AMG_GEN_A ? A[level] : which == AMG_GEN_P ? P[level] : Rm[level];
   };
   auto rows_of = [&](int which, int level) {
      const int pl = (which == AMG_GEN_R) ? level + 1 : level;
      return part.rs[pl][me + 1] - part.rs[pl][me];
   };
   auto local = [&](int which, int level, HostRows &h) -> int {
      const amg_csr_part &m = pick(which, level);
      AMG_ARG(m.nrows == rows_of(which, level) && m.rowptr && (m.nnz == 0 || (m.col && m.val)),
              "amg_dist_hier_create: operator %d of level %d: %d local rows, partition says %lld",
              which, level, m.nrows, (long long)rows_of(which, level));
      AMG_ARG(m.rowptr[0] == 0 && m.rowptr[m.nrows] == m.nnz,
              "amg_dist_hier_create: operator %d of level %d: rowptr must run 0..nnz", which, level);
      h.rp.assign(m.rowptr, m.rowptr + m.nrows + 1);
      h.cj.assign(m.col, m.col + m.nnz);
      h.cv.assign(m.val, m.val + m.nnz);
      if (h.cj.empty()) {
         h.cj.push_back(0);
         h.cv.push_back(0.0);
      }
      return AMG_OK;
   };
   auto full = [&](int which, int level, amg_mat **mout) -> int {
      // gather every rank's rows of this (small) operator
      const amg_csr_part &m = pick(which, level);
      AMG_ARG(m.nrows == rows_of(which, level), "amg_dist_hier_create: operator %d of level %d row count",
              which, level);
      std::vector<char> all;
      std::vector<long long> sz;
      std::vector<int> rl(m.rowptr + 1, m.rowptr + m.nrows + 1); // row lengths via ends
      for (int i = m.nrows - 1; i >= 0; i--) rl[i] -= m.rowptr[i];
      AMG_TRY(host_allgatherv(c, rl.data(), (long long)rl.size() * 4, all, sz));
      std::vector<int> rp(1, 0);
      for (size_t k = 0; k < all.size() / 4; k++) rp.push_back(rp.back() + ((int *)all.data())[k]);
      AMG_TRY(host_allgatherv(c, m.col, m.nnz * 4, all, sz));
      std::vector<int> cj((int *)all.data(), (int *)all.data() + all.size() / 4);
      AMG_TRY(host_allgatherv(c, m.val, m.nnz * 8, all, sz));
      std::vector<double> cv((double *)all.data(), (double *)all.data() + all.size() / 8);
      const int pl_rows = (which == AMG_GEN_R) ? level + 1 : level;
      const int pl_cols = (which == AMG_GEN_P) ? level + 1 : level;
      const long long nr = part.total(pl_rows), nc = part.total(pl_cols);
      AMG_ARG((long long)rp.size() == nr + 1 && (long long)cj.size() == rp.back(),
              "amg_dist_hier_create: gathered operator %d of level %d is inconsistent", which, level);
      if (cj.empty()) {
         cj.push_back(0);
         cv.push_back(0.0);
      }
      return amg_csr_register(c, (int)nr, (int)nc, rp.back(), rp.data(), cj.data(), cv.data(), 1, mout);
   };
   return build_hier(c, L, part, opts, local, full, out); // the lambdas read part: copy it
}

extern "C" int amg_dist_hier_free(amg_dist_hier *D)
{
   if (!D) return AMG_OK;
   hipStreamSynchronize(D->ctx->stream);
   hipStreamSynchronize(D->ctx->comm_stream);
   for (auto s : D->ctx->level_streams) hipStreamSynchronize(s);
   if (D->links) link_free(D->links); // collective (a barrier between unmapping and freeing)
   if (D->ajac_links) link_free(D->ajac_links);
   // the rest under the process-wide teardown lock (not link_free: a peer
   // blocked in its barrier would hold it)
   std::lock_guard<std::recursive_mutex> td(amg_teardown_mutex());
   for (auto *a : {&D->grid.al}) {
      if (a->ev_ready) hipEventDestroy(a->ev_ready);
      if (a->ev_done) hipEventDestroy(a->ev_done);
   }
   for (auto &a : D->al) {
      if (a.ev_ready) hipEventDestroy(a.ev_ready);
      if (a.ev_done) hipEventDestroy(a.ev_done);
   }
   for (auto &v : D->lv)
      for (DistMat *M : {&v.A, &v.P, &v.R})
         if (M->A) amg_mat_free(M->A);
   if (D->coarse) amg_hier_free(D->coarse);
   for (auto *m : D->coarse_mats) amg_mat_free(m);
   for (void *p : D->allocs) hipFree(p);
   for (int k = 0; k < 5; k++)
      for (auto &e : D->pend[k]) {
         hipEventDestroy(e.first);
         hipEventDestroy(e.second);
      }
   if (D->ev_pack) hipEventDestroy(D->ev_pack);
   if (D->ev_comm) hipEventDestroy(D->ev_comm);
   delete D;
   return AMG_OK;
}

extern "C" int amg_dist_hier_matrix_info(amg_dist_hier *D, int level, long long *nnz, int *value_index,
                                         int *dict_index, int *row_pattern)
{
   AMG_ARG(D && level >= 0 && level < D->L, "amg_dist_hier_matrix_info: bad level");
   const amg_mat *A = level < D->Ld ? D->lv[level].A.A : D->cA[level - D->Ld];
   if (nnz) *nnz = A->nnz;
   if (value_index) *value_index = A->vi_n;
   if (dict_index) *dict_index = A->dc_n;
   if (row_pattern) *row_pattern = A->rp_n;
   return AMG_OK;
}

extern "C" int amg_dist_hier_pair_pattern(amg_dist_hier *D, int level, int *pair_pattern)
{
   AMG_ARG(D && pair_pattern && level >= 0 && level < D->L, "amg_dist_hier_pair_pattern: bad argument");
   const amg_mat *A = level < D->Ld ? D->lv[level].A.A : D->cA[level - D->Ld];
   *pair_pattern = A->pp_n;
   return AMG_OK;
}

extern "C" int amg_dist_hier_local_rows(amg_dist_hier *D, int level, int *row0, int *nrows)
{
   AMG_ARG(D && level >= 0 && level < D->L, "amg_dist_hier_local_rows: bad level");
   const int me = D->ctx->xport->rank;
   if (row0) *row0 = (int)D->part.rows_begin(level, me);
   if (nrows) *nrows = (int)(D->part.rows_end(level, me) - D->part.rows_begin(level, me));
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// cycle
// ---------------------------------------------------------------------------
namespace {

int d_spgemv(amg_dist_hier *D, DistMat &M, double *x, const double *b, const amgk::Gemv &g,
             double *y, double *partials)
{
   hipStream_t s = D->ctx->stream;
   return split_launch(D, M, x, [&](int rb, int re, int poff) {
      amgk::spgemv(s, M.A, x, b, g, y, rb, re, partials ? partials + poff : nullptr);
   });
}

bool d_reuse(const amg_dist_hier *D)
{
   return D->o.reuse_outer_residual && D->o.num_pre_smooth_sweeps > 0 && !dist_mult_accel(D);
}

// SMEM_Sync_Parfor_Jacobi on a distributed level (ping-pong)
int d_smooth(amg_dist_hier *D, int l, const double *f, int sweeps, bool allow_reuse)
{
   DLevel &v = D->lv[l];
   hipStream_t s = D->ctx->stream;
   const bool l1 = D->o.smoother == AMG_L1_JACOBI;
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && v.zero_flag == 1) {
         amgk::jacobi_zero(s, v.A.A->diag, f, l1 ? v.l1 : nullptr, D->o.smooth_weight, v.u, 0, v.n, 0);
      } else if (k == 0 && allow_reuse && D->pre_ready) {
         std::swap(v.u, v.u_alt);
         D->pre_ready = false;
      } else {
         DProf pr(D, 1, l == 0);
         double *x = v.u, *out = v.u_alt;
         AMG_TRY(split_launch(D, v.A, x, [&](int rb, int re, int) {
            amgk::jacobi_sweep(s, v.A.A, f, x, l1 ? v.l1 : nullptr, D->o.smooth_weight, out, rb, re);
         }));
         std::swap(v.u, v.u_alt);
      }
   }
   return AMG_OK;
}

// SMEM_Sync_Parfor_Vcycle on the distributed levels.  precond: the cycle runs
// on the outer residual r0 from a zero level-0 guess (precond_flag, the form
// DMEM_MultCycle takes with precond_zero_init_guess = 1) and leaves the
// correction in lv[0].u
int d_vcycle(amg_dist_hier *D, bool precond)
{
   if (D->slab) return slab_vcycle(D, precond);
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   const int L = D->L, Ld = D->Ld;
   const amgk::Gemv res_mode = amgk::gemv_mode(-1.0, 1.0);
   const amgk::Gemv mv_mode = amgk::gemv_mode(1.0, 0.0);
   const amgk::Gemv pro_mode = amgk::gemv_mode(1.0, 1.0);
   for (int l = 0; l < Ld && l < L - 1; l++) {
      DLevel &v = D->lv[l];
      const double *fl = (l == 0 && precond) ? D->r0 : v.f;
      v.zero_flag = (l == 0 && !precond) ? 0 : 1;
      AMG_TRY(d_smooth(D, l, fl, D->o.num_pre_smooth_sweeps, l == 0 && d_reuse(D)));
      {
         DProf pr(D, 0, l == 0);
         AMG_TRY(d_spgemv(D, v.A, v.u, fl, res_mode, v.r_fine, nullptr));
      }
      {
         DProf pr(D, 2, l == 0);
         double *dst = (l + 1 < Ld) ? D->lv[l + 1].f : D->gath_buf + (size_t)D->gath_blk * c->xport->nranks;
         AMG_TRY(d_spgemv(D, v.R, v.r_fine, nullptr, mv_mode, dst, nullptr));
         if (l + 1 == Ld) {
            // assemble the replicated level-Ld right-hand side on every rank
            const int R = c->xport->nranks;
            AMG_TRY(xp_allgather(c, s, dst, D->gath_buf, (long long)D->gath_blk * 8));
            scatter_blocks_k<<<std::max(1, std::min(4096, (D->gath_blk * R + 255) / 256)), 256, 0, s>>>(
               D->gath_buf, D->gath_blk, D->d_gcnt, D->d_gdsp, R, D->f_rep);
         }
      }
   }
   const double *u_rep = nullptr;
   if (Ld < L) {
      AMG_TRY(amg_hier_subcycle(D->coarse, s, D->f_rep, &u_rep));
   } else {
      // single distributed level: SMEM_Sync_Parfor_Vcycle smooths the coarsest
      DLevel &v = D->lv[L - 1];
      const double *fl = (L == 1 && precond) ? D->r0 : v.f;
      AMG_TRY(d_smooth(D, L - 1, fl, D->o.num_pre_smooth_sweeps + D->o.num_post_smooth_sweeps, false));
   }
   for (int l = std::min(Ld, L - 1) - 1; l >= 0; l--) {
      DLevel &v = D->lv[l];
      v.zero_flag = 0;
      {
         DProf pr(D, 3, l == 0);
         double *xc = (l + 1 < Ld) ? D->lv[l + 1].u : const_cast<double *>(u_rep);
         AMG_TRY(d_spgemv(D, v.P, xc, v.u, pro_mode, v.u, nullptr));
      }
      AMG_TRY(d_smooth(D, l, (l == 0 && precond) ? D->r0 : v.f, D->o.num_post_smooth_sweeps, false));
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int d_outer_residual(amg_dist_hier *D, int slot)
{
   if (D->slab) return slab_outer_residual(D, slot);
   amg_ctx *c = D->ctx;
   hipStream_t s = c->stream;
   DLevel &v = D->lv[0];
   double *p;
   const int np = nparts(v.A);
   AMG_TRY(amg_ctx_partials(c, np + 1, &p));
   {
      DProf pr(D, 4, true);
      if (d_reuse(D) && D->L > 1) {
         const bool l1 = D->o.smoother == AMG_L1_JACOBI;
         // reuse_outer_residual 2: the MULT cycle never reads r0 outside
         // preconditioner mode (excluded by d_reuse), so it is not written
         double *r0 = (D->o.reuse_outer_residual >= 2 && D->o.solver == AMG_MULT) ? nullptr : D->r0;
         double *x = v.u, *un = v.u_alt;
         AMG_TRY(split_launch(D, v.A, x, [&](int rb, int re, int poff) {
            amgk::residual_jacobi(s, v.A.A, v.f, x, l1 ? v.l1 : nullptr, D->o.smooth_weight, r0,
                                  un, rb, re, p + poff);
         }));
         D->pre_ready = true;
      } else {
         AMG_TRY(d_spgemv(D, v.A, dist_iterate(D), v.f, amgk::gemv_mode(-1.0, 1.0), D->r0, p));
         D->pre_ready = false;
      }
   }
   double *sum = D->d_hist + slot;
   amgk::reduce_partials(s, p, np, sum, 0, c->d_scalars + 4096);
   AMG_TRY(xp_allreduce(c, s, sum, 1));
   sqrt_to_k<<<1, 1, 0, s>>>(sum, sum);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

} // namespace

int amgd::dist_outer_residual(amg_dist_hier *D, int slot) { return d_outer_residual(D, slot); }

bool amgd::dist_mult_accel(const amg_dist_hier *D)
{
   return D->o.solver == AMG_MULT && D->o.accel_type != AMG_NO_ACCEL;
}

double *amgd::dist_iterate(amg_dist_hier *D) { return dist_mult_accel(D) ? D->x_acc : D->lv[0].u; }

bool amgd::AccelState::next(const amg_opts &o, double *om1, double *omd)
{
   if (cycle++ == 0) return false; // DMEM_Misc.cpp:627-631
   const double mu = o.cheby_mu, delta = o.cheby_delta;
   double omega;
   if (o.accel_type == AMG_RICHARD_ACCEL) {
      omega = 2.0 / (1.0 + std::sqrt(1.0 - std::pow(mu, -2.0))); // :634-636
   } else {
      const double c_temp = c; // :638-641
      c = 2.0 * mu * c - c_prev;
      c_prev = c_temp;
      omega = 2.0 * mu * c_prev / c;
   }
   *om1 = omega - 1.0;
   *omd = omega * delta;
   return true;
}

int amgd::dist_solve_begin(amg_dist_hier *D, const double *f_local)
{
   if (D->slab) return slab_solve_begin(D, f_local);
   amg_ctx *c = D->ctx;
   for (auto &v : D->lv) {
      for (double *p : {v.f, v.u, v.u_alt, v.r_fine}) amgk::vset(c->stream, p, 0.0, 0, v.cap);
      v.zero_flag = 0;
   }
   AMG_TRY(h2d(c->stream, D->lv[0].f, f_local, (size_t)D->lv[0].n * sizeof(double)));
   // InitVectors on the replicated levels (the coarsest iterate carries over
   // between cycles, so a new solve starts it from zero as one GPU does)
   if (D->coarse) AMG_TRY(amg_hier_reset(D->coarse));
   if (D->x_acc) {
      amgk::vset(c->stream, D->x_acc, 0.0, 0, D->lv[0].cap);
      amgk::vset(c->stream, D->d_acc, 0.0, 0, std::max(1, D->lv[0].n));
   }
   D->acc.reset(D->o);
   D->iter = 0;
   AMG_TRY(d_outer_residual(D, 0));
   AMG_TRY(d2h(c->stream, c->h_pinned, D->d_hist, sizeof(double)));
   D->r0norm = c->h_pinned[0];
   D->have_state = true;
   return AMG_OK;
}

extern "C" int amg_dist_solve_start(amg_dist_hier *D, const double *f_local, double *r0norm)
{
   AMG_ARG(D && f_local, "amg_dist_solve_start: null argument");
   AMG_ARG(D->o.solver == AMG_MULT, "amg_dist_solve_start: MULT hierarchies (ASYNC_*: amg_dist_async_solve)");
   AMG_TRY(dist_solve_begin(D, f_local));
   if (r0norm) *r0norm = D->r0norm;
   return AMG_OK;
}

// DMEM_DelayProc (DMEM_Misc.cpp:668-684): before every cycle the rank waits
// delay_usec (every rank; delay_rank >= 0: that rank only, the commented-out
// delay_id test) -- here a wait on the stream the cycle runs on
void amgd::dist_delay(amg_dist_hier *D, hipStream_t s)
{
   const amg_opts &o = D->o;
   if (o.delay_type == AMG_DELAY_NONE || o.delay_usec <= 0) return;
   if (o.delay_rank >= 0 && o.delay_rank != D->ctx->xport->rank) return;
   amgk::delay(s, (double)o.delay_usec, D->ctx->wall_khz);
}

extern "C" int amg_dist_solve_iterate(amg_dist_hier *D, int k)
{
   AMG_ARG(D && D->have_state, "amg_dist_solve_iterate: call amg_dist_solve_start first");
   const bool accel = dist_mult_accel(D);
   for (int i = 0; i < k; i++) {
      dist_delay(D, D->ctx->stream); // DMEM_Mult.cpp:40
      if (accel) {
         // DMEM_Mult.cpp:40-55: e = 0; e = M r; x += e; ChebyUpdate(d, e); x += d
         DLevel &v = D->lv[0];
         amgk::vset(D->ctx->stream, v.u, 0.0, 0, v.n);
         AMG_TRY(d_vcycle(D, true));
         double om1 = 0.0, omd = 0.0;
         const bool upd = D->acc.next(D->o, &om1, &omd);
         amgk::dmem_mult_accel(D->ctx->stream, D->x_acc, v.u, D->d_acc, v.n, upd ? 0 : 1, om1, omd);
      } else {
         AMG_TRY(d_vcycle(D, false));
      }
      D->iter++;
      AMG_TRY(d_outer_residual(D, D->iter % (D->hist_cap - 1)));
   }
   return AMG_OK;
}

extern "C" int amg_dist_solve_resnorm(amg_dist_hier *D, double *out)
{
   AMG_ARG(D && out && D->have_state, "amg_dist_solve_resnorm: no solve state");
   amg_ctx *c = D->ctx;
   AMG_HIP(hipMemcpyAsync(c->h_pinned, D->d_hist + D->iter % (D->hist_cap - 1), sizeof(double),
                          hipMemcpyDeviceToHost, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   *out = c->h_pinned[0];
   return AMG_OK;
}

extern "C" int amg_dist_get_u(amg_dist_hier *D, double *u_local)
{
   AMG_ARG(D && u_local, "amg_dist_get_u: null argument");
   AMG_HIP(hipStreamSynchronize(D->ctx->stream));
   AMG_TRY(d2h(D->ctx->stream, u_local, dist_iterate(D), (size_t)D->lv[0].n * sizeof(double)));
   return AMG_OK;
}

extern "C" int amg_dist_profile_read(amg_dist_hier *D, double *ms, long long *launches, int reset)
{
   AMG_ARG(D, "amg_dist_profile_read: null hierarchy");
   AMG_HIP(hipStreamSynchronize(D->ctx->stream));
   for (int k = 0; k < 5; k++) {
      for (auto &e : D->pend[k]) {
         float t = 0.f;
         hipEventSynchronize(e.second);
         if (hipEventElapsedTime(&t, e.first, e.second) == hipSuccess) {
            D->prof_ms[k] += t;
            D->prof_n[k]++;
         }
         hipEventDestroy(e.first);
         hipEventDestroy(e.second);
      }
      D->pend[k].clear();
      if (ms) ms[k] = D->prof_ms[k];
      if (launches) launches[k] = D->prof_n[k];
      if (reset) {
         D->prof_ms[k] = 0;
         D->prof_n[k] = 0;
      }
   }
   return AMG_OK;
}

extern "C" int amg_dist_fine_spmv(amg_dist_hier *D, int reps, double *ms)
{
   AMG_ARG(D && ms && reps >= 1, "amg_dist_fine_spmv: bad argument");
   if (D->slab) return slab_fine_spmv(D, reps, ms);
   amg_ctx *c = D->ctx;
   DLevel &v = D->lv[0];
   hipEvent_t a, b;
   AMG_HIP(hipEventCreate(&a));
   AMG_HIP(hipEventCreate(&b));
   const amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   AMG_HIP(hipEventRecord(a, c->stream));
   for (int r = 0; r < reps; r++) AMG_TRY(d_spgemv(D, v.A, v.u, nullptr, mv, v.r_fine, nullptr));
   AMG_HIP(hipEventRecord(b, c->stream));
   AMG_HIP(hipEventSynchronize(b));
   float t = 0.f;
   AMG_HIP(hipEventElapsedTime(&t, a, b));
   hipEventDestroy(a);
   hipEventDestroy(b);
   *ms = (double)t / reps;
   return AMG_OK;
}
