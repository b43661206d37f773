// amg_grid.cpp -- the level-grouped asynchronous additive solver of the
// distributed reference (DMEM_Add, DMEM_Add.cpp:20-944; message engine
// DMEM_Comm.cpp:11-382; grid assignment DMEM_Setup.cpp:1638-1735; message
// classes DMEM_Setup.cpp:990-1140).
//
// Ranks (one per GPU) are split into grids, one grid per level k.  Every grid
// holds the WHOLE fine problem, row-partitioned among its own ranks (an
// amg_dist_hier over the grid's transport: halo exchange inside the grid), and
// computes only level k's additive correction (AddCycle).  Between grids the
// corrections travel as messages between the ranks whose row ranges overlap
// (gridjToGridk_Correct_outside{Send,Recv}): each message carries the
// accumulated correction of the overlap, a done flag (0 running, 1 my grid
// done, 2 all done) and one spare slot, and a sender keeps at most
// max_inflight messages in flight per destination (data accumulates while
// every slot is busy).  Termination follows CheckConverge / AddResNorm's
// InnerProdFlag / AsyncRecvCleanup.  The protocol runs on the host over a
// non-blocking transport with MPI point-to-point semantics (amg_nb_transport:
// isend / irecv / test / wait and a sum over the grid's ranks); the numerics of
// a grid run on its GPU (or, for protocol tests, a host model).
//
// Device-resident messages (amg_devhub, amg_grid_add_create_devhub): the
// correction accumulators and the in-flight send slots live in device memory,
// and a receiver's accumulate kernel reads a message straight from the sender's
// slot (peer-mapped: ranks are threads of one process sharing the device(s)).
// Completion is by events -- the slot written on the sender's stream, the slot
// read on the receiver's -- polled by test(); the done flag travels as a host
// word of the match.  No payload passes through host memory and no copy is
// made.  The host transport remains the path across processes.
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "amg_dist_internal.h"

namespace {

constexpr int GRIDJ_TO_GRIDK_CORRECT_TAG = 7; // one tag for the correction class
enum Op { ACCUMULATE, WRITE };

// ---- numerics of one grid rank -----------------------------------------------
// vectors of the grid's local rows: x (iterate), b, r (F[0]), y (outgoing
// corrections), e (incoming), d (ChebyUpdate direction of the cheby grid)
struct Backend {
   virtual ~Backend() {}
   virtual int n() const = 0;
   virtual int begin(const double *b, const double *x0) = 0; // y = e = d = 0, r = b - A x
   virtual int cycle() = 0;                                   // AddCycle: u = M_k r (+ ChebyUpdate)
   virtual int y_add_u() = 0;                                 // y += u
   virtual int x_add_u() = 0;                                 // x += u
   virtual int get_y(double *host) = 0;                       // y -> host, then y = 0
   virtual int add_e(const double *host, bool to_d) = 0;      // x += e (d += e)
   virtual int residual(double *rr) = 0;                      // r = b - A x; *rr = local r.r
   virtual int get_x(double *host) = 0;
   // device-resident messages (DistBackend only)
   virtual double *y_dev() { return nullptr; }
   virtual int add_e_dev(const double *, bool) { return AMG_ERR_ARG; }
   virtual hipStream_t dstream() const { return nullptr; }
};

// GPU: the grid's distributed hierarchy
struct DistBackend : Backend {
   amg_dist_hier *D;
   double *x = nullptr, *b = nullptr, *r = nullptr, *y = nullptr, *e = nullptr, *d = nullptr;
   double *u = nullptr; // U[0] of the last cycle
   double *dot = nullptr;
   amgd::AccelState acc;
   bool cheby_mine = false;
   std::vector<double> tmp;
   int n0 = 0;
   explicit DistBackend(amg_dist_hier *D_) : D(D_) {}
   int n() const override { return n0; }
   int init(int k)
   {
      AMG_TRY(amgd::grid_prepare(D, k));
      n0 = D->lv[0].n;
      const size_t cap = std::max(1, D->lv[0].cap);
      AMG_TRY(amgd::dvec(D, cap, &x));
      AMG_TRY(amgd::dvec(D, cap, &b));
      AMG_TRY(amgd::dvec(D, cap, &r));
      AMG_TRY(amgd::dvec(D, cap, &y));
      AMG_TRY(amgd::dvec(D, cap, &e));
      AMG_TRY(amgd::dvec(D, cap, &d));
      AMG_TRY(amgd::dvec(D, 1, &dot));
      tmp.assign(std::max(1, n0), 0.0);
      cheby_mine = k == std::min(D->o.cheby_grid, D->L - 1);
      return AMG_OK;
   }
   hipStream_t st() const { return D->ctx->stream; }
   int begin(const double *bh, const double *x0) override
   {
      AMG_TRY(amgd::h2d(st(), b, bh, (size_t)n0 * 8));
      AMG_TRY(amgd::h2d(st(), x, x0, (size_t)n0 * 8));
      amgk::vset(st(), y, 0.0, 0, n0);
      amgk::vset(st(), e, 0.0, 0, n0);
      amgk::vset(st(), d, 0.0, 0, n0);
      acc.reset(D->o);
      double rr;
      return residual(&rr);
   }
   int cycle() override
   {
      AMG_TRY(amgd::grid_cycle(D, r, &u));
      if (D->o.accel_type != AMG_NO_ACCEL) {
         // DMEM_Add.cpp:319-324: ChebyUpdate(gridk.d, U_array[0]) (async
         // branch, DMEM_Misc.cpp:650-663: only cheby_grid keeps d)
         double om1 = 0.0, omd = 0.0;
         if (acc.next(D->o, &om1, &omd))
            amgk::dmem_cheby_update(st(), d, u, n0, cheby_mine ? 1 : 2, om1, omd);
         else if (cheby_mine)
            amgk::vcopy(st(), u, d, 0, n0);
      }
      AMG_HIP(hipGetLastError());
      return AMG_OK;
   }
   int y_add_u() override
   {
      amgk::vaxpy(st(), 1.0, u, y, 0, n0);
      return AMG_OK;
   }
   int x_add_u() override
   {
      amgk::vaxpy(st(), 1.0, u, x, 0, n0);
      return AMG_OK;
   }
   int get_y(double *host) override
   {
      AMG_TRY(amgd::d2h(st(), host, y, (size_t)n0 * 8));
      amgk::vset(st(), y, 0.0, 0, n0);
      return AMG_OK;
   }
   int add_e(const double *host, bool to_d) override
   {
      AMG_TRY(amgd::h2d(st(), e, host, (size_t)n0 * 8));
      amgk::vaxpy(st(), 1.0, e, x, 0, n0);
      if (to_d) amgk::vaxpy(st(), 1.0, e, d, 0, n0);
      return AMG_OK;
   }
   int residual(double *rr) override
   {
      AMG_TRY(amgd::grid_residual(D, x, b, r));
      double *part;
      AMG_TRY(amg_ctx_partials(D->ctx, 4096 + 1024, &part));
      int np = 0;
      amgk::sumsq_partials(st(), r, n0, part, &np);
      amgk::reduce_partials(st(), part, np, dot, 0, part + 4096);
      AMG_TRY(amgd::d2h(st(), rr, dot, 8));
      return AMG_OK;
   }
   int get_x(double *host) override { return amgd::d2h(st(), host, x, (size_t)n0 * 8); }
   double *y_dev() override { return y; }
   int add_e_dev(const double *ed, bool to_d) override
   {
      amgk::vaxpy(st(), 1.0, ed, x, 0, n0);
      if (to_d) amgk::vaxpy(st(), 1.0, ed, d, 0, n0);
      return AMG_OK;
   }
   hipStream_t dstream() const override { return st(); }
};

// host model for protocol tests: A = diag(a); grid k corrects its own share of
// the rows (global row % number of grids == k) by u = w r ./ a -- the grids
// act on complementary subspaces, as the levels of an additive cycle do
struct HostBackend : Backend {
   std::vector<double> a, x, b, r, y, u, d;
   std::vector<char> mine;
   double w;
   explicit HostBackend(const double *diag, int n, double weight) : a(diag, diag + n), w(weight) {}
   int n() const override { return (int)a.size(); }
   int begin(const double *bh, const double *x0) override
   {
      const int m = n();
      b.assign(bh, bh + m);
      x.assign(x0, x0 + m);
      y.assign(m, 0.0);
      u.assign(m, 0.0);
      d.assign(m, 0.0);
      r.assign(m, 0.0);
      double rr;
      return residual(&rr);
   }
   int cycle() override
   {
      for (int i = 0; i < n(); i++) u[i] = mine[i] ? w * r[i] / a[i] : 0.0;
      return AMG_OK;
   }
   int y_add_u() override
   {
      for (int i = 0; i < n(); i++) y[i] += u[i];
      return AMG_OK;
   }
   int x_add_u() override
   {
      for (int i = 0; i < n(); i++) x[i] += u[i];
      return AMG_OK;
   }
   int get_y(double *host) override
   {
      std::memcpy(host, y.data(), y.size() * 8);
      std::fill(y.begin(), y.end(), 0.0);
      return AMG_OK;
   }
   int add_e(const double *host, bool to_d) override
   {
      for (int i = 0; i < n(); i++) {
         x[i] += host[i];
         if (to_d) d[i] += host[i];
      }
      return AMG_OK;
   }
   int residual(double *rr) override
   {
      double s = 0.0;
      for (int i = 0; i < n(); i++) {
         r[i] = b[i] - a[i] * x[i];
         s += r[i] * r[i];
      }
      *rr = s;
      return AMG_OK;
   }
   int get_x(double *host) override
   {
      std::memcpy(host, x.data(), x.size() * 8);
      return AMG_OK;
   }
};

// ---- one message class (DMEM_CommData) -----------------------------------------
struct CommClass {
   bool send = false;
   std::vector<int> procs, start, len;
   std::vector<int> done_flags, recv_flags, message_count;
   std::vector<std::vector<double>> data;    // [i][len + 2]
   std::vector<long long> requests;          // outstanding receive per peer
   std::vector<int> max_inflight, num_inflight, next_inflight;
   std::vector<std::vector<std::vector<double>>> data_inflight; // [i][j][len + 2]
   std::vector<std::vector<long long>> requests_inflight;
   std::vector<std::vector<int>> inflight_flags;
   // device-resident messages: accumulators / receive buffers and send slots
   std::vector<double *> dd;
   std::vector<std::vector<double *>> dslot;
   std::vector<double *> dpool; // one allocation per peer holding its slots (IPC-mappable)
   std::vector<std::vector<double>> dflag; // the slots' done flags (host words of the messages)
};

} // namespace

// ---- device message hub (ranks as threads of one process) -------------------
// A message is the sender's in-flight slot itself: the receiver's accumulate
// kernel reads the payload straight from it (no copy), and two events order the
// slot's life -- `written` (recorded on the sender's stream after the slot is
// filled) is waited for on the receiver's stream before the read, `consumed`
// (recorded on the receiver's stream after the read) completes the send, so the
// slot is refilled only after it was read.  A receive completes at its match.  Posted sends and receives match per (destination,
// source, tag) in order, as MPI's do; the done flag rides in the match.
struct amg_devhub {
   struct Msg {
      const double *src = nullptr;
      int src_rank = -1;
      long long n = 0;
      double flag = 0.0;
      hipEvent_t written = nullptr, consumed = nullptr;
      bool matched = false;
      ~Msg()
      {
         for (hipEvent_t e : {written, consumed})
            if (e) hipEventDestroy(e);
      }
   };
   using Key = std::tuple<int, int, int>; // (dst, src, tag)
   struct Grid {
      int n = 0, arrived = 0, readers = 0;
      long long gen = 0;
      std::vector<double> acc, out;
   };
   int world = 0;
   std::vector<int> rank_grid;
   std::vector<int> device;   // each rank's device (registered at create)
   std::mutex mu;
   std::condition_variable cv;
   // round-robin schedule (async_schedule = AMG_SCHED_ROUND_ROBIN): the rank
   // holding the token runs; it passes the token at the oracle's points
   int token = 0;
   std::vector<char> finished;
   void wait_turn(int me)
   {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return token == me; });
   }
   void pass_turn(int me, bool fin)
   {
      std::lock_guard<std::mutex> lk(mu);
      if (fin) finished[me] = 1;
      int nx = -1;
      for (int q = 1; q <= world; q++) {
         const int c = (me + q) % world;
         if (!finished[c]) {
            nx = c;
            break;
         }
      }
      if (nx < 0) { // every rank is through: ready for the next solve
         std::fill(finished.begin(), finished.end(), 0);
         nx = 0;
      }
      token = nx;
      cv.notify_all();
   }
   std::map<Key, std::deque<std::shared_ptr<Msg>>> sends, recvs;
   std::map<long long, std::shared_ptr<Msg>> sreq, rreq;
   long long next = 1;
   std::map<int, Grid> grids;

   static int mark(hipStream_t s, hipEvent_t *e)
   {
      AMG_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
      AMG_HIP(hipEventRecord(*e, s));
      return AMG_OK;
   }
   static int ready(hipEvent_t e, bool *ok) // non-blocking completion of e
   {
      *ok = false;
      if (!e) return AMG_OK;
      const hipError_t r = hipEventQuery(e);
      if (r == hipErrorNotReady) return AMG_OK;
      AMG_HIP(r);
      *ok = true;
      return AMG_OK;
   }
   // post a send of src[0:n) (filled by work already queued on stream s) with
   // the message's done flag
   int isend(int me, int peer, int tag, const double *src, long long n, double flag, hipStream_t s,
             long long *req)
   {
      auto m = std::make_shared<Msg>();
      m->src = src;
      m->src_rank = me;
      m->n = n;
      m->flag = flag;
      AMG_TRY(mark(s, &m->written));
      std::lock_guard<std::mutex> lk(mu);
      auto &q = recvs[Key(peer, me, tag)];
      if (!q.empty()) {
         // hand the payload to the receiver's posted request
         auto r = q.front();
         q.pop_front();
         r->src = m->src;
         r->src_rank = me;
         r->n = std::min(r->n, n);
         r->flag = flag;
         r->written = m->written;
         m->written = nullptr;
         r->matched = true;
         m = r;
      } else {
         sends[Key(peer, me, tag)].push_back(m);
      }
      *req = next++;
      sreq[*req] = m;
      return AMG_OK;
   }
   int irecv(int me, int peer, int tag, long long n, long long *req)
   {
      std::lock_guard<std::mutex> lk(mu);
      auto &q = sends[Key(me, peer, tag)];
      std::shared_ptr<Msg> m;
      if (!q.empty()) {
         m = q.front();
         q.pop_front();
         m->n = std::min(m->n, n);
         m->matched = true;
      } else {
         m = std::make_shared<Msg>();
         m->n = n;
         recvs[Key(me, peer, tag)].push_back(m);
      }
      *req = next++;
      rreq[*req] = m;
      return AMG_OK;
   }
   // MPI_Test of a receive: done once a send has matched it (the sender's
   // slot write is queued on its stream).  The receiver's stream then waits for
   // that write (in stream order: the event was recorded before this wait is
   // queued, so waits never form a cycle) and reads *src until consume()
   int test_recv(long long req, hipStream_t s, int *done, double *flag, const double **src, long long *n)
   {
      std::lock_guard<std::mutex> lk(mu);
      auto it = rreq.find(req);
      AMG_ARG(it != rreq.end(), "amg_devhub: unknown receive %lld", req);
      const auto &m = it->second;
      *done = m->matched;
      if (m->matched) {
         // the receiver's kernel reads the sender's slot in place: a sender on
         // another device must be peer-accessible from this one
         const int sd = m->src_rank >= 0 ? device[m->src_rank] : -1;
         int cur = -1;
         AMG_HIP(hipGetDevice(&cur));
         if (sd >= 0 && sd != cur) {
            int can = 0;
            AMG_HIP(hipDeviceCanAccessPeer(&can, cur, sd));
            AMG_ARG(can, "amg_devhub: device %d cannot read device %d's message slots", cur, sd);
            const hipError_t e = hipDeviceEnablePeerAccess(sd, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
               return amg_set_error(AMG_ERR_HIP, "amg_devhub: hipDeviceEnablePeerAccess(%d): %s", sd,
                                    hipGetErrorString(e));
            (void)hipGetLastError();
         }
         AMG_HIP(hipStreamWaitEvent(s, m->written, 0));
         *flag = m->flag;
         *src = m->src;
         *n = m->n;
      }
      return AMG_OK;
   }
   // the receiver's kernels reading the slot are queued on s: the send completes
   // when they have run
   int consume(long long req, hipStream_t s)
   {
      hipEvent_t e;
      AMG_TRY(mark(s, &e));
      std::lock_guard<std::mutex> lk(mu);
      auto it = rreq.find(req);
      AMG_ARG(it != rreq.end(), "amg_devhub: unknown receive %lld", req);
      it->second->consumed = e;
      rreq.erase(it);
      return AMG_OK;
   }
   // MPI_Test of a send
   int test_send(long long req, int *done)
   {
      std::lock_guard<std::mutex> lk(mu);
      auto it = sreq.find(req);
      AMG_ARG(it != sreq.end(), "amg_devhub: unknown send %lld", req);
      bool ok = false;
      AMG_TRY(ready(it->second->consumed, &ok));
      *done = ok;
      if (ok) sreq.erase(it); // the record (and its events) goes with the last side
      return AMG_OK;
   }
   int wait_send(long long req)
   {
      for (;;) {
         int done = 0;
         AMG_TRY(test_send(req, &done));
         if (done) return AMG_OK;
         std::this_thread::yield();
      }
   }
   // InnerProdFlag over the caller's grid
   int grid_sum(int me, double *vals, int n)
   {
      std::unique_lock<std::mutex> lk(mu);
      Grid &g = grids[rank_grid[me]];
      cv.wait(lk, [&] { return g.readers == 0; }); // the previous sum fully read
      if (g.arrived == 0) g.acc.assign(n, 0.0);
      for (int i = 0; i < n; i++) g.acc[i] += vals[i];
      const long long gen = g.gen;
      if (++g.arrived == g.n) {
         g.out = g.acc;
         g.arrived = 0;
         g.readers = g.n;
         g.gen++;
         cv.notify_all();
      } else {
         cv.wait(lk, [&] { return g.gen != gen; });
      }
      for (int i = 0; i < n; i++) vals[i] = g.out[i];
      if (--g.readers == 0) cv.notify_all();
      return AMG_OK;
   }
};

extern "C" int amg_devhub_create(int world, const int *rank_grid, amg_devhub **out)
{
   AMG_ARG(world >= 1 && rank_grid && out, "amg_devhub_create: bad argument");
   auto h = std::make_unique<amg_devhub>();
   h->world = world;
   h->rank_grid.assign(rank_grid, rank_grid + world);
   h->finished.assign(world, 0);
   h->device.assign(world, -1);
   for (int r = 0; r < world; r++) h->grids[rank_grid[r]].n++;
   *out = h.release();
   return AMG_OK;
}

extern "C" int amg_devhub_free(amg_devhub *h)
{
   delete h;
   return AMG_OK;
}

namespace {

constexpr int IPC_ACK_TAG = GRIDJ_TO_GRIDK_CORRECT_TAG + 1;    // receiver -> sender: slot read
constexpr int IPC_HANDLE_TAG = GRIDJ_TO_GRIDK_CORRECT_TAG + 2; // the slot pools' IPC handles

// the payload path of device-resident messages: a message is sender slot
// `slot` (device memory), read in place by the receiver's kernel
struct MsgLink {
   virtual ~MsgLink() = default;
   virtual int isend(int peer, const double *src, int slot, long long n, double flag, hipStream_t s,
                     long long *req) = 0;
   virtual int irecv(int peer, long long n, long long *req) = 0;
   // done: *src may be read by work queued on s from now on, until consume()
   virtual int test_recv(long long req, hipStream_t s, int *done, double *flag, const double **src,
                         long long *n) = 0;
   virtual int consume(long long req, hipStream_t s) = 0;
   virtual int test_send(long long req, int *done) = 0;
   virtual int grid_sum(double *v, int n) = 0;
   virtual int flush() { return AMG_OK; } // outstanding acknowledgements, at the end of a solve
   int wait_send(long long req)
   {
      for (;;) {
         int done = 0;
         AMG_TRY(test_send(req, &done));
         if (done) return AMG_OK;
         std::this_thread::yield();
      }
   }
};

// ranks as threads of one process: the hub
struct HubLink : MsgLink {
   amg_devhub *h;
   int me;
   HubLink(amg_devhub *h_, int me_) : h(h_), me(me_) {}
   int isend(int peer, const double *src, int, long long n, double flag, hipStream_t s, long long *req) override
   {
      return h->isend(me, peer, GRIDJ_TO_GRIDK_CORRECT_TAG, src, n, flag, s, req);
   }
   int irecv(int peer, long long n, long long *req) override
   {
      return h->irecv(me, peer, GRIDJ_TO_GRIDK_CORRECT_TAG, n, req);
   }
   int test_recv(long long req, hipStream_t s, int *done, double *flag, const double **src, long long *n) override
   {
      return h->test_recv(req, s, done, flag, src, n);
   }
   int consume(long long req, hipStream_t s) override { return h->consume(req, s); }
   int test_send(long long req, int *done) override { return h->test_send(req, done); }
   int grid_sum(double *v, int n) override { return h->grid_sum(me, v, n); }
};

int xp(int st, const char *what)
{
   return st == 0 ? AMG_OK : amg_set_error(AMG_ERR_ARG, "amg_grid_add: transport %s failed (%d)", what, st);
}

// ranks as processes: every send slot pool is mapped into its receiver's
// address space once (hipIpcGetMemHandle / hipIpcOpenMemHandle, handles
// exchanged over the host transport at creation).  Per message the host
// transport carries only a control word pair (slot, done flag) -- sent once
// the slot's write has run on the sender's stream -- and an acknowledgement
// back once the receiver's read of the slot has run on its stream; the send
// completes with the acknowledgement, so the slot is refilled only after it
// was read.  The payload never leaves device memory.
struct IpcLink : MsgLink {
   amg_nb_transport t;
   struct Peer {
      const double *base = nullptr; // the sender's slot pool, mapped here
      long long len = 0;            // doubles per slot
   };
   std::map<int, Peer> peers; // receive peers
   struct SendRec {
      int peer = 0;
      hipEvent_t written = nullptr; // the slot's write, on the sender's stream
      bool ctl_sent = false;        // the control word goes out once `written` has run
      long long ctl_req = 0, ack_req = 0;
      double ctl[2] = {0.0, 0.0}, ack = 0.0;
      bool ctl_done = false, ack_done = false;
   };
   struct RecvRec {
      long long req = 0;
      int peer = 0;
      double ctl[2] = {0.0, 0.0};
   };
   struct AckRec {
      int peer = 0;
      hipEvent_t ev = nullptr;
      bool sent = false;
      long long req = 0;
      double buf = 1.0;
   };
   std::map<long long, std::unique_ptr<SendRec>> sends;
   std::map<long long, std::unique_ptr<RecvRec>> recvs;
   std::deque<std::unique_ptr<AckRec>> acks;
   std::vector<void *> opened;
   long long next = 1;
   explicit IpcLink(const amg_nb_transport &t_) : t(t_) {}
   ~IpcLink() override
   {
      for (auto &a : acks)
         if (a->ev) hipEventDestroy(a->ev);
      for (auto &sr : sends)
         if (sr.second->written) hipEventDestroy(sr.second->written);
      for (void *p : opened) hipIpcCloseMemHandle(p);
   }
   // send the control word of every slot whose write has run (in issue order:
   // the writes are on one stream, so they complete in order); acknowledge
   // every read that has run; retire sent acknowledgements
   int progress()
   {
      for (auto &kv : sends) {
         SendRec &r = *kv.second;
         if (r.ctl_sent) continue;
         const hipError_t q = hipEventQuery(r.written);
         if (q == hipErrorNotReady) break;
         AMG_HIP(q);
         AMG_TRY(xp(t.isend(t.user, r.peer, GRIDJ_TO_GRIDK_CORRECT_TAG, r.ctl, 2, &r.ctl_req), "isend"));
         r.ctl_sent = true;
         hipEventDestroy(r.written);
         r.written = nullptr;
      }
      for (auto it = acks.begin(); it != acks.end();) {
         AckRec &a = **it;
         if (!a.sent) {
            const hipError_t q = hipEventQuery(a.ev);
            if (q == hipErrorNotReady) {
               ++it;
               continue;
            }
            AMG_HIP(q);
            AMG_TRY(xp(t.isend(t.user, a.peer, IPC_ACK_TAG, &a.buf, 1, &a.req), "isend"));
            a.sent = true;
         }
         int done = 0;
         AMG_TRY(xp(t.test(t.user, a.req, &done), "test"));
         if (done) {
            hipEventDestroy(a.ev);
            it = acks.erase(it);
         } else {
            ++it;
         }
      }
      return AMG_OK;
   }
   int isend(int peer, const double *, int slot, long long, double flag, hipStream_t s, long long *req) override
   {
      // the control word waits for the slot's write (an event, polled by
      // progress()) -- the host never blocks on the grid's stream here
      auto r = std::make_unique<SendRec>();
      r->peer = peer;
      r->ctl[0] = (double)slot;
      r->ctl[1] = flag;
      AMG_HIP(hipEventCreateWithFlags(&r->written, hipEventDisableTiming));
      AMG_HIP(hipEventRecord(r->written, s));
      AMG_TRY(xp(t.irecv(t.user, peer, IPC_ACK_TAG, &r->ack, 1, &r->ack_req), "irecv"));
      *req = next++;
      sends[*req] = std::move(r);
      return progress();
   }
   int irecv(int peer, long long, long long *req) override
   {
      auto r = std::make_unique<RecvRec>();
      r->peer = peer;
      AMG_TRY(xp(t.irecv(t.user, peer, GRIDJ_TO_GRIDK_CORRECT_TAG, r->ctl, 2, &r->req), "irecv"));
      *req = next++;
      recvs[*req] = std::move(r);
      return AMG_OK;
   }
   int test_recv(long long req, hipStream_t, int *done, double *flag, const double **src, long long *n) override
   {
      AMG_TRY(progress());
      auto it = recvs.find(req);
      AMG_ARG(it != recvs.end(), "amg_grid_add: unknown receive %lld", req);
      RecvRec &r = *it->second;
      AMG_TRY(xp(t.test(t.user, r.req, done), "test"));
      if (*done) {
         const Peer &p = peers.at(r.peer);
         *flag = r.ctl[1];
         *src = p.base + (long long)r.ctl[0] * p.len;
         *n = p.len;
      }
      return AMG_OK;
   }
   int consume(long long req, hipStream_t s) override
   {
      auto it = recvs.find(req);
      AMG_ARG(it != recvs.end(), "amg_grid_add: unknown receive %lld", req);
      auto a = std::make_unique<AckRec>();
      a->peer = it->second->peer;
      AMG_HIP(hipEventCreateWithFlags(&a->ev, hipEventDisableTiming));
      AMG_HIP(hipEventRecord(a->ev, s));
      acks.push_back(std::move(a));
      recvs.erase(it);
      return progress();
   }
   int test_send(long long req, int *done) override
   {
      AMG_TRY(progress());
      auto it = sends.find(req);
      AMG_ARG(it != sends.end(), "amg_grid_add: unknown send %lld", req);
      SendRec &r = *it->second;
      int d = 0;
      if (!r.ctl_sent) {
         *done = 0;
         return AMG_OK;
      }
      if (!r.ctl_done) {
         AMG_TRY(xp(t.test(t.user, r.ctl_req, &d), "test"));
         r.ctl_done = d;
      }
      if (!r.ack_done) {
         AMG_TRY(xp(t.test(t.user, r.ack_req, &d), "test"));
         r.ack_done = d;
      }
      *done = r.ctl_done && r.ack_done;
      if (*done) sends.erase(it);
      return AMG_OK;
   }
   int grid_sum(double *v, int n) override { return xp(t.grid_allreduce(t.user, v, n), "grid_allreduce"); }
   int flush() override
   {
      auto unsent = [&] {
         for (auto &kv : sends)
            if (!kv.second->ctl_sent) return true;
         return false;
      };
      while (!acks.empty() || unsent()) {
         AMG_TRY(progress());
         if (!acks.empty() || unsent()) std::this_thread::yield();
      }
      return AMG_OK;
   }
};

} // namespace

struct amg_grid_add {
   amg_nb_transport t{};
   std::unique_ptr<MsgLink> link; // device-resident messages (else the host transport t)
   amg_devhub *hub = nullptr;     // the in-process hub (round-robin schedule)
   bool rr = false;               // async_schedule = AMG_SCHED_ROUND_ROBIN
   bool dev = false;
   double *ehd = nullptr, *zd = nullptr; // incoming corrections / zeros (device)
   amg_opts o{};
   int my_grid = 0, world = 1, me = 0, grid_size = 1;
   long long row0 = 0, row1 = 0; // my global rows in my grid's partition
   std::unique_ptr<Backend> be;
   CommClass send, recv;
   // DMEM_AllData iter / comm state
   int all_done_flag = 0, outside_done_flag = 0, grid_done_flag = 0, converge_flag = 0;
   int r_local_converge_flag = 0, cycle = 0;
   double r0_norm2 = 1.0, r_local = 1.0;
   long long messages_sent = 0, messages_recv = 0;
   std::vector<double> yh, eh;
};

namespace {

// round robin (the oracle's or_dmem_add sched 1): at each of the oracle's
// yield points the rank finishes its queued work (so every event a peer may
// test has completed), hands the token on and waits for it to come back
int rr_yield(amg_grid_add *G)
{
   if (!G->rr) return AMG_OK;
   AMG_HIP(hipStreamSynchronize(G->be->dstream()));
   G->hub->pass_turn(G->me, false);
   G->hub->wait_turn(G->me);
   return AMG_OK;
}

int xp_err(int st, const char *what)
{
   return st == 0 ? AMG_OK : amg_set_error(AMG_ERR_ARG, "amg_grid_add: transport %s failed (%d)", what, st);
}

// the message transport: the device hub or the caller's host transport
int tp_test(amg_grid_add *G, long long req, int *done)
{
   if (G->dev) return G->link->test_send(req, done);
   return xp_err(G->t.test(G->t.user, req, done), "test");
}

int tp_sum(amg_grid_add *G, double *v, int n)
{
   if (G->dev) return G->link->grid_sum(v, n);
   return xp_err(G->t.grid_allreduce(G->t.user, v, n), "grid_allreduce");
}

int tp_irecv(amg_grid_add *G, CommClass &cd, int i)
{
   if (G->dev) return G->link->irecv(cd.procs[i], cd.len[i], &cd.requests[i]);
   return xp_err(G->t.irecv(G->t.user, cd.procs[i], GRIDJ_TO_GRIDK_CORRECT_TAG, cd.data[i].data(), cd.len[i] + 2,
                            &cd.requests[i]),
                 "irecv");
}

// CheckInFlight (DMEM_Comm.cpp:25-63)
int check_inflight(amg_grid_add *G, CommClass &cd, int i)
{
   while (true) {
      int break_flag = 0;
      if (G->all_done_flag == 0)
         break_flag = 1;
      else if (cd.num_inflight[i] < cd.max_inflight[i])
         break;
      for (int j = 0; j < cd.max_inflight[i]; j++) {
         if (cd.inflight_flags[i][j] == 1) {
            int flag = 0;
            AMG_TRY(tp_test(G, cd.requests_inflight[i][j], &flag));
            if (flag) {
               cd.inflight_flags[i][j] = 0;
               cd.num_inflight[i]--;
               if (j < cd.next_inflight[i]) cd.next_inflight[i] = j;
               if (G->all_done_flag == 1) {
                  break_flag = 1;
                  break;
               }
            }
         } else if (G->all_done_flag == 1) {
            break_flag = 1;
            break;
         }
      }
      if (break_flag) break;
      AMG_TRY(rr_yield(G));
   }
   return AMG_OK;
}

// SetNextInFlight (DMEM_Comm.cpp:65-75)
void set_next_inflight(CommClass &cd, int i)
{
   for (int j = 0; j < cd.max_inflight[i]; j++)
      if (cd.inflight_flags[i][j] == 0) {
         cd.next_inflight[i] = j;
         return;
      }
   cd.next_inflight[i] = cd.max_inflight[i];
}

// SendRecv, asynchronous outside classes (DMEM_Comm.cpp:77-348); v holds the
// grid's local rows (device memory in device mode); returns the recv / send flag
int send_recv(amg_grid_add *G, CommClass &cd, double *v, Op op, int *ret)
{
   const bool local = G->o.converge_test_type != AMG_GLOBAL;
   const bool dev = G->dev;
   const hipStream_t s = dev ? G->be->dstream() : nullptr;
   int return_flag = 0;
   for (int i = 0; i < (int)cd.procs.size(); i++) {
      const int ip = cd.procs[i], vs = cd.start[i], vl = cd.len[i];
      cd.recv_flags[i] = 0;
      if (cd.send) {
         if (cd.done_flags[i] >= 2) continue;
         if (dev) {
            // the accumulator of what could not be sent yet, on the grid's stream
            // (adding the cleanup's zeros is skipped: it changes nothing)
            if (op == WRITE)
               amgk::vcopy(s, v + vs, cd.dd[i], 0, vl);
            else if (v != G->zd)
               amgk::vaxpy(s, 1.0, v + vs, cd.dd[i], 0, vl);
         } else if (op == WRITE) {
            std::memcpy(cd.data[i].data(), v + vs, (size_t)vl * 8);
         } else {
            for (int j = 0; j < vl; j++) cd.data[i][j] += v[vs + j];
         }
         AMG_TRY(check_inflight(G, cd, i));
         if (cd.num_inflight[i] >= cd.max_inflight[i]) continue;
         const int nx = cd.next_inflight[i];
         double *flw;
         if (dev) {
            amgk::vcopy(s, cd.dd[i], cd.dslot[i][nx], 0, vl);
            amgk::vset(s, cd.dd[i], 0.0, 0, vl);
            flw = &cd.dflag[i][nx];
         } else {
            std::vector<double> &slot = cd.data_inflight[i][nx];
            std::memcpy(slot.data(), cd.data[i].data(), (size_t)vl * 8);
            std::fill(cd.data[i].begin(), cd.data[i].begin() + vl, 0.0);
            flw = &slot[vl];
         }
         if (G->grid_done_flag == 1) {
            *flw = 1.0;
            if (local) {
               cd.done_flags[i] = 2;
            } else {
               cd.done_flags[i] = 1;
               if (G->all_done_flag == 1) {
                  cd.done_flags[i] = 2;
                  *flw = 2.0;
               }
            }
         }
         if (dev)
            AMG_TRY(G->link->isend(ip, cd.dslot[i][nx], nx, vl, *flw, s, &cd.requests_inflight[i][nx]));
         else
            AMG_TRY(xp_err(G->t.isend(G->t.user, ip, GRIDJ_TO_GRIDK_CORRECT_TAG, cd.data_inflight[i][nx].data(),
                                      vl + 2, &cd.requests_inflight[i][nx]),
                           "isend"));
         cd.inflight_flags[i][nx] = 1;
         cd.num_inflight[i]++;
         set_next_inflight(cd, i);
         cd.message_count[i]++;
         G->messages_sent++;
         return_flag = 1;
      } else {
         if (cd.done_flags[i] >= 2) continue;
         while (true) {
            int flag = 0;
            double fl = 0.0;
            const double *src = nullptr;
            long long got = 0;
            if (dev)
               AMG_TRY(G->link->test_recv(cd.requests[i], s, &flag, &fl, &src, &got));
            else
               AMG_TRY(tp_test(G, cd.requests[i], &flag));
            if (!flag) break;
            cd.message_count[i]++;
            G->messages_recv++;
            if (dev) {
               // read the payload from the sender's slot, then release it
               amgk::vaxpy(s, 1.0, src, v + vs, 0, (int)std::min<long long>(got, vl));
               AMG_TRY(G->link->consume(cd.requests[i], s));
            } else {
               for (int j = 0; j < vl; j++) v[vs + j] += cd.data[i][j];
               fl = cd.data[i][vl];
            }
            if (local) {
               if (fl == 1.0) {
                  cd.done_flags[i] = 2;
                  break;
               }
            } else {
               if (fl == 1.0) {
                  cd.done_flags[i] = 1;
               } else if (fl == 2.0) {
                  cd.done_flags[i] = 2;
                  break;
               }
            }
            AMG_TRY(tp_irecv(G, cd, i));
            cd.recv_flags[i] = 1;
            return_flag = 1;
            if (G->o.async_type == AMG_SEMI_ASYNC && G->all_done_flag == 0) break;
         }
      }
   }
   *ret = return_flag;
   return AMG_OK;
}

// DMEM_AddCheckComm (DMEM_Add.cpp:460-528)
int add_check_comm(amg_grid_add *G)
{
   const bool to_d = G->o.accel_type != AMG_NO_ACCEL && G->my_grid == G->o.cheby_grid;
   int recv_flag = 0;
   if (G->dev) {
      amgk::vset(G->be->dstream(), G->ehd, 0.0, 0, G->be->n());
      AMG_TRY(send_recv(G, G->recv, G->ehd, ACCUMULATE, &recv_flag));
      if (recv_flag == 1) AMG_TRY(G->be->add_e_dev(G->ehd, to_d));
   } else {
      std::fill(G->eh.begin(), G->eh.end(), 0.0);
      AMG_TRY(send_recv(G, G->recv, G->eh.data(), ACCUMULATE, &recv_flag));
      if (recv_flag == 1) AMG_TRY(G->be->add_e(G->eh.data(), to_d));
   }
   for (int i = 0; i < (int)G->send.procs.size(); i++) AMG_TRY(check_inflight(G, G->send, i));
   return AMG_OK;
}

// DMEM_AddCorrect_LocalRes (DMEM_Add.cpp:391-458)
int add_correct(amg_grid_add *G)
{
   AMG_TRY(G->be->y_add_u());
   if (G->converge_flag == 1 || G->cycle % std::max(1, G->o.async_comm_save_divisor) == 0) {
      int f;
      if (G->dev) {
         double *y = G->be->y_dev();
         AMG_TRY(send_recv(G, G->send, y, ACCUMULATE, &f));
         amgk::vset(G->be->dstream(), y, 0.0, 0, G->be->n());
      } else {
         AMG_TRY(G->be->get_y(G->yh.data()));
         AMG_TRY(send_recv(G, G->send, G->yh.data(), ACCUMULATE, &f));
      }
   }
   AMG_TRY(G->be->x_add_u());
   return add_check_comm(G);
}

// DMEM_CheckOutsideDoneFlag (DMEM_Add.cpp:741-749)
void check_outside_done(amg_grid_add *G)
{
   auto none0 = [](const CommClass &cd) {
      for (int f : cd.done_flags)
         if (f == 0) return false;
      return true;
   };
   if (none0(G->send) && none0(G->recv)) G->outside_done_flag = 1;
}

// CheckConverge (DMEM_Add.cpp:905-944)
int check_converge(amg_grid_add *G)
{
   const amg_opts &o = G->o;
   if (o.converge_test_type == AMG_GLOBAL) {
      if (G->all_done_flag == 0) {
         if (G->grid_done_flag == 0 && (G->cycle >= o.num_cycles - 1 || G->r_local_converge_flag == 1))
            G->grid_done_flag = 1;
         if (G->grid_done_flag == 1 && G->outside_done_flag == 0) check_outside_done(G);
         return 0;
      }
      return 1;
   }
   if (G->cycle >= o.num_cycles - 1 || G->r_local_converge_flag == 1) {
      G->grid_done_flag = 1;
      return 1;
   }
   return 0;
}

// AddResNorm, async FULL_ASYNC branch (DMEM_Add.cpp:331-389): InnerProdFlag
// sums (r.r, outside_done_flag) over the grid's ranks
int add_res_norm(amg_grid_add *G, double rr)
{
   if (G->o.async_type == AMG_SEMI_ASYNC) return AMG_OK; // :346-358: not computed
   double v[2] = {rr, (double)G->outside_done_flag};
   AMG_TRY(tp_sum(G, v, 2));
   G->r_local = std::sqrt(v[0]) / G->r0_norm2;
   if (G->r_local < G->o.tol) G->r_local_converge_flag = 1;
   if ((int)v[1] == G->grid_size) G->all_done_flag = 1;
   return AMG_OK;
}

// AsyncRecvCleanup (DMEM_Add.cpp:829-884) + CompleteInFlight (DMEM_Comm.cpp:11-23)
int async_end(amg_grid_add *G)
{
   const bool local = G->o.converge_test_type != AMG_GLOBAL;
   auto all2 = [](const CommClass &cd) {
      for (int f : cd.done_flags)
         if (f != 2) return false;
      return true;
   };
   std::vector<double> zero;
   double *eh = G->ehd, *z = G->zd;
   if (G->dev) {
      amgk::vset(G->be->dstream(), G->ehd, 0.0, 0, G->be->n());
   } else {
      std::fill(G->eh.begin(), G->eh.end(), 0.0);
      zero.assign(G->yh.size(), 0.0);
      eh = G->eh.data();
      z = zero.data();
   }
   for (long long spin = 0;; spin++) {
      if (local ? (all2(G->recv) && all2(G->send)) : all2(G->recv)) break;
      int f;
      AMG_TRY(send_recv(G, G->recv, eh, ACCUMULATE, &f));
      if (local) AMG_TRY(send_recv(G, G->send, z, ACCUMULATE, &f));
      AMG_TRY(rr_yield(G));
      if (spin > (1LL << 34)) return amg_set_error(AMG_ERR_ARG, "amg_grid_add: cleanup never completed");
   }
   if (G->dev)
      AMG_TRY(G->be->add_e_dev(G->ehd, false));
   else
      AMG_TRY(G->be->add_e(G->eh.data(), false));
   for (int i = 0; i < (int)G->send.procs.size(); i++)
      for (int j = 0; j < G->send.max_inflight[i]; j++)
         if (G->send.inflight_flags[i][j] == 1) {
            if (G->rr) {
               for (;;) {
                  int done = 0;
                  AMG_TRY(G->link->test_send(G->send.requests_inflight[i][j], &done));
                  if (done) break;
                  AMG_TRY(rr_yield(G));
               }
            } else if (G->dev)
               AMG_TRY(G->link->wait_send(G->send.requests_inflight[i][j]));
            else
               AMG_TRY(xp_err(G->t.wait(G->t.user, G->send.requests_inflight[i][j]), "wait"));
            G->send.inflight_flags[i][j] = 0;
         }
   if (G->dev) AMG_TRY(G->link->flush()); // acknowledge the last reads
   return AMG_OK;
}

// the outside classes: every rank of another grid whose row range overlaps
// mine (DMEM_Setup.cpp:996-1047 send, :1106-1140 receive); start / len in my
// local rows
int build_classes(amg_grid_add *G, const int *rank_grid, const long long *rank_rows)
{
   for (CommClass *cd : {&G->send, &G->recv}) {
      const bool send = cd == &G->send;
      cd->send = send;
      for (int p = 0; p < G->world; p++) {
         if (rank_grid[p] == G->my_grid) continue;
         const long long ps = rank_rows[2 * p], pe = rank_rows[2 * p + 1];
         const long long s = std::max(ps, G->row0), e = std::min(pe, G->row1);
         if (e <= s) continue;
         cd->procs.push_back(p);
         cd->start.push_back((int)(s - G->row0));
         cd->len.push_back((int)(e - s));
      }
      const size_t np = cd->procs.size();
      cd->done_flags.assign(np, 0);
      cd->recv_flags.assign(np, 0);
      cd->message_count.assign(np, 0);
      // host payload buffers (device mode: in device memory, alloc_dev)
      const auto hl = [&](size_t i) { return G->dev ? (size_t)2 : (size_t)cd->len[i] + 2; };
      cd->data.resize(np);
      for (size_t i = 0; i < np; i++) cd->data[i].assign(hl(i), 0.0);
      if (send) {
         const int mi = std::max(1, G->o.max_inflight);
         cd->max_inflight.assign(np, mi);
         cd->num_inflight.assign(np, 0);
         cd->next_inflight.assign(np, 0);
         cd->data_inflight.resize(np);
         cd->requests_inflight.assign(np, std::vector<long long>(mi, 0));
         cd->inflight_flags.assign(np, std::vector<int>(mi, 0));
         for (size_t i = 0; i < np; i++) cd->data_inflight[i].assign(mi, std::vector<double>(hl(i), 0.0));
         cd->dflag.assign(np, std::vector<double>(mi, 0.0));
      } else {
         cd->requests.assign(np, 0);
      }
   }
   return AMG_OK;
}

void reset_classes(amg_grid_add *G)
{
   for (CommClass *cd : {&G->send, &G->recv}) {
      std::fill(cd->done_flags.begin(), cd->done_flags.end(), 0);
      std::fill(cd->recv_flags.begin(), cd->recv_flags.end(), 0);
      std::fill(cd->message_count.begin(), cd->message_count.end(), 0);
      for (auto &v : cd->data) std::fill(v.begin(), v.end(), 0.0);
      for (auto &f : cd->inflight_flags) std::fill(f.begin(), f.end(), 0);
      std::fill(cd->num_inflight.begin(), cd->num_inflight.end(), 0);
      std::fill(cd->next_inflight.begin(), cd->next_inflight.end(), 0);
      for (auto &pool : cd->data_inflight)
         for (auto &v : pool) std::fill(v.begin(), v.end(), 0.0);
      for (auto &f : cd->dflag) std::fill(f.begin(), f.end(), 0.0);
   }
   if (G->dev) {
      // the device accumulators / receive buffers start from zero
      const hipStream_t s = G->be->dstream();
      for (CommClass *cd : {&G->send, &G->recv})
         for (size_t i = 0; i < cd->dd.size(); i++) amgk::vset(s, cd->dd[i], 0.0, 0, cd->len[i]);
   }
}

// device-mode buffers, from the grid's hierarchy's pool (freed with it)
int alloc_dev(amg_grid_add *G, amg_dist_hier *D)
{
   const int n = std::max(1, G->be->n());
   AMG_TRY(amgd::dvec(D, n, &G->ehd));
   AMG_TRY(amgd::dvec(D, n, &G->zd));
   amgk::vset(G->be->dstream(), G->zd, 0.0, 0, n);
   // send side only: the receiver reads the sender's slots
   CommClass &cd = G->send;
   const size_t np = cd.procs.size();
   cd.dd.assign(np, nullptr);
   cd.dslot.assign(np, {});
   cd.dpool.assign(np, nullptr);
   for (size_t i = 0; i < np; i++) {
      const int len = std::max(1, cd.len[i]), mi = cd.max_inflight[i];
      AMG_TRY(amgd::dvec(D, len, &cd.dd[i]));
      AMG_TRY(amgd::dvec(D, (size_t)len * mi, &cd.dpool[i]));
      cd.dslot[i].assign(mi, nullptr);
      for (int j = 0; j < mi; j++) cd.dslot[i][j] = cd.dpool[i] + (size_t)j * len;
   }
   return AMG_OK;
}

int create_common(amg_grid_add *G, int my_grid, int world, int me, const int *rank_grid,
                  const long long *rank_rows, const amg_nb_transport *t)
{
   AMG_ARG(G->dev || (t && t->isend && t->irecv && t->test && t->wait && t->grid_allreduce),
           "amg_grid_add: incomplete transport");
   AMG_ARG(rank_grid && rank_rows && world >= 1 && me >= 0 && me < world && rank_grid[me] == my_grid,
           "amg_grid_add: bad rank layout");
   AMG_ARG(!(G->o.async_type == AMG_SEMI_ASYNC && G->o.converge_test_type == AMG_GLOBAL),
           "amg_grid_add: SEMI_ASYNC with converge_test GLOBAL never terminates in the reference "
           "(AddResNorm computes no flags for SEMI_ASYNC, DMEM_Add.cpp:346-358)");
   if (t) G->t = *t;
   G->my_grid = my_grid;
   G->world = world;
   G->me = me;
   G->grid_size = 0;
   for (int p = 0; p < world; p++) G->grid_size += rank_grid[p] == my_grid;
   G->row0 = rank_rows[2 * me];
   G->row1 = rank_rows[2 * me + 1];
   AMG_ARG(G->row1 - G->row0 == G->be->n(), "amg_grid_add: row range %lld..%lld vs %d local rows", G->row0,
           G->row1, G->be->n());
   G->yh.assign(std::max(1, G->be->n()), 0.0);
   G->eh.assign(std::max(1, G->be->n()), 0.0);
   return build_classes(G, rank_grid, rank_rows);
}

} // namespace

// DMEM_Setup.cpp:1638-1735 (assign_procs_type default): ranks per grid from the
// levels' work fractions, grids in level order, at least one rank each
extern "C" int amg_grid_partition(int num_procs, int num_grids, const double *frac_work, int *procs_per_grid)
{
   AMG_ARG(num_procs >= num_grids && num_grids >= 1 && frac_work && procs_per_grid,
           "amg_grid_partition: %d ranks cannot hold %d grids", num_procs, num_grids);
   int count = num_procs;
   for (int level = 0; level < num_grids; level++) {
      int cur;
      if (level == num_grids - 1 || count == 1) {
         cur = count;
      } else if (count == num_grids - level) {
         cur = 1;
      } else {
         cur = std::max((int)std::ceil(frac_work[level] * (double)num_procs), 1);
         while (true) {
            const int next = cur - 1;
            const double next_frac = (double)next / (double)num_procs;
            const double diff_cur = std::fabs(frac_work[level] - (double)cur / (double)num_procs);
            const double diff_next = std::fabs(frac_work[level] - next_frac);
            if (count - cur <= num_grids - level) {
               cur = count - (num_grids - level) + 1;
               break;
            }
            if (diff_cur <= diff_next || cur == 1) break;
            cur--;
         }
      }
      procs_per_grid[level] = cur;
      count -= cur;
   }
   return AMG_OK;
}

extern "C" int amg_grid_add_create(amg_dist_hier *D, int my_grid, int world_nranks, int world_rank,
                                   const int *rank_grid, const long long *rank_rows, const amg_nb_transport *t,
                                   amg_grid_add **out)
{
   AMG_ARG(D && out, "amg_grid_add_create: null argument");
   AMG_ARG(D->o.solver == AMG_ASYNC_MULTADD, "amg_grid_add_create: ASYNC_MULTADD hierarchies only");
   auto G = std::make_unique<amg_grid_add>();
   G->o = D->o;
   auto be = std::make_unique<DistBackend>(D);
   AMG_TRY(be->init(my_grid));
   G->be = std::move(be);
   AMG_TRY(create_common(G.get(), my_grid, world_nranks, world_rank, rank_grid, rank_rows, t));
   *out = G.release();
   return AMG_OK;
}

// the same, with device-resident correction messages over an in-process hub
extern "C" int amg_grid_add_create_devhub(amg_dist_hier *D, int my_grid, int world_nranks, int world_rank,
                                          const int *rank_grid, const long long *rank_rows, amg_devhub *hub,
                                          amg_grid_add **out)
{
   AMG_ARG(D && hub && out, "amg_grid_add_create_devhub: null argument");
   AMG_ARG(D->o.solver == AMG_ASYNC_MULTADD, "amg_grid_add_create_devhub: ASYNC_MULTADD hierarchies only");
   AMG_ARG(world_nranks == hub->world && rank_grid && world_rank >= 0 && world_rank < world_nranks,
           "amg_grid_add_create_devhub: rank layout does not match the hub's %d ranks", hub->world);
   for (int p = 0; p < world_nranks; p++)
      AMG_ARG(rank_grid[p] == hub->rank_grid[p], "amg_grid_add_create_devhub: rank %d's grid differs from the hub's",
              p);
   auto G = std::make_unique<amg_grid_add>();
   G->o = D->o;
   G->link = std::make_unique<HubLink>(hub, world_rank);
   G->hub = hub;
   {
      std::lock_guard<std::mutex> lk(hub->mu);
      hub->device[world_rank] = D->ctx->device;
   }
   G->dev = true;
   auto be = std::make_unique<DistBackend>(D);
   AMG_TRY(be->init(my_grid));
   G->be = std::move(be);
   AMG_TRY(create_common(G.get(), my_grid, world_nranks, world_rank, rank_grid, rank_rows, nullptr));
   AMG_TRY(alloc_dev(G.get(), D));
   *out = G.release();
   return AMG_OK;
}

// the same across processes: slot pools mapped into their receivers by IPC
// handles exchanged over t at creation (every rank of the world calls this
// together); t then carries only control words, acknowledgements and the grid
// sums
extern "C" int amg_grid_add_create_ipc(amg_dist_hier *D, int my_grid, int world_nranks, int world_rank,
                                       const int *rank_grid, const long long *rank_rows, const amg_nb_transport *t,
                                       amg_grid_add **out)
{
   AMG_ARG(D && t && out, "amg_grid_add_create_ipc: null argument");
   AMG_ARG(D->o.solver == AMG_ASYNC_MULTADD, "amg_grid_add_create_ipc: ASYNC_MULTADD hierarchies only");
   AMG_ARG(t->isend && t->irecv && t->test && t->wait && t->grid_allreduce,
           "amg_grid_add_create_ipc: incomplete transport");
   auto G = std::make_unique<amg_grid_add>();
   G->o = D->o;
   G->dev = true;
   auto be = std::make_unique<DistBackend>(D);
   AMG_TRY(be->init(my_grid));
   G->be = std::move(be);
   AMG_TRY(create_common(G.get(), my_grid, world_nranks, world_rank, rank_grid, rank_rows, t));
   AMG_TRY(alloc_dev(G.get(), D));
   AMG_HIP(hipStreamSynchronize(G->be->dstream()));
   auto link = std::make_unique<IpcLink>(*t);
   // exchange the slot pools' handles with every outside peer
   constexpr int HW = 8; // doubles per handle
   static_assert(sizeof(hipIpcMemHandle_t) <= HW * sizeof(double), "IPC handle size");
   const CommClass &sd = G->send, &rd = G->recv;
   std::vector<std::vector<double>> sb(sd.procs.size(), std::vector<double>(HW, 0.0)),
      rb(rd.procs.size(), std::vector<double>(HW, 0.0));
   std::vector<long long> reqs;
   for (size_t i = 0; i < rd.procs.size(); i++) {
      long long q;
      AMG_TRY(xp(t->irecv(t->user, rd.procs[i], IPC_HANDLE_TAG, rb[i].data(), HW, &q), "irecv"));
      reqs.push_back(q);
   }
   for (size_t i = 0; i < sd.procs.size(); i++) {
      hipIpcMemHandle_t h;
      AMG_HIP(hipIpcGetMemHandle(&h, sd.dpool[i]));
      std::memcpy(sb[i].data(), &h, sizeof h);
      long long q;
      AMG_TRY(xp(t->isend(t->user, sd.procs[i], IPC_HANDLE_TAG, sb[i].data(), HW, &q), "isend"));
      reqs.push_back(q);
   }
   for (long long q : reqs) AMG_TRY(xp(t->wait(t->user, q), "wait"));
   for (size_t i = 0; i < rd.procs.size(); i++) {
      hipIpcMemHandle_t h;
      std::memcpy(&h, rb[i].data(), sizeof h);
      void *p = nullptr;
      AMG_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      link->opened.push_back(p);
      link->peers[rd.procs[i]] = IpcLink::Peer{(const double *)p, (long long)std::max(1, rd.len[i])};
   }
   G->link = std::move(link);
   *out = G.release();
   return AMG_OK;
}

extern "C" int amg_grid_add_create_host(int nrows, const double *diag, double weight, const amg_opts *opts,
                                        int my_grid, int world_nranks, int world_rank, const int *rank_grid,
                                        const long long *rank_rows, const amg_nb_transport *t,
                                        amg_grid_add **out)
{
   AMG_ARG(diag && opts && out && nrows >= 0, "amg_grid_add_create_host: bad argument");
   for (int i = 0; i < nrows; i++) AMG_ARG(diag[i] != 0.0, "amg_grid_add_create_host: zero diagonal at %d", i);
   auto G = std::make_unique<amg_grid_add>();
   G->o = *opts;
   auto hb = std::make_unique<HostBackend>(diag, nrows, weight);
   AMG_ARG(rank_grid && rank_rows && world_rank >= 0 && world_rank < world_nranks,
           "amg_grid_add_create_host: bad rank layout");
   int ngrids = 0;
   for (int p = 0; p < world_nranks; p++) ngrids = std::max(ngrids, rank_grid[p] + 1);
   hb->mine.assign(nrows, 0);
   for (int i = 0; i < nrows; i++) hb->mine[i] = (rank_rows[2 * world_rank] + i) % ngrids == my_grid;
   G->be = std::move(hb);
   AMG_TRY(create_common(G.get(), my_grid, world_nranks, world_rank, rank_grid, rank_rows, t));
   *out = G.release();
   return AMG_OK;
}

// DMEM_Add (DMEM_Add.cpp:20-178), asynchronous branch
extern "C" int amg_grid_add_solve(amg_grid_add *G, const double *b_local, double *x_local, int *cycles,
                                  double *relres_local, long long *messages)
{
   AMG_ARG(G && b_local && x_local, "amg_grid_add_solve: null argument");
   G->rr = G->o.async_schedule == AMG_SCHED_ROUND_ROBIN;
   AMG_ARG(!G->rr || (G->hub && G->grid_size == 1),
           "amg_grid_add_solve: the round-robin schedule needs the device hub and one rank per grid");
   AMG_ARG(G->o.async_schedule == AMG_SCHED_FREE || G->rr, "amg_grid_add_solve: async_schedule %d (free or "
                                                          "round robin)", G->o.async_schedule);
   G->all_done_flag = G->outside_done_flag = G->grid_done_flag = G->converge_flag = 0;
   G->r_local_converge_flag = 0;
   G->cycle = 0;
   G->messages_sent = G->messages_recv = 0;
   reset_classes(G);
   // r = b - A x0 and its norm over the grid (the whole problem: every grid
   // holds all rows) -- output.r0_norm2
   AMG_TRY(G->be->begin(b_local, x_local));
   double rr;
   AMG_TRY(G->be->residual(&rr));
   double v[1] = {rr};
   AMG_TRY(tp_sum(G, v, 1));
   G->r0_norm2 = std::sqrt(v[0]);
   if (G->r0_norm2 == 0.0) G->r0_norm2 = 1.0;
   G->r_local = 1.0;
   // AsyncStart: post every outside receive
   for (int i = 0; i < (int)G->recv.procs.size(); i++) AMG_TRY(tp_irecv(G, G->recv, i));
   const long long cap = 1000LL * std::max(1, G->o.num_cycles) + 1000;
   if (G->rr) G->hub->wait_turn(G->me);
   while (true) {
      G->converge_flag = check_converge(G);
      if (G->o.delay_type != AMG_DELAY_NONE && G->o.delay_usec > 0 &&
          (G->o.delay_rank < 0 || G->o.delay_rank == G->me)) {
         // DMEM_DelayProc (DMEM_Misc.cpp:668-684)
         DistBackend *db = dynamic_cast<DistBackend *>(G->be.get());
         if (db) amgk::delay(db->st(), (double)G->o.delay_usec, db->D->ctx->wall_khz);
      }
      AMG_TRY(G->be->cycle());
      AMG_TRY(add_correct(G));
      AMG_TRY(G->be->residual(&rr)); // DMEM_AddResidual_LocalRes
      if (G->all_done_flag == 0) AMG_TRY(add_res_norm(G, rr));
      G->cycle++;
      AMG_TRY(rr_yield(G));
      if (G->converge_flag == 1) break;
      if (G->cycle > cap) return amg_set_error(AMG_ERR_ARG, "amg_grid_add_solve: no termination after %d cycles",
                                               G->cycle);
   }
   AMG_TRY(async_end(G));
   if (G->rr) {
      AMG_HIP(hipStreamSynchronize(G->be->dstream()));
      G->hub->pass_turn(G->me, true);
   }
   AMG_TRY(G->be->residual(&rr));
   v[0] = rr;
   AMG_TRY(tp_sum(G, v, 1));
   AMG_TRY(G->be->get_x(x_local));
   if (cycles) *cycles = G->cycle;
   if (relres_local) *relres_local = std::sqrt(v[0]) / G->r0_norm2;
   if (messages) {
      messages[0] = G->messages_sent;
      messages[1] = G->messages_recv;
   }
   return AMG_OK;
}

extern "C" int amg_grid_add_peers(const amg_grid_add *G, int *nsend, int *nrecv)
{
   AMG_ARG(G, "amg_grid_add_peers: null handle");
   if (nsend) *nsend = (int)G->send.procs.size();
   if (nrecv) *nrecv = (int)G->recv.procs.size();
   return AMG_OK;
}

extern "C" int amg_grid_add_free(amg_grid_add *G)
{
   delete G;
   return AMG_OK;
}
