// amg_link.cpp -- per-level device-resident mailboxes of the asynchronous
// distributed additive solve: the MPI_Test analogue.
//
// Reference: every grid (level) of DMEM_Add runs on its own MPI ranks and polls
// its own messages (MPI_Test in SendRecv / CheckInFlight, DMEM_Comm.cpp:81-348);
// the ghost data of DMEM_AsyncSmooth travels independently of the other
// message classes (DMEM_Smooth.cpp:165-269).  Here every GPU holds a z-slab of
// every level and each level group runs its correction loop on its own host
// thread and HIP stream; its exchanges (ghost planes, the allgather into the
// replicated levels) go through its OWN channels, so one level waiting for a
// neighbour never holds another level back.
//
// A channel (level group k, sender a -> receiver b):
//   * payload: a ring of NS slots in b's device memory (fine-grained, so writes
//     arriving over xGMI are coherent with b's kernels), mapped into a -- the
//     same pointer in one process, peer access across devices, an IPC handle
//     across processes.  a's copy kernel writes the message straight into the
//     slot: no RCCL, no host staging;
//   * two sequence words in b's control block, on their own cache lines:
//     `arrived` (written by a's host once the copy kernel's event has
//     completed: message seq is in slot seq % NS) and `acked` (written by b's
//     host once its unpack kernel, slot -> its vector's ghost rows, has
//     completed: the slot may be reused).  Control blocks are host memory: a
//     malloc'ed block shared by ranks that are threads of one process, a POSIX
//     shared-memory segment between processes of one node.  No device code
//     ever writes host memory or polls.
//   * send(seq): wait (polling) until acked >= seq - NS, launch the copy,
//     record an event; the event is published as `arrived` by progress().
//     recv(seq): poll `arrived` >= seq (publishing this thread's own completed
//     sends and unpacks meanwhile -- the MPI_Test loop), launch the unpack,
//     record an event, published as `acked` by progress().
// Waits are bounded (AMG_LINK_TIMEOUT_S, default 300 s) and an error in one
// rank's level raises an abort word every peer polls, so no thread spins
// forever.  Each level group's channels are touched by exactly one host
// thread, so the links need no locks.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "amg_dist_internal.h"

using namespace amgd;

namespace {

constexpr int NS_DEFAULT = 2;      // slots per channel (link_create's nslots)
constexpr int NS_MAX = 8;
constexpr size_t LINE = 64;        // one sequence word per cache line
constexpr int MAX_EV = 2 * NS_MAX; // event ring per channel direction (at most 2 ns in flight)

struct alignas(64) Word {
   std::atomic<unsigned long long> v;
   char pad[LINE - sizeof(std::atomic<unsigned long long>)];
};
static_assert(sizeof(Word) == LINE, "word layout");

// control block of a rank: words [k][src][{arrived, acked}] of the channels
// src -> rank, then one abort word
size_t ctrl_words(int K, int R) { return (size_t)K * R * 2 + 1; }

__global__ void link_copy_k(const double *__restrict__ src, double *__restrict__ dst, long long n)
{
   const long long stride = (long long)gridDim.x * blockDim.x;
   for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

void launch_copy(hipStream_t s, const double *src, double *dst, long long n)
{
   if (n <= 0) return;
   const long long nb = std::min<long long>(4096, (n + 255) / 256);
   link_copy_k<<<(unsigned)nb, 256, 0, s>>>(src, dst, n);
}

} // namespace

double amgd::link_timeout_s()
{
   static const double t = [] {
      const char *e = std::getenv("AMG_LINK_TIMEOUT_S");
      return e ? std::atof(e) : 300.0;
   }();
   return t;
}

namespace {

struct RankInfo {
   long long pid;
   long long hostid;
   int device;
   int pad;
   unsigned long long ctrl; // control block address (same process)
   unsigned long long slots; // slot region address (same process)
   char ipc[64];            // slot region IPC handle (other processes)
};

} // namespace

struct Chan {
   // receive side (peer -> me)
   double *rslot = nullptr; // my slot ring for this channel
   long long rcap = 0;
   Word *r_arrived = nullptr, *r_acked = nullptr;
   unsigned long long rseq = 0, r_pub = 0;
   hipEvent_t rev[MAX_EV] = {};
   // send side (me -> peer)
   double *sslot = nullptr; // the peer's slot ring for me (mapped)
   long long scap = 0;
   Word *s_arrived = nullptr, *s_acked = nullptr;
   unsigned long long sseq = 0, s_pub = 0;
   hipEvent_t sev[MAX_EV] = {};
};

struct amgd::LinkSet {
   amg_dist_hier *D = nullptr;
   int K = 0, R = 1, me = 0;
   std::vector<Chan> ch;           // [k * R + peer]
   Word *my_ctrl = nullptr;        // my control block
   std::vector<Word *> ctrl;       // every rank's control block as mapped here
   std::vector<std::string> shm_names;
   std::vector<void *> shm_maps;
   std::vector<size_t> shm_bytes;
   bool own_ctrl_malloc = false;
   double *slots = nullptr;        // my receive slot region
   std::vector<double *> ipc_open; // opened peer regions (closed at free)
   bool one_thread = false;        // every level group on one host thread: progress serves them all
   int ns = NS_DEFAULT;            // slots per channel
   Chan &c(int k, int p) { return ch[(size_t)k * R + p]; }
   Word *abort_word(int r) { return ctrl[r] + ctrl_words(K, R) - 1; }
};

namespace {

bool aborted(LinkSet *L, int peer)
{
   if (L->abort_word(L->me)->v.load(std::memory_order_acquire)) return true;
   return peer >= 0 && L->abort_word(peer)->v.load(std::memory_order_acquire);
}

// publish this level group's completed sends (arrived) and unpacks (acked);
// with one host thread for every group, all groups' (a group whose thread has
// moved on to another level must still publish: its peer may be waiting)
int progress_one(LinkSet *L, int k);
int progress(LinkSet *L, int k)
{
   if (!L->one_thread) return progress_one(L, k);
   for (int q = 0; q < L->K; q++) AMG_TRY(progress_one(L, q));
   return AMG_OK;
}

int progress_one(LinkSet *L, int k)
{
   for (int p = 0; p < L->R; p++) {
      Chan &c = L->c(k, p);
      // message seq's event is ev[seq % MAX_EV]: the next to publish is s_pub + 1
      while (c.s_pub < c.sseq) {
         const hipError_t q = hipEventQuery(c.sev[(c.s_pub + 1) % MAX_EV]);
         if (q == hipErrorNotReady) break;
         if (q != hipSuccess) return amg_set_error(AMG_ERR_HIP, "link send event: %s", hipGetErrorString(q));
         c.s_pub++;
         c.s_arrived->v.store(c.s_pub, std::memory_order_release);
      }
      while (c.r_pub < c.rseq) {
         const hipError_t q = hipEventQuery(c.rev[(c.r_pub + 1) % MAX_EV]);
         if (q == hipErrorNotReady) break;
         if (q != hipSuccess) return amg_set_error(AMG_ERR_HIP, "link unpack event: %s", hipGetErrorString(q));
         c.r_pub++;
         c.r_acked->v.store(c.r_pub, std::memory_order_release);
      }
   }
   return AMG_OK;
}

// poll until pred() holds, publishing this group's completions meanwhile
template <class F>
int wait_for(LinkSet *L, int k, int peer, const char *what, F pred)
{
   auto t0 = std::chrono::steady_clock::now();
   for (long long it = 0;; it++) {
      if (pred()) return AMG_OK;
      AMG_TRY(progress(L, k));
      if (pred()) return AMG_OK;
      if (aborted(L, peer)) return amg_set_error(AMG_ERR_RCCL, "link: %s (level %d, rank %d <-> %d): aborted", what,
                                                 k, L->me, peer);
      if ((it & 1023) == 1023) {
         const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
         if (dt > link_timeout_s())
            return amg_set_error(AMG_ERR_RCCL, "link: %s (level %d, rank %d <-> %d) timed out after %.0f s", what, k,
                                 L->me, peer, dt);
      }
      if (it < 64)
         sched_yield();
      else
         std::this_thread::sleep_for(std::chrono::microseconds(it < 4096 ? 2 : 20));
   }
}

// a host allgather of fixed-size records through the hierarchy's transport
int allgather_bytes(amg_dist_hier *D, const void *mine, size_t bytes, std::vector<char> &all)
{
   amg_ctx *c = D->ctx;
   const int R = c->xport->nranks;
   char *d = nullptr;
   AMG_HIP(hipMalloc(&d, bytes * (R + 1)));
   int st = h2d(c->stream, d + bytes * R, mine, bytes);
   if (st == AMG_OK) st = xp_allgather(c, c->stream, d + bytes * R, d, (long long)bytes);
   all.assign(bytes * R, 0);
   if (st == AMG_OK) st = d2h(c->stream, all.data(), d, bytes * R);
   hipFree(d);
   return st;
}

long long host_id()
{
   char h[256] = {0};
   gethostname(h, sizeof(h) - 1);
   unsigned long long x = 1469598103934665603ULL;
   for (char *p = h; *p; p++) x = (x ^ (unsigned char)*p) * 1099511628211ULL;
   return (long long)(x & 0x7fffffffffffffffULL);
}

} // namespace

// caps[k * R + src]: doubles of the largest message src sends me in level
// group k (0: no channel); identical on the sending side by construction
// every rank of the job on this node (collective): the device-resident links
// need it; callers fall back to the transport's send / recv otherwise
int amgd::link_single_node(amg_dist_hier *D, bool *one)
{
   const long long me = host_id();
   std::vector<char> all;
   AMG_TRY(allgather_bytes(D, &me, sizeof(me), all));
   const int R = D->ctx->xport->nranks;
   *one = true;
   for (int r = 0; r < R; r++) {
      long long h = 0;
      std::memcpy(&h, all.data() + (size_t)r * sizeof(h), sizeof(h));
      if (h != me) *one = false;
   }
   return AMG_OK;
}

static int link_create_into(amg_dist_hier *D, int K, const std::vector<long long> &caps, LinkSet *L, int nslots);

// *out is set only on success; a failed creation is torn down (collectively,
// as link_free) and leaves *out null
int amgd::link_create(amg_dist_hier *D, int K, const std::vector<long long> &caps, LinkSet **out, int nslots)
{
   *out = nullptr;
   AMG_ARG(nslots >= 1 && nslots <= NS_MAX, "link_create: %d slots per channel (1 .. %d)", nslots, NS_MAX);
   auto *L = new LinkSet();
   L->D = D;
   const int st = link_create_into(D, K, caps, L, nslots);
   if (st != AMG_OK) {
      const std::string msg = amg_last_error();
      link_free(L);
      return amg_set_error(st, "%s", msg.c_str());
   }
   *out = L;
   return AMG_OK;
}

static int link_create_into(amg_dist_hier *D, int K, const std::vector<long long> &caps, LinkSet *L, int nslots)
{
   amg_ctx *c = D->ctx;
   const int R = c->xport->nranks, me = c->xport->rank;
   const int NS = nslots;
   L->ns = NS;
   L->K = K;
   L->R = R;
   L->me = me;
   L->ch.resize((size_t)K * R);
   // who shares my process (the control block's home and the slots' kind)
   RankInfo mine{};
   mine.pid = (long long)getpid();
   mine.hostid = host_id();
   mine.device = c->device;
   std::vector<char> infos_raw;
   AMG_TRY(allgather_bytes(D, &mine, sizeof(mine), infos_raw));
   std::vector<RankInfo> info(R);
   std::memcpy(info.data(), infos_raw.data(), sizeof(RankInfo) * R);
   bool all_local = true;
   for (int r = 0; r < R; r++) {
      AMG_ARG(info[r].hostid == mine.hostid, "amg_dist_async_solve: rank %d is on another node (device-resident links "
                                             "need one node)", r);
      if (info[r].pid != mine.pid) all_local = false;
   }
   // receive slot region: channels (k, src) in order.  Ranks of one process:
   // fine-grained memory, coherent for writes arriving from a peer device;
   // across processes the region must be IPC-exportable (hipMalloc)
   std::vector<long long> off((size_t)K * R, 0);
   long long tot = 0;
   for (size_t i = 0; i < off.size(); i++) {
      off[i] = tot;
      tot += NS * caps[i];
   }
   const size_t rbytes = (size_t)std::max<long long>(tot, 8) * sizeof(double);
   if (!all_local || hipExtMallocWithFlags((void **)&L->slots, rbytes, hipDeviceMallocFinegrained) != hipSuccess) {
      (void)hipGetLastError();
      AMG_HIP(hipMalloc(&L->slots, rbytes));
   }
   mine.slots = (unsigned long long)(uintptr_t)L->slots;
   if (!all_local) AMG_HIP(hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t *>(mine.ipc), L->slots));
   // the job tag names the shared-memory segments: rank 0's draw
   unsigned long long tag = std::random_device{}() ^ ((unsigned long long)getpid() << 20);
   {
      std::vector<char> all;
      AMG_TRY(allgather_bytes(D, &tag, sizeof(tag), all));
      std::memcpy(&tag, all.data(), sizeof(tag));
   }
   // control block
   const size_t cbytes = ctrl_words(K, R) * sizeof(Word);
   if (all_local) {
      void *p = nullptr;
      if (posix_memalign(&p, 4096, cbytes) != 0) return amg_set_error(AMG_ERR_OOM, "link control block");
      std::memset(p, 0, cbytes);
      L->my_ctrl = static_cast<Word *>(p);
      L->own_ctrl_malloc = true;
   } else {
      char name[96];
      std::snprintf(name, sizeof(name), "/amg_link_%llx_%d", tag, me);
      const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
      AMG_ARG(fd >= 0, "link: shm_open(%s): %s", name, std::strerror(errno));
      if (ftruncate(fd, (off_t)cbytes) != 0) {
         close(fd);
         shm_unlink(name);
         return amg_set_error(AMG_ERR_OOM, "link: ftruncate(%s)", name);
      }
      void *p = mmap(nullptr, cbytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      AMG_ARG(p != MAP_FAILED, "link: mmap(%s)", name);
      L->my_ctrl = static_cast<Word *>(p);
      L->shm_names.push_back(name);
      L->shm_maps.push_back(p);
      L->shm_bytes.push_back(cbytes);
   }
   mine.ctrl = (unsigned long long)(uintptr_t)L->my_ctrl;
   AMG_TRY(allgather_bytes(D, &mine, sizeof(mine), infos_raw));
   std::memcpy(info.data(), infos_raw.data(), sizeof(RankInfo) * R);
   // every rank's control block and (for the peers I send to) slot region
   L->ctrl.assign(R, nullptr);
   std::vector<double *> peer_slots(R, nullptr);
   std::vector<bool> sends_to(R, false);
   for (int k = 0; k < K; k++)
      for (int p = 0; p < R; p++)
         if (p != me && caps[(size_t)k * R + p] > 0) sends_to[p] = true; // symmetric channel sets
   for (int r = 0; r < R; r++) {
      if (r == me) {
         L->ctrl[r] = L->my_ctrl;
         peer_slots[r] = L->slots;
         continue;
      }
      if (info[r].pid == mine.pid) {
         L->ctrl[r] = reinterpret_cast<Word *>((uintptr_t)info[r].ctrl);
      } else {
         char name[96];
         std::snprintf(name, sizeof(name), "/amg_link_%llx_%d", tag, r);
         const int fd = shm_open(name, O_RDWR, 0600);
         AMG_ARG(fd >= 0, "link: shm_open(%s) of rank %d: %s", name, r, std::strerror(errno));
         void *p = mmap(nullptr, cbytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
         close(fd);
         AMG_ARG(p != MAP_FAILED, "link: mmap(%s)", name);
         L->ctrl[r] = static_cast<Word *>(p);
         L->shm_maps.push_back(p);
         L->shm_bytes.push_back(cbytes);
      }
      if (!sends_to[r]) continue;
      if (info[r].pid == mine.pid) {
         peer_slots[r] = reinterpret_cast<double *>((uintptr_t)info[r].slots);
         if (info[r].device != c->device) {
            int can = 0;
            AMG_HIP(hipDeviceCanAccessPeer(&can, c->device, info[r].device));
            AMG_ARG(can, "link: device %d cannot access device %d (rank %d)", c->device, info[r].device, r);
            const hipError_t e = hipDeviceEnablePeerAccess(info[r].device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
               return amg_set_error(AMG_ERR_HIP, "link: hipDeviceEnablePeerAccess(%d): %s", info[r].device,
                                    hipGetErrorString(e));
            (void)hipGetLastError();
         }
      } else {
         hipIpcMemHandle_t h;
         std::memcpy(&h, info[r].ipc, sizeof(h));
         void *p = nullptr;
         AMG_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
         peer_slots[r] = static_cast<double *>(p);
         L->ipc_open.push_back(static_cast<double *>(p));
      }
   }
   // the peers' slot offsets: every rank's caps of its incoming channels
   std::vector<char> caps_raw;
   AMG_TRY(allgather_bytes(D, caps.data(), caps.size() * sizeof(long long), caps_raw));
   const long long *allcaps = reinterpret_cast<const long long *>(caps_raw.data());
   for (int k = 0; k < K; k++)
      for (int p = 0; p < R; p++) {
         if (p == me) continue;
         Chan &ch = L->c(k, p);
         ch.rcap = caps[(size_t)k * R + p];
         ch.rslot = L->slots + off[(size_t)k * R + p];
         ch.r_arrived = L->my_ctrl + ((size_t)k * R + p) * 2;
         ch.r_acked = ch.r_arrived + 1;
         // my channel into p: entry (k, me) of p's table
         const long long *pc = allcaps + (size_t)p * K * R;
         long long o = 0;
         for (size_t i = 0; i < (size_t)k * R + me; i++) o += NS * pc[i];
         ch.scap = pc[(size_t)k * R + me];
         ch.sslot = ch.scap > 0 ? peer_slots[p] + o : nullptr;
         ch.s_arrived = L->ctrl[p] + ((size_t)k * R + me) * 2;
         ch.s_acked = ch.s_arrived + 1;
         for (int q = 0; q < MAX_EV; q++) {
            if (ch.rcap > 0) AMG_HIP(hipEventCreateWithFlags(&ch.rev[q], hipEventDisableTiming));
            if (ch.scap > 0) AMG_HIP(hipEventCreateWithFlags(&ch.sev[q], hipEventDisableTiming));
         }
      }
   // every rank has mapped every segment: the names can go (the mappings stay)
   {
      std::vector<char> all;
      int one = 1;
      AMG_TRY(allgather_bytes(D, &one, sizeof(one), all));
   }
   for (auto &n : L->shm_names) shm_unlink(n.c_str());
   L->shm_names.clear();
   AMG_HIP(hipStreamSynchronize(c->stream));
   return AMG_OK;
}

// reset the sequence numbers before a solve (every rank calls it, then a
// barrier through the transport, so no peer still reads the old words);
// one_thread: every level group is driven by the calling thread
int amgd::link_reset(LinkSet *L, bool one_thread)
{
   L->one_thread = one_thread;
   for (auto &c : L->ch) {
      c.rseq = c.r_pub = c.sseq = c.s_pub = 0;
   }
   const size_t n = ctrl_words(L->K, L->R);
   for (size_t i = 0; i < n; i++) L->my_ctrl[i].v.store(0, std::memory_order_relaxed);
   std::atomic_thread_fence(std::memory_order_seq_cst);
   std::vector<char> all;
   int one = 1;
   return allgather_bytes(L->D, &one, sizeof(one), all);
}

int amgd::link_send(LinkSet *L, int k, int peer, const double *src, long long n, hipStream_t s)
{
   Chan &c = L->c(k, peer);
   const unsigned long long NS = (unsigned long long)L->ns, EV = 2 * NS;
   AMG_ARG(n <= c.scap && c.sslot, "link_send: %lld doubles to rank %d on level %d (capacity %lld)", n, peer, k,
           c.scap);
   const unsigned long long seq = c.sseq + 1;
   // the slot seq % NS is free once the peer acknowledged message seq - NS;
   // the event ring holds at most MAX_EV unpublished sends
   AMG_TRY(wait_for(L, k, peer, "send slot", [&] {
      return (seq <= NS || c.s_acked->v.load(std::memory_order_acquire) >= seq - NS) && c.sseq - c.s_pub < EV;
   }));
   launch_copy(s, src, c.sslot + (long long)(seq % NS) * c.scap, n);
   AMG_HIP(hipGetLastError());
   AMG_HIP(hipEventRecord(c.sev[seq % MAX_EV], s));
   c.sseq = seq;
   return AMG_OK;
}

int amgd::link_recv(LinkSet *L, int k, int peer, double *dst, long long n, hipStream_t s)
{
   Chan &c = L->c(k, peer);
   const unsigned long long NS = (unsigned long long)L->ns, EV = 2 * NS;
   AMG_ARG(n <= c.rcap, "link_recv: %lld doubles from rank %d on level %d (capacity %lld)", n, peer, k, c.rcap);
   const unsigned long long seq = c.rseq + 1;
   AMG_TRY(wait_for(L, k, peer, "receive", [&] {
      return c.r_arrived->v.load(std::memory_order_acquire) >= seq && c.rseq - c.r_pub < EV;
   }));
   launch_copy(s, c.rslot + (long long)(seq % NS) * c.rcap, dst, n);
   AMG_HIP(hipGetLastError());
   AMG_HIP(hipEventRecord(c.rev[seq % MAX_EV], s));
   c.rseq = seq;
   return AMG_OK;
}

int amgd::link_try_recv(LinkSet *L, int k, int peer, double *dst, long long n, hipStream_t s, int *got)
{
   Chan &c = L->c(k, peer);
   const unsigned long long NS = (unsigned long long)L->ns, EV = 2 * NS;
   AMG_ARG(n <= c.rcap, "link_try_recv: %lld doubles from rank %d on level %d (capacity %lld)", n, peer, k, c.rcap);
   *got = 0;
   AMG_TRY(progress(L, k));
   const unsigned long long seq = c.rseq + 1;
   if (c.r_arrived->v.load(std::memory_order_acquire) < seq || c.rseq - c.r_pub >= EV) {
      if (aborted(L, peer)) return amg_set_error(AMG_ERR_RCCL, "link: receive (level %d, rank %d <-> %d): aborted", k,
                                                 L->me, peer);
      return AMG_OK;
   }
   launch_copy(s, c.rslot + (long long)(seq % NS) * c.rcap, dst, n);
   AMG_HIP(hipGetLastError());
   AMG_HIP(hipEventRecord(c.rev[seq % MAX_EV], s));
   c.rseq = seq;
   *got = 1;
   return AMG_OK;
}

int amgd::link_can_send(LinkSet *L, int k, int peer, int *ok)
{
   Chan &c = L->c(k, peer);
   const unsigned long long NS = (unsigned long long)L->ns, EV = 2 * NS;
   AMG_TRY(progress(L, k));
   const unsigned long long seq = c.sseq + 1;
   *ok = (seq <= NS || c.s_acked->v.load(std::memory_order_acquire) >= seq - NS) && c.sseq - c.s_pub < EV;
   if (!*ok && aborted(L, peer))
      return amg_set_error(AMG_ERR_RCCL, "link: send (level %d, rank %d <-> %d): aborted", k, L->me, peer);
   return AMG_OK;
}

int amgd::link_drain(LinkSet *L, int k)
{
   for (int p = 0; p < L->R; p++) {
      Chan &c = L->c(k, p);
      AMG_TRY(wait_for(L, k, p, "drain", [&] { return c.s_pub == c.sseq && c.r_pub == c.rseq; }));
   }
   return AMG_OK;
}

void amgd::link_abort(LinkSet *L)
{
   if (L && L->my_ctrl) L->abort_word(L->me)->v.store(1, std::memory_order_release);
}

// collective: every rank unmaps its peers' slot regions, then (after a
// barrier) frees its own -- no region is freed while another rank maps it
void amgd::link_free(LinkSet *L)
{
   if (!L) return;
   for (auto &c : L->ch)
      for (int q = 0; q < MAX_EV; q++) {
         if (c.rev[q]) hipEventDestroy(c.rev[q]);
         if (c.sev[q]) hipEventDestroy(c.sev[q]);
      }
   for (double *p : L->ipc_open) hipIpcCloseMemHandle(p);
   {
      std::vector<char> all;
      int one = 1;
      (void)allgather_bytes(L->D, &one, sizeof(one), all);
   }
   for (size_t i = 0; i < L->shm_maps.size(); i++) munmap(L->shm_maps[i], L->shm_bytes[i]);
   for (auto &n : L->shm_names) shm_unlink(n.c_str());
   if (L->own_ctrl_malloc) free(L->my_ctrl);
   if (L->slots) hipFree(L->slots);
   delete L;
}

// ghost planes of a slab vector (slab_xchg's exchange) through level group
// k's channels: both sends, then both receives
int amgd::link_xchg_planes(LinkSet *L, int k, hipStream_t s, double *x, long long n_own, long long cP,
                           const std::vector<int> &nlo, const std::vector<int> &nhi)
{
   const int me = L->me, R = L->R;
   if (me > 0 && nhi[me - 1] > 0) AMG_TRY(link_send(L, k, me - 1, x, (long long)nhi[me - 1] * cP, s));
   if (me < R - 1 && nlo[me + 1] > 0)
      AMG_TRY(link_send(L, k, me + 1, x + n_own - (long long)nlo[me + 1] * cP, (long long)nlo[me + 1] * cP, s));
   if (me > 0 && nlo[me] > 0) AMG_TRY(link_recv(L, k, me - 1, x - (long long)nlo[me] * cP, (long long)nlo[me] * cP, s));
   if (me < R - 1 && nhi[me] > 0) AMG_TRY(link_recv(L, k, me + 1, x + n_own, (long long)nhi[me] * cP, s));
   return AMG_OK;
}

// allgather of equal blocks (gath = [rank 0 block | rank 1 block | ...]) through
// level group k's channels
int amgd::link_allgather(LinkSet *L, int k, hipStream_t s, const double *mine, double *gath, long long blk)
{
   const int me = L->me, R = L->R;
   for (int p = 0; p < R; p++)
      if (p != me) AMG_TRY(link_send(L, k, p, mine, blk, s));
   if (blk > 0) AMG_HIP(hipMemcpyAsync(gath + (long long)me * blk, mine, blk * sizeof(double), hipMemcpyDeviceToDevice, s));
   for (int p = 0; p < R; p++)
      if (p != me) AMG_TRY(link_recv(L, k, p, gath + (long long)p * blk, blk, s));
   return AMG_OK;
}
