// amg_api.cpp -- C-ABI: context, matrices, vectors and the per-kernel entry
// points that replace the reference's SEQ_* / SMEM_* kernels.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "amg_internal.h"

#include <csignal>
#include <execinfo.h>
#include <unistd.h>

// AMG_SEGV_TRACE=1: a host SIGSEGV / SIGBUS / SIGABRT prints the native backtrace
// (frames as libamg_mi355x.so(+offset), for addr2line), then hands the signal
// to the handler that was installed before (Python's faulthandler prints the
// threads' Python stacks) -- the diagnostic for teardown faults of multi-rank
// tests.  backtrace() is called once at install so that libgcc is loaded
// before any fault (loading it inside the handler would allocate).
namespace {
struct sigaction g_prev_segv, g_prev_bus, g_prev_abrt;
void amg_fault_trace(int sig, siginfo_t *si, void *uc)
{
   char msg[96];
   const int m = snprintf(msg, sizeof(msg), "[amg] signal %d at address %p, native backtrace:\n", sig, si->si_addr);
   if (m > 0) (void)!write(2, msg, (size_t)m);
   void *buf[64];
   const int n = backtrace(buf, 64);
   backtrace_symbols_fd(buf, n, 2);
   const struct sigaction &prev = sig == SIGSEGV ? g_prev_segv : sig == SIGBUS ? g_prev_bus : g_prev_abrt;
   if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) {
      prev.sa_sigaction(sig, si, uc);
   } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler) {
      prev.sa_handler(sig);
   }
   signal(sig, SIG_DFL);
   raise(sig);
}
__attribute__((constructor)) void amg_fault_trace_init()
{
   const char *e = std::getenv("AMG_SEGV_TRACE");
   if (!e || std::atoi(e) == 0) return;
   void *warm[4];
   (void)backtrace(warm, 4);
   struct sigaction sa;
   std::memset(&sa, 0, sizeof(sa));
   sa.sa_sigaction = amg_fault_trace;
   sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
   sigaction(SIGSEGV, &sa, &g_prev_segv);
   sigaction(SIGBUS, &sa, &g_prev_bus);
   sigaction(SIGABRT, &sa, &g_prev_abrt); // heap-check / assertion aborts
}
} // namespace

static thread_local std::string g_last_error;

int amg_set_error(int code, const char *fmt, ...)
{
   char buf[1024];
   va_list ap;
   va_start(ap, fmt);
   vsnprintf(buf, sizeof(buf), fmt, ap);
   va_end(ap);
   g_last_error = buf;
   return code;
}

extern "C" const char *amg_last_error(void) { return g_last_error.c_str(); }
extern "C" int amg_version(void) { return 1; }

extern "C" void amg_opts_default(amg_opts *o)
{
   std::memset(o, 0, sizeof(*o));
   // SMEM_Main.cpp:65-105
   o->solver = AMG_MULT;
   o->smoother = AMG_JACOBI;
   o->num_pre_smooth_sweeps = 1;
   o->num_post_smooth_sweeps = 1;
   o->num_fine_smooth_sweeps = 1;
   o->num_coarse_smooth_sweeps = 1;
   o->smooth_weight = 1.0;
   o->num_cycles = 20;
   o->tol = 1e-9;
   o->check_resnorm = 1;
   o->cheby_flag = 0;
   o->num_threads = 1;
   o->jgs_block_rows = 64;
   o->reuse_outer_residual = 0;
   o->async_type = AMG_FULL_ASYNC;
   o->profile = 0;
   o->accel_type = AMG_NO_ACCEL; // DMEM_Main.cpp:130
   o->cheby_grid = 0;            // DMEM_Main.cpp:142
   o->delay_type = AMG_DELAY_NONE; // SMEM_Main.cpp:98-101
   o->delay_usec = 0;
   o->delay_frac = 0.0;
   o->fail_iter = 0;
   o->delay_rank = -1; // DMEM_DelayProc: every rank (DMEM_Misc.cpp:670-676)
   o->max_inflight = 1;            // DMEM_Main.cpp:113
   o->async_comm_save_divisor = 1; // DMEM_Main.cpp:123
   o->sps_probability_type = AMG_SPS_EXPONENTIAL; // DMEM_Main.cpp:119-121
   o->sps_alpha = 1.0;
   o->sps_min_prob = 0.0;
   o->delay_level = -1;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
extern "C" int amg_init(amg_ctx **out, int device, int nstreams)
{
   AMG_ARG(out, "amg_init: null out");
   int ndev = 0;
   AMG_HIP(hipGetDeviceCount(&ndev));
   AMG_ARG(device >= 0 && device < ndev, "amg_init: device %d of %d", device, ndev);
   AMG_HIP(hipSetDevice(device));
   amg_ctx *c = new amg_ctx();
   c->device = device;
   AMG_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
   // AMG_COMM_PRIORITY=1: the communication stream at the greatest priority
   // (a hardware queue of its own).  Measured at 512^3, 2 ranks, the box's
   // default 4 queues (profiles/r06/ajac): high priority 0.67-0.92 of each
   // sweep's exchange hidden with 0.10 ms exchange windows, normal priority
   // 0.92 with 0.02-0.03 ms windows -- normal is the default
   {
      int least = 0, greatest = 0;
      const char *v = std::getenv("AMG_COMM_PRIORITY");
      const bool hi = v && std::atoi(v) != 0;
      if (hi && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least) {
         AMG_HIP(hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, greatest));
      } else {
         (void)hipGetLastError();
         AMG_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
      }
   }
   for (int i = 0; i < std::max(0, nstreams); i++) {
      hipStream_t s;
      AMG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      c->level_streams.push_back(s);
   }
   AMG_HIP(hipMalloc(&c->d_scalars, 8192 * sizeof(double)));
   AMG_HIP(hipMemset(c->d_scalars, 0, 8192 * sizeof(double)));
   AMG_HIP(hipMalloc(&c->d_err, 64));
   AMG_HIP(hipMemset(c->d_err, 0, 64));
   AMG_HIP(hipHostMalloc(&c->h_pinned, 1024 * sizeof(double)));
   hipDeviceProp_t prop;
   if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
   if (hipDeviceGetAttribute(&c->wall_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || c->wall_khz <= 0)
      c->wall_khz = 100000; // gfx9 s_memrealtime: 100 MHz
   if (const char *v = std::getenv("AMG_VALUE_INDEX")) c->value_index = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_DICT_INDEX")) c->dict_index = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_ROW_PATTERN")) c->row_pattern = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_PAIR_PATTERN")) c->pair_pattern = std::min(2, std::max(0, std::atoi(v)));
   if (const char *v = std::getenv("AMG_MASTER_PATTERN")) c->master_pattern = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_PAIR_ANCHOR16")) c->pair_anchor16 = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_PLANE_MARCH")) {
      c->plane_march = std::atoi(v) > 0;
      if (std::atoi(v) > 1) c->mz_zc = std::min(std::atoi(v), 64), c->mz_zc_auto = 0;
   }
   if (const char *v = std::getenv("AMG_PLANE_MARCH_XCD")) c->mz_xcd = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_FUSE_TRANSFER")) c->fuse_transfer = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_FUSE_XFER")) c->fuse_xfer = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_GRAPHS")) c->graphs = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_LONG_FORM")) c->long_form = std::max(0, std::min(2, std::atoi(v)));
   if (const char *v = std::getenv("AMG_LONG_XCD")) c->long_xcd = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_OUTER_SLAB")) c->outer_slab = std::max(1, std::atoi(v));
   if (const char *v = std::getenv("AMG_FUSE_OUTER")) c->fuse_outer = std::max(0, std::min(3, std::atoi(v)));
   if (const char *v = std::getenv("AMG_FUSE_XFP_SLAB")) c->fuse_xfp_slab = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_FUSE_PROLONG")) c->fuse_prolong = std::max(0, std::min(7, std::atoi(v)));
   if (const char *v = std::getenv("AMG_JGS_SMALL")) c->jgs_small = std::max(0, std::min(2, std::atoi(v)));
   if (const char *v = std::getenv("AMG_JGS_WAVE")) c->jgs_wave = std::max(0, std::min(3, std::atoi(v)));
   if (const char *v = std::getenv("AMG_JGS_FOLD")) c->jgs_fold = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_BSR3")) c->bsr3 = std::max(0, std::min(std::atoi(v), 2));
   if (const char *v = std::getenv("AMG_BSR3_XS")) c->bsr3_xs = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_MZ_EDGE")) c->mz_edge = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_MZ27_OCC")) c->mz27_occ = std::max(-1, std::min(8, std::atoi(v)));
   if (const char *v = std::getenv("AMG_MZ_OCC")) c->mz_occ = std::max(-1, std::min(8, std::atoi(v)));
   if (const char *v = std::getenv("AMG_MZ_PF")) c->mz_pf = std::atoi(v) == 2 ? 2 : (std::atoi(v) == 1 ? 1 : 3);
   if (const char *v = std::getenv("AMG_MZ27_PF")) c->mz27_pf = std::atoi(v) == 1 ? 1 : (std::atoi(v) == 3 ? 3 : 2);
   if (const char *v = std::getenv("AMG_RR_LINES")) c->rr_lines = std::atoi(v) == 2 ? 2 : 1;
   if (const char *v = std::getenv("AMG_RR_OCC")) c->rr_occ = std::atoi(v);
   if (const char *v = std::getenv("AMG_RR_FPF")) c->rr_fpf = std::atoi(v);
   if (const char *v = std::getenv("AMG_RR_ZC")) c->rr_zc = std::max(0, std::min(std::atoi(v), 32));
   if (const char *v = std::getenv("AMG_RR_RING")) c->rr_ring = std::atoi(v) != 0;
   if (const char *v = std::getenv("AMG_MZ_NT")) c->mz_nt = std::atoi(v) & 3;
   if (const char *v = std::getenv("AMG_MZ_LINES")) c->mz_lines = std::atoi(v) == 4 ? 4 : std::atoi(v) == 2 ? 2 : 1;
   if (const char *v = std::getenv("AMG_MZ_LINES_GEMV"))
      c->mz_lines_gemv = std::atoi(v) == 4 ? 4 : std::atoi(v) == 2 ? 2 : 1;
   *out = c;
   return AMG_OK;
}

// one process-wide lock around teardown (contexts, hierarchies, matrices):
// ranks that are threads of one process free concurrently, and the runtime's
// free / destroy paths are kept out of each other's way
std::recursive_mutex &amg_teardown_mutex()
{
   static std::recursive_mutex m;
   return m;
}

extern "C" int amg_finalize(amg_ctx *c)
{
   if (!c) return AMG_OK;
   std::lock_guard<std::recursive_mutex> td(amg_teardown_mutex());
   hipSetDevice(c->device);
   hipStreamSynchronize(c->stream);
   if (c->comm_stream) hipStreamSynchronize(c->comm_stream);
   for (auto s : c->level_streams) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
   }
   if (c->comm_stream) hipStreamDestroy(c->comm_stream);
   hipStreamDestroy(c->stream);
   hipFree(c->d_partials);
   hipFree(c->d_scalars);
   hipFree(c->d_err);
   hipHostFree(c->h_pinned);
   delete c;
   return AMG_OK;
}

// device-side range-check flags since the last call (bit 0: a zero-guess fold
// write outside the coarse level's rows, dropped), cleared on read
extern "C" int amg_device_errors(amg_ctx *c, int *flags)
{
   AMG_ARG(c && flags, "amg_device_errors: null argument");
   int h[16];
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_HIP(hipMemcpy(h, c->d_err, sizeof(h), hipMemcpyDeviceToHost));
   AMG_HIP(hipMemset(c->d_err, 0, sizeof(h)));
   *flags = h[0];
   return AMG_OK;
}

extern "C" int amg_sync(amg_ctx *c)
{
   AMG_ARG(c, "amg_sync: null ctx");
   AMG_HIP(hipStreamSynchronize(c->stream));
   return AMG_OK;
}

int amg_ctx_partials(amg_ctx *c, size_t n, double **out)
{
   if (n > c->partials_cap) {
      // grow only at points where the stream may be synchronised
      AMG_HIP(hipStreamSynchronize(c->stream));
      hipFree(c->d_partials);
      c->d_partials = nullptr;
      size_t cap = std::max<size_t>(n, 1 << 16);
      AMG_HIP(hipMalloc(&c->d_partials, cap * sizeof(double)));
      c->partials_cap = cap;
   }
   *out = c->d_partials;
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// matrices
// ---------------------------------------------------------------------------
static int mat_alloc(amg_ctx *c, int nrows, int ncols, long long nnz, amg_mat **out)
{
   amg_mat *A = new amg_mat();
   A->ctx = c;
   A->nrows = nrows;
   A->ncols = ncols;
   A->nnz = nnz;
   size_t np = (size_t)nnz + AMG_NNZ_PAD;
   hipError_t e = hipMalloc(&A->rowptr, ((size_t)nrows + 1) * sizeof(int));
   if (e == hipSuccess) e = hipMalloc(&A->col, np * sizeof(int));
   if (e == hipSuccess) e = hipMalloc(&A->val, np * sizeof(double));
   if (e == hipSuccess) e = hipMalloc(&A->diag, std::max(1, nrows) * sizeof(double));
   if (e != hipSuccess) {
      hipFree(A->rowptr); hipFree(A->col); hipFree(A->val); hipFree(A->diag);
      delete A;
      return amg_set_error(AMG_ERR_OOM, "amg_csr_register: device allocation of %lld nnz failed: %s",
                           nnz, hipGetErrorString(e));
   }
   // padding: col 0 (a valid x index), val 0
   AMG_HIP(hipMemsetAsync(A->col + nnz, 0, AMG_NNZ_PAD * sizeof(int), c->stream));
   AMG_HIP(hipMemsetAsync(A->val + nnz, 0, AMG_NNZ_PAD * sizeof(double), c->stream));
   *out = A;
   return AMG_OK;
}

// value-indexed CSR (CSR-VI): when the matrix holds at most 256 distinct
// values (by bit pattern) the hot kernels stream one byte per entry instead
// of eight and read the value from an LDS table -- bit-identical products.
// val stays resident for the other kernels and for amg_mat_download.
static int build_value_index(amg_mat *A)
{
   amg_ctx *c = A->ctx;
   hipStream_t s = c->stream;
   constexpr int NS = 4096;
   unsigned long long *slots = nullptr;
   AMG_HIP(hipMalloc(&slots, NS * sizeof(unsigned long long) + 64));
   int *count = reinterpret_cast<int *>(slots + NS);
   AMG_HIP(hipMemsetAsync(slots, 0xff, NS * sizeof(unsigned long long), s));
   AMG_HIP(hipMemsetAsync(count, 0, sizeof(int), s));
   amgk::vi_collect(s, A->val, A->nnz, slots, NS, count);
   std::vector<unsigned long long> h(NS);
   int cnt = 0;
   AMG_HIP(hipMemcpyAsync(h.data(), slots, NS * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(&cnt, count, sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   if (cnt < 1 || cnt > 256) {
      hipFree(slots);
      return AMG_OK; // plain CSR
   }
   std::vector<unsigned long long> keys;
   for (auto k : h)
      if (k != ~0ULL) keys.push_back(k);
   std::sort(keys.begin(), keys.end());
   const int T = (int)keys.size();
   std::vector<double> tab(256, 0.0);
   std::memcpy(tab.data(), keys.data(), T * sizeof(double));
   hipError_t e = hipMalloc(&A->vidx, (size_t)A->nnz + 64);
   if (e == hipSuccess) e = hipMalloc(&A->vtab, 256 * sizeof(double));
   if (e != hipSuccess) { // not enough room: keep plain CSR
      hipFree(A->vidx);
      hipFree(A->vtab);
      A->vidx = nullptr;
      A->vtab = nullptr;
      hipFree(slots);
      (void)hipGetLastError();
      return AMG_OK;
   }
   AMG_HIP(hipMemcpyAsync(slots, keys.data(), T * sizeof(unsigned long long), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->vtab, tab.data(), 256 * sizeof(double), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemsetAsync(A->vidx + A->nnz, 0, 64, s));
   amgk::vi_encode(s, A->val, A->nnz, slots, T, A->vidx);
   AMG_HIP(hipStreamSynchronize(s));
   hipFree(slots);
   A->vi_n = T;
   return AMG_OK;
}

// dictionary-coded CSR (CSR-DC) on top of the value index: when every entry's
// (col - row, value) pair comes from at most 256 distinct pairs and no row
// holds more than AMG_DC_MAXROW entries, each entry becomes one byte and the
// lane-per-row kernel reads x[row + off] coalesced across a wave.
static int build_dict_index(amg_mat *A)
{
   amg_ctx *c = A->ctx;
   hipStream_t s = c->stream;
   constexpr int NS = 4096;
   unsigned long long *slots = nullptr;
   AMG_HIP(hipMalloc(&slots, NS * sizeof(unsigned long long) + 64));
   int *count = reinterpret_cast<int *>(slots + NS);
   AMG_HIP(hipMemsetAsync(slots, 0xff, NS * sizeof(unsigned long long), s));
   AMG_HIP(hipMemsetAsync(count, 0, 3 * sizeof(int), s));
   amgk::dc_collect(s, A, slots, NS, count, count + 1);
   std::vector<unsigned long long> h(NS);
   int cm[3] = {0, 0, 0}; // distinct pairs, longest row, some anchor != row
   AMG_HIP(hipMemcpyAsync(h.data(), slots, NS * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(cm, count, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   if (cm[0] < 1 || cm[0] > 256 || cm[1] > AMG_DC_MAXROW) {
      hipFree(slots);
      return AMG_OK;
   }
   std::vector<unsigned long long> keys;
   for (auto k : h)
      if (k != ~0ULL) keys.push_back(k);
   std::sort(keys.begin(), keys.end());
   const int T = (int)keys.size();
   std::vector<double> vt(256, 0.0);
   AMG_HIP(hipMemcpy(vt.data(), A->vtab, 256 * sizeof(double), hipMemcpyDeviceToHost));
   std::vector<int> off(256, 0);
   std::vector<double> dv(256, 0.0);
   for (int t = 0; t < T; t++) {
      off[t] = (int)(unsigned int)(keys[t] >> 8);
      dv[t] = vt[keys[t] & 0xff];
   }
   // anchors only where some row does not start at its own index (the
   // transfers); a distributed slab [owned | ghost] keeps anchor = row
   const bool need_anchor = cm[2] != 0;
   hipError_t e = hipMalloc(&A->didx, (size_t)A->nnz + 64);
   if (e == hipSuccess) e = hipMalloc(&A->doff, 256 * sizeof(int));
   if (e == hipSuccess) e = hipMalloc(&A->dval, 256 * sizeof(double));
   if (e == hipSuccess && need_anchor) e = hipMalloc(&A->danch, std::max(1, A->nrows) * sizeof(int));
   if (e != hipSuccess) {
      hipFree(A->didx);
      hipFree(A->doff);
      hipFree(A->dval);
      hipFree(A->danch);
      A->didx = nullptr;
      A->doff = nullptr;
      A->dval = nullptr;
      A->danch = nullptr;
      hipFree(slots);
      (void)hipGetLastError();
      return AMG_OK;
   }
   AMG_HIP(hipMemcpyAsync(slots, keys.data(), T * sizeof(unsigned long long), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->doff, off.data(), 256 * sizeof(int), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->dval, dv.data(), 256 * sizeof(double), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemsetAsync(A->didx + A->nnz, 0, 64, s));
   amgk::dc_encode(s, A, slots, T, A->didx, A->danch);
   AMG_HIP(hipStreamSynchronize(s));
   hipFree(slots);
   A->dc_n = T;
   A->dc_maxrow = cm[1];
   return AMG_OK;
}

// row-pattern-coded CSR: when every row is non-empty and the rows' dictionary
// sequences take at most 256 distinct values, one byte per row names the
// sequence.  Lossless: the kernels walk the same entries in
// the same order.
static int build_row_pattern(amg_mat *A)
{
   amg_ctx *c = A->ctx;
   hipStream_t s = c->stream;
   constexpr int NS = 4096;
   unsigned long long *slots = nullptr;
   AMG_HIP(hipMalloc(&slots, NS * sizeof(unsigned long long) + NS * sizeof(int) + 64));
   int *rep = reinterpret_cast<int *>(slots + NS);
   int *count = rep + NS;
   AMG_HIP(hipMemsetAsync(slots, 0xff, NS * sizeof(unsigned long long), s));
   AMG_HIP(hipMemsetAsync(count, 0, 2 * sizeof(int), s));
   amgk::rp_collect(s, A, slots, rep, NS, count, count + 1);
   std::vector<unsigned long long> h(NS);
   std::vector<int> hr(NS);
   int cb[2] = {0, 0}; // distinct row sequences, rows that cannot be coded
   AMG_HIP(hipMemcpyAsync(h.data(), slots, NS * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(hr.data(), rep, NS * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(cb, count, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   if (cb[0] < 1 || cb[0] > 256 || cb[1] != 0) {
      hipFree(slots);
      return AMG_OK;
   }
   std::vector<std::pair<unsigned long long, int>> kr;
   for (int i = 0; i < NS; i++)
      if (h[i] != ~0ULL) kr.push_back({h[i], hr[i]});
   std::sort(kr.begin(), kr.end());
   const int T = (int)kr.size();
   std::vector<unsigned long long> keys(T);
   std::vector<int> reps(T);
   for (int t = 0; t < T; t++) {
      keys[t] = kr[t].first;
      reps[t] = kr[t].second;
   }
   hipError_t e = hipMalloc(&A->rpat, std::max(1, A->nrows));
   if (e == hipSuccess) e = hipMalloc(&A->ptab, 256 * AMG_RP_STRIDE);
   if (e != hipSuccess) {
      hipFree(A->rpat);
      hipFree(A->ptab);
      A->rpat = A->ptab = nullptr;
      hipFree(slots);
      (void)hipGetLastError();
      return AMG_OK;
   }
   AMG_HIP(hipMemsetAsync(A->ptab, 0, 256 * AMG_RP_STRIDE, s));
   AMG_HIP(hipMemcpyAsync(slots, keys.data(), T * sizeof(unsigned long long), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(rep, reps.data(), T * sizeof(int), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemsetAsync(count + 1, 0, sizeof(int), s));
   amgk::rp_table(s, A, rep, T, A->ptab);
   amgk::rp_encode(s, A, slots, T, A->ptab, A->rpat, count + 1);
   AMG_HIP(hipMemcpyAsync(cb, count, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   hipFree(slots);
   if (cb[1] != 0) { // a hash collision: keep the dictionary-coded form
      hipFree(A->rpat);
      hipFree(A->ptab);
      A->rpat = A->ptab = nullptr;
      return AMG_OK;
   }
   A->rp_n = T;
   return AMG_OK;
}

// paired-row-pattern CSR on top of the row patterns: rows 2t and 2t+1 share
// one merged entry list in which an entry of row 2t at column c and an entry
// of row 2t+1 at column c + 1 are one 16-byte x load.
// Columns are relative to row 2t's anchor (the row itself for square
// diagonal-first operators); row 2t+1's anchor is da further.  The merge is a
// shortest common supersequence of the two rows' entry lists (matched on
// column), so each row still sums its own entries in its CSR order:
// bit-identical to the single-row kernel.
static void pair_merge(const unsigned char *a, int la, const unsigned char *b, int lb, int da,
                       const std::vector<int> &off, std::vector<unsigned int> &out)
{
   int dp[AMG_PP_MAXROW + 2][AMG_PP_MAXROW + 2] = {};
   auto match = [&](int i, int j) { return off[b[j]] + da == off[a[i]] + 1; };
   for (int i = la - 1; i >= 0; i--)
      for (int j = lb - 1; j >= 0; j--)
         dp[i][j] = match(i, j) ? dp[i + 1][j + 1] + 1 : std::max(dp[i + 1][j], dp[i][j + 1]);
   int i = 0, j = 0;
   while (i < la || j < lb) {
      if (i < la && j < lb && match(i, j) && dp[i][j] == dp[i + 1][j + 1] + 1) {
         out.push_back(a[i] | (unsigned)b[j] << 8 | 3u << 16);
         i++;
         j++;
      } else if (j >= lb || (i < la && dp[i + 1][j] >= dp[i][j + 1])) {
         out.push_back(a[i] | 1u << 16);
         i++;
      } else {
         out.push_back((unsigned)b[j] << 8 | 2u << 16);
         j++;
      }
   }
}

// Slab-compressed anchors for the paired kernel (amg_internal.h): anchor(2t)
// = pbase[2t >> 9] + pdelta[t].  Kept only when every 512-row slab's anchors
// span at most 65535 (interpolation: a fine line maps to half a coarse line).
static int compress_pair_anchors(amg_mat *A)
{
   hipStream_t s = A->ctx->stream;
   const size_t ns = ((size_t)A->nrows + 511) / 512, np = ((size_t)A->nrows + 1) / 2;
   int *ok = nullptr;
   hipError_t e = hipMalloc(&A->pbase, ns * sizeof(int));
   if (e == hipSuccess) e = hipMalloc(&A->pdelta, np * sizeof(unsigned short));
   if (e == hipSuccess) e = hipMalloc(&ok, sizeof(int));
   int okh = 0;
   if (e == hipSuccess) {
      const int one = 1;
      AMG_HIP(hipMemcpyAsync(ok, &one, sizeof(int), hipMemcpyHostToDevice, s));
      amgk::pp_anchor_compress(s, A, A->pbase, A->pdelta, ok);
      AMG_HIP(hipMemcpyAsync(&okh, ok, sizeof(int), hipMemcpyDeviceToHost, s));
      AMG_HIP(hipStreamSynchronize(s));
   }
   hipFree(ok);
   if (e != hipSuccess || !okh) {
      hipFree(A->pbase);
      hipFree(A->pdelta);
      A->pbase = nullptr;
      A->pdelta = nullptr;
      (void)hipGetLastError();
   }
   return AMG_OK;
}

static int build_pair_pattern(amg_mat *A)
{
   amg_ctx *c = A->ctx;
   hipStream_t s = c->stream;
   constexpr int NK = AMG_PP_NK;
   unsigned char *flags = nullptr;
   AMG_HIP(hipMalloc(&flags, 2 * (size_t)NK + 1 + 256 * sizeof(unsigned long long) + 8));
   unsigned char *map = flags + NK + 1;
   unsigned long long *counts = reinterpret_cast<unsigned long long *>(
      (reinterpret_cast<uintptr_t>(map + NK) + 7) & ~(uintptr_t)7);
   AMG_HIP(hipMemsetAsync(flags, 0, NK + 1, s));
   amgk::pp_collect(s, A, flags);
   std::vector<unsigned char> hf(NK + 1), pt(256 * AMG_RP_STRIDE);
   std::vector<int> off(256);
   AMG_HIP(hipMemcpyAsync(hf.data(), flags, NK + 1, hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(pt.data(), A->ptab, pt.size(), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(off.data(), A->doff, 256 * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   std::vector<unsigned char> hm(NK, 0);
   std::vector<unsigned int> tab;
   const int PS = amg_pp_stride(A->dc_maxrow);
   int T = hf[NK] ? 257 : 0; // an anchor delta out of range: not pair-coded
   bool centre0 = !A->danch; // square diagonal-first: is entry 0 the diagonal of both rows?
   std::vector<int> msz(256, 0), ssz(256, 0); // per pattern: merged entries, the longer row's
   for (int k = 0; k < NK && T <= 256; k++) {
      if (!hf[k]) continue;
      if (T == 256) {
         T++;
         break;
      }
      const int pk = k / AMG_PP_NDA, da = k % AMG_PP_NDA - AMG_PP_DA0;
      const int p0 = pk / 257, p1 = pk % 257;
      const unsigned char *a = pt.data() + p0 * AMG_RP_STRIDE;
      std::vector<unsigned int> el;
      if (p1 < 256) {
         const unsigned char *b = pt.data() + p1 * AMG_RP_STRIDE;
         pair_merge(a + 1, a[0], b + 1, b[0], A->danch ? da : 1, off, el);
         msz[T] = (int)el.size();
         ssz[T] = std::max<int>(a[0], b[0]);
      } else {
         for (int j = 0; j < a[0]; j++) el.push_back(a[1 + j] | 1u << 16);
      }
      // header: nel | first dictionary entry of row 2t << 8 | of row 2t+1 << 16
      // | row 2t+1 present << 24 | (anchor delta + 16) << 25
      std::vector<unsigned int> w(PS, 0);
      w[0] = (unsigned)el.size() | (unsigned)a[1] << 8 |
             (p1 < 256 ? (unsigned)pt[p1 * AMG_RP_STRIDE + 1] << 16 | 1u << 24 : 0u) |
             (unsigned)(da + 16) << 25;
      for (size_t e = 0; e < el.size(); e++) w[1 + e] = el[e];
      centre0 = centre0 && !el.empty() && off[el[0] & 0xff] == 0 && (el[0] >> 16 & 1) &&
                (p1 == 256 || (el[0] >> 16 & 3) == 3);
      tab.insert(tab.end(), w.begin(), w.end());
      hm[k] = (unsigned char)T++;
   }
   if (T < 1 || T > 256 || (size_t)T * PS * 4 > (size_t)AMG_PP_LDS) {
      hipFree(flags);
      return AMG_OK;
   }
   const size_t np = ((size_t)A->nrows + 1) / 2;
   hipError_t e = hipMalloc(&A->ppat, std::max<size_t>(1, np));
   if (e == hipSuccess) e = hipMalloc(&A->pptab, tab.size() * sizeof(unsigned int));
   if (e != hipSuccess) {
      hipFree(A->ppat);
      hipFree(A->pptab);
      A->ppat = nullptr;
      A->pptab = nullptr;
      hipFree(flags);
      (void)hipGetLastError();
      return AMG_OK;
   }
   AMG_HIP(hipMemcpyAsync(map, hm.data(), NK, hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->pptab, tab.data(), tab.size() * sizeof(unsigned int), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemsetAsync(counts, 0, 256 * sizeof(unsigned long long), s));
   amgk::pp_encode(s, A, map, A->ppat, counts);
   std::vector<unsigned long long> cnt(256);
   AMG_HIP(hipMemcpyAsync(cnt.data(), counts, 256 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   hipFree(flags);
   // a pair lane walks the merged list: worth it only when it is hardly
   // longer than the longer of its rows, counted over all row pairs (7-pt /
   // 27-pt operators and interpolation: as long; restriction, anchors 2
   // apart: 4/3 as long, and slower than one row per lane)
   double merged = 0.0, single = 0.0;
   for (int t = 0; t < T; t++) {
      merged += (double)cnt[t] * msz[t];
      single += (double)cnt[t] * ssz[t];
   }
   if (merged > AMG_PP_MAXFILL * single) {
      hipFree(A->ppat);
      hipFree(A->pptab);
      A->ppat = nullptr;
      A->pptab = nullptr;
      return AMG_OK;
   }
   A->pp_n = T;
   A->pp_stride = PS;
   A->pp_centre0 = centre0 ? 1 : 0;
   if (A->ctx->pair_anchor16 && A->danch && A->nrows > 0) AMG_TRY(compress_pair_anchors(A));
   return AMG_OK;
}

// Master-pattern form on top of the pair patterns of a square,
// diagonal-first operator: every row's column offsets (relative to the row)
// must follow the master order -- 0 first, then ascending -- so a row's
// entries are an ordered subsequence of the master list and walking the
// master with per-row use bits adds exactly the row's products in its CSR
// order (bit-identical).  Offsets then become wave-uniform scalars and the
// per-entry LDS lookups of the pair kernel disappear.
static int build_master_pattern(amg_mat *A)
{
   if (!A->ppat || A->danch || A->nrows != A->ncols || A->nrows < 2 || A->pp_n < 1) return AMG_OK;
   hipStream_t s = A->ctx->stream;
   const int T = A->pp_n, PS = A->pp_stride, D = A->dc_n;
   std::vector<unsigned int> tab((size_t)T * PS);
   std::vector<int> off(256);
   std::vector<double> val(256);
   AMG_HIP(hipMemcpyAsync(tab.data(), A->pptab, tab.size() * 4, hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(off.data(), A->doff, 256 * sizeof(int), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipMemcpyAsync(val.data(), A->dval, 256 * sizeof(double), hipMemcpyDeviceToHost, s));
   AMG_HIP(hipStreamSynchronize(s));
   std::vector<int> mo;
   for (int d = 0; d < D; d++) mo.push_back(off[d]);
   std::sort(mo.begin(), mo.end());
   mo.erase(std::unique(mo.begin(), mo.end()), mo.end());
   auto z = std::find(mo.begin(), mo.end(), 0);
   if (z == mo.end() || (int)mo.size() > AMG_MP_MAXJ) return AMG_OK;
   mo.erase(z);
   mo.insert(mo.begin(), 0);
   const int J = (int)mo.size();
   auto pos = [&](int o) { return (int)(std::find(mo.begin(), mo.end(), o) - mo.begin()); };
   std::vector<unsigned long long> mask(T, 0);
   std::vector<double> mv((size_t)T * J * 2, 0.0);
   std::vector<unsigned long long> uni_bits(J, 0);
   std::vector<int> uni_set(J, 0);
   bool uni = true;
   for (int t = 0; t < T; t++) {
      const unsigned int *w = tab.data() + (size_t)t * PS;
      const int nel = w[0] & 0xff;
      const bool two = (w[0] >> 24) & 1;
      int last[2] = {-1, -1};
      for (int e = 0; e < nel; e++) {
         const unsigned int en = w[1 + e];
         for (int r = 0; r < 2; r++) {
            if (!(en >> (16 + r) & 1)) continue;
            const int d = r ? (en >> 8 & 0xff) : (en & 0xff);
            const int j = pos(off[d]);
            if (j <= last[r]) return AMG_OK; // not an ordered subsequence of the master
            last[r] = j;
            mask[t] |= 1ULL << (2 * j + r);
            mv[((size_t)t * J + j) * 2 + r] = val[d];
            unsigned long long bits;
            std::memcpy(&bits, &val[d], 8);
            if (!uni_set[j]) {
               uni_set[j] = 1;
               uni_bits[j] = bits;
            } else if (uni_bits[j] != bits) {
               uni = false;
            }
         }
      }
      // a_ii = A_data[A_i[i]] and x_i come from master entry 0 (the diagonal)
      if (!(mask[t] & 1ULL) || (two && !(mask[t] & 2ULL))) return AMG_OK;
   }
   if (!uni && (size_t)T * J * 16 > (size_t)AMG_MP_LDS) return AMG_OK;
   hipError_t e = hipMalloc(&A->mpmask, (size_t)T * 8);
   if (e == hipSuccess && !uni) e = hipMalloc(&A->mpval, mv.size() * 8);
   if (e != hipSuccess) {
      hipFree(A->mpmask);
      hipFree(A->mpval);
      A->mpmask = nullptr;
      A->mpval = nullptr;
      (void)hipGetLastError();
      return AMG_OK;
   }
   AMG_HIP(hipMemcpyAsync(A->mpmask, mask.data(), (size_t)T * 8, hipMemcpyHostToDevice, s));
   if (!uni) AMG_HIP(hipMemcpyAsync(A->mpval, mv.data(), mv.size() * 8, hipMemcpyHostToDevice, s));
   AMG_HIP(hipStreamSynchronize(s));
   for (int j = 0; j < J; j++) {
      A->mp_off[j] = mo[j];
      std::memcpy(&A->mp_val[j], &uni_bits[j], 8);
   }
   A->mp_uni = uni ? 1 : 0;
   A->mp_J = J;
   // plane-marching form: master [0, -P, -S, -1, +1, +S, +P], whole planes of
   // P rows (P % 512 == 0: a workgroup's 512 positions never straddle planes)
   // (S even: every pair's +-S operand pair is one aligned-in-range 16-byte load)
   if (A->ctx->plane_march && J == 7 && mo[3] == -1 && mo[4] == 1 && mo[1] == -mo[6] &&
       mo[2] == -mo[5] && mo[5] > 1 && mo[5] % 2 == 0 && mo[6] > mo[5] && mo[6] % 512 == 0 &&
       A->nrows % mo[6] == 0 && A->nrows / mo[6] >= 2 && A->nrows < (1 << 29)) { // 32-bit byte offsets
      A->mz_P = mo[6];
      A->mz_S = mo[5];
   }
   // 27-pt plane march: master [0, dz P + dy S + dx ascending (centre skipped)]
   if (A->ctx->plane_march && J == 27 && A->nrows < (1 << 29) && (uni || T <= 64)) {
      const int S = mo[16], P = mo[22];
      bool ok = S >= 4 && S % 2 == 0 && P % 512 == 0 && P % S == 0 && P / S >= 3 && A->nrows % P == 0 &&
                A->nrows / P >= 2;
      for (int L = 0, j = 1; ok && L < 27; L++) {
         if (L == 13) continue;
         const int o = (L / 9 - 1) * P + ((L / 3) % 3 - 1) * S + (L % 3 - 1);
         ok = mo[j++] == o;
      }
      int dom = -1;
      if (ok && !uni) {
         // the most frequent pattern using all 27 entries in both rows with
         // bit-equal values in the two rows
         std::vector<unsigned char> pp((size_t)(A->nrows / 2));
         AMG_HIP(hipMemcpy(pp.data(), A->ppat, pp.size(), hipMemcpyDeviceToHost));
         std::vector<long long> cnt(T, 0);
         for (unsigned char q : pp) cnt[q]++;
         const unsigned long long full = (1ull << 54) - 1;
         for (int t = 0; t < T; t++) {
            if (mask[t] != full) continue;
            bool same = true;
            for (int j = 0; j < J && same; j++)
               same = std::memcmp(&mv[((size_t)t * J + j) * 2], &mv[((size_t)t * J + j) * 2 + 1], 8) == 0;
            if (same && (dom < 0 || cnt[t] > cnt[dom])) dom = t;
         }
         if (dom >= 0)
            for (int j = 0; j < J; j++) A->mz_domval[j] = mv[((size_t)dom * J + j) * 2];
         // x-edge pair patterns (the waves at both ends of every line)
         if (dom >= 0) {
            unsigned long long lo_x = 0, hi_y = 0; // row 2t's mask without dx = -1, row 2t+1's without +1
            for (int j = 0; j < 27; j++) {
               const int L = j == 0 ? 13 : (j <= 13 ? j - 1 : j), dx = L % 3 - 1;
               if (dx != -1) lo_x |= 1ull << (2 * j);
               if (dx != 1) hi_y |= 2ull << (2 * j);
            }
            const unsigned long long even = 0x5555555555555555ull & full, odd = 0xAAAAAAAAAAAAAAAAull & full;
            long long best_lo = 0, best_hi = 0;
            for (int t = 0; t < T; t++) {
               auto same = [&](int j, int r) {
                  return std::memcmp(&mv[((size_t)t * J + j) * 2 + r], &A->mz_domval[j], 8) == 0;
               };
               if (mask[t] == (lo_x | odd) && cnt[t] > best_lo) {
                  bool ok = true;
                  for (int j = 0; j < J && ok; j++) ok = same(j, 1) && (!((lo_x >> (2 * j)) & 1) || same(j, 0));
                  if (ok) A->mz_xlo = t, best_lo = cnt[t];
               }
               if (mask[t] == (even | hi_y) && cnt[t] > best_hi) {
                  bool ok = true;
                  for (int j = 0; j < J && ok; j++) ok = same(j, 0);
                  if (ok) {
                     A->mz_xhi = t, best_hi = cnt[t];
                     for (int j = 0; j < J; j++) A->mz_hival[j] = mv[((size_t)t * J + j) * 2 + 1];
                  }
               }
            }
         }
      }
      if (ok) {
         A->mz_P = P;
         A->mz_S = S;
         A->mz27 = 1;
         A->mz_dom = dom;
      }
   }
   return AMG_OK;
}

// back to the row-pattern form (pair / master / march forms dropped)
static void drop_pair_forms(amg_mat *A)
{
   hipFree(A->ppat);
   hipFree(A->pptab);
   hipFree(A->mpmask);
   hipFree(A->mpval);
   A->ppat = nullptr;
   A->pptab = nullptr;
   A->mpmask = nullptr;
   A->mpval = nullptr;
   A->pp_n = A->pp_stride = A->pp_centre0 = 0;
   A->mp_J = A->mp_uni = 0;
   A->mz_P = A->mz_S = A->mz27 = 0;
   A->mz_dom = -1;
   A->mz_xlo = A->mz_xhi = -1;
}

int amg_mat_finish(amg_mat *A)
{
   amgk::extract_diag(A->ctx->stream, A);
   AMG_HIP(hipGetLastError());
   {
      int *d = nullptr;
      AMG_HIP(hipMalloc(&d, 2 * sizeof(int)));
      AMG_HIP(hipMemsetAsync(d, 0, 2 * sizeof(int), A->ctx->stream));
      amgk::row_max(A->ctx->stream, A, d);
      amgk::diag_uniform(A->ctx->stream, A, d + 1);
      int h[2] = {0, 0};
      double d0 = 0.0;
      hipError_t e = hipMemcpyAsync(h, d, 2 * sizeof(int), hipMemcpyDeviceToHost, A->ctx->stream);
      if (e == hipSuccess && A->nrows > 0)
         e = hipMemcpyAsync(&d0, A->diag, sizeof(double), hipMemcpyDeviceToHost, A->ctx->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(A->ctx->stream);
      hipFree(d);
      if (e != hipSuccess) return amg_set_error(AMG_ERR_HIP, "amg_mat_finish: %s", hipGetErrorString(e));
      A->maxrow = h[0];
      A->diag_uni = A->nrows > 0 && h[1] == 0;
      A->diag_u = d0;
   }
   if (A->ctx->value_index && A->nnz > 0) AMG_TRY(build_value_index(A));
   if (A->ctx->dict_index && A->vidx) AMG_TRY(build_dict_index(A));
   if (A->ctx->row_pattern && A->didx) AMG_TRY(build_row_pattern(A));
   const bool pp = A->dc_maxrow <= 8 || A->nrows >= AMG_PP_LONG_MIN_ROWS || A->ctx->pair_pattern == 2;
   // long-row operators below the pair-coding size still try the 27-pt march
   // (kept only if it applies: the pair kernel itself is slower there)
   const bool try27 = !pp && A->ctx->plane_march && A->ctx->master_pattern;
   if (A->ctx->pair_pattern && A->rpat && A->dc_maxrow <= AMG_PP_MAXROW && (pp || try27))
      AMG_TRY(build_pair_pattern(A));
   if (A->ctx->master_pattern && A->ppat) AMG_TRY(build_master_pattern(A));
   if (try27 && A->ppat && !A->mz27 && !A->pbase) drop_pair_forms(A);
   return AMG_OK;
}

extern "C" int amg_set_row_pattern(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_row_pattern: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->row_pattern = enable ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_mat_row_pattern(const amg_mat *A)
{
   return A ? A->rp_n : 0;
}

extern "C" int amg_set_pair_pattern(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_pair_pattern: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->pair_pattern = enable < 0 ? 0 : enable > 2 ? 2 : enable;
   return AMG_OK;
}

extern "C" int amg_mat_pair_pattern(const amg_mat *A)
{
   return A ? A->pp_n : 0;
}

extern "C" int amg_set_pair_anchor16(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_pair_anchor16: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->pair_anchor16 = enable ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_mat_pair_anchor16(const amg_mat *A)
{
   return (A && A->pdelta) ? 1 : 0;
}

extern "C" int amg_set_master_pattern(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_master_pattern: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->master_pattern = enable ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_mat_master_pattern(const amg_mat *A)
{
   return A ? A->mp_J * (A->mp_uni ? -1 : 1) : 0;
}

extern "C" int amg_set_plane_march(amg_ctx *c, int enable, int zc, int xcd)
{
   AMG_ARG(c, "amg_set_plane_march: null context");
   AMG_ARG(zc >= -1 && zc <= 64, "amg_set_plane_march: planes per chunk %d outside [1, 64] (0: keep, -1: auto)",
           zc);
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->plane_march = enable ? 1 : 0;
   if (zc > 0) c->mz_zc = zc, c->mz_zc_auto = 0;
   if (zc == -1) c->mz_zc = 16, c->mz_zc_auto = 1;
   if (xcd >= 0) c->mz_xcd = xcd ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_set_jgs_wave(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_jgs_wave: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->jgs_wave = std::max(0, std::min(3, enable));
   return AMG_OK;
}

extern "C" int amg_set_jgs_small(amg_ctx *c, int form)
{
   AMG_ARG(c, "amg_set_jgs_small: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->jgs_small = std::max(0, std::min(2, form));
   return AMG_OK;
}

extern "C" int amg_set_jgs_fold(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_jgs_fold: null context");
   c->knob_gen++;
   c->jgs_fold = enable != 0;
   return AMG_OK;
}

extern "C" int amg_set_fuse_prolong(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_fuse_prolong: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->fuse_prolong = std::max(0, std::min(7, enable));
   return AMG_OK;
}

extern "C" int amg_set_march_lines(amg_ctx *c, int lines)
{
   AMG_ARG(c && (lines == 1 || lines == 2 || lines == 4), "amg_set_march_lines: lines must be 1, 2 or 4");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->mz_lines = lines;
   c->mz_lines_gemv = lines;
   return AMG_OK;
}

extern "C" int amg_set_march_lines_gemv(amg_ctx *c, int lines)
{
   AMG_ARG(c && (lines == 1 || lines == 2 || lines == 4), "amg_set_march_lines_gemv: lines must be 1, 2 or 4");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->mz_lines_gemv = lines;
   return AMG_OK;
}

extern "C" int amg_set_fuse_outer(amg_ctx *c, int mode)
{
   AMG_ARG(c && mode >= 0 && mode <= 3, "amg_set_fuse_outer: mode 0, 1, 2 or 3");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->fuse_outer = mode;
   return AMG_OK;
}

extern "C" int amg_set_outer_slab(amg_ctx *c, int planes)
{
   AMG_ARG(c && planes >= 1, "amg_set_outer_slab: planes must be >= 1");
   c->knob_gen++;
   c->outer_slab = planes;
   return AMG_OK;
}

extern "C" int amg_set_long_form(amg_ctx *c, int form, int xcd)
{
   AMG_ARG(c && form >= 0 && form <= 2, "amg_set_long_form: form 0, 1 or 2");
   c->knob_gen++;
   c->long_form = form;
   c->long_xcd = xcd != 0;
   return AMG_OK;
}

extern "C" int amg_set_graphs(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_graphs: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->graphs = enable != 0;
   return AMG_OK;
}

extern "C" int amg_set_march_tuning(amg_ctx *c, int mz_pf, int mz27_pf, int mz_occ, int mz27_occ)
{
   AMG_ARG(c, "amg_set_march_tuning: null context");
   AMG_ARG(mz_pf == -2 || (mz_pf >= 1 && mz_pf <= 3), "amg_set_march_tuning: 7-pt prefetch distance %d", mz_pf);
   AMG_ARG(mz27_pf == -2 || mz27_pf == 1 || mz27_pf == 2 || mz27_pf == 3,
           "amg_set_march_tuning: 27-pt prefetch distance %d (3: the LDS plane ring)",
           mz27_pf);
   AMG_ARG(mz_occ >= -2 && mz_occ <= 8 && mz27_occ >= -2 && mz27_occ <= 8,
           "amg_set_march_tuning: occupancy %d / %d outside [-1, 8]", mz_occ, mz27_occ);
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   if (mz_pf != -2) c->mz_pf = mz_pf;
   if (mz27_pf != -2) c->mz27_pf = mz27_pf;
   if (mz_occ != -2) c->mz_occ = mz_occ;
   if (mz27_occ != -2) c->mz27_occ = mz27_occ;
   return AMG_OK;
}

extern "C" int amg_set_fuse_transfer(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_fuse_transfer: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->fuse_transfer = enable ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_mat_plane_march(const amg_mat *A)
{
   return A ? A->mz_P : 0;
}

extern "C" int amg_mat_march_points(const amg_mat *A)
{
   return (A && A->mz_P) ? (A->mz27 ? 27 : 7) : 0;
}

extern "C" int amg_set_dict_index(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_dict_index: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->dict_index = enable ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_mat_dict_index(const amg_mat *A)
{
   return A ? A->dc_n : 0;
}

extern "C" int amg_set_value_index(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_value_index: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->value_index = enable ? 1 : 0;
   return AMG_OK;
}

extern "C" int amg_mat_value_index(const amg_mat *A)
{
   return A ? A->vi_n : 0;
}

int amg_mat_create_device(amg_ctx *c, int nrows, int ncols, long long nnz, amg_mat **out)
{
   return mat_alloc(c, nrows, ncols, nnz, out);
}

// 3x3 block form of a square, diagonal-first operator with num_functions = 3
// (dofs byVDIM: rows 3t..3t+2 are the three components of node t, e.g. the
// DMEM elasticity problem, DMEM_BuildMatrix.cpp:442-719): block row t is
// blocked when its three rows hold exactly the columns 3j..3j+2 of the same
// node set {j} -- each row diagonal first, then ascending, so walking the
// blocks (ascending j, components ascending) with the diagonal taken first
// adds every row's products in its CSR order (bit-identical).  Other block
// rows (the identity rows of fixed dofs) keep the CSR form.  Used only when
// at least 90% of the block rows are blocked.
static int build_bsr3(amg_mat *A, const int *rowptr, const int *col, const double *val)
{
   const int n = A->nrows, nb = n / 3;
   if (!A->ctx->bsr3 || n % 3 || n != A->ncols || !A->diag_first || n < 3 || A->nnz < 24LL * n) return AMG_OK;
   std::vector<int> bptr(nb + 1, 0), bdiag(nb, -1), bcol;
   std::vector<unsigned char> mode(nb, 1);
   std::vector<long long> src; // CSR position of every block entry (row-major 3x3), -1 unused
   std::vector<int> js;
   long long blocked = 0;
   for (int t = 0; t < nb; t++) {
      bptr[t + 1] = bptr[t];
      const int r0 = 3 * t;
      const int len = rowptr[r0 + 1] - rowptr[r0];
      if (len < 3 || len % 3) continue;
      bool ok = true;
      js.clear();
      for (int c = 0; c < 3 && ok; c++) {
         const int r = r0 + c, b = rowptr[r], e = rowptr[r + 1];
         ok = e - b == len && col[b] == r;
         // the row minus its diagonal, ascending, with the diagonal reinserted
         // at its sorted place: 3j, 3j+1, 3j+2 per node j
         int prev = -1, k = b + 1;
         std::vector<int> cols;
         cols.reserve(len);
         bool ins = false;
         for (int q = 0; q < len - 1 && ok; q++, k++) {
            const int cc = col[k];
            if (!ins && r < cc) cols.push_back(r), ins = true;
            ok = cc > prev && cc != r;
            prev = cc;
            cols.push_back(cc);
         }
         if (!ins) cols.push_back(r);
         for (int q = 0; q < len && ok; q += 3) {
            ok = cols[q] % 3 == 0 && cols[q + 1] == cols[q] + 1 && cols[q + 2] == cols[q] + 2;
            if (ok && c == 0) js.push_back(cols[q] / 3);
            if (ok && c > 0) ok = js[q / 3] == cols[q] / 3;
         }
      }
      if (!ok) continue;
      mode[t] = 0;
      blocked++;
      for (size_t q = 0; q < js.size(); q++) {
         if (js[q] == t) bdiag[t] = bptr[t + 1];
         bcol.push_back(js[q]);
         bptr[t + 1]++;
      }
      if (bdiag[t] < 0) return AMG_OK; // unreachable: every row holds its diagonal
      // CSR positions: row r's entry for column 3j + cc
      const size_t base = src.size();
      src.resize(base + js.size() * 9, -1);
      for (int c = 0; c < 3; c++) {
         const int r = r0 + c, b = rowptr[r], e = rowptr[r + 1];
         for (int k = b; k < e; k++) {
            const int j = col[k] / 3, cc = col[k] % 3;
            const size_t q = std::lower_bound(js.begin(), js.end(), j) - js.begin();
            src[base + q * 9 + 3 * c + cc] = k;
         }
      }
   }
   if (blocked * 10 < 9LL * nb) return AMG_OK;
   // sliced layout (21 block rows per slice -- a lane per row -- or, value-indexed
   // with ctx->bsr3 == 2, 64 -- a lane per block row; padded to the slice's longest)
   const int SL = A->ctx->bsr3 == 2 && A->vidx ? 64 : 21;
   A->bsl = SL;
   const int ns = (nb + SL - 1) / SL;
   std::vector<long long> soff(ns + 1, 0);
   for (int sl = 0; sl < ns; sl++) {
      int w = 0;
      for (int t = sl * SL; t < std::min(nb, (sl + 1) * SL); t++) w = std::max(w, bptr[t + 1] - bptr[t]);
      soff[sl + 1] = soff[sl] + (long long)w * SL;
   }
   const size_t nslot = (size_t)soff[ns];
   std::vector<int> scol(std::max<size_t>(nslot, 1), 0), bdk(nb, 0);
   std::vector<unsigned char> bcnt(nb, 0);
   for (int t = 0; t < nb; t++) {
      const int cnt = bptr[t + 1] - bptr[t];
      if (cnt > 255) return AMG_OK; // block rows of more than 255 blocks: keep CSR
      bcnt[t] = (unsigned char)cnt;
      bdk[t] = mode[t] ? 0 : bdiag[t] - bptr[t];
      const int sl = t / SL, q = t % SL;
      const int w = (int)((soff[sl + 1] - soff[sl]) / SL);
      for (int k = 0; k < w; k++) scol[(size_t)soff[sl] + (size_t)k * SL + q] = k < cnt ? bcol[bptr[t] + k] : t;
   }
   hipStream_t s = A->ctx->stream;
   auto fail = [&]() {
      hipFree(A->soff), hipFree(A->bcol), hipFree(A->bdiag), hipFree(A->bmode), hipFree(A->bvi), hipFree(A->bval);
      A->soff = nullptr;
      A->bcol = A->bdiag = nullptr;
      A->bmode = nullptr;
      A->bvi = nullptr;
      A->bval = nullptr;
      (void)hipGetLastError();
      return AMG_OK; // not enough room: keep the CSR forms
   };
   hipError_t e = hipMalloc(&A->soff, (ns + 1) * sizeof(long long));
   if (e == hipSuccess) e = hipMalloc(&A->bcol, scol.size() * sizeof(int));
   if (e == hipSuccess) e = hipMalloc(&A->bdiag, nb * sizeof(int));
   if (e == hipSuccess) e = hipMalloc(&A->bmode, nb);
   if (e != hipSuccess) return fail();
   // slot of block k of block row t
   auto slot = [&](int t, int k) { return (size_t)soff[t / SL] + (size_t)k * SL + t % SL; };
   if (A->vidx) {
      // block entries as indices into the value table (3 rows x 4 bytes)
      std::vector<double> tab(256);
      AMG_HIP(hipMemcpy(tab.data(), A->vtab, 256 * sizeof(double), hipMemcpyDeviceToHost));
      std::vector<unsigned long long> keys(A->vi_n);
      std::memcpy(keys.data(), tab.data(), A->vi_n * 8);
      std::vector<unsigned int> bvi(std::max<size_t>(nslot * 3, 1), 0);
      for (int t = 0; t < nb; t++)
         for (int k = 0; k < bptr[t + 1] - bptr[t]; k++)
            for (int q = 0; q < 9; q++) {
               const long long sp = src[(size_t)(bptr[t] + k) * 9 + q];
               if (sp < 0) continue;
               unsigned long long b;
               std::memcpy(&b, &val[sp], 8);
               const size_t idx = std::lower_bound(keys.begin(), keys.end(), b) - keys.begin();
               bvi[slot(t, k) * 3 + q / 3] |= (unsigned int)idx << (8 * (q % 3));
            }
      e = hipMalloc(&A->bvi, bvi.size() * 4);
      if (e != hipSuccess) return fail();
      AMG_HIP(hipMemcpyAsync(A->bvi, bvi.data(), bvi.size() * 4, hipMemcpyHostToDevice, s));
      AMG_HIP(hipStreamSynchronize(s));
      A->bsr3 = 1;
   } else {
      std::vector<double> bv(std::max<size_t>(nslot * 9, 1), 0.0);
      for (int t = 0; t < nb; t++)
         for (int k = 0; k < bptr[t + 1] - bptr[t]; k++)
            for (int q = 0; q < 9; q++) {
               const long long sp = src[(size_t)(bptr[t] + k) * 9 + q];
               if (sp >= 0) bv[slot(t, k) * 9 + q] = val[sp];
            }
      e = hipMalloc(&A->bval, bv.size() * 8);
      if (e != hipSuccess) return fail();
      AMG_HIP(hipMemcpyAsync(A->bval, bv.data(), bv.size() * 8, hipMemcpyHostToDevice, s));
      AMG_HIP(hipStreamSynchronize(s));
      A->bsr3 = 2;
   }
   for (int t = 0; t < nb; t++) bcnt[t] = mode[t] ? 0 : bcnt[t];
   AMG_HIP(hipMemcpyAsync(A->soff, soff.data(), (ns + 1) * sizeof(long long), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->bcol, scol.data(), scol.size() * sizeof(int), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->bdiag, bdk.data(), nb * sizeof(int), hipMemcpyHostToDevice, s));
   AMG_HIP(hipMemcpyAsync(A->bmode, bcnt.data(), nb, hipMemcpyHostToDevice, s));
   AMG_HIP(hipStreamSynchronize(s));
   return AMG_OK;
}

extern "C" int amg_set_bsr3(amg_ctx *c, int enable)
{
   AMG_ARG(c, "amg_set_bsr3: null context");
   c->knob_gen++; // cached hipGraphs were captured with the old setting
   c->bsr3 = enable == 2 ? 2 : (enable ? 1 : 0);
   return AMG_OK;
}

extern "C" int amg_mat_bsr3(const amg_mat *A)
{
   return A ? A->bsr3 : 0;
}

extern "C" int amg_mat_bsr3_slice(const amg_mat *A)
{
   return A && A->bsr3 ? A->bsl : 0;
}

extern "C" int amg_csr_register(amg_ctx *c, int nrows, int ncols, long long nnz, const int *rowptr,
                                const int *col, const double *val, int diag_first, amg_mat **out)
{
   AMG_ARG(c && out && rowptr && (nnz == 0 || (col && val)), "amg_csr_register: null argument");
   AMG_ARG(nrows >= 0 && ncols >= 0 && nnz >= 0, "amg_csr_register: negative size");
   AMG_ARG(nnz < (1LL << 31) - AMG_NNZ_PAD, "amg_csr_register: nnz %lld exceeds int32 CSR", nnz);
   AMG_ARG(rowptr[nrows] == nnz && rowptr[0] == 0, "amg_csr_register: rowptr[0]=%d rowptr[n]=%d nnz=%lld",
           rowptr[0], rowptr[nrows], nnz);
   AMG_ARG(nrows == 0 || ncols > 0, "amg_csr_register: ncols must be positive");
   amg_mat *A = nullptr;
   AMG_TRY(mat_alloc(c, nrows, ncols, nnz, &A));
   A->diag_first = diag_first;
   AMG_HIP(hipMemcpyAsync(A->rowptr, rowptr, ((size_t)nrows + 1) * sizeof(int),
                          hipMemcpyHostToDevice, c->stream));
   if (nnz) {
      AMG_HIP(hipMemcpyAsync(A->col, col, (size_t)nnz * sizeof(int), hipMemcpyHostToDevice, c->stream));
      AMG_HIP(hipMemcpyAsync(A->val, val, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice,
                             c->stream));
   }
   AMG_TRY(amg_mat_finish(A));
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_TRY(build_bsr3(A, rowptr, col, val));
   *out = A;
   return AMG_OK;
}

extern "C" int amg_mat_free(amg_mat *A)
{
   std::lock_guard<std::recursive_mutex> td(amg_teardown_mutex());
   if (!A) return AMG_OK;
   if (A->trans) amg_mat_free(A->trans);
   hipFree(A->rowptr);
   hipFree(A->col);
   hipFree(A->val);
   hipFree(A->diag);
   hipFree(A->vidx);
   hipFree(A->vtab);
   hipFree(A->didx);
   hipFree(A->doff);
   hipFree(A->dval);
   hipFree(A->danch);
   hipFree(A->rpat);
   hipFree(A->ptab);
   hipFree(A->ppat);
   hipFree(A->pptab);
   hipFree(A->mpmask);
   hipFree(A->mpval);
   hipFree(A->soff);
   hipFree(A->bcol);
   hipFree(A->bdiag);
   hipFree(A->bmode);
   hipFree(A->bvi);
   hipFree(A->bval);
   hipFree(A->pbase);
   hipFree(A->pdelta);
   delete A;
   return AMG_OK;
}

extern "C" int amg_mat_info(const amg_mat *A, int *nrows, int *ncols, long long *nnz)
{
   AMG_ARG(A, "amg_mat_info: null matrix");
   if (nrows) *nrows = A->nrows;
   if (ncols) *ncols = A->ncols;
   if (nnz) *nnz = A->nnz;
   return AMG_OK;
}

extern "C" int amg_mat_download(amg_ctx *c, const amg_mat *A, int *rowptr, int *col, double *val)
{
   AMG_ARG(c && A, "amg_mat_download: null argument");
   AMG_HIP(hipStreamSynchronize(c->stream));
   if (rowptr)
      AMG_HIP(hipMemcpy(rowptr, A->rowptr, ((size_t)A->nrows + 1) * sizeof(int), hipMemcpyDeviceToHost));
   if (col && A->nnz) AMG_HIP(hipMemcpy(col, A->col, (size_t)A->nnz * sizeof(int), hipMemcpyDeviceToHost));
   if (val && A->nnz) AMG_HIP(hipMemcpy(val, A->val, (size_t)A->nnz * sizeof(double), hipMemcpyDeviceToHost));
   return AMG_OK;
}

// ---------------------------------------------------------------------------
// vectors
// ---------------------------------------------------------------------------
extern "C" int amg_vec_create(amg_ctx *c, int n, amg_vec **out)
{
   AMG_ARG(c && out && n >= 0, "amg_vec_create: bad argument");
   amg_vec *v = new amg_vec();
   v->ctx = c;
   v->n = n;
   hipError_t e = hipMalloc(&v->d, std::max(1, n) * sizeof(double));
   if (e != hipSuccess) {
      delete v;
      return amg_set_error(AMG_ERR_OOM, "amg_vec_create(%d): %s", n, hipGetErrorString(e));
   }
   AMG_HIP(hipMemsetAsync(v->d, 0, std::max(1, n) * sizeof(double), c->stream));
   *out = v;
   return AMG_OK;
}

extern "C" int amg_vec_free(amg_vec *v)
{
   if (!v) return AMG_OK;
   if (v->owns) hipFree(v->d);
   delete v;
   return AMG_OK;
}

extern "C" int amg_vec_size(const amg_vec *v) { return v ? v->n : -1; }

extern "C" int amg_vec_upload(amg_ctx *c, amg_vec *v, const double *h)
{
   AMG_ARG(c && v && h, "amg_vec_upload: null argument");
   AMG_HIP(hipMemcpyAsync(v->d, h, (size_t)v->n * sizeof(double), hipMemcpyHostToDevice, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   return AMG_OK;
}

extern "C" int amg_vec_download(amg_ctx *c, const amg_vec *v, double *h)
{
   AMG_ARG(c && v && h, "amg_vec_download: null argument");
   AMG_HIP(hipMemcpyAsync(h, v->d, (size_t)v->n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   return AMG_OK;
}

extern "C" int amg_vec_set(amg_ctx *c, amg_vec *v, double a)
{
   AMG_ARG(c && v, "amg_vec_set: null argument");
   amgk::vset(c->stream, v->d, a, 0, v->n);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_vec_copy(amg_ctx *c, const amg_vec *x, amg_vec *y)
{
   AMG_ARG(c && x && y && x->n == y->n, "amg_vec_copy: size mismatch");
   amgk::vcopy(c->stream, x->d, y->d, 0, x->n);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_vec_axpy(amg_ctx *c, double a, const amg_vec *x, amg_vec *y)
{
   AMG_ARG(c && x && y && x->n == y->n, "amg_vec_axpy: size mismatch");
   amgk::vaxpy(c->stream, a, x->d, y->d, 0, x->n);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_vec_ivaxpy(amg_ctx *c, const amg_vec *x, const amg_vec *s, amg_vec *y)
{
   AMG_ARG(c && x && s && y && x->n == y->n && s->n == y->n, "amg_vec_ivaxpy: size mismatch");
   amgk::vivaxpy(c->stream, x->d, s->d, y->d, 0, y->n);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_vec_scale(amg_ctx *c, double a, amg_vec *y)
{
   AMG_ARG(c && y, "amg_vec_scale: null argument");
   amgk::vscale(c->stream, a, y->d, 0, y->n);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int amg_reduce_to_host(amg_ctx *c, const double *partials, int np, int do_sqrt, double *out)
{
   amgk::reduce_partials(c->stream, partials, np, c->d_scalars, do_sqrt, c->d_scalars + 4096);
   AMG_HIP(hipGetLastError());
   AMG_HIP(hipMemcpyAsync(c->h_pinned, c->d_scalars, sizeof(double), hipMemcpyDeviceToHost, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   *out = c->h_pinned[0];
   return AMG_OK;
}

extern "C" int amg_vec_norm2(amg_ctx *c, const amg_vec *x, double *out)
{
   AMG_ARG(c && x && out, "amg_vec_norm2: null argument");
   double *p;
   AMG_TRY(amg_ctx_partials(c, 1024, &p));
   int np = 0;
   amgk::sumsq_partials(c->stream, x->d, x->n, p, &np);
   return amg_reduce_to_host(c, p, np, 1, out);
}

extern "C" int amg_vec_dot(amg_ctx *c, const amg_vec *x, const amg_vec *y, double *out)
{
   AMG_ARG(c && x && y && out && x->n == y->n, "amg_vec_dot: size mismatch");
   double *p;
   AMG_TRY(amg_ctx_partials(c, 1024, &p));
   int np = 0;
   amgk::dot_partials(c->stream, x->d, y->d, x->n, p, &np);
   return amg_reduce_to_host(c, p, np, 0, out);
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
static int check_range(const amg_mat *A, int rb, int re)
{
   AMG_ARG(rb >= 0 && re <= A->nrows && rb <= re, "row range [%d,%d) outside [0,%d)", rb, re,
           A->nrows);
   return AMG_OK;
}

extern "C" int amg_matvec(amg_ctx *c, const amg_mat *A, const amg_vec *x, amg_vec *y, int rb, int re)
{
   AMG_ARG(c && A && x && y, "amg_matvec: null argument");
   AMG_ARG(x->n >= A->ncols && y->n >= A->nrows, "amg_matvec: vector sizes %d/%d vs %dx%d", x->n,
           y->n, A->nrows, A->ncols);
   AMG_TRY(check_range(A, rb, re));
   amgk::spgemv(c->stream, A, x->d, nullptr, amgk::gemv_mode(1.0, 0.0), y->d, rb, re, nullptr);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_matvec_timed(amg_ctx *c, const amg_mat *A, const amg_vec *x, amg_vec *y,
                                int reps, double *ms)
{
   AMG_ARG(c && A && x && y && ms && reps >= 1, "amg_matvec_timed: bad argument");
   AMG_ARG(x->n >= A->ncols && y->n >= A->nrows, "amg_matvec_timed: vector sizes");
   hipEvent_t a, b;
   AMG_HIP(hipEventCreate(&a));
   AMG_HIP(hipEventCreate(&b));
   const amgk::Gemv g = amgk::gemv_mode(1.0, 0.0);
   AMG_HIP(hipEventRecord(a, c->stream));
   for (int r = 0; r < reps; r++)
      amgk::spgemv(c->stream, A, x->d, nullptr, g, y->d, 0, A->nrows, nullptr);
   AMG_HIP(hipEventRecord(b, c->stream));
   AMG_HIP(hipEventSynchronize(b));
   float t = 0.f;
   AMG_HIP(hipEventElapsedTime(&t, a, b));
   hipEventDestroy(a);
   hipEventDestroy(b);
   *ms = (double)t / reps;
   return AMG_OK;
}

// measurement helpers (declared in the header): PMC calibration streams
// (tools/pmc_traffic.py) and the STREAM-triad ceiling bench.py reports
extern "C" int amg_pmc_calib(amg_ctx *c, int mode, long long bytes)
{
   AMG_ARG(c && mode >= 0 && mode <= 4 && bytes > 0, "amg_pmc_calib: bad argument");
   void *buf = nullptr;
   AMG_HIP(hipMalloc(&buf, (size_t)bytes));
   AMG_HIP(hipMemsetAsync(buf, 1, (size_t)bytes, c->stream));
   amgk::calib_stream(c->stream, mode, buf, bytes, c->d_scalars + 8000);
   AMG_HIP(hipStreamSynchronize(c->stream));
   hipFree(buf);
   return AMG_OK;
}

extern "C" int amg_stream_triad(amg_ctx *c, long long n, int reps, double *gbs)
{
   AMG_ARG(c && n >= 2 && reps >= 1 && gbs, "amg_stream_triad: bad argument");
   n &= ~1LL;
   double *a = nullptr, *b = nullptr, *d = nullptr;
   AMG_HIP(hipMalloc(&a, (size_t)n * 8));
   if (hipMalloc(&b, (size_t)n * 8) != hipSuccess || hipMalloc(&d, (size_t)n * 8) != hipSuccess) {
      hipFree(a);
      hipFree(b);
      return amg_set_error(AMG_ERR_OOM, "amg_stream_triad: %lld doubles", n);
   }
   hipEvent_t e0, e1;
   hipEventCreate(&e0);
   hipEventCreate(&e1);
   hipMemsetAsync(b, 0, (size_t)n * 8, c->stream);
   hipMemsetAsync(d, 0, (size_t)n * 8, c->stream);
   amgk::stream_triad(c->stream, a, b, d, 3.0, n); // warm
   float best = 1e30f;
   for (int r = 0; r < reps; r++) {
      hipEventRecord(e0, c->stream);
      amgk::stream_triad(c->stream, a, b, d, 3.0, n);
      hipEventRecord(e1, c->stream);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      best = std::min(best, ms);
   }
   const hipError_t err = hipGetLastError();
   hipEventDestroy(e0);
   hipEventDestroy(e1);
   hipFree(a);
   hipFree(b);
   hipFree(d);
   AMG_HIP(err);
   *gbs = 24.0 * (double)n / (best * 1e-3) / 1e9;
   return AMG_OK;
}

#ifdef AMG_DEV_TUNE
// development-only tuning entry points (tools/tune_spmv.py), only in the
// development build lib/libamg_mi355x_dev.so (make dev); not in the header
namespace amgk {
int num_tune_variants();
const char *tune_variant_name(int v);
void launch_tune_variant(hipStream_t s, int v, const amg_mat *A, const double *x, double *y);
} // namespace amgk

extern "C" int amg_dev_tune_count(void) { return amgk::num_tune_variants(); }

extern "C" const char *amg_dev_tune_name(int v) { return amgk::tune_variant_name(v); }
extern "C" int amg_dev_tune_spmv(amg_ctx *c, const amg_mat *A, const amg_vec *x, amg_vec *y,
                                 int variant, int reps, double *ms)
{
   AMG_ARG(c && A && x && y && ms && reps >= 1, "amg_dev_tune_spmv: bad argument");
   AMG_ARG(variant >= 0 && variant < amgk::num_tune_variants(), "amg_dev_tune_spmv: variant");
   hipEvent_t a, b;
   AMG_HIP(hipEventCreate(&a));
   AMG_HIP(hipEventCreate(&b));
   AMG_HIP(hipEventRecord(a, c->stream));
   for (int r = 0; r < reps; r++) amgk::launch_tune_variant(c->stream, variant, A, x->d, y->d);
   AMG_HIP(hipEventRecord(b, c->stream));
   AMG_HIP(hipEventSynchronize(b));
   AMG_HIP(hipGetLastError());
   float t = 0.f;
   AMG_HIP(hipEventElapsedTime(&t, a, b));
   hipEventDestroy(a);
   hipEventDestroy(b);
   *ms = (double)t / reps;
   return AMG_OK;
}
#endif // AMG_DEV_TUNE

extern "C" int amg_spgemv(amg_ctx *c, const amg_mat *A, const amg_vec *x, const amg_vec *b,
                          double alpha, double beta, amg_vec *y, int rb, int re)
{
   AMG_ARG(c && A && x && y, "amg_spgemv: null argument");
   AMG_ARG(x->n >= A->ncols && y->n >= A->nrows, "amg_spgemv: vector sizes");
   AMG_TRY(check_range(A, rb, re));
   amgk::Gemv g = amgk::gemv_mode(alpha, beta);
   AMG_ARG(g.init == 0 || (b && b->n >= A->nrows), "amg_spgemv: b required when beta != 0");
   amgk::spgemv(c->stream, A, x->d, b ? b->d : nullptr, g, y->d, rb, re, nullptr);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_residual(amg_ctx *c, const amg_mat *A, const amg_vec *b, const amg_vec *x,
                            amg_vec *y, amg_vec *r, int rb, int re)
{
   AMG_ARG(c && A && b && x && y && r, "amg_residual: null argument");
   AMG_TRY(check_range(A, rb, re));
   // SMEM_Residual: y = A x over [rb,re), then r = b - y
   amgk::spgemv(c->stream, A, x->d, nullptr, amgk::gemv_mode(1.0, 0.0), y->d, rb, re, nullptr);
   amgk::vsub(c->stream, b->d, y->d, r->d, rb, re);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

static int build_transpose(amg_mat *A);

extern "C" int amg_matvec_t(amg_ctx *c, const amg_mat *A, const amg_vec *x, amg_vec *y, int T)
{
   AMG_ARG(c && A && x && y, "amg_matvec_t: null argument");
   AMG_ARG(x->n >= A->nrows && y->n >= A->ncols, "amg_matvec_t: vector sizes");
   amg_mat *Am = const_cast<amg_mat *>(A);
   if (!Am->trans) AMG_TRY(build_transpose(Am));
   amgk::matvec_t_chunked(c->stream, Am->trans, x->d, y->d, A->nrows, T);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

// transpose on the host once (setup-time; rows of A^T list source rows ascending)
static int build_transpose(amg_mat *A)
{
   amg_ctx *c = A->ctx;
   std::vector<int> rp(A->nrows + 1), cj(A->nnz);
   std::vector<double> cv(A->nnz);
   AMG_TRY(amg_mat_download(c, A, rp.data(), cj.data(), cv.data()));
   std::vector<int> trp(A->ncols + 1, 0), tcj(A->nnz);
   std::vector<double> tcv(A->nnz);
   for (long long k = 0; k < A->nnz; k++) trp[cj[k] + 1]++;
   for (int i = 0; i < A->ncols; i++) trp[i + 1] += trp[i];
   std::vector<int> pos(trp.begin(), trp.end());
   for (int r = 0; r < A->nrows; r++)
      for (int k = rp[r]; k < rp[r + 1]; k++) {
         int col = cj[k];
         tcj[pos[col]] = r;
         tcv[pos[col]] = cv[k];
         pos[col]++;
      }
   return amg_csr_register(c, A->ncols, A->nrows, A->nnz, trp.data(), tcj.data(), tcv.data(), 0,
                           &A->trans);
}

extern "C" int amg_jacobi(amg_ctx *c, const amg_mat *A, const amg_vec *f, amg_vec *u,
                          amg_vec *u_prev, double omega, int sweeps, int zero_first, int rb,
                          int re, int variant)
{
   AMG_ARG(c && A && f && u && u_prev, "amg_jacobi: null argument");
   AMG_TRY(check_range(A, rb, re));
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zero_first == 1) {
         amgk::jacobi_zero(c->stream, A->diag, f->d, nullptr, omega, u->d, rb, re, variant);
      } else {
         // u_prev = u; u = J(u_prev) (SMEM_Smooth.cpp:33-46)
         amgk::vcopy(c->stream, u->d, u_prev->d, 0, u->n);
         amgk::jacobi_sweep(c->stream, A, f->d, u_prev->d, nullptr, omega, u->d, rb, re);
      }
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_l1_jacobi(amg_ctx *c, const amg_mat *A, const amg_vec *f, amg_vec *u,
                             amg_vec *u_prev, const amg_vec *l1, int sweeps, int zero_first,
                             int rb, int re, int variant)
{
   AMG_ARG(c && A && f && u && u_prev && l1, "amg_l1_jacobi: null argument");
   AMG_TRY(check_range(A, rb, re));
   for (int k = 0; k < sweeps; k++) {
      if (k == 0 && zero_first == 1) {
         amgk::jacobi_zero(c->stream, A->diag, f->d, l1->d, 1.0, u->d, rb, re, variant);
      } else {
         amgk::vcopy(c->stream, u->d, u_prev->d, 0, u->n);
         amgk::jacobi_sweep(c->stream, A, f->d, u_prev->d, l1->d, 1.0, u->d, rb, re);
      }
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

int amg_hybrid_jgs_dev(amg_ctx *c, hipStream_t s, const amg_mat *A, const double *f, double *u,
                       double *u_prev, int n_vec, const int *d_blk, int nblk, int blk_lo,
                       int blk_hi, const double *ds, double weight, int sweeps, int zero_first,
                       int reverse, double *apply_u = nullptr, double *apply_priv = nullptr,
                       bool *applied = nullptr, unsigned long long *stamp = nullptr)
{
   bool ap = false;
   for (int k = 0; k < sweeps; k++) {
      const int zero = (k == 0 && zero_first == 1);
      if (!zero) amgk::vcopy(s, u, u_prev, blk_lo, blk_hi);
      const bool last = k == sweeps - 1;
      ap = amgk::hybrid_jgs(s, A, f, u, u_prev, d_blk, nblk, ds, weight, zero, reverse, last ? apply_u : nullptr,
                            last ? apply_priv : nullptr, last ? stamp : nullptr);
   }
   if (applied) *applied = ap;
   (void)n_vec;
   (void)c;
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_hybrid_jgs(amg_ctx *c, const amg_mat *A, const amg_vec *f, amg_vec *u,
                              amg_vec *u_prev, const int *blk, int nblk, const amg_vec *diag_scale,
                              double weight, int sweeps, int zero_first, int reverse)
{
   AMG_ARG(c && A && f && u && u_prev && blk && nblk > 0, "amg_hybrid_jgs: null argument");
   for (int b = 0; b < nblk; b++)
      AMG_ARG(blk[b] <= blk[b + 1] && blk[b] >= 0 && blk[b + 1] <= A->nrows,
              "amg_hybrid_jgs: bad block %d [%d,%d)", b, blk[b], blk[b + 1]);
   int *d_blk = nullptr;
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_HIP(hipMalloc((void **)&d_blk, (nblk + 1) * sizeof(int)));
   AMG_HIP(hipMemcpyAsync(d_blk, blk, (nblk + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream));
   AMG_HIP(hipStreamSynchronize(c->stream));
   int s = amg_hybrid_jgs_dev(c, c->stream, A, f->d, u->d, u_prev->d, u->n, d_blk, nblk, blk[0],
                              blk[nblk], diag_scale ? diag_scale->d : nullptr, weight, sweeps,
                              zero_first, reverse);
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_HIP(hipFree(d_blk));
   return s;
}

extern "C" int amg_gauss_seidel(amg_ctx *c, const amg_mat *A, const amg_vec *f, amg_vec *u,
                                int sweeps)
{
   AMG_ARG(c && A && f && u, "amg_gauss_seidel: null argument");
   // SEQ_GaussSeidel == one hybrid block covering every row (no out-of-block terms)
   int blk[2] = {0, A->nrows};
   return amg_hybrid_jgs(c, A, f, u, u, blk, 1, nullptr, 1.0, sweeps, 0, 0);
}

extern "C" int amg_async_gauss_seidel(amg_ctx *c, const amg_mat *A, const amg_vec *f, amg_vec *u,
                                      const int *blk, int nblk, int sweeps, int semi, int reverse)
{
   AMG_ARG(c && A && f && u && blk && nblk > 0 && sweeps >= 0, "amg_async_gauss_seidel: bad argument");
   AMG_ARG(f->n >= A->nrows && u->n >= A->nrows && A->nrows == A->ncols,
           "amg_async_gauss_seidel: square matrix and vectors of its size");
   for (int b = 0; b < nblk; b++)
      AMG_ARG(blk[b] <= blk[b + 1] && blk[b] >= 0 && blk[b + 1] <= A->nrows,
              "amg_async_gauss_seidel: bad block %d [%d,%d)", b, blk[b], blk[b + 1]);
   int *d_blk = nullptr;
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_HIP(hipMalloc((void **)&d_blk, (nblk + 1) * sizeof(int)));
   AMG_HIP(hipMemcpyAsync(d_blk, blk, (nblk + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream));
   amgk::async_gs(c->stream, A, f->d, u->d, d_blk, nblk, sweeps, semi, reverse);
   AMG_HIP(hipStreamSynchronize(c->stream));
   AMG_HIP(hipFree(d_blk));
   return AMG_OK;
}

int amg_sym_jacobi_dev(hipStream_t s, const amg_mat *A, const double *f, double *u, double *y,
                       double *r, double omega, const double *l1, int sweeps, int zero_first,
                       int rb, int re, int variant)
{
   const int seq = (variant == 1);
   amgk::Gemv mv = amgk::gemv_mode(1.0, 0.0);
   int k = 0;
   if (seq || zero_first == 1) {
      amgk::vcopy(s, f, r, rb, re);
   } else {
      amgk::spgemv(s, A, u, nullptr, mv, y, rb, re, nullptr);
      amgk::vsub(s, f, y, r, rb, re);
   }
   while (true) {
      amgk::sym_scale(s, A->diag, l1, omega, r, rb, re, seq);
      amgk::spgemv(s, A, r, nullptr, mv, y, rb, re, nullptr);
      amgk::sym_update(s, A->diag, l1, omega, r, y, u, rb, re, seq, (!seq && zero_first == 1));
      k++;
      if (k == sweeps) break;
      amgk::spgemv(s, A, u, nullptr, mv, y, rb, re, nullptr);
      amgk::vsub(s, f, y, r, rb, re);
   }
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_sym_jacobi(amg_ctx *c, const amg_mat *A, const amg_vec *f, amg_vec *u,
                              amg_vec *y, amg_vec *r, double omega, const amg_vec *l1, int sweeps,
                              int zero_first, int rb, int re, int variant)
{
   AMG_ARG(c && A && f && u && y && r && sweeps >= 1, "amg_sym_jacobi: bad argument");
   AMG_TRY(check_range(A, rb, re));
   return amg_sym_jacobi_dev(c->stream, A, f->d, u->d, y->d, r->d, omega, l1 ? l1->d : nullptr,
                             sweeps, zero_first, rb, re, variant);
}

extern "C" int amg_l1_norms(amg_ctx *c, const amg_mat *A, amg_vec *out)
{
   AMG_ARG(c && A && out && out->n >= A->nrows, "amg_l1_norms: bad argument");
   amgk::l1_norms(c->stream, A, out->d);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}

extern "C" int amg_a_diag(amg_ctx *c, const amg_mat *A, double omega, amg_vec *out)
{
   AMG_ARG(c && A && out && out->n >= A->nrows, "amg_a_diag: bad argument");
   amgk::a_diag(c->stream, A->diag, omega, out->d, A->nrows);
   AMG_HIP(hipGetLastError());
   return AMG_OK;
}
