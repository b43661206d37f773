// amg_spgemm.hip -- Galerkin products of the classical setup on the GPU
// (the R (A P) of HYPRE_BoomerAMGSetup's hypre_BoomerAMGBuildCoarseOperator,
// SMEM_Setup.cpp:55-70 / DMEM_Setup.cpp:169-173, restated host-side in
// amg_classical.cpp::spgemm).
//
// C = A B with one lane per row of C, exactly the host's Gustavson order: the
// lane walks its row's (A entry, B entry) products in order and adds each into
// its column's slot of an open-addressing table in global scratch (a column's
// first contribution lands on 0.0, like the host's acc[c] = 0.0), so every
// entry of C is the same sum of the same rounded products in the same order --
// bit-identical to the host.  The row's distinct columns are then sorted
// ascending (shell sort in the lane's scratch), the diagonal moved first for
// square products, and rows packed by an exclusive scan of their counts.  Rows
// run in batches sized to a scratch budget (upper bound per row: the sum of
// the B rows its A entries name).
#include <algorithm>
#include <numeric>
#include <vector>

#include "amg_internal.h"

namespace {

// ub[r] = sum of |B row k| over the entries (r, k) of A
__global__ void spgemm_ub_k(const int *__restrict__ arp, const int *__restrict__ acj, const int *__restrict__ brp,
                            int n, long long *__restrict__ ub)
{
   const int r = blockIdx.x * blockDim.x + threadIdx.x;
   if (r >= n) return;
   long long s = 0;
   for (int k = arp[r]; k < arp[r + 1]; k++) s += brp[acj[k] + 1] - brp[acj[k]];
   ub[r] = s;
}

// rows [r0, r0 + nr): the hash tables at hoff[r - r0] (capacity cap = power of
// two >= 2 ub), then the row's sorted entries at the table's start; cnt[r - r0]
__global__ void spgemm_row_k(const int *__restrict__ arp, const int *__restrict__ acj,
                             const double *__restrict__ av, const int *__restrict__ brp,
                             const int *__restrict__ bcj, const double *__restrict__ bv, int r0, int nr,
                             const long long *__restrict__ hoff, int *__restrict__ hcol,
                             double *__restrict__ hval, int *__restrict__ cnt, int square)
{
   const int q = blockIdx.x * blockDim.x + threadIdx.x;
   if (q >= nr) return;
   const int r = r0 + q;
   const long long base = hoff[q];
   const int cap = (int)(hoff[q + 1] - base);
   int *hc = hcol + base;
   double *hv = hval + base;
   for (int i = 0; i < cap; i++) hc[i] = -1;
   const unsigned mask = (unsigned)cap - 1u;
   for (int ka = arp[r]; ka < arp[r + 1]; ka++) {
      const int k = acj[ka];
      const double a = av[ka];
      for (int kb = brp[k]; kb < brp[k + 1]; kb++) {
         const int c = bcj[kb];
         unsigned h = ((unsigned)c * 2654435761u) & mask;
         while (hc[h] != c && hc[h] != -1) h = (h + 1) & mask;
         if (hc[h] == -1) {
            hc[h] = c;
            hv[h] = 0.0;
         }
         hv[h] += a * bv[kb];
      }
   }
   // compact the occupied slots to the table's start (scan order), then sort
   int m = 0;
   for (int i = 0; i < cap; i++)
      if (hc[i] != -1) {
         const int c = hc[i];
         const double v = hv[i];
         hc[m] = c;
         hv[m] = v;
         m++;
      }
   // shell sort by column (columns are distinct)
   for (int gap = m / 2; gap > 0; gap /= 2)
      for (int i = gap; i < m; i++) {
         const int c = hc[i];
         const double v = hv[i];
         int j = i;
         for (; j >= gap && hc[j - gap] > c; j -= gap) {
            hc[j] = hc[j - gap];
            hv[j] = hv[j - gap];
         }
         hc[j] = c;
         hv[j] = v;
      }
   if (square) {
      // diag_first: the diagonal moved to the front, the rest keeping order
      for (int i = 0; i < m; i++)
         if (hc[i] == r) {
            const double v = hv[i];
            for (int j = i; j > 0; j--) {
               hc[j] = hc[j - 1];
               hv[j] = hv[j - 1];
            }
            hc[0] = r;
            hv[0] = v;
            break;
         }
   }
   cnt[q] = m;
}

__global__ void spgemm_pack_k(const long long *__restrict__ hoff, const int *__restrict__ hcol,
                              const double *__restrict__ hval, const long long *__restrict__ ooff, int nr,
                              int *__restrict__ ocol, double *__restrict__ oval)
{
   const int q = blockIdx.x;
   if (q >= nr) return;
   const long long b = hoff[q], o = ooff[q], m = ooff[q + 1] - o;
   for (long long i = threadIdx.x; i < m; i += blockDim.x) {
      ocol[o + i] = hcol[b + i];
      oval[o + i] = hval[b + i];
   }
}

template <class T>
int dupload(hipStream_t s, const std::vector<T> &h, T **d)
{
   AMG_HIP(hipMalloc(d, std::max<size_t>(h.size(), 1) * sizeof(T)));
   if (!h.empty()) AMG_HIP(hipMemcpyAsync(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
   return AMG_OK;
}

// C = A B with every operand on the device: A An x (B's rows), B with Bm
// columns; C's rowptr / col / val allocated here (*d_crp, *d_ccj, *d_cv) and
// its entry count in *nnz
int spgemm_dev(hipStream_t s, int An, const int *d_arp, const int *d_acj, const double *d_av, const int *d_brp,
               const int *d_bcj, const double *d_bv, int Bm, int **d_crp, int **d_ccj, double **d_cv, long long *nnz)
{
   long long *d_ub = nullptr, *d_hoff = nullptr, *d_ooff = nullptr;
   int *d_hcol = nullptr, *d_cnt = nullptr, *d_ocol = nullptr;
   double *d_hval = nullptr, *d_oval = nullptr;
   int *c_col = nullptr;
   double *c_val = nullptr;
   long long c_cap = 0;
   auto cleanup = [&]() {
      hipStreamSynchronize(s);
      for (void *p : {(void *)d_ub, (void *)d_hoff, (void *)d_ooff, (void *)d_hcol, (void *)d_cnt, (void *)d_ocol,
                      (void *)d_hval, (void *)d_oval})
         hipFree(p);
   };
   auto run = [&]() -> int {
      AMG_HIP(hipMalloc(&d_ub, std::max(An, 1) * sizeof(long long)));
      if (An > 0) spgemm_ub_k<<<(An + 255) / 256, 256, 0, s>>>(d_arp, d_acj, d_brp, An, d_ub);
      std::vector<long long> ub(An);
      if (An > 0) AMG_HIP(hipMemcpyAsync(ub.data(), d_ub, An * sizeof(long long), hipMemcpyDeviceToHost, s));
      AMG_HIP(hipStreamSynchronize(s));
      // table capacity per row: a power of two >= 2 ub (>= 2)
      std::vector<long long> capr(An);
      for (int r = 0; r < An; r++) {
         long long c = 2;
         while (c < 2 * ub[r]) c <<= 1;
         capr[r] = c;
      }
      // batches of rows within the scratch budget (12 bytes per slot)
      const long long budget = 1LL << 29; // slots: 6 GiB of scratch
      long long maxb = 1;
      for (int r0 = 0; r0 < An;) {
         long long tot = 0;
         int r1 = r0;
         while (r1 < An && (r1 == r0 || tot + capr[r1] <= budget)) tot += capr[r1++];
         maxb = std::max(maxb, tot);
         r0 = r1;
      }
      AMG_HIP(hipMalloc(&d_hcol, maxb * sizeof(int)));
      AMG_HIP(hipMalloc(&d_hval, maxb * sizeof(double)));
      AMG_HIP(hipMalloc(&d_hoff, (size_t)(An + 1) * sizeof(long long)));
      AMG_HIP(hipMalloc(&d_ooff, (size_t)(An + 1) * sizeof(long long)));
      AMG_HIP(hipMalloc(&d_cnt, std::max(An, 1) * sizeof(int)));
      AMG_HIP(hipMalloc(&d_ocol, maxb * sizeof(int)));
      AMG_HIP(hipMalloc(&d_oval, maxb * sizeof(double)));
      std::vector<int> crp(An + 1, 0);
      long long used = 0;
      for (int r0 = 0; r0 < An;) {
         long long tot = 0;
         int r1 = r0;
         while (r1 < An && (r1 == r0 || tot + capr[r1] <= budget)) tot += capr[r1++];
         const int nr = r1 - r0;
         std::vector<long long> hoff(nr + 1, 0);
         for (int q = 0; q < nr; q++) hoff[q + 1] = hoff[q] + capr[r0 + q];
         AMG_HIP(hipMemcpyAsync(d_hoff, hoff.data(), (nr + 1) * sizeof(long long), hipMemcpyHostToDevice, s));
         spgemm_row_k<<<(nr + 127) / 128, 128, 0, s>>>(d_arp, d_acj, d_av, d_brp, d_bcj, d_bv, r0, nr, d_hoff,
                                                       d_hcol, d_hval, d_cnt, An == Bm ? 1 : 0);
         AMG_HIP(hipGetLastError());
         std::vector<int> cnt(nr);
         AMG_HIP(hipMemcpyAsync(cnt.data(), d_cnt, nr * sizeof(int), hipMemcpyDeviceToHost, s));
         AMG_HIP(hipStreamSynchronize(s));
         std::vector<long long> ooff(nr + 1, 0);
         for (int q = 0; q < nr; q++) ooff[q + 1] = ooff[q] + cnt[q];
         AMG_HIP(hipMemcpyAsync(d_ooff, ooff.data(), (nr + 1) * sizeof(long long), hipMemcpyHostToDevice, s));
         spgemm_pack_k<<<nr, 64, 0, s>>>(d_hoff, d_hcol, d_hval, d_ooff, nr, d_ocol, d_oval);
         // append the batch to C (grown by doubling, device to device)
         if (used + ooff[nr] > c_cap) {
            const long long cap = std::max(used + ooff[nr], 2 * c_cap);
            int *nc = nullptr;
            double *nv = nullptr;
            AMG_HIP(hipMalloc(&nc, std::max(cap, 1LL) * sizeof(int)));
            if (hipMalloc(&nv, std::max(cap, 1LL) * sizeof(double)) != hipSuccess) {
               hipFree(nc);
               return amg_set_error(AMG_ERR_OOM, "spgemm_dev: %lld entries", cap);
            }
            if (used) {
               AMG_HIP(hipMemcpyAsync(nc, c_col, used * sizeof(int), hipMemcpyDeviceToDevice, s));
               AMG_HIP(hipMemcpyAsync(nv, c_val, used * sizeof(double), hipMemcpyDeviceToDevice, s));
            }
            AMG_HIP(hipStreamSynchronize(s));
            hipFree(c_col);
            hipFree(c_val);
            c_col = nc;
            c_val = nv;
            c_cap = cap;
         }
         if (ooff[nr]) {
            AMG_HIP(hipMemcpyAsync(c_col + used, d_ocol, ooff[nr] * sizeof(int), hipMemcpyDeviceToDevice, s));
            AMG_HIP(hipMemcpyAsync(c_val + used, d_oval, ooff[nr] * sizeof(double), hipMemcpyDeviceToDevice, s));
         }
         AMG_HIP(hipStreamSynchronize(s));
         for (int q = 0; q < nr; q++) crp[r0 + q + 1] = crp[r0 + q] + cnt[q];
         used += ooff[nr];
         r0 = r1;
      }
      if (!c_col) {
         AMG_HIP(hipMalloc(&c_col, sizeof(int)));
         AMG_HIP(hipMalloc(&c_val, sizeof(double)));
      }
      int *rp = nullptr;
      AMG_TRY(dupload(s, crp, &rp));
      AMG_HIP(hipStreamSynchronize(s));
      *d_crp = rp;
      *d_ccj = c_col;
      *d_cv = c_val;
      *nnz = used;
      c_col = nullptr;
      c_val = nullptr;
      return AMG_OK;
   };
   const int st = run();
   hipFree(c_col);
   hipFree(c_val);
   cleanup();
   return st;
}

template <class T>
int download(hipStream_t s, const T *d, size_t n, std::vector<T> &h)
{
   h.resize(n);
   if (n) AMG_HIP(hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
   return AMG_OK;
}

} // namespace

// C = A B on device `device` (host CSR in and out; bit-identical to the host
// Gustavson spgemm).  An x Am, B Am x Bm.
int amg_spgemm_device(int device, int An, const std::vector<int> &arp, const std::vector<int> &acj,
                      const std::vector<double> &av, int Bn, const std::vector<int> &brp,
                      const std::vector<int> &bcj, const std::vector<double> &bv, int Bm, std::vector<int> &crp,
                      std::vector<int> &ccj, std::vector<double> &cv)
{
   (void)Bn;
   AMG_HIP(hipSetDevice(device));
   hipStream_t s;
   AMG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
   std::vector<void *> mem;
   int *d_arp = nullptr, *d_acj = nullptr, *d_brp = nullptr, *d_bcj = nullptr, *d_crp = nullptr, *d_ccj = nullptr;
   double *d_av = nullptr, *d_bv = nullptr, *d_cv = nullptr;
   long long nnz = 0;
   auto run = [&]() -> int {
      AMG_TRY(dupload(s, arp, &d_arp));
      AMG_TRY(dupload(s, acj, &d_acj));
      AMG_TRY(dupload(s, av, &d_av));
      AMG_TRY(dupload(s, brp, &d_brp));
      AMG_TRY(dupload(s, bcj, &d_bcj));
      AMG_TRY(dupload(s, bv, &d_bv));
      AMG_TRY(spgemm_dev(s, An, d_arp, d_acj, d_av, d_brp, d_bcj, d_bv, Bm, &d_crp, &d_ccj, &d_cv, &nnz));
      AMG_TRY(download(s, d_crp, (size_t)An + 1, crp));
      AMG_TRY(download(s, d_ccj, (size_t)nnz, ccj));
      AMG_TRY(download(s, d_cv, (size_t)nnz, cv));
      AMG_HIP(hipStreamSynchronize(s));
      return AMG_OK;
   };
   const int st = run();
   hipStreamSynchronize(s);
   for (void *p : {(void *)d_arp, (void *)d_acj, (void *)d_av, (void *)d_brp, (void *)d_bcj, (void *)d_bv,
                   (void *)d_crp, (void *)d_ccj, (void *)d_cv})
      hipFree(p);
   hipStreamDestroy(s);
   return st;
}

// A_c = R (A P) on device `device`: A, P, R uploaded once, A P kept on the
// device between the two products, only A_c downloaded (host CSR in and out;
// bit-identical to the host's two Gustavson products)
int amg_rap_device(int device, int An, const std::vector<int> &arp, const std::vector<int> &acj,
                   const std::vector<double> &av, const std::vector<int> &prp, const std::vector<int> &pcj,
                   const std::vector<double> &pv, int Pm, int Rn, const std::vector<int> &rrp,
                   const std::vector<int> &rcj, const std::vector<double> &rv, std::vector<int> &crp,
                   std::vector<int> &ccj, std::vector<double> &cv)
{
   AMG_HIP(hipSetDevice(device));
   hipStream_t s;
   AMG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
   int *d_arp = nullptr, *d_acj = nullptr, *d_prp = nullptr, *d_pcj = nullptr, *d_rrp = nullptr, *d_rcj = nullptr;
   int *d_aprp = nullptr, *d_apcj = nullptr, *d_crp = nullptr, *d_ccj = nullptr;
   double *d_av = nullptr, *d_pv = nullptr, *d_rv = nullptr, *d_apv = nullptr, *d_cv = nullptr;
   long long apnz = 0, cnz = 0;
   auto run = [&]() -> int {
      AMG_TRY(dupload(s, arp, &d_arp));
      AMG_TRY(dupload(s, acj, &d_acj));
      AMG_TRY(dupload(s, av, &d_av));
      AMG_TRY(dupload(s, prp, &d_prp));
      AMG_TRY(dupload(s, pcj, &d_pcj));
      AMG_TRY(dupload(s, pv, &d_pv));
      AMG_TRY(spgemm_dev(s, An, d_arp, d_acj, d_av, d_prp, d_pcj, d_pv, Pm, &d_aprp, &d_apcj, &d_apv, &apnz));
      // A is not needed any more: give its memory back before the second product
      AMG_HIP(hipStreamSynchronize(s));
      hipFree(d_acj), d_acj = nullptr;
      hipFree(d_av), d_av = nullptr;
      AMG_TRY(dupload(s, rrp, &d_rrp));
      AMG_TRY(dupload(s, rcj, &d_rcj));
      AMG_TRY(dupload(s, rv, &d_rv));
      AMG_TRY(spgemm_dev(s, Rn, d_rrp, d_rcj, d_rv, d_aprp, d_apcj, d_apv, Pm, &d_crp, &d_ccj, &d_cv, &cnz));
      AMG_TRY(download(s, d_crp, (size_t)Rn + 1, crp));
      AMG_TRY(download(s, d_ccj, (size_t)cnz, ccj));
      AMG_TRY(download(s, d_cv, (size_t)cnz, cv));
      AMG_HIP(hipStreamSynchronize(s));
      return AMG_OK;
   };
   const int st = run();
   hipStreamSynchronize(s);
   for (void *p : {(void *)d_arp, (void *)d_acj, (void *)d_av, (void *)d_prp, (void *)d_pcj, (void *)d_pv,
                   (void *)d_rrp, (void *)d_rcj, (void *)d_rv, (void *)d_aprp, (void *)d_apcj, (void *)d_apv,
                   (void *)d_crp, (void *)d_ccj, (void *)d_cv})
      hipFree(p);
   hipStreamDestroy(s);
   return st;
}
