// mz27_probe.hip -- the level-1 27-point plane march (csr_mz27_kernel's
// memory pipeline) in isolation: y = b - A x on a 256^3 box, every row the
// full 27-point stencil (uniform values, SGPR kernel arguments), plane chunks
// marched by 256-lane workgroups of 512 in-plane positions (2 per lane).
//  V0: the library's form -- each of the 9 marched lines (planes k-1..k+1 x
//      lines y-1..y+1) held as 4 doubles (x-1, x, x+1, x+2; the +-1 neighbours
//      shuffled in when the line is loaded), the new plane's 3 lines
//      prefetched PF planes ahead into registers.
//  V1: lean lines -- each marched line held as its pair (2 doubles) plus the
//      wave-edge double; the +-1 neighbours taken at use by wave-wide DPP
//      shifts (wave_shr:1 / wave_shl:1), PF = 2 or 3 planes ahead.
// Both add the 27 terms in the same order: bit-identical outputs.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/mz27_probe.hip -o tools/_mz27_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef double v2d __attribute__((ext_vector_type(2)));
typedef double v2du __attribute__((ext_vector_type(2), aligned(8)));

#define CK(x)                                                                                                      \
   do {                                                                                                            \
      hipError_t e_ = (x);                                                                                         \
      if (e_ != hipSuccess) {                                                                                      \
         printf("%s -> %s\n", #x, hipGetErrorString(e_));                                                          \
         exit(1);                                                                                                  \
      }                                                                                                            \
   } while (0)

struct V27 {
   double v[27];
};

__device__ __forceinline__ v2d ld2u(const double *b, unsigned i) { return *reinterpret_cast<const v2du *>(b + i); }

// ---------------------------------------------------------------- V0
struct Ln4 {
   double l, a, b, r;
};
__device__ __forceinline__ void ld_line(const double *__restrict__ x, long long idx, unsigned Nu, int lane, v2d &v,
                                        double &e)
{
   const unsigned i = idx < 0 ? 0u : (idx + 2 > (long long)Nu ? Nu - 2 : (unsigned)idx);
   v = ld2u(x, i);
   e = 0.0;
   if (lane == 0 && i > 0) e = x[i - 1];
   if (lane == 63 && i + 2 < Nu) e = x[i + 2];
}
__device__ __forceinline__ Ln4 mk_line(v2d v, double e, int lane)
{
   double l = __shfl_up(v.y, 1, 64);
   double r = __shfl_down(v.x, 1, 64);
   if (lane == 0) l = e;
   if (lane == 63) r = e;
   return Ln4{l, v.x, v.y, r};
}

template <int PF>
__global__ __launch_bounds__(256) void v0_k(const double *__restrict__ x, const double *__restrict__ b,
                                            double *__restrict__ y, int P, int S, int nz, int zc, int npb, V27 W)
{
   const int tid = threadIdx.x, lane = tid & 63;
   const int G = gridDim.x;
   int lg = blockIdx.x;
   if ((G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   const int pos = pblk * 512 + 2 * tid;
   const unsigned Nu = (unsigned)((long long)nz * P);
   Ln4 X[3][3];
#pragma unroll
   for (int m = 0; m < 3; m++)
#pragma unroll
      for (int d = 0; d < 3; d++) {
         const int p = k0 - 1 + m;
         v2d v{0.0, 0.0};
         double e = 0.0;
         if (p >= 0 && p < nz) ld_line(x, (long long)p * P + pos + (d - 1) * S, Nu, lane, v, e);
         X[m][d] = mk_line(v, e, lane);
      }
   v2d qv[3] = {{0, 0}, {0, 0}, {0, 0}};
   double qe[3] = {0, 0, 0};
   if (PF == 2 && k0 + 2 < nz && k0 + 1 < k1)
#pragma unroll
      for (int d = 0; d < 3; d++) ld_line(x, (long long)(k0 + 2) * P + pos + (d - 1) * S, Nu, lane, qv[d], qe[d]);
   for (int k = k0; k < k1; k++) {
      const unsigned row = (unsigned)k * P + pos;
      v2d nv[3] = {{0, 0}, {0, 0}, {0, 0}};
      double ne[3] = {0, 0, 0};
      if (k + PF + 1 < nz && k + PF < k1)
#pragma unroll
         for (int d = 0; d < 3; d++) ld_line(x, (long long)row + (PF + 1LL) * P + (d - 1) * S, Nu, lane, nv[d], ne[d]);
      v2d acc = ld2u(b, row);
#pragma unroll
      for (int m = 0; m < 3; m++)
#pragma unroll
         for (int d = 0; d < 3; d++) {
            const Ln4 &q = X[m][d];
            const double w0 = W.v[m * 9 + d * 3], w1 = W.v[m * 9 + d * 3 + 1], w2 = W.v[m * 9 + d * 3 + 2];
            acc.x = acc.x - w0 * q.l;
            acc.y = acc.y - w0 * q.a;
            acc.x = acc.x - w1 * q.a;
            acc.y = acc.y - w1 * q.b;
            acc.x = acc.x - w2 * q.b;
            acc.y = acc.y - w2 * q.r;
         }
      *reinterpret_cast<v2d *>(y + row) = acc;
#pragma unroll
      for (int d = 0; d < 3; d++) {
         X[0][d] = X[1][d];
         X[1][d] = X[2][d];
         if (PF == 2) {
            X[2][d] = mk_line(qv[d], qe[d], lane);
            qv[d] = nv[d];
            qe[d] = ne[d];
         } else {
            X[2][d] = mk_line(nv[d], ne[d], lane);
         }
      }
   }
}

// ---------------------------------------------------------------- V1
// wave-wide DPP shifts of a double: lane l <- lane l - 1 (shr) / l + 1 (shl);
// the vacated lane gets `fill`
__device__ __forceinline__ double wshr1(double v, double fill)
{
   const unsigned long long b = (unsigned long long)__double_as_longlong(v);
   const unsigned long long f = (unsigned long long)__double_as_longlong(fill);
   const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)f, (int)(unsigned)b, 0x138, 0xf, 0xf, false);
   const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(f >> 32), (int)(unsigned)(b >> 32), 0x138, 0xf, 0xf,
                                              false);
   return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wshl1(double v, double fill)
{
   const unsigned long long b = (unsigned long long)__double_as_longlong(v);
   const unsigned long long f = (unsigned long long)__double_as_longlong(fill);
   const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)f, (int)(unsigned)b, 0x130, 0xf, 0xf, false);
   const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(f >> 32), (int)(unsigned)(b >> 32), 0x130, 0xf, 0xf,
                                              false);
   return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

struct Ln3 {
   v2d v;
   double e; // lane 0: x at pair - 1; lane 63: x at pair + 2
};

template <int PF>
__global__ __launch_bounds__(256) void v1_k(const double *__restrict__ x, const double *__restrict__ b,
                                            double *__restrict__ y, int P, int S, int nz, int zc, int npb, V27 W)
{
   const int tid = threadIdx.x, lane = tid & 63;
   const int G = gridDim.x;
   int lg = blockIdx.x;
   if ((G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   const int pos = pblk * 512 + 2 * tid;
   const unsigned Nu = (unsigned)((long long)nz * P);
   Ln3 X[3][3];
   Ln3 Q[PF - 1][3]; // planes k + 2 .. k + PF (PF - 1 of them loaded ahead)
#pragma unroll
   for (int m = 0; m < 3; m++)
#pragma unroll
      for (int d = 0; d < 3; d++) {
         const int p = k0 - 1 + m;
         X[m][d].v = v2d{0.0, 0.0};
         X[m][d].e = 0.0;
         if (p >= 0 && p < nz) ld_line(x, (long long)p * P + pos + (d - 1) * S, Nu, lane, X[m][d].v, X[m][d].e);
      }
#pragma unroll
   for (int q = 0; q < PF - 1; q++)
#pragma unroll
      for (int d = 0; d < 3; d++) {
         const int p = k0 + 2 + q;
         Q[q][d].v = v2d{0.0, 0.0};
         Q[q][d].e = 0.0;
         if (p < nz && p <= k1) ld_line(x, (long long)p * P + pos + (d - 1) * S, Nu, lane, Q[q][d].v, Q[q][d].e);
      }
   for (int k = k0; k < k1; k++) {
      const unsigned row = (unsigned)k * P + pos;
      Ln3 nv[3];
#pragma unroll
      for (int d = 0; d < 3; d++) {
         nv[d].v = v2d{0.0, 0.0};
         nv[d].e = 0.0;
      }
      if (k + PF + 1 < nz && k + PF < k1)
#pragma unroll
         for (int d = 0; d < 3; d++)
            ld_line(x, (long long)row + (PF + 1LL) * P + (d - 1) * S, Nu, lane, nv[d].v, nv[d].e);
      v2d acc = ld2u(b, row);
#pragma unroll
      for (int m = 0; m < 3; m++)
#pragma unroll
         for (int d = 0; d < 3; d++) {
            const Ln3 &q = X[m][d];
            const double l = wshr1(q.v.y, q.e), r = wshl1(q.v.x, q.e);
            const double w0 = W.v[m * 9 + d * 3], w1 = W.v[m * 9 + d * 3 + 1], w2 = W.v[m * 9 + d * 3 + 2];
            acc.x = acc.x - w0 * l;
            acc.y = acc.y - w0 * q.v.x;
            acc.x = acc.x - w1 * q.v.x;
            acc.y = acc.y - w1 * q.v.y;
            acc.x = acc.x - w2 * q.v.y;
            acc.y = acc.y - w2 * r;
         }
      *reinterpret_cast<v2d *>(y + row) = acc;
#pragma unroll
      for (int d = 0; d < 3; d++) {
         X[0][d] = X[1][d];
         X[1][d] = X[2][d];
         X[2][d] = Q[0][d];
#pragma unroll
         for (int q = 0; q < PF - 2; q++) Q[q][d] = Q[q + 1][d];
         Q[PF - 2][d] = nv[d];
      }
   }
}

// ---------------------------------------------------------------- V2
// V0's pipeline + the library's per-pair pattern byte: a wave whose pairs are
// all the dominant pattern (or an x-edge pattern, whose edge row is redone
// with its own values Hv) computes; any other wave-plane is skipped and
// appended to a fix-up list (the full kernel's slow path, not measured here)
template <int PF>
__global__ __launch_bounds__(256) void v2_k(const double *__restrict__ x, const double *__restrict__ b,
                                            double *__restrict__ y, int P, int S, int nz, int zc, int npb, V27 W,
                                            V27 Hv, const unsigned char *__restrict__ ppat, int dom, int xlo, int xhi,
                                            unsigned *__restrict__ fix, unsigned *__restrict__ nfix)
{
   const int tid = threadIdx.x, lane = tid & 63;
   const int G = gridDim.x;
   int lg = blockIdx.x;
   if ((G & 7) == 0) lg = (lg & 7) * (G >> 3) + (lg >> 3);
   const int pblk = lg % npb, chunk = lg / npb;
   const int k0 = chunk * zc, k1 = min(k0 + zc, nz);
   const int pos = pblk * 512 + 2 * tid;
   const unsigned Nu = (unsigned)((long long)nz * P);
   Ln4 X[3][3];
#pragma unroll
   for (int m = 0; m < 3; m++)
#pragma unroll
      for (int d = 0; d < 3; d++) {
         const int p = k0 - 1 + m;
         v2d v{0.0, 0.0};
         double e = 0.0;
         if (p >= 0 && p < nz) ld_line(x, (long long)p * P + pos + (d - 1) * S, Nu, lane, v, e);
         X[m][d] = mk_line(v, e, lane);
      }
   v2d qv[3] = {{0, 0}, {0, 0}, {0, 0}};
   double qe[3] = {0, 0, 0};
   if (PF == 2 && k0 + 2 < nz && k0 + 1 < k1)
#pragma unroll
      for (int d = 0; d < 3; d++) ld_line(x, (long long)(k0 + 2) * P + pos + (d - 1) * S, Nu, lane, qv[d], qe[d]);
   for (int k = k0; k < k1; k++) {
      const unsigned row = (unsigned)k * P + pos;
      v2d nv[3] = {{0, 0}, {0, 0}, {0, 0}};
      double ne[3] = {0, 0, 0};
      if (k + PF + 1 < nz && k + PF < k1)
#pragma unroll
         for (int d = 0; d < 3; d++) ld_line(x, (long long)row + (PF + 1LL) * P + (d - 1) * S, Nu, lane, nv[d], ne[d]);
      const int pid = ppat[row >> 1];
      const bool fast = __all(pid == dom || pid == xlo || pid == xhi);
      if (fast) {
         const v2d acc0 = ld2u(b, row);
         v2d acc = acc0;
#pragma unroll
         for (int m = 0; m < 3; m++)
#pragma unroll
            for (int d = 0; d < 3; d++) {
               const Ln4 &q = X[m][d];
               const double w0 = W.v[m * 9 + d * 3], w1 = W.v[m * 9 + d * 3 + 1], w2 = W.v[m * 9 + d * 3 + 2];
               acc.x = acc.x - w0 * q.l;
               acc.y = acc.y - w0 * q.a;
               acc.x = acc.x - w1 * q.a;
               acc.y = acc.y - w1 * q.b;
               acc.x = acc.x - w2 * q.b;
               acc.y = acc.y - w2 * q.r;
            }
         if (pid == xlo) {
            acc.x = acc0.x;
#pragma unroll
            for (int m = 0; m < 3; m++)
#pragma unroll
               for (int d = 0; d < 3; d++) {
                  const Ln4 &q = X[m][d];
                  acc.x = acc.x - W.v[m * 9 + d * 3 + 1] * q.a;
                  acc.x = acc.x - W.v[m * 9 + d * 3 + 2] * q.b;
               }
         }
         if (pid == xhi) {
            acc.y = acc0.y;
#pragma unroll
            for (int m = 0; m < 3; m++)
#pragma unroll
               for (int d = 0; d < 3; d++) {
                  const Ln4 &q = X[m][d];
                  acc.y = acc.y - Hv.v[m * 9 + d * 3] * q.a;
                  acc.y = acc.y - Hv.v[m * 9 + d * 3 + 1] * q.b;
               }
         }
         *reinterpret_cast<v2d *>(y + row) = acc;
      } else if (lane == 0) {
         const unsigned q = atomicAdd(nfix, 1u);
         fix[q] = (unsigned)(row - 2 * lane); // the wave's first row
      }
#pragma unroll
      for (int d = 0; d < 3; d++) {
         X[0][d] = X[1][d];
         X[1][d] = X[2][d];
         if (PF == 2) {
            X[2][d] = mk_line(qv[d], qe[d], lane);
            qv[d] = nv[d];
            qe[d] = ne[d];
         } else {
            X[2][d] = mk_line(nv[d], ne[d], lane);
         }
      }
   }
}

int main(int argc, char **argv)
{
   const int n = argc > 1 ? atoi(argv[1]) : 256;
   const long long N = (long long)n * n * n;
   const int P = n * n, S = n, nz = n;
   std::vector<double> hx(N), hb(N);
   srand(1);
   for (long long i = 0; i < N; i++) {
      hx[i] = rand() / (double)RAND_MAX - 0.5;
      hb[i] = rand() / (double)RAND_MAX - 0.5;
   }
   V27 W;
   for (int j = 0; j < 27; j++) W.v[j] = j == 13 ? 8.0 / 3.0 : -1.0 / 3.0 + 0.01 * j;
   double *x, *b, *y0, *y1;
   CK(hipMalloc(&x, N * 8));
   CK(hipMalloc(&b, N * 8));
   CK(hipMalloc(&y0, N * 8));
   CK(hipMalloc(&y1, N * 8));
   CK(hipMemcpy(x, hx.data(), N * 8, hipMemcpyHostToDevice));
   CK(hipMemcpy(b, hb.data(), N * 8, hipMemcpyHostToDevice));
   const int npb = P / 512;
   hipEvent_t e0, e1;
   CK(hipEventCreate(&e0));
   CK(hipEventCreate(&e1));
   const double bytes = 3.0 * 8.0 * (double)N;
   auto run = [&](const char *name, auto launch, double *y) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipDeviceSynchronize());
      const int R = 20;
      CK(hipEventRecord(e0));
      for (int r = 0; r < R; r++) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= R;
      printf("%-28s %8.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
             bytes / (ms * 1e-3) / 8e12);
      (void)y;
   };
   int zcs[] = {16, 22, 32, 43, 64};
   for (int zc : zcs) {
      const int nch = (nz + zc - 1) / zc, nb = npb * nch;
      char nm[64];
      snprintf(nm, sizeof nm, "V0 PF2 zc=%d (%d WG)", zc, nb);
      run(nm, [&] { v0_k<2><<<nb, 256>>>(x, b, y0, P, S, nz, zc, npb, W); }, y0);
      snprintf(nm, sizeof nm, "V1 PF2 zc=%d", zc);
      run(nm, [&] { v1_k<2><<<nb, 256>>>(x, b, y1, P, S, nz, zc, npb, W); }, y1);
      snprintf(nm, sizeof nm, "V1 PF3 zc=%d", zc);
      run(nm, [&] { v1_k<3><<<nb, 256>>>(x, b, y1, P, S, nz, zc, npb, W); }, y1);
      snprintf(nm, sizeof nm, "V1 PF4 zc=%d", zc);
      run(nm, [&] { v1_k<4><<<nb, 256>>>(x, b, y1, P, S, nz, zc, npb, W); }, y1);
   }
   // V2: pattern bytes of a 27-pt Galerkin box operator (0: interior, 1 / 2: the
   // x-edge pairs, 3: any face row in y or z)
   {
      std::vector<unsigned char> hp(N / 2);
      for (long long i = 0; i < N; i += 2) {
         const int xx = (int)(i % n), yy = (int)((i / n) % n), zz = (int)(i / P);
         unsigned char c = 0;
         if (yy == 0 || yy == n - 1 || zz == 0 || zz == n - 1) c = 3;
         else if (xx == 0) c = 1;
         else if (xx == n - 2) c = 2;
         hp[i / 2] = c;
      }
      unsigned char *pp;
      unsigned *fix, *nfix;
      CK(hipMalloc(&pp, N / 2));
      CK(hipMalloc(&fix, 4 * (N / 64)));
      CK(hipMalloc(&nfix, 4));
      CK(hipMemcpy(pp, hp.data(), N / 2, hipMemcpyHostToDevice));
      V27 H = W;
      for (int zc : zcs) {
         const int nch = (nz + zc - 1) / zc, nb = npb * nch;
         char nm[64];
         snprintf(nm, sizeof nm, "V2 PF2 zc=%d", zc);
         run(nm, [&] {
            hipMemsetAsync(nfix, 0, 4);
            v2_k<2><<<nb, 256>>>(x, b, y1, P, S, nz, zc, npb, W, H, pp, 0, 1, 2, fix, nfix);
         }, y1);
      }
      unsigned hn = 0;
      CK(hipMemcpy(&hn, nfix, 4, hipMemcpyDeviceToHost));
      printf("V2: %u wave-planes left to the fix-up of %lld\n", hn, N / 128);
   }
   // bitwise check of V1 against V0
   {
      const int zc = 32, nch = (nz + zc - 1) / zc, nb = npb * nch;
      v0_k<2><<<nb, 256>>>(x, b, y0, P, S, nz, zc, npb, W);
      v1_k<3><<<nb, 256>>>(x, b, y1, P, S, nz, zc, npb, W);
      CK(hipDeviceSynchronize());
      std::vector<double> a(N), c(N);
      CK(hipMemcpy(a.data(), y0, N * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(c.data(), y1, N * 8, hipMemcpyDeviceToHost));
      long long bad = 0;
      for (long long i = 0; i < N; i++) bad += memcmp(&a[i], &c[i], 8) != 0;
      printf("V1 vs V0: %lld differing of %lld\n", bad, N);
   }
   return 0;
}
