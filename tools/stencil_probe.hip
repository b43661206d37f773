// stencil_probe.hip -- ceiling probe for the structured residual r = f - A x
// with wave-uniform (scalar) stencil offsets and values: how fast can a
// 27-pt (level 1, 256^3) and a 7-pt (level 0, 512^3) residual go when the
// offsets/values are SGPR operands instead of per-lane LDS lookups?
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/stencil_probe.hip -o tools/_stencil_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double v2d __attribute__((ext_vector_type(2)));
typedef double v2du __attribute__((ext_vector_type(2), aligned(8)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Sten { int off[32]; double val[32]; int m; };

// pair per lane, all offsets uniform (kernel argument -> SGPRs)
template <int M>
__global__ __launch_bounds__(256) void pair_k(const double *__restrict__ f, const double *__restrict__ x,
                                              double *__restrict__ r, long long n, Sten s)
{
   const long long i = 2 * ((long long)blockIdx.x * 256 + threadIdx.x);
   if (i >= n) return;
   v2d acc = *reinterpret_cast<const v2d *>(f + i);
   v2d xv[M];
#pragma unroll
   for (int j = 0; j < M; j++) xv[j] = *reinterpret_cast<const v2du *>(x + i + s.off[j]);
#pragma unroll
   for (int j = 0; j < M; j++) {
      acc.x -= s.val[j] * xv[j].x;
      acc.y -= s.val[j] * xv[j].y;
   }
   *reinterpret_cast<v2d *>(r + i) = acc;
}

// pair per lane with a per-lane entry mask from a per-pair pattern byte (LDS
// mask table): the master-pattern form
template <int M>
__global__ __launch_bounds__(256) void pair_mask_k(const double *__restrict__ f, const double *__restrict__ x,
                                                   double *__restrict__ r, long long n, Sten s,
                                                   const unsigned char *__restrict__ pat,
                                                   const unsigned long long *__restrict__ mtab, int np)
{
   __shared__ unsigned long long mt[256];
   if (threadIdx.x < np) mt[threadIdx.x] = mtab[threadIdx.x];
   __syncthreads();
   const long long i = 2 * ((long long)blockIdx.x * 256 + threadIdx.x);
   if (i >= n) return;
   const unsigned long long mk = mt[pat[i >> 1]];
   v2d acc = *reinterpret_cast<const v2d *>(f + i);
   v2d xv[M];
#pragma unroll
   for (int j = 0; j < M; j++) {
      xv[j] = v2d{0.0, 0.0};
      if ((mk >> (2 * j)) & 3) xv[j] = *reinterpret_cast<const v2du *>(x + i + s.off[j]);
   }
#pragma unroll
   for (int j = 0; j < M; j++) {
      if ((mk >> (2 * j)) & 1) acc.x -= s.val[j] * xv[j].x;
      if ((mk >> (2 * j + 1)) & 1) acc.y -= s.val[j] * xv[j].y;
   }
   *reinterpret_cast<v2d *>(r + i) = acc;
}

// pair per lane, f streamed in and r streamed out with nontemporal hints so
// the L2 keeps the x windows (NT=1: f and r, NT=2: r only)
template <int M, int NT, bool XCD>
__global__ __launch_bounds__(256) void pair_nt_k(const double *__restrict__ f, const double *__restrict__ x,
                                                 double *__restrict__ r, long long n, Sten s)
{
   int b = blockIdx.x;
   if (XCD) {
      const int nb = gridDim.x, per = nb / 8;
      if (b < per * 8) b = (b % 8) * per + b / 8;
   }
   const long long i = 2 * ((long long)b * 256 + threadIdx.x);
   if (i >= n) return;
   v2d acc;
   if (NT == 1)
      acc = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(f + i));
   else
      acc = *reinterpret_cast<const v2d *>(f + i);
   v2d xv[M];
#pragma unroll
   for (int j = 0; j < M; j++) xv[j] = *reinterpret_cast<const v2du *>(x + i + s.off[j]);
#pragma unroll
   for (int j = 0; j < M; j++) {
      acc.x -= s.val[j] * xv[j].x;
      acc.y -= s.val[j] * xv[j].y;
   }
   if (NT >= 1)
      __builtin_nontemporal_store(acc, reinterpret_cast<v2d *>(r + i));
   else
      *reinterpret_cast<v2d *>(r + i) = acc;
}

// four rows per lane (two 16-byte loads per offset)
template <int M, int NT>
__global__ __launch_bounds__(256) void quad_k(const double *__restrict__ f, const double *__restrict__ x,
                                              double *__restrict__ r, long long n, Sten s)
{
   const long long i = 4 * ((long long)blockIdx.x * 256 + threadIdx.x);
   if (i >= n) return;
   v2d a0 = *reinterpret_cast<const v2d *>(f + i), a1 = *reinterpret_cast<const v2d *>(f + i + 2);
   v2d xv[M], xw[M];
#pragma unroll
   for (int j = 0; j < M; j++) {
      xv[j] = *reinterpret_cast<const v2du *>(x + i + s.off[j]);
      xw[j] = *reinterpret_cast<const v2du *>(x + i + 2 + s.off[j]);
   }
#pragma unroll
   for (int j = 0; j < M; j++) {
      a0.x -= s.val[j] * xv[j].x;
      a0.y -= s.val[j] * xv[j].y;
      a1.x -= s.val[j] * xw[j].x;
      a1.y -= s.val[j] * xw[j].y;
   }
   if (NT) {
      __builtin_nontemporal_store(a0, reinterpret_cast<v2d *>(r + i));
      __builtin_nontemporal_store(a1, reinterpret_cast<v2d *>(r + i + 2));
   } else {
      *reinterpret_cast<v2d *>(r + i) = a0;
      *reinterpret_cast<v2d *>(r + i + 2) = a1;
   }
}

// triad a = b + s c, plain and nontemporal
template <int NT>
__global__ __launch_bounds__(256) void triad_k(const double *__restrict__ b, const double *__restrict__ c,
                                               double *__restrict__ a, long long n)
{
   const long long i = 2 * ((long long)blockIdx.x * 256 + threadIdx.x);
   if (i >= n) return;
   const v2d bv = *reinterpret_cast<const v2d *>(b + i), cv = *reinterpret_cast<const v2d *>(c + i);
   const v2d o = bv + 3.0 * cv;
   if (NT)
      __builtin_nontemporal_store(o, reinterpret_cast<v2d *>(a + i));
   else
      *reinterpret_cast<v2d *>(a + i) = o;
}

// one row per lane
template <int M>
__global__ __launch_bounds__(256) void row_k(const double *__restrict__ f, const double *__restrict__ x,
                                             double *__restrict__ r, long long n, Sten s)
{
   const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
   if (i >= n) return;
   double acc = f[i];
   double xv[M];
#pragma unroll
   for (int j = 0; j < M; j++) xv[j] = x[i + s.off[j]];
#pragma unroll
   for (int j = 0; j < M; j++) acc -= s.val[j] * xv[j];
   r[i] = acc;
}

template <class F>
static float timeit(F launch, int reps)
{
   hipEvent_t a, b;
   CK(hipEventCreate(&a));
   CK(hipEventCreate(&b));
   launch();
   launch();
   CK(hipEventRecord(a));
   for (int k = 0; k < reps; k++) launch();
   CK(hipEventRecord(b));
   CK(hipEventSynchronize(b));
   float ms;
   CK(hipEventElapsedTime(&ms, a, b));
   return ms / reps;
}

static void run(int nn, int pts)
{
   const long long n = (long long)nn * nn * nn, pad = (long long)nn * nn + nn + 8;
   double *f, *x, *r;
   CK(hipMalloc(&f, n * 8));
   CK(hipMalloc(&r, n * 8));
   CK(hipMalloc(&x, (n + 2 * pad) * 8));
   CK(hipMemset(f, 0, n * 8));
   CK(hipMemset(x, 0, (n + 2 * pad) * 8));
   double *xc = x + pad;
   Sten s{};
   s.m = 0;
   for (int dz = -1; dz <= 1; dz++)
      for (int dy = -1; dy <= 1; dy++)
         for (int dx = -1; dx <= 1; dx++) {
            const int nz = (dx != 0) + (dy != 0) + (dz != 0);
            if (pts == 7 && nz > 1) continue;
            s.off[s.m] = dz * nn * nn + dy * nn + dx;
            s.val[s.m] = nz == 0 ? 6.0 : -1.0 / (1 + nz);
            s.m++;
         }
   unsigned char *pat;
   unsigned long long *mt;
   CK(hipMalloc(&pat, n / 2));
   CK(hipMemset(pat, 0, n / 2));
   std::vector<unsigned long long> hm(4, ~0ULL);
   hm[1] = ~0ULL ^ 1;
   CK(hipMalloc(&mt, 32));
   CK(hipMemcpy(mt, hm.data(), 32, hipMemcpyHostToDevice));
   const double bytes = 24.0 * n;
   const int gp = (int)((n / 2 + 255) / 256), gr = (int)((n + 255) / 256);
   if (pts == 7) {
      const int gq = (int)((n / 4 + 255) / 256);
      for (int rep = 0; rep < 2; rep++) {
         const float a = timeit([&] { pair_nt_k<7, 0, false><<<gp, 256>>>(f, xc, r, n, s); }, 20);
         const float b = timeit([&] { pair_nt_k<7, 1, false><<<gp, 256>>>(f, xc, r, n, s); }, 20);
         const float c = timeit([&] { pair_nt_k<7, 2, false><<<gp, 256>>>(f, xc, r, n, s); }, 20);
         const float d = timeit([&] { pair_nt_k<7, 1, true><<<gp, 256>>>(f, xc, r, n, s); }, 20);
         const float e = timeit([&] { quad_k<7, 0><<<gq, 256>>>(f, xc, r, n, s); }, 20);
         const float g = timeit([&] { quad_k<7, 1><<<gq, 256>>>(f, xc, r, n, s); }, 20);
         const float t0 = timeit([&] { triad_k<0><<<gp, 256>>>(f, xc, r, n); }, 20);
         const float t1 = timeit([&] { triad_k<1><<<gp, 256>>>(f, xc, r, n); }, 20);
         printf("%d^3 7-pt variants (GB/s of 24n): pair %.0f  nt(f,r) %.0f  nt(r) %.0f  nt+xcd %.0f  quad %.0f  "
                "quad+nt %.0f | triad %.0f  triad+nt %.0f\n",
                nn, bytes / a / 1e6, bytes / b / 1e6, bytes / c / 1e6, bytes / d / 1e6, bytes / e / 1e6,
                bytes / g / 1e6, bytes / t0 / 1e6, bytes / t1 / 1e6);
      }
   }
   for (int rep = 0; rep < 3; rep++) {
      float t1, t2, t3;
      if (pts == 27) {
         t1 = timeit([&] { pair_k<27><<<gp, 256>>>(f, xc, r, n, s); }, 20);
         t2 = timeit([&] { pair_mask_k<27><<<gp, 256>>>(f, xc, r, n, s, pat, mt, 4); }, 20);
         t3 = timeit([&] { row_k<27><<<gr, 256>>>(f, xc, r, n, s); }, 20);
      } else {
         t1 = timeit([&] { pair_k<7><<<gp, 256>>>(f, xc, r, n, s); }, 20);
         t2 = timeit([&] { pair_mask_k<7><<<gp, 256>>>(f, xc, r, n, s, pat, mt, 4); }, 20);
         t3 = timeit([&] { row_k<7><<<gr, 256>>>(f, xc, r, n, s); }, 20);
      }
      printf("%d^3 %2d-pt: pair %.3f ms (%.0f GB/s)  pair+mask %.3f ms  row %.3f ms (%.0f GB/s)\n", nn, pts, t1,
             bytes / t1 / 1e6, t2, t3, bytes / t3 / 1e6);
   }
   CK(hipFree(f));
   CK(hipFree(r));
   CK(hipFree(x));
   CK(hipFree(pat));
   CK(hipFree(mt));
}

int main()
{
   run(256, 27);
   run(512, 7);
   run(256, 7);
   return 0;
}
