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
