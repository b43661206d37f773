// amg_setup.cpp -- structured problem and hierarchy generator (setup phase).
//
// The reference builds its 7-pt Laplacian with hypre's GenerateLaplacian
// (BuildHypreMatrix.cpp:250-275, diag 6 / off -1, lexicographic x fastest,
// diagonal first) and takes its level operators from BoomerAMG.  BoomerAMG
// is not available here, so the hierarchy is an INPUT of the hot path: this
// file provides a deterministic geometric one.  Every operator is a Kronecker
// sum of 1-D tridiagonals,
//     A_l = T_x (x) M_y (x) M_z + M_x (x) T_y (x) M_z + M_x (x) M_y (x) T_z,
// with A_0 the 7-pt Laplacian (T = tridiag(-1,2,-1), M = I), P_l the tensor
// product of 1-D linear interpolation (or 2:1 aggregation) and the Galerkin
// product A_{l+1} = P_l^T A_l P_l evaluated axis by axis:
// T_{l+1} = P1^T T_l P1, M_{l+1} = P1^T M_l P1.  All entries are dyadic
// rationals with few significant bits, so the values are exactly those a
// generic CSR SpGEMM R*A*P produces (tests/test_generator.py checks this bit
// for bit against the oracle's SpGEMM).  Rows hold the diagonal first, then
// the remaining columns ascending (hypre's convention); R = P^T holds its
// columns ascending.
#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "amg_internal.h"

namespace {

struct Tri {
   std::vector<double> lo, di, up; // lo[i] = M[i][i-1], up[i] = M[i][i+1]
   int n() const { return (int)di.size(); }
   double at(int i, int d) const
   {
      if (d == 0) return di[i];
      if (d < 0) return i > 0 ? lo[i] : 0.0;
      return i + 1 < n() ? up[i] : 0.0;
   }
};

struct P1 {
   int nf = 0, nc = 0;
   // fine row i: cnt[i] entries (col, w) in ascending col order
   std::vector<int> cnt;
   std::vector<std::array<int, 2>> col;
   std::vector<std::array<double, 2>> w;
   // transpose: coarse row c: fine entries ascending
   std::vector<std::vector<std::pair<int, double>>> tr;
};

P1 make_p1(int nf, int interp)
{
   P1 p;
   p.nf = nf;
   p.nc = (interp == AMG_INTERP_AGGREGATE) ? (nf + 1) / 2 : nf / 2;
   p.cnt.assign(nf, 0);
   p.col.assign(nf, {0, 0});
   p.w.assign(nf, {0.0, 0.0});
   for (int i = 0; i < nf; i++) {
      if (interp == AMG_INTERP_AGGREGATE) {
         p.cnt[i] = 1;
         p.col[i][0] = i / 2;
         p.w[i][0] = 1.0;
      } else if (i & 1) {
         p.cnt[i] = 1;
         p.col[i][0] = (i - 1) / 2;
         p.w[i][0] = 1.0;
      } else {
         const int k = i / 2;
         int c = 0;
         if (k - 1 >= 0) {
            p.col[i][c] = k - 1;
            p.w[i][c] = 0.5;
            c++;
         }
         if (k < p.nc) {
            p.col[i][c] = k;
            p.w[i][c] = 0.5;
            c++;
         }
         p.cnt[i] = c;
      }
   }
   p.tr.assign(p.nc, {});
   for (int i = 0; i < nf; i++)
      for (int q = 0; q < p.cnt[i]; q++) p.tr[p.col[i][q]].push_back({i, p.w[i][q]});
   return p;
}

Tri galerkin(const P1 &p, const Tri &T)
{
   Tri c;
   c.lo.assign(p.nc, 0.0);
   c.di.assign(p.nc, 0.0);
   c.up.assign(p.nc, 0.0);
   for (int i = 0; i < p.nf; i++)
      for (int qa = 0; qa < p.cnt[i]; qa++) {
         const int a = p.col[i][qa];
         const double wa = p.w[i][qa];
         for (int d = -1; d <= 1; d++) {
            const int j = i + d;
            if (j < 0 || j >= p.nf) continue;
            const double t = T.at(i, d);
            if (t == 0.0) continue;
            for (int qb = 0; qb < p.cnt[j]; qb++) {
               const int b = p.col[j][qb];
               const double v = (wa * t) * p.w[j][qb];
               if (b == a)
                  c.di[a] += v;
               else if (b == a - 1)
                  c.lo[a] += v;
               else if (b == a + 1)
                  c.up[a] += v;
               else
                  std::abort(); // not tridiagonal: impossible for these P1
            }
         }
      }
   return c;
}

template <class F>
void parallel_for(int n, int nthreads, F f)
{
   if (nthreads <= 0) nthreads = (int)std::min(32u, std::max(1u, std::thread::hardware_concurrency()));
   nthreads = std::max(1, std::min(nthreads, n));
   if (nthreads == 1) {
      for (int i = 0; i < n; i++) f(i);
      return;
   }
   std::atomic<int> next{0};
   std::vector<std::thread> th;
   for (int t = 0; t < nthreads; t++)
      th.emplace_back([&]() {
         for (int i; (i = next.fetch_add(1)) < n;) f(i);
      });
   for (auto &t : th) t.join();
}

} // namespace

struct amg_gen {
   int L = 0;
   int interp = 0;
   std::vector<std::array<int, 3>> dims;
   std::vector<std::array<Tri, 3>> T, M;
   std::vector<std::array<P1, 3>> P; // level l: fine l -> coarse l+1
};

extern "C" int amg_gen_create(int nx, int ny, int nz, int interp, int max_levels, int max_coarse,
                              amg_gen **out)
{
   AMG_ARG(out && nx >= 1 && ny >= 1 && nz >= 1, "amg_gen_create: bad dimensions");
   AMG_ARG(interp == AMG_INTERP_LINEAR || interp == AMG_INTERP_AGGREGATE, "amg_gen_create: interp");
   AMG_ARG((long long)nx * ny * nz < (1LL << 31), "amg_gen_create: more than 2^31 rows");
   if (max_levels <= 0) max_levels = 25;  // SMEM_Main.cpp:28 hypre.max_levels
   if (max_coarse <= 0) max_coarse = 9;   // hypre default max coarse size
   amg_gen *g = new amg_gen();
   g->interp = interp;
   std::array<int, 3> d = {nx, ny, nz};
   std::array<Tri, 3> T0, M0;
   for (int a = 0; a < 3; a++) {
      const int n = d[a];
      T0[a].lo.assign(n, -1.0);
      T0[a].di.assign(n, 2.0);
      T0[a].up.assign(n, -1.0);
      M0[a].lo.assign(n, 0.0);
      M0[a].di.assign(n, 1.0);
      M0[a].up.assign(n, 0.0);
   }
   g->dims.push_back(d);
   g->T.push_back(T0);
   g->M.push_back(M0);
   while ((int)g->dims.size() < max_levels) {
      const auto &cd = g->dims.back();
      const long long rows = (long long)cd[0] * cd[1] * cd[2];
      if (rows <= max_coarse) break;
      bool ok = true;
      for (int a = 0; a < 3; a++) ok = ok && cd[a] >= 2;
      if (!ok) break;
      std::array<P1, 3> p;
      std::array<int, 3> nd;
      std::array<Tri, 3> Tn, Mn;
      for (int a = 0; a < 3; a++) {
         p[a] = make_p1(cd[a], interp);
         nd[a] = p[a].nc;
         Tn[a] = galerkin(p[a], g->T.back()[a]);
         Mn[a] = galerkin(p[a], g->M.back()[a]);
      }
      g->P.push_back(p);
      g->dims.push_back(nd);
      g->T.push_back(Tn);
      g->M.push_back(Mn);
   }
   g->L = (int)g->dims.size();
   *out = g;
   return AMG_OK;
}

extern "C" int amg_gen_free(amg_gen *g)
{
   delete g;
   return AMG_OK;
}

extern "C" int amg_gen_num_levels(const amg_gen *g) { return g ? g->L : -1; }

extern "C" int amg_gen_dims(const amg_gen *g, int level, int *nx, int *ny, int *nz)
{
   AMG_ARG(g && level >= 0 && level < g->L, "amg_gen_dims: bad level");
   if (nx) *nx = g->dims[level][0];
   if (ny) *ny = g->dims[level][1];
   if (nz) *nz = g->dims[level][2];
   return AMG_OK;
}

namespace {

// row (x,y,z) of A_l: calls emit(col, val) diag first then ascending
template <class E>
inline void a_row(const amg_gen *g, int l, int x, int y, int z, E emit)
{
   const auto &d = g->dims[l];
   const Tri &Tx = g->T[l][0], &Ty = g->T[l][1], &Tz = g->T[l][2];
   const Tri &Mx = g->M[l][0], &My = g->M[l][1], &Mz = g->M[l][2];
   const long long nx = d[0], nxy = (long long)d[0] * d[1];
   const long long row = x + nx * y + nxy * z;
   auto value = [&](int dx, int dy, int dz) {
      const double tx = Tx.at(x, dx), ty = Ty.at(y, dy), tz = Tz.at(z, dz);
      const double mx = Mx.at(x, dx), my = My.at(y, dy), mz = Mz.at(z, dz);
      return ((tx * my) * mz + (mx * ty) * mz) + (mx * my) * tz;
   };
   emit((int)row, value(0, 0, 0));
   for (int dz = -1; dz <= 1; dz++) {
      if (z + dz < 0 || z + dz >= d[2]) continue;
      for (int dy = -1; dy <= 1; dy++) {
         if (y + dy < 0 || y + dy >= d[1]) continue;
         for (int dx = -1; dx <= 1; dx++) {
            if (x + dx < 0 || x + dx >= d[0]) continue;
            if (dx == 0 && dy == 0 && dz == 0) continue;
            const double v = value(dx, dy, dz);
            if (v == 0.0) continue;
            emit((int)(row + dx + nx * dy + nxy * dz), v);
         }
      }
   }
}

template <class E>
inline void p_row(const amg_gen *g, int l, int x, int y, int z, E emit)
{
   const auto &cd = g->dims[l + 1];
   const P1 &px = g->P[l][0], &py = g->P[l][1], &pz = g->P[l][2];
   const long long cnx = cd[0], cnxy = (long long)cd[0] * cd[1];
   for (int qz = 0; qz < pz.cnt[z]; qz++)
      for (int qy = 0; qy < py.cnt[y]; qy++)
         for (int qx = 0; qx < px.cnt[x]; qx++) {
            const double v = (px.w[x][qx] * py.w[y][qy]) * pz.w[z][qz];
            emit((int)(px.col[x][qx] + cnx * py.col[y][qy] + cnxy * pz.col[z][qz]), v);
         }
}

template <class E>
inline void r_row(const amg_gen *g, int l, int cx, int cy, int cz, E emit)
{
   const auto &fd = g->dims[l];
   const P1 &px = g->P[l][0], &py = g->P[l][1], &pz = g->P[l][2];
   const long long nx = fd[0], nxy = (long long)fd[0] * fd[1];
   for (const auto &ez : pz.tr[cz])
      for (const auto &ey : py.tr[cy])
         for (const auto &ex : px.tr[cx]) {
            const double v = (ex.second * ey.second) * ez.second;
            emit((int)(ex.first + nx * ey.first + nxy * ez.first), v);
         }
}

template <class E>
inline void any_row(const amg_gen *g, int which, int l, int x, int y, int z, E emit)
{
   if (which == AMG_GEN_A)
      a_row(g, l, x, y, z, emit);
   else if (which == AMG_GEN_P)
      p_row(g, l, x, y, z, emit);
   else
      r_row(g, l, x, y, z, emit);
}

// grid whose rows the operator has
inline const std::array<int, 3> &row_grid(const amg_gen *g, int which, int l)
{
   return (which == AMG_GEN_R) ? g->dims[l + 1] : g->dims[l];
}

int check_op(const amg_gen *g, int which, int l, int z0, int z1)
{
   AMG_ARG(g, "amg_gen: null generator");
   AMG_ARG(which >= 0 && which <= 2, "amg_gen: bad operator %d", which);
   AMG_ARG(l >= 0 && l < g->L && (which == AMG_GEN_A || l < g->L - 1), "amg_gen: bad level %d", l);
   const auto &d = row_grid(g, which, l);
   AMG_ARG(z0 >= 0 && z1 <= d[2] && z0 <= z1, "amg_gen: plane range [%d,%d) of %d", z0, z1, d[2]);
   return AMG_OK;
}

long long plane_nnz(const amg_gen *g, int which, int l, int z)
{
   const auto &d = row_grid(g, which, l);
   long long c = 0;
   for (int y = 0; y < d[1]; y++)
      for (int x = 0; x < d[0]; x++) any_row(g, which, l, x, y, z, [&](int, double) { c++; });
   return c;
}

} // namespace

extern "C" long long amg_gen_nnz(const amg_gen *g, int which, int level, int z0, int z1)
{
   if (check_op(g, which, level, z0, z1) != AMG_OK) return -1;
   std::vector<long long> pc(z1 - z0, 0);
   parallel_for(z1 - z0, 0, [&](int i) { pc[i] = plane_nnz(g, which, level, z0 + i); });
   long long s = 0;
   for (auto v : pc) s += v;
   return s;
}

extern "C" int amg_gen_fill(const amg_gen *g, int which, int level, int z0, int z1, int *rowptr,
                            int *col, double *val, int nthreads)
{
   AMG_TRY(check_op(g, which, level, z0, z1));
   AMG_ARG(rowptr && col && val, "amg_gen_fill: null output");
   const auto &d = row_grid(g, which, level);
   const long long plane = (long long)d[0] * d[1];
   const int np = z1 - z0;
   std::vector<long long> pc(np + 1, 0);
   parallel_for(np, nthreads, [&](int i) { pc[i + 1] = plane_nnz(g, which, level, z0 + i); });
   for (int i = 0; i < np; i++) pc[i + 1] += pc[i];
   AMG_ARG(pc[np] < (1LL << 31), "amg_gen_fill: %lld nnz exceeds int32 CSR", pc[np]);
   rowptr[0] = 0;
   parallel_for(np, nthreads, [&](int i) {
      const int z = z0 + i;
      long long k = pc[i];
      long long r = plane * i;
      for (int y = 0; y < d[1]; y++)
         for (int x = 0; x < d[0]; x++) {
            any_row(g, which, level, x, y, z, [&](int c, double v) {
               col[k] = c;
               val[k] = v;
               k++;
            });
            rowptr[++r] = (int)k;
         }
   });
   return AMG_OK;
}

// RandDouble(lo,hi) after srand(0) (SMEM_Setup.cpp:1729-1745, Misc.cpp:282-285):
// entries [r0, r1) of the global sequence
extern "C" int amg_rhs_rand(long long r0, long long r1, double lo, double hi, double *out)
{
   AMG_ARG(out && r0 >= 0 && r1 >= r0, "amg_rhs_rand: bad range");
   srand(0);
   for (long long i = 0; i < r0; i++) (void)rand();
   for (long long i = r0; i < r1; i++) out[i - r0] = lo + (hi - lo) * ((double)rand() / RAND_MAX);
   return AMG_OK;
}

// device-side generation: rows computed on the host in plane batches and
// streamed into the device CSR (keeps host memory bounded for 512^3).
int amg_mat_create_device(amg_ctx *c, int nrows, int ncols, long long nnz, amg_mat **out);
int amg_mat_finish(amg_mat *A);

// Rows of planes [e0, e1) of the operator's row grid (rows of planes outside
// [o0, o1) are "ghost" rows: A keeps its whole row when every column lies in
// the column planes -- the fused residual + restriction forms residuals of the
// first ghost plane -- else only its diagonal entry; P / R keep none),
// columns shifted to planes [ce0, ce1) of the column grid (every kept column
// must lie there).  The whole operator: e0 = o0 = 0, e1 = o1 = nz, ce0 = 0,
// ce1 = nz of the column grid.  A z-slab's extended operator: the owned planes
// [o0, o1) plus ghost planes around them (amg_dist.cpp, slab hierarchies).
int amg_gen_register_ext(amg_ctx *ctx, const amg_gen *g, int which, int level, int e0, int e1, int o0, int o1,
                         int ce0, int ce1, amg_mat **out)
{
   AMG_TRY(check_op(g, which, level, e0, e1));
   AMG_ARG(ctx && out, "amg_gen_register: null argument");
   AMG_ARG(e0 <= o0 && o0 <= o1 && o1 <= e1, "amg_gen_register: owned planes [%d,%d) outside [%d,%d)", o0, o1, e0,
           e1);
   const auto &d = row_grid(g, which, level);
   const long long plane = (long long)d[0] * d[1];
   const long long nrows = plane * (e1 - e0);
   const auto &cdim = (which == AMG_GEN_A) ? g->dims[level]
                      : (which == AMG_GEN_P) ? g->dims[level + 1]
                                             : g->dims[level];
   const long long cplane = (long long)cdim[0] * cdim[1];
   AMG_ARG(ce0 >= 0 && ce0 <= ce1 && ce1 <= cdim[2], "amg_gen_register: column planes [%d,%d) of %d", ce0, ce1,
           cdim[2]);
   const long long ncols = cplane * (ce1 - ce0), cshift = cplane * ce0;
   // A's ghost rows: the whole row if it fits the column planes, else the diagonal
   auto ghost_keep = [&](const int *rp, const int *cj, long long r, long long &cnt) {
      const long long kb = rp[r], ke = rp[r + 1];
      bool fits = true;
      for (long long k = kb; k < ke; k++) {
         const long long c = (long long)cj[k] - cshift;
         fits = fits && c >= 0 && c < ncols;
      }
      cnt = fits ? ke - kb : std::min(ke - kb, 1LL);
      return fits;
   };
   long long ghost_nnz = 0;
   if (which == AMG_GEN_A) {
      for (int z = e0; z < e1; z++) {
         if (z >= o0 && z < o1) continue;
         const long long pn = amg_gen_nnz(g, which, level, z, z + 1);
         std::vector<int> rp(plane + 1), cj(std::max(1LL, pn));
         std::vector<double> cv(std::max(1LL, pn));
         AMG_TRY(amg_gen_fill(g, which, level, z, z + 1, rp.data(), cj.data(), cv.data(), 0));
         for (long long q = 0; q < plane; q++) {
            long long cnt;
            ghost_keep(rp.data(), cj.data(), q, cnt);
            ghost_nnz += cnt;
         }
      }
   }
   const long long nnz = amg_gen_nnz(g, which, level, o0, o1) + ghost_nnz;
   AMG_ARG(nnz >= 0 && nnz < (1LL << 31) - AMG_NNZ_PAD, "amg_gen_register: nnz %lld", nnz);
   AMG_ARG(nrows < (1LL << 31) && ncols < (1LL << 31), "amg_gen_register: %lld x %lld exceeds int32", nrows, ncols);
   amg_mat *A = nullptr;
   AMG_TRY(amg_mat_create_device(ctx, (int)nrows, (int)std::max(1LL, ncols), nnz, &A));
   // batches of planes, double-buffered through pinned host memory
   const int np = e1 - e0;
   // ~16M entries (~190 MB of pinned staging) per batch
   const int batch =
      std::max(1, (int)std::min<long long>(np, (16LL << 20) / 27 / std::max(1LL, plane)));
   std::vector<int> rp_all(nrows + 1);
   int *hcol[2] = {nullptr, nullptr};
   double *hval[2] = {nullptr, nullptr};
   const long long cap = (long long)batch * plane * 27 + 64;
   for (int b = 0; b < 2; b++) {
      AMG_HIP(hipHostMalloc(&hcol[b], cap * sizeof(int)));
      AMG_HIP(hipHostMalloc(&hval[b], cap * sizeof(double)));
   }
   hipEvent_t done[2];
   AMG_HIP(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
   AMG_HIP(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
   long long base = 0;
   int buf = 0;
   bool used[2] = {false, false};
   int bad = 0;
   for (int zb = 0; zb < np; zb += batch) {
      const int nb = std::min(batch, np - zb);
      if (used[buf]) AMG_HIP(hipEventSynchronize(done[buf]));
      std::vector<int> rp(nb * plane + 1);
      AMG_TRY(amg_gen_fill(g, which, level, e0 + zb, e0 + zb + nb, rp.data(), hcol[buf], hval[buf], 0));
      // ghost rows and the column shift, compacted in place (k_out <= k_in)
      long long ko = 0;
      for (int pz = 0; pz < nb; pz++) {
         const int z = e0 + zb + pz;
         const bool ghost = z < o0 || z >= o1;
         for (long long q = 0; q < plane; q++) {
            const long long r = (long long)pz * plane + q;
            const long long kb = rp[r], ke = rp[r + 1];
            long long keep_to = ke;
            if (ghost) {
               long long cnt = 0;
               if (which == AMG_GEN_A) ghost_keep(rp.data(), hcol[buf], r, cnt);
               keep_to = kb + cnt;
            }
            for (long long k = kb; k < keep_to; k++) {
               const long long c = (long long)hcol[buf][k] - cshift;
               if (c < 0 || c >= ncols) bad = 1;
               hcol[buf][ko] = (int)c;
               hval[buf][ko] = hval[buf][k];
               ko++;
            }
            rp_all[zb * plane + r + 1] = (int)(base + ko);
         }
      }
      AMG_ARG(!bad, "amg_gen_register: a column of an owned row lies outside column planes [%d,%d)", ce0, ce1);
      AMG_HIP(hipMemcpyAsync(A->col + base, hcol[buf], ko * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
      AMG_HIP(hipMemcpyAsync(A->val + base, hval[buf], ko * sizeof(double), hipMemcpyHostToDevice,
                             ctx->stream));
      AMG_HIP(hipEventRecord(done[buf], ctx->stream));
      used[buf] = true;
      base += ko;
      buf ^= 1;
   }
   AMG_ARG(base == nnz, "amg_gen_register: %lld entries written, %lld expected", base, nnz);
   rp_all[0] = 0;
   AMG_HIP(hipMemcpyAsync(A->rowptr, rp_all.data(), (nrows + 1) * sizeof(int), hipMemcpyHostToDevice,
                          ctx->stream));
   AMG_TRY(amg_mat_finish(A));
   AMG_HIP(hipStreamSynchronize(ctx->stream));
   for (int b = 0; b < 2; b++) {
      hipHostFree(hcol[b]);
      hipHostFree(hval[b]);
      hipEventDestroy(done[b]);
   }
   *out = A;
   return AMG_OK;
}

extern "C" int amg_gen_register(amg_ctx *ctx, const amg_gen *g, int which, int level, int z0,
                                int z1, amg_mat **out)
{
   AMG_TRY(check_op(g, which, level, z0, z1));
   const int cl = (which == AMG_GEN_P) ? level + 1 : level;
   return amg_gen_register_ext(ctx, g, which, level, z0, z1, z0, z1, 0, g->dims[cl][2], out);
}
