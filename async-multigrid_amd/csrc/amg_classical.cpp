// amg_classical.cpp -- in-house classical AMG setup (host, C++): the hierarchy
// the reference obtains from hypre BoomerAMG (SMEM_Setup.cpp:55-70 with the
// parameters of SMEM_Main.cpp:29-35 / SMEM_Setup.cpp:1670-1690, DMEM_Main.cpp:38-49
// / DMEM_Setup.cpp:530-552).  hypre is not part of the reference tree, so its
// published algorithms are restated here; agreement with hypre's own output is
// parity unpinned.
//
//   strength     classical, theta, max_row_sum (hypre CreateS), one function
//                per unknown (num_functions, "unknown" approach)
//   coarsening   HMIS (coarsen_type 10: Ruge-Stueben first pass; in one process
//                it decides every point) or PMIS (8 / 9: independent sets of a
//                random-perturbed measure on S + S^T)
//   interpolation extended+i (interp_type 6, De Sterck, Falgout, Nolting, Yang,
//                "Distance-two interpolation for parallel algebraic multigrid",
//                NLAA 2008) or direct (interp_type 3)
//   Galerkin     A_c = R A P with R = P^T (construct_R_flag, SMEM_Setup.cpp:1405-1419),
//                Gustavson products accumulated in row-entry order, columns
//                sorted, diagonal first
// Levels are built until the coarse operator has at most max_coarse_size rows,
// coarsening stalls, or max_levels is reached.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <set>
#include <thread>
#include <vector>

#include "amg_internal.h"

// amg_spgemm.hip: C = A B on a GPU, bit-identical to spgemm() below
int amg_spgemm_device(int device, int An, const std::vector<int> &arp, const std::vector<int> &acj,
                      const std::vector<double> &av, int Bn, const std::vector<int> &brp,
                      const std::vector<int> &bcj, const std::vector<double> &bv, int Bm, std::vector<int> &crp,
                      std::vector<int> &ccj, std::vector<double> &cv);
// A_c = R (A P) on a GPU with A P kept on the device, bit-identical to two spgemm() calls
int amg_rap_device(int device, int An, const std::vector<int> &arp, const std::vector<int> &acj,
                   const std::vector<double> &av, const std::vector<int> &prp, const std::vector<int> &pcj,
                   const std::vector<double> &pv, int Pm, int Rn, const std::vector<int> &rrp,
                   const std::vector<int> &rcj, const std::vector<double> &rv, std::vector<int> &crp,
                   std::vector<int> &ccj, std::vector<double> &cv);

namespace {

struct HCsr {
   int n = 0, m = 0;
   std::vector<int> rp{0}, cj;
   std::vector<double> v;
   long long nnz() const { return (long long)cj.size(); }
};

constexpr int CF_U = 0, CF_C = 1, CF_F = -1;

// host threads for the row-parallel setup phases (strength, interpolation):
// AMG_SETUP_THREADS (any level of at least 64 rows), else the hardware's, at
// most 16, on levels of at least 16384 rows
int setup_threads(int n)
{
   if (const char *v = std::getenv("AMG_SETUP_THREADS"))
      return n < 64 ? 1 : std::max(1, std::min(64, std::atoi(v)));
   if (n < 16384) return 1;
   return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// M's rows built in parallel over contiguous row ranges: fn(r0, r1, cnt, cj, v)
// appends rows r0..r1-1 in order to its own cj / v and sets cnt[r]; the ranges
// are then concatenated in row order, so M is the same as a sequential build
template <class Fn>
void rows_parallel(int n, HCsr &M, Fn fn)
{
   const int T = setup_threads(n);
   std::vector<std::vector<int>> cjs(T);
   std::vector<std::vector<double>> vs(T);
   std::vector<int> cnt(n, 0);
   std::vector<std::thread> th;
   for (int t = 0; t < T; t++) {
      const int r0 = (int)((long long)n * t / T), r1 = (int)((long long)n * (t + 1) / T);
      if (T == 1)
         fn(r0, r1, cnt, cjs[t], vs[t]);
      else
         th.emplace_back([&, t, r0, r1] { fn(r0, r1, cnt, cjs[t], vs[t]); });
   }
   for (auto &x : th) x.join();
   M.rp.assign(n + 1, 0);
   for (int i = 0; i < n; i++) M.rp[i + 1] = M.rp[i] + cnt[i];
   M.cj.clear();
   M.v.clear();
   M.cj.reserve(M.rp[n]);
   for (int t = 0; t < T; t++) {
      M.cj.insert(M.cj.end(), cjs[t].begin(), cjs[t].end());
      M.v.insert(M.v.end(), vs[t].begin(), vs[t].end());
   }
}

// hypre_BoomerAMGCreateS (serial): row scale = most negative off-diagonal for
// a non-negative diagonal (most positive for a negative one); a_ij is strong
// when it exceeds theta times that scale in the diagonal's opposite sign.
// With max_row_sum < 1 a row whose |row sum| exceeds max_row_sum |a_ii| has
// only weak connections.  Different functions never couple.
void strength(const HCsr &A, double theta, double max_row_sum, int nfun, HCsr &S)
{
   S = HCsr();
   S.n = S.m = A.n;
   rows_parallel(A.n, S, [&](int r0, int r1, std::vector<int> &cnt, std::vector<int> &cj, std::vector<double> &) {
      for (int i = r0; i < r1; i++) {
         const size_t before = cj.size();
         double diag = 0.0, row_scale = 0.0, row_sum = 0.0;
         for (int k = A.rp[i]; k < A.rp[i + 1]; k++)
            if (A.cj[k] == i) diag = A.v[k];
         for (int k = A.rp[i]; k < A.rp[i + 1]; k++) {
            const int j = A.cj[k];
            row_sum += A.v[k];
            if (j == i || j % nfun != i % nfun) continue;
            row_scale = diag < 0 ? std::max(row_scale, A.v[k]) : std::min(row_scale, A.v[k]);
         }
         const bool all_weak = max_row_sum < 1.0 && std::fabs(row_sum) > std::fabs(diag) * max_row_sum;
         if (!all_weak)
            for (int k = A.rp[i]; k < A.rp[i + 1]; k++) {
               const int j = A.cj[k];
               if (j == i || j % nfun != i % nfun) continue;
               const bool strong = diag < 0 ? A.v[k] > theta * row_scale : A.v[k] < theta * row_scale;
               if (strong) cj.push_back(j);
            }
         cnt[i] = (int)(cj.size() - before);
      }
   });
}

void transpose_pattern(const HCsr &S, HCsr &T)
{
   T = HCsr();
   T.n = S.m;
   T.m = S.n;
   T.rp.assign(T.n + 1, 0);
   for (int j : S.cj) T.rp[j + 1]++;
   for (int c = 0; c < T.n; c++) T.rp[c + 1] += T.rp[c];
   T.cj.resize(S.cj.size());
   std::vector<int> pos(T.rp.begin(), T.rp.end() - 1);
   for (int r = 0; r < S.n; r++)
      for (int k = S.rp[r]; k < S.rp[r + 1]; k++) T.cj[pos[S.cj[k]]++] = r;
}

// counting-sort transpose with values; rows of the result hold ascending source rows
void transpose(const HCsr &A, HCsr &T)
{
   T = HCsr();
   T.n = A.m;
   T.m = A.n;
   T.rp.assign(T.n + 1, 0);
   for (int j : A.cj) T.rp[j + 1]++;
   for (int c = 0; c < T.n; c++) T.rp[c + 1] += T.rp[c];
   T.cj.resize(A.cj.size());
   T.v.resize(A.cj.size());
   std::vector<int> pos(T.rp.begin(), T.rp.end() - 1);
   for (int r = 0; r < A.n; r++)
      for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
         const int p = pos[A.cj[k]]++;
         T.cj[p] = r;
         T.v[p] = A.v[k];
      }
}

void diag_first(HCsr &M)
{
   if (M.n != M.m) return;
   for (int r = 0; r < M.n; r++) {
      const int s = M.rp[r], e = M.rp[r + 1];
      for (int k = s; k < e; k++)
         if (M.cj[k] == r) {
            const int cj = M.cj[k];
            const double cv = M.v[k];
            for (int q = k; q > s; q--) {
               M.cj[q] = M.cj[q - 1];
               M.v[q] = M.v[q - 1];
            }
            M.cj[s] = cj;
            M.v[s] = cv;
            break;
         }
   }
}

// Gustavson C = A B: accumulation in (A row entry, B row entry) order, columns
// of each row sorted, diagonal first when square
void spgemm(const HCsr &A, const HCsr &B, HCsr &C)
{
   C = HCsr();
   C.n = A.n;
   C.m = B.m;
   C.rp.assign(A.n + 1, 0);
   std::vector<int> mark(B.m, -1), cols;
   std::vector<double> acc(B.m, 0.0);
   cols.reserve(256);
   for (int r = 0; r < A.n; r++) {
      cols.clear();
      for (int ka = A.rp[r]; ka < A.rp[r + 1]; ka++) {
         const int k = A.cj[ka];
         const double av = A.v[ka];
         for (int kb = B.rp[k]; kb < B.rp[k + 1]; kb++) {
            const int c = B.cj[kb];
            if (mark[c] != r) {
               mark[c] = r;
               acc[c] = 0.0;
               cols.push_back(c);
            }
            acc[c] += av * B.v[kb];
         }
      }
      std::sort(cols.begin(), cols.end());
      for (int c : cols) {
         C.cj.push_back(c);
         C.v.push_back(acc[c]);
      }
      C.rp[r + 1] = (int)C.cj.size();
   }
   diag_first(C);
}

uint64_t splitmix64(uint64_t x)
{
   x += 0x9e3779b97f4a7c15ULL;
   x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
   x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
   return x ^ (x >> 31);
}

// Ruge-Stueben first pass (the whole of HMIS in one process): pick the
// undecided point of largest measure |S^T_i| (ties: the larger index), make it
// C, its undecided strong dependents F, and raise the measure of the points
// those new F points depend on; points the new C point depends on lose one.
// Points of measure 0 are F.
void coarsen_rs(const HCsr &S, const HCsr &ST, std::vector<int> &cf)
{
   const int n = S.n;
   cf.assign(n, CF_U);
   std::vector<int> meas(n);
   std::set<std::pair<int, int>> q; // (measure, index)
   for (int i = 0; i < n; i++) {
      meas[i] = ST.rp[i + 1] - ST.rp[i];
      if (meas[i] == 0)
         cf[i] = CF_F;
      else
         q.insert({meas[i], i});
   }
   auto bump = [&](int k, int d) {
      q.erase({meas[k], k});
      meas[k] += d;
      if (meas[k] <= 0) {
         cf[k] = CF_F;
      } else {
         q.insert({meas[k], k});
      }
   };
   while (!q.empty()) {
      const int i = std::prev(q.end())->second;
      q.erase(std::prev(q.end()));
      cf[i] = CF_C;
      for (int a = ST.rp[i]; a < ST.rp[i + 1]; a++) {
         const int j = ST.cj[a];
         if (cf[j] != CF_U) continue;
         q.erase({meas[j], j});
         cf[j] = CF_F;
         for (int b = S.rp[j]; b < S.rp[j + 1]; b++) {
            const int k = S.cj[b];
            if (cf[k] == CF_U) bump(k, +1);
         }
      }
      for (int a = S.rp[i]; a < S.rp[i + 1]; a++) {
         const int j = S.cj[a];
         if (cf[j] == CF_U) bump(j, -1);
      }
   }
}

// PMIS: measure |S^T_i| + a uniform [0,1) draw per point (splitmix64 of the
// seed and the index); points below 1 are F; then repeatedly every undecided
// point whose measure beats all undecided neighbours in S + S^T becomes C and
// its undecided strong dependents become F.
void coarsen_pmis(const HCsr &S, const HCsr &ST, uint64_t seed, std::vector<int> &cf)
{
   const int n = S.n;
   cf.assign(n, CF_U);
   std::vector<double> meas(n);
   int left = 0;
   for (int i = 0; i < n; i++) {
      const double r = (double)(splitmix64(seed ^ (uint64_t)i * 0x2545f4914f6cdd1dULL) >> 11) * 0x1.0p-53;
      meas[i] = (ST.rp[i + 1] - ST.rp[i]) + r;
      if (meas[i] < 1.0)
         cf[i] = CF_F;
      else
         left++;
   }
   std::vector<int> newc;
   while (left > 0) {
      newc.clear();
      for (int i = 0; i < n; i++) {
         if (cf[i] != CF_U) continue;
         bool best = true;
         for (int a = S.rp[i]; best && a < S.rp[i + 1]; a++) {
            const int j = S.cj[a];
            if (cf[j] == CF_U && meas[j] >= meas[i]) best = false;
         }
         for (int a = ST.rp[i]; best && a < ST.rp[i + 1]; a++) {
            const int j = ST.cj[a];
            if (cf[j] == CF_U && meas[j] >= meas[i]) best = false;
         }
         if (best) newc.push_back(i);
      }
      if (newc.empty()) break; // cannot happen with distinct measures
      for (int c : newc) {
         cf[c] = CF_C;
         left--;
      }
      for (int c : newc)
         for (int a = ST.rp[c]; a < ST.rp[c + 1]; a++) {
            const int j = ST.cj[a];
            if (cf[j] == CF_U) {
               cf[j] = CF_F;
               left--;
            }
         }
   }
   for (int i = 0; i < n; i++)
      if (cf[i] == CF_U) cf[i] = CF_F;
}

// interpolation: C rows inject; F rows follow extended+i (interp 6) or direct
// (interp 3).  ext+i for F point i, with S_i its strong neighbours:
//   C^_i = (S_i n C) u U_{k in S_i n F} (S_k n C)
//   abar_kl = a_kl when a_kl and a_kk differ in sign, else 0
//   d_k = sum_{l in C^_i u {i}} abar_kl       (k a strong F neighbour)
//   atil_ii = a_ii + sum of a_in over neighbours n outside C^_i u (S_i n F)
//             + sum_k a_ik abar_ki / d_k
//   w_ij = -(a_ij + sum_k a_ik abar_kj / d_k) / atil_ii,   j in C^_i
// a strong F neighbour with d_k = 0 is lumped into atil_ii; couplings to
// another function are left out.  Direct: C^_i = S_i n C,
//   w_ij = -(sum_{n != i} a_in / sum_{j in C^_i} a_ij) a_ij / a_ii.
void interpolation(const HCsr &A, const HCsr &S, const std::vector<int> &cf, int type, int nfun, HCsr &P,
                   int *nc_out)
{
   const int n = A.n;
   std::vector<int> cidx(n, -1);
   int nc = 0;
   for (int i = 0; i < n; i++)
      if (cf[i] == CF_C) cidx[i] = nc++;
   *nc_out = nc;
   P = HCsr();
   P.n = n;
   P.m = nc;
   auto aval = [&](int k, int l) -> double { // a_kl by search (rows are short)
      for (int q = A.rp[k]; q < A.rp[k + 1]; q++)
         if (A.cj[q] == l) return A.v[q];
      return 0.0;
   };
   auto diag_of = [&](int k) { return aval(k, k); };
   rows_parallel(n, P, [&](int r0, int r1, std::vector<int> &cnt, std::vector<int> &pcj, std::vector<double> &pv) {
   std::vector<int> mark(n, -1), smark(n, -1), chat;
   std::vector<double> num(n, 0.0);
   for (int i = r0; i < r1; i++) {
      const size_t before = pcj.size();
      if (cf[i] == CF_C) {
         pcj.push_back(cidx[i]);
         pv.push_back(1.0);
         cnt[i] = 1;
         continue;
      }
      for (int a = S.rp[i]; a < S.rp[i + 1]; a++) smark[S.cj[a]] = i;
      chat.clear();
      auto add_c = [&](int j) {
         if (mark[j] != i) {
            mark[j] = i;
            num[j] = 0.0;
            chat.push_back(j);
         }
      };
      const double aii = diag_of(i);
      if (type == 3) { // direct
         double sum_all = 0.0, sum_c = 0.0;
         for (int q = A.rp[i]; q < A.rp[i + 1]; q++) {
            const int j = A.cj[q];
            if (j == i || j % nfun != i % nfun) continue;
            sum_all += A.v[q];
            if (smark[j] == i && cf[j] == CF_C) {
               add_c(j);
               num[j] += A.v[q];
               sum_c += A.v[q];
            }
         }
         std::sort(chat.begin(), chat.end());
         if (sum_c != 0.0 && aii != 0.0) {
            const double alpha = sum_all / sum_c;
            for (int j : chat) {
               pcj.push_back(cidx[j]);
               pv.push_back(-alpha * num[j] / aii);
            }
         }
         cnt[i] = (int)(pcj.size() - before);
         continue;
      }
      // extended+i
      for (int a = S.rp[i]; a < S.rp[i + 1]; a++) {
         const int k = S.cj[a];
         if (cf[k] == CF_C) {
            add_c(k);
         } else {
            for (int b = S.rp[k]; b < S.rp[k + 1]; b++)
               if (cf[S.cj[b]] == CF_C) add_c(S.cj[b]);
         }
      }
      double atil = aii;
      for (int q = A.rp[i]; q < A.rp[i + 1]; q++) {
         const int j = A.cj[q];
         if (j == i) continue;
         const double aij = A.v[q];
         if (j % nfun != i % nfun) {
            continue; // another function: not part of the unknown's operator (hypre skips it)
         } else if (mark[j] == i) {
            num[j] += aij; // j in C^_i: interpolation target
         } else if (smark[j] == i && cf[j] == CF_F) {
            const int k = j; // strong F neighbour: distribute over C^_i u {i}
            const double akk = diag_of(k);
            double dk = 0.0;
            for (int r = A.rp[k]; r < A.rp[k + 1]; r++) {
               const int l = A.cj[r];
               const double akl = A.v[r];
               if ((l == i || mark[l] == i) && akl * akk < 0.0) dk += akl;
            }
            if (dk == 0.0) {
               atil += aij;
               continue;
            }
            for (int r = A.rp[k]; r < A.rp[k + 1]; r++) {
               const int l = A.cj[r];
               const double akl = A.v[r];
               if (akl * akk >= 0.0) continue;
               if (l == i)
                  atil += aij * akl / dk;
               else if (mark[l] == i)
                  num[l] += aij * akl / dk;
            }
         } else {
            atil += aij; // weak neighbour outside C^_i
         }
      }
      std::sort(chat.begin(), chat.end());
      if (atil != 0.0)
         for (int j : chat) {
            pcj.push_back(cidx[j]);
            pv.push_back(-num[j] / atil);
         }
      cnt[i] = (int)(pcj.size() - before);
   }
   });
}

} // namespace

struct amg_classical {
   std::vector<HCsr> A, P, R;
   std::vector<std::vector<int>> cf;
};

extern "C" void amg_classical_opts_default(amg_classical_opts *o)
{
   // SMEM_Main.cpp:29-35 + SMEM_Setup.cpp:1678 (HMIS, ext+i, theta 0.25, max row sum 1)
   o->coarsen_type = AMG_COARSEN_HMIS;
   o->interp_type = AMG_CLASSICAL_EXT_I;
   o->strong_threshold = 0.25;
   o->max_row_sum = 1.0;
   o->max_levels = 25;
   o->max_coarse_size = 9; // hypre's default
   o->num_functions = 1;
   o->seed = 2747;
   o->device = -1;
}

extern "C" int amg_classical_setup(const amg_classical_opts *o, int n, const int *rowptr, const int *col,
                                   const double *val, amg_classical **out)
{
   AMG_ARG(o && out && rowptr && n > 0, "amg_classical_setup: bad argument");
   AMG_ARG(o->coarsen_type == AMG_COARSEN_HMIS || o->coarsen_type == AMG_COARSEN_PMIS ||
              o->coarsen_type == AMG_COARSEN_PMIS_FIXED,
           "amg_classical_setup: coarsen_type %d (8 PMIS, 9 PMIS fixed seed, 10 HMIS)", o->coarsen_type);
   AMG_ARG(o->interp_type == AMG_CLASSICAL_EXT_I || o->interp_type == AMG_CLASSICAL_DIRECT,
           "amg_classical_setup: interp_type %d (3 direct, 6 extended+i)", o->interp_type);
   AMG_ARG(o->num_functions >= 1 && n % o->num_functions == 0, "amg_classical_setup: num_functions %d",
           o->num_functions);
   AMG_ARG(o->max_levels >= 1, "amg_classical_setup: max_levels %d", o->max_levels);
   const long long nnz = rowptr[n];
   AMG_ARG(rowptr[0] == 0 && nnz >= 0, "amg_classical_setup: rowptr");
   auto *H = new amg_classical();
   HCsr A0;
   A0.n = A0.m = n;
   A0.rp.assign(rowptr, rowptr + n + 1);
   A0.cj.assign(col, col + nnz);
   A0.v.assign(val, val + nnz);
   for (long long k = 0; k < nnz; k++)
      if (A0.cj[k] < 0 || A0.cj[k] >= n) {
         delete H;
         return amg_set_error(AMG_ERR_ARG, "amg_classical_setup: column %d out of range", A0.cj[k]);
      }
   H->A.push_back(std::move(A0));
   const uint64_t seed = o->coarsen_type == AMG_COARSEN_PMIS ? o->seed + 0x9e37ULL : o->seed;
   for (int l = 0; l + 1 < o->max_levels; l++) {
      const HCsr &A = H->A.back();
      if (A.n <= o->max_coarse_size) break;
      const int nfun = A.n % o->num_functions == 0 ? o->num_functions : 1;
      HCsr S, ST;
      const bool tm = std::getenv("AMG_CLASSICAL_TIMING") != nullptr;
      auto now = [] { return std::chrono::steady_clock::now(); };
      auto t0 = now();
      strength(A, o->strong_threshold, o->max_row_sum, nfun, S);
      transpose_pattern(S, ST);
      auto t1 = now();
      std::vector<int> cf;
      if (o->coarsen_type == AMG_COARSEN_HMIS)
         coarsen_rs(S, ST, cf);
      else
         coarsen_pmis(S, ST, seed + (uint64_t)l * 7919ULL, cf);
      auto t2 = now();
      HCsr P;
      int nc = 0;
      interpolation(A, S, cf, o->interp_type, nfun, P, &nc);
      auto t3 = now();
      if (nc == 0 || nc == A.n) break; // coarsening stalled
      HCsr R, AP, Ac;
      transpose(P, R);
      if (o->device >= 0) {
         Ac.n = R.n, Ac.m = P.m;
         const int st = amg_rap_device(o->device, A.n, A.rp, A.cj, A.v, P.rp, P.cj, P.v, P.m, R.n, R.rp, R.cj, R.v,
                                       Ac.rp, Ac.cj, Ac.v);
         if (st != AMG_OK) {
            delete H;
            return st;
         }
      } else {
         spgemm(A, P, AP);
         spgemm(R, AP, Ac);
      }
      auto t4 = now();
      if (tm) {
         auto d = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
         std::fprintf(stderr, "[classical] level %d n=%d: strength %.2fs coarsen %.2fs interp %.2fs RAP %.2fs\n", l,
                      A.n, d(t0, t1), d(t1, t2), d(t2, t3), d(t3, t4));
      }
      H->cf.push_back(std::move(cf));
      H->P.push_back(std::move(P));
      H->R.push_back(std::move(R));
      H->A.push_back(std::move(Ac));
   }
   *out = H;
   return AMG_OK;
}

extern "C" int amg_classical_levels(const amg_classical *H) { return H ? (int)H->A.size() : -1; }

static const HCsr *pick(const amg_classical *H, int which, int level)
{
   if (!H || level < 0) return nullptr;
   const auto &v = which == AMG_GEN_A ? H->A : which == AMG_GEN_P ? H->P : which == AMG_GEN_R ? H->R : H->A;
   if (which != AMG_GEN_A && which != AMG_GEN_P && which != AMG_GEN_R) return nullptr;
   return level < (int)v.size() ? &v[level] : nullptr;
}

extern "C" int amg_classical_get(const amg_classical *H, int which, int level, int *nrows, int *ncols,
                                 long long *nnz, const int **rowptr, const int **col, const double **val)
{
   const HCsr *M = pick(H, which, level);
   AMG_ARG(M, "amg_classical_get: no operator %d on level %d", which, level);
   if (nrows) *nrows = M->n;
   if (ncols) *ncols = M->m;
   if (nnz) *nnz = M->nnz();
   if (rowptr) *rowptr = M->rp.data();
   if (col) *col = M->cj.data();
   if (val) *val = M->v.data();
   return AMG_OK;
}

extern "C" int amg_classical_register(amg_ctx *ctx, const amg_classical *H, int which, int level,
                                      amg_mat **out)
{
   const HCsr *M = pick(H, which, level);
   AMG_ARG(ctx && out && M, "amg_classical_register: no operator %d on level %d", which, level);
   return amg_csr_register(ctx, M->n, M->m, M->nnz(), M->rp.data(), M->cj.data(), M->v.data(),
                           which == AMG_GEN_A ? 1 : 0, out);
}

extern "C" int amg_classical_cf_marker(const amg_classical *H, int level, int *cf)
{
   AMG_ARG(H && cf && level >= 0 && level < (int)H->cf.size(), "amg_classical_cf_marker: bad level");
   std::copy(H->cf[level].begin(), H->cf[level].end(), cf);
   return AMG_OK;
}

extern "C" int amg_classical_free(amg_classical *H)
{
   delete H;
   return AMG_OK;
}
