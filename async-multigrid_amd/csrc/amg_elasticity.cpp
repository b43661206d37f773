// amg_elasticity.cpp -- the DMEM elasticity test problem (config 5), generated
// on the host: DMEM_BuildMfemMatrix (DMEM_BuildMatrix.cpp:442-719) assembles it
// with MFEM, which is not in the reference tree, so the discretisation is
// restated from its description there (parity unpinned):
//   * mesh: MFEM's beam-hex, [0,8] x [0,1] x [0,1] in 8 x 1 x 1 hexahedra, the
//     first four of material attribute 1, the rest attribute 2
//     (DMEM_BuildMatrix.cpp:461), refined uniformly `refine` times -> cubes of
//     side h = 2^-refine, (8 / h) x (1 / h) x (1 / h) elements;
//   * Q1 vector H1 space, Ordering::byVDIM: dof = 3 * node + component, nodes
//     numbered lexicographically (x fastest; MFEM's refined numbering differs);
//   * ElasticityIntegrator with lambda = mu = 1, times 50 on attribute 1
//     (:540-547): K[(a,i),(b,j)] = int lambda d_i phi_a d_j phi_b
//       + mu (delta_ij grad phi_a . grad phi_b + d_j phi_a d_i phi_b),
//     2 x 2 x 2 Gauss points (exact for these cubes);
//   * essential boundary attribute 1 (the face x = 0) fixed (:519-521): its rows
//     become identity rows and its columns are removed (FormLinearSystem);
//   * load: pull force -1e-2 in z on boundary attribute 2 (the face x = 8,
//     :523-533), b = int f . phi over the face; zero on the fixed dofs.
// Rows are diagonal first, then ascending columns; num_functions = 3.
#include <algorithm>
#include <cmath>
#include <vector>

#include "amg_internal.h"

struct amg_elast {
   int nx = 0, ny = 0, nz = 0; // elements per direction
   std::vector<int> rp, cj;
   std::vector<double> v, rhs;
};

namespace {

// reference cube [0,1]^3 stiffness parts for lambda = 1 (KL) and mu = 1 (KM),
// dof (a, i) -> 3 a + i, node a = (ax, ay, az) bits (x fastest)
void reference_stiffness(double KL[24][24], double KM[24][24])
{
   const double g = 0.5 / std::sqrt(3.0);
   const double qp[2] = {0.5 - g, 0.5 + g}; // weights 1/2 each -> 1/8 per point
   for (int r = 0; r < 24; r++)
      for (int c = 0; c < 24; c++) KL[r][c] = KM[r][c] = 0.0;
   for (int qz = 0; qz < 2; qz++)
      for (int qy = 0; qy < 2; qy++)
         for (int qx = 0; qx < 2; qx++) {
            const double p[3] = {qp[qx], qp[qy], qp[qz]};
            double grad[8][3];
            for (int a = 0; a < 8; a++) {
               const int b[3] = {a & 1, (a >> 1) & 1, (a >> 2) & 1};
               double f[3], df[3];
               for (int d = 0; d < 3; d++) {
                  f[d] = b[d] ? p[d] : 1.0 - p[d];
                  df[d] = b[d] ? 1.0 : -1.0;
               }
               grad[a][0] = df[0] * f[1] * f[2];
               grad[a][1] = f[0] * df[1] * f[2];
               grad[a][2] = f[0] * f[1] * df[2];
            }
            for (int a = 0; a < 8; a++)
               for (int i = 0; i < 3; i++)
                  for (int b = 0; b < 8; b++)
                     for (int j = 0; j < 3; j++) {
                        const double dot = grad[a][0] * grad[b][0] + grad[a][1] * grad[b][1] +
                                           grad[a][2] * grad[b][2];
                        KL[3 * a + i][3 * b + j] += 0.125 * (grad[a][i] * grad[b][j]);
                        KM[3 * a + i][3 * b + j] +=
                           0.125 * ((i == j ? dot : 0.0) + grad[a][j] * grad[b][i]);
                     }
         }
}

} // namespace

extern "C" int amg_elast_create(int refine, amg_elast **out)
{
   AMG_ARG(out && refine >= 0 && refine <= 8, "amg_elast_create: refine %d (0..8)", refine);
   const int s = 1 << refine;
   auto *E = new amg_elast();
   E->nx = 8 * s;
   E->ny = E->nz = s;
   const int px = E->nx + 1, py = E->ny + 1, pz = E->nz + 1;
   const long long nodes = (long long)px * py * pz;
   const long long n = 3 * nodes;
   if (n > (1LL << 31) - 1 || n * 81 > (1LL << 31) - 64) {
      delete E;
      return amg_set_error(AMG_ERR_ARG, "amg_elast_create: %lld dofs exceed int32 CSR", n);
   }
   const double h = 1.0 / s;
   double KL[24][24], KM[24][24];
   reference_stiffness(KL, KM);
   // element stiffness per material: h * (lambda KL + mu KM) (3-D scaling of the cube)
   double K[2][24][24];
   for (int m = 0; m < 2; m++) {
      const double lam = m == 0 ? 50.0 : 1.0, mu = lam;
      for (int r = 0; r < 24; r++)
         for (int c = 0; c < 24; c++) K[m][r][c] = h * (lam * KL[r][c] + mu * KM[r][c]);
   }
   auto node = [&](int x, int y, int z) -> long long { return ((long long)z * py + y) * px + x; };
   auto fixed = [&](long long d) { return (d / 3) % px == 0; }; // node on x = 0
   // row i couples to the 27 (or fewer) neighbour nodes: assemble row by row,
   // element contributions in a fixed order (elements z, y, x ascending)
   E->rp.assign(n + 1, 0);
   E->cj.reserve(n * 81);
   E->v.reserve(n * 81);
   std::vector<double> acc(81);
   for (long long d = 0; d < n; d++) {
      const long long nd = d / 3;
      const int comp = (int)(d % 3);
      const int x = (int)(nd % px), y = (int)((nd / px) % py), z = (int)(nd / ((long long)px * py));
      if (fixed(d)) { // essential dof: identity row
         E->cj.push_back((int)d);
         E->v.push_back(1.0);
         E->rp[d + 1] = (int)E->cj.size();
         continue;
      }
      std::fill(acc.begin(), acc.end(), 0.0);
      // elements containing node (x,y,z): (ex, ey, ez) with ex in {x-1, x}
      for (int ez = z - 1; ez <= z; ez++)
         for (int ey = y - 1; ey <= y; ey++)
            for (int ex = x - 1; ex <= x; ex++) {
               if (ex < 0 || ey < 0 || ez < 0 || ex >= E->nx || ey >= E->ny || ez >= E->nz) continue;
               const int mat = ex < E->nx / 2 ? 0 : 1; // attribute 1: the first half of the beam
               const int la = (x - ex) | ((y - ey) << 1) | ((z - ez) << 2);
               for (int lb = 0; lb < 8; lb++) {
                  const int bx = ex + (lb & 1), by = ey + ((lb >> 1) & 1), bz = ez + ((lb >> 2) & 1);
                  const int slot = ((bz - z + 1) * 3 + (by - y + 1)) * 3 + (bx - x + 1);
                  for (int j = 0; j < 3; j++) acc[slot * 3 + j] += K[mat][3 * la + comp][3 * lb + j];
               }
            }
      // diagonal first, then ascending columns; fixed columns removed
      E->cj.push_back((int)d);
      E->v.push_back(acc[13 * 3 + comp]);
      for (int sl = 0; sl < 27; sl++) {
         const int bx = x + sl % 3 - 1, by = y + (sl / 3) % 3 - 1, bz = z + sl / 9 - 1;
         if (bx < 0 || by < 0 || bz < 0 || bx >= px || by >= py || bz >= pz) continue;
         for (int j = 0; j < 3; j++) {
            const long long c = 3 * node(bx, by, bz) + j;
            if (c == d || fixed(c)) continue;
            E->cj.push_back((int)c);
            E->v.push_back(acc[sl * 3 + j]);
         }
      }
      E->rp[d + 1] = (int)E->cj.size();
   }
   // load: f_z = -1e-2 on the face x = 8, bilinear face shape functions
   // integrate to h^2 / 4 per face corner
   E->rhs.assign(n, 0.0);
   for (int ez = 0; ez < E->nz; ez++)
      for (int ey = 0; ey < E->ny; ey++)
         for (int c = 0; c < 4; c++) {
            const long long nd = node(E->nx, ey + (c & 1), ez + (c >> 1));
            E->rhs[3 * nd + 2] += -1.0e-2 * h * h * 0.25;
         }
   *out = E;
   return AMG_OK;
}

extern "C" int amg_elast_get(const amg_elast *E, int *n, long long *nnz, const int **rowptr, const int **col,
                             const double **val, const double **rhs)
{
   AMG_ARG(E, "amg_elast_get: null problem");
   if (n) *n = (int)E->rhs.size();
   if (nnz) *nnz = (long long)E->cj.size();
   if (rowptr) *rowptr = E->rp.data();
   if (col) *col = E->cj.data();
   if (val) *val = E->v.data();
   if (rhs) *rhs = E->rhs.data();
   return AMG_OK;
}

extern "C" int amg_elast_free(amg_elast *E)
{
   delete E;
   return AMG_OK;
}
