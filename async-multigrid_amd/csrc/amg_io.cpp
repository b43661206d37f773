// amg_io.cpp -- binary triplet matrix files (-problem file): the reference's
// readers and writers restated on host arrays (no hypre / MPI / METIS).
//
//   record  = {int32 i, int32 j, double val}  (16 bytes, Triplet_AOS,
//             Main.hpp:433-437), 1-based i, j
//   record 0 = header: i = number of rows (PrintCSRMatrix writes
//             {num_rows, num_cols, nnz}, Misc.cpp:766-770)
//
// amg_triplet_read        ReadBinary_fread_HypreParCSR   Misc.cpp:800-915
// amg_triplet_read_part   ParReadBinary_fread            DMEM_BuildMatrix.cpp:1488-1560
// amg_triplet_write       PrintCSRMatrix                 Misc.cpp:753-797
// amg_triplet_text_to_bin TextToBin main                 TextToBin.cpp:5-39
//
// Both readers hand every row's (col, val) list, in file order, to hypre's
// IJ interface (HYPRE_IJMatrixSetValues + Assemble, third party): a column
// set twice keeps its first position and the last value, and the assembled
// diag block stores each row's diagonal first.  That assembly is restated
// here (parity unpinned: hypre is not in the reference tree); the rows come
// out diagonal-first, the convention every kernel relies on (a_ii =
// A_data[A_i[i]]).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "amg_internal.h"

namespace {

struct Trip {
   int i, j;
   double val;
};
static_assert(sizeof(Trip) == 16, "Triplet_AOS is 16 bytes");

int read_records(const char *path, std::vector<Trip> &buf)
{
   FILE *fp = std::fopen(path, "rb");
   if (!fp) return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: cannot open \"%s\"", path);
   std::fseek(fp, 0, SEEK_END);
   const long size = std::ftell(fp);
   std::rewind(fp);
   const size_t nrec = size > 0 ? (size_t)size / sizeof(Trip) : 0;
   buf.resize(nrec);
   const size_t got = nrec ? std::fread(buf.data(), sizeof(Trip), nrec, fp) : 0;
   std::fclose(fp);
   if (got != nrec) return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: short read of \"%s\"", path);
   if (nrec < 1 || buf[0].i < 0)
      return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: \"%s\" has no header record", path);
   return AMG_OK;
}

// HYPRE_IJMatrixSetValues per row, then the assembly: first position, last
// value; the diagonal (column == global row) moved to the front
int assemble(int nrows, int ncols, int row0, std::vector<std::vector<int>> &cols,
             std::vector<std::vector<double>> &vals, amg_host_csr *out)
{
   std::vector<int> rowptr(nrows + 1, 0);
   std::vector<int> col;
   std::vector<double> val;
   std::unordered_map<int, size_t> seen;
   for (int r = 0; r < nrows; r++) {
      seen.clear();
      const size_t start = col.size();
      for (size_t k = 0; k < cols[r].size(); k++) {
         const int c = cols[r][k];
         if (c < 0 || c >= ncols)
            return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: column %d of row %d outside [1, %d]", c + 1,
                                 r + row0 + 1, ncols);
         auto it = seen.find(c);
         if (it != seen.end()) {
            val[it->second] = vals[r][k];
         } else {
            seen.emplace(c, col.size());
            col.push_back(c);
            val.push_back(vals[r][k]);
         }
      }
      for (size_t k = start; k < col.size(); k++) {
         if (col[k] != r + row0) continue;
         for (size_t q = k; q > start; q--) {
            std::swap(col[q], col[q - 1]);
            std::swap(val[q], val[q - 1]);
         }
         break;
      }
      rowptr[r + 1] = (int)col.size();
      std::vector<int>().swap(cols[r]);
      std::vector<double>().swap(vals[r]);
   }
   out->nrows = nrows;
   out->ncols = ncols;
   out->nnz = (long long)col.size();
   out->rowptr = (int *)std::malloc(sizeof(int) * (nrows + 1));
   out->col = (int *)std::malloc(sizeof(int) * std::max<size_t>(col.size(), 1));
   out->val = (double *)std::malloc(sizeof(double) * std::max<size_t>(val.size(), 1));
   if (!out->rowptr || !out->col || !out->val) {
      amg_host_csr_free(out);
      return amg_set_error(AMG_ERR_OOM, "amg_triplet_read: out of host memory");
   }
   std::memcpy(out->rowptr, rowptr.data(), sizeof(int) * (nrows + 1));
   if (!col.empty()) {
      std::memcpy(out->col, col.data(), sizeof(int) * col.size());
      std::memcpy(out->val, val.data(), sizeof(double) * val.size());
   }
   return AMG_OK;
}

} // namespace

extern "C" void amg_host_csr_free(amg_host_csr *M)
{
   if (!M) return;
   std::free(M->rowptr);
   std::free(M->col);
   std::free(M->val);
   M->rowptr = M->col = nullptr;
   M->val = nullptr;
   M->nrows = M->ncols = 0;
   M->nnz = 0;
}

// ReadBinary_fread_HypreParCSR (Misc.cpp:800-915)
extern "C" int amg_triplet_read(const char *path, int symm, int remove_disconnected, amg_host_csr *out)
{
   AMG_ARG(path && out, "amg_triplet_read: null argument");
   *out = amg_host_csr{};
   std::vector<Trip> buf;
   AMG_TRY(read_records(path, buf));
   const int lines = (int)buf.size();
   int num_rows = buf[0].i;
   std::vector<int> col_count(num_rows, 0);
   std::vector<char> flag(lines, 0);
   for (int k = 1; k < lines; k++) {
      const int r = buf[k].i, c = buf[k].j;
      if (r < 1 || r > num_rows || c < 1 || c > num_rows)
         return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: record %d (%d, %d) outside [1, %d]", k, r, c,
                              num_rows);
      // every record counts, zero values included (the |elem| > 0 test is
      // commented out at Misc.cpp:827)
      col_count[c - 1]++;
      flag[k] = 1;
   }
   std::vector<int> shift(num_rows, 0);
   if (remove_disconnected) {
      // Misc.cpp:846-871: a record whose row has <= 1 entries in its COLUMN
      // count is dropped and the row renumbered away; num_rows drops once per
      // such record (the reference's "TODO: fix this")
      std::vector<int> disc(num_rows, 0);
      for (int k = 1; k < lines; k++) {
         if (!flag[k]) continue;
         const int r = buf[k].i;
         if (col_count[r - 1] <= 1) {
            flag[k] = 0;
            disc[r - 1] = 1;
            num_rows--;
         }
      }
      std::partial_sum(disc.begin(), disc.end(), shift.begin());
   }
   if (num_rows < 0) return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: row count below zero");
   std::vector<std::vector<int>> cols(num_rows);
   std::vector<std::vector<double>> vals(num_rows);
   for (int k = 1; k < lines; k++) {
      if (!flag[k]) continue;
      const int r = buf[k].i - shift[buf[k].i - 1], c = buf[k].j - shift[buf[k].j - 1];
      if (r < 1 || r > num_rows || c < 1 || c > num_rows)
         return amg_set_error(AMG_ERR_ARG, "amg_triplet_read: record %d renumbered outside the matrix", k);
      cols[r - 1].push_back(c - 1);
      vals[r - 1].push_back(buf[k].val);
      if (symm && r != c) {
         cols[c - 1].push_back(r - 1);
         vals[c - 1].push_back(buf[k].val);
      }
   }
   return assemble(num_rows, num_rows, 0, cols, vals, out);
}

// ParReadBinary_fread (DMEM_BuildMatrix.cpp:1488-1560): one rank's file of
// its own rows [min_row, max_row] (global, 1-based in the file); records with
// a zero value are skipped.  *first_row = min_row - 1 (0-based).
extern "C" int amg_triplet_read_part(const char *path, int ncols, int *first_row, amg_host_csr *out)
{
   AMG_ARG(path && out && first_row && ncols > 0, "amg_triplet_read_part: bad argument");
   *out = amg_host_csr{};
   std::vector<Trip> buf;
   AMG_TRY(read_records(path, buf));
   const int lines = (int)buf.size();
   if (lines < 2) return amg_set_error(AMG_ERR_ARG, "amg_triplet_read_part: \"%s\" holds no entries", path);
   int min_row = buf[1].i, max_row = 0;
   for (int k = 1; k < lines; k++) {
      if (!(std::fabs(buf[k].val) > 0)) continue;
      min_row = std::min(min_row, buf[k].i);
      max_row = std::max(max_row, buf[k].i);
   }
   const int nloc = std::max(0, max_row - min_row + 1);
   std::vector<std::vector<int>> cols(nloc);
   std::vector<std::vector<double>> vals(nloc);
   for (int k = 1; k < lines; k++) {
      if (!(std::fabs(buf[k].val) > 0)) continue;
      cols[buf[k].i - min_row].push_back(buf[k].j - 1);
      vals[buf[k].i - min_row].push_back(buf[k].val);
   }
   *first_row = min_row - 1;
   return assemble(nloc, ncols, min_row - 1, cols, vals, out);
}

// PrintCSRMatrix (Misc.cpp:753-797): header {num_rows, num_cols, nnz}, then
// (row + 1, col + 1, value) per entry in CSR order; binary or "%d %d %.16e"
extern "C" int amg_triplet_write(const char *path, int nrows, int ncols, const int *rowptr, const int *col,
                                 const double *val, int binary)
{
   AMG_ARG(path && rowptr && nrows >= 0, "amg_triplet_write: bad argument");
   FILE *fp = std::fopen(path, binary ? "wb" : "w");
   if (!fp) return amg_set_error(AMG_ERR_ARG, "amg_triplet_write: cannot open \"%s\"", path);
   const int nnz = rowptr[nrows];
   bool ok = true;
   if (binary) {
      // the reference writes nnz with sizeof(double) from an int; here the
      // header's value slot holds nnz in its low word and zero above
      Trip h{nrows, ncols, 0.0};
      long long w = (unsigned int)nnz;
      std::memcpy(&h.val, &w, 8);
      ok = std::fwrite(&h, sizeof(Trip), 1, fp) == 1;
   } else {
      ok = std::fprintf(fp, "%d %d %d\n", nrows, ncols, nnz) > 0;
   }
   for (int i = 0; ok && i < nrows; i++)
      for (int k = rowptr[i]; ok && k < rowptr[i + 1]; k++) {
         if (binary) {
            const Trip t{i + 1, col[k] + 1, val[k]};
            ok = std::fwrite(&t, sizeof(Trip), 1, fp) == 1;
         } else {
            ok = std::fprintf(fp, "%d %d %.16e\n", i + 1, col[k] + 1, val[k]) > 0;
         }
      }
   if (std::fclose(fp) != 0) ok = false;
   return ok ? AMG_OK : amg_set_error(AMG_ERR_ARG, "amg_triplet_write: write to \"%s\" failed", path);
}

// TextToBin (TextToBin.cpp:5-39): "row col value" lines to binary records,
// the first line included (the header record)
extern "C" int amg_triplet_text_to_bin(const char *in_path, const char *out_path)
{
   AMG_ARG(in_path && out_path, "amg_triplet_text_to_bin: null path");
   FILE *in = std::fopen(in_path, "r");
   if (!in) return amg_set_error(AMG_ERR_ARG, "amg_triplet_text_to_bin: cannot open \"%s\"", in_path);
   FILE *out = std::fopen(out_path, "wb");
   if (!out) {
      std::fclose(in);
      return amg_set_error(AMG_ERR_ARG, "amg_triplet_text_to_bin: cannot open \"%s\"", out_path);
   }
   Trip t{};
   bool ok = true;
   while (ok && std::fscanf(in, "%d %d %lg", &t.i, &t.j, &t.val) == 3) ok = std::fwrite(&t, sizeof(Trip), 1, out) == 1;
   std::fclose(in);
   if (std::fclose(out) != 0) ok = false;
   return ok ? AMG_OK : amg_set_error(AMG_ERR_ARG, "amg_triplet_text_to_bin: write failed");
}
