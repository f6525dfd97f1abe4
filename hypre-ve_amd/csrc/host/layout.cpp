// Host-side construction of the HBM layouts consumed by the device runtime.
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "hve_host.hpp"
#include "layout.hpp"

namespace hve {

// SELL-64: slices of 64 consecutive rows, padded to the longest row of the
// slice; entry k of lane r at slice_ptr[s] + 64*k + r; padding col = -1.
static void sell_order(const CSR& A, int sigma, std::vector<int>& perm) {
  const int n = A.nrows;
  perm.resize(n);
  for (int r = 0; r < n; ++r) perm[r] = r;
  if (sigma <= 0) return;
#pragma omp parallel for schedule(static)
  for (int w0 = 0; w0 < n; w0 += sigma) {
    const int w1 = std::min(n, w0 + sigma);
    std::stable_sort(perm.begin() + w0, perm.begin() + w1, [&](int x, int y) {
      return A.i[x + 1] - A.i[x] > A.i[y + 1] - A.i[y];
    });
  }
}

int64_t sell_padded_nnz(const CSR& A, int sigma) {
  std::vector<int> perm;
  sell_order(A, sigma, perm);
  int64_t tot = 0;
  for (int s0 = 0; s0 < A.nrows; s0 += 64) {
    int w = 0;
    for (int r = s0; r < std::min(A.nrows, s0 + 64); ++r) w = std::max(w, A.i[perm[r] + 1] - A.i[perm[r]]);
    tot += (int64_t)w * 64;
  }
  return tot;
}

void build_sell_host(const CSR& A, int sigma, std::vector<int>& perm, std::vector<int>& slice_ptr,
                     std::vector<int>& col, std::vector<double>& val) {
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  sell_order(A, sigma, perm);
  slice_ptr.assign(ns + 1, 0);
  std::vector<int64_t> sp(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int w = 0;
    const int r1 = std::min(n, (s + 1) * 64);
    for (int r = s * 64; r < r1; ++r) w = std::max(w, A.i[perm[r] + 1] - A.i[perm[r]]);
    sp[s + 1] = sp[s] + (int64_t)w * 64;
  }
  if (sp[ns] > 0x7fffffffLL) throw std::runtime_error("padded operator exceeds 2^31 entries on one GPU");
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  col.assign((size_t)sp[ns], -1);
  val.assign((size_t)sp[ns], 0.0);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    const int r1 = std::min(n, (s + 1) * 64);
    for (int r = s * 64; r < r1; ++r) {
      const int lane = r & 63, src = perm[r];
      for (int k = A.i[src]; k < A.i[src + 1]; ++k) {
        const size_t pos = (size_t)slice_ptr[s] + (size_t)(k - A.i[src]) * 64 + lane;
        col[pos] = A.j[k];
        val[pos] = A.a[k];
      }
    }
  }
  if (sigma <= 0) perm.clear();
}

// hypre_gselim (sstruct_ls/gselim.h) forward elimination of the matrix alone:
// records each multiplier factor = A[j][k] * (1/A[k][k]) that the reference
// applies to x (mask = 1 where it applies one) and the eliminated matrix whose
// upper triangle the back substitution reads.
void gselim_factor(int n, const std::vector<double>& dense, std::vector<double>& L,
                   std::vector<unsigned char>& mask, std::vector<double>& U) {
  U = dense;
  L.assign((size_t)n * n, 0.0);
  mask.assign((size_t)n * n, 0);
  if (n <= 1) return;
  for (int k = 0; k < n - 1; ++k) {
    if (U[(size_t)k * n + k] != 0.0) {
      const double divA = 1.0 / U[(size_t)k * n + k];
      for (int j = k + 1; j < n; ++j) {
        if (U[(size_t)j * n + k] != 0.0) {
          const double factor = U[(size_t)j * n + k] * divA;
          for (int m = k + 1; m < n; ++m) U[(size_t)j * n + m] -= factor * U[(size_t)k * n + m];
          L[(size_t)j * n + k] = factor;
          mask[(size_t)j * n + k] = 1;
        }
      }
    }
  }
}

// Dense row-major copy of a (small) CSR operator, as hypre_GaussElimSetup
// (par_gauss_elim.c:84) assembles A_mat.
void csr_to_dense(const CSR& A, std::vector<double>& dense) {
  const int n = A.nrows;
  dense.assign((size_t)n * n, 0.0);
  for (int r = 0; r < n; ++r)
    for (int k = A.i[r]; k < A.i[r + 1]; ++k) dense[(size_t)r * n + A.j[k]] = A.a[k];
}

}  // namespace hve
