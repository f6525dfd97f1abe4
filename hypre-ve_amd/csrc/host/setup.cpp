#include <memory>
// BoomerAMG setup phase on the host: strength, PMIS coarsening, extended+i
// interpolation, truncation and the Galerkin product.  Every routine follows the
// single-process (num_procs == 1) branch of the cited hypre routine statement for
// statement, including entry order inside rows and the floating-point
// accumulation order, so that the resulting hierarchy (and therefore the
// complexities and convergence the reference reports) is reproduced exactly.
#include "hve_host.hpp"
#include "setup_dev.hpp"
#include "layout.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <stdexcept>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace hve {
int knob(int id);  // kernels.hip (tests' knobs)


// ---------------------------------------------------------------------------
// Problem generators
// ---------------------------------------------------------------------------

// parcsr_ls/par_laplace.c:15 GenerateLaplacian with P=Q=R=1, values from
// test/ij.c:7790 (values[0] = 2cx+2cy+2cz for dims > 1, off-diag -c).
void generate_laplacian_7pt(int nx, int ny, int nz, double cx, double cy, double cz, CSR& A) {
  const int64_t n64 = (int64_t)nx * ny * nz;
  if (n64 > 0x7fffffff) throw std::runtime_error("grid too large for 32-bit rows");
  const int n = (int)n64;
  double v0 = 0.0;
  if (nx > 1) v0 += 2.0 * cx;
  if (ny > 1) v0 += 2.0 * cy;
  if (nz > 1) v0 += 2.0 * cz;
  const double v1 = -cx, v2 = -cy, v3 = -cz;
  A.resize_rows(n, n);
  // first pass: row lengths (boundary-dependent), computed per row in parallel
  const int64_t nxny = (int64_t)nx * ny;
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    int ix = r % nx, iy = (r / nx) % ny, iz = (int)(r / nxny);
    int c = 1 + (iz > 0) + (iy > 0) + (ix > 0) + (ix + 1 < nx) + (iy + 1 < ny) + (iz + 1 < nz);
    A.i[r + 1] = c;
  }
  for (int r = 0; r < n; ++r) A.i[r + 1] += A.i[r];
  if ((int64_t)A.i[n] < 0) throw std::runtime_error("nnz overflow");
  A.j.resize(A.i[n]);
  A.a.resize(A.i[n]);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    int ix = r % nx, iy = (r / nx) % ny, iz = (int)(r / nxny);
    int k = A.i[r];
    A.j[k] = r; A.a[k++] = v0;
    if (iz > 0) { A.j[k] = r - (int)nxny; A.a[k++] = v3; }
    if (iy > 0) { A.j[k] = r - nx; A.a[k++] = v2; }
    if (ix > 0) { A.j[k] = r - 1; A.a[k++] = v1; }
    if (ix + 1 < nx) { A.j[k] = r + 1; A.a[k++] = v1; }
    if (iy + 1 < ny) { A.j[k] = r + nx; A.a[k++] = v2; }
    if (iz + 1 < nz) { A.j[k] = r + (int)nxny; A.a[k++] = v3; }
  }
}

// Process-grid block (p,q,r) of GenerateLaplacian (par_laplace.c:15) with
// hypre_GeneratePartitioning (seq_mv/genpart.c:18) and the global numbering of
// hypre_map (par_laplace.c:363).  Rows come out with GLOBAL column indices,
// each row's entries in the serial order (diag, z-, y-, x-, x+, y+, z+), so
// the gathered matrix equals the one-process matrix for a z-slab partition.
static std::vector<int64_t> gen_part(int64_t len, int np) {
  std::vector<int64_t> part(np + 1, 0);
  const int64_t size = len / np, rest = len - size * np;
  for (int i = 0; i < np; ++i) part[i + 1] = part[i] + size + (i < rest ? 1 : 0);
  return part;
}
void generate_laplacian_7pt_block(int nx, int ny, int nz, int P, int Q, int R, int p, int q, int r,
                                  const double* value, CSR& A, int64_t& first_row) {
  const auto xp = gen_part(nx, P), yp = gen_part(ny, Q), zp = gen_part(nz, R);
  auto map = [&](int64_t ix, int64_t iy, int64_t iz, int pp, int qq, int rr) -> int64_t {
    const int64_t nxl = xp[pp + 1] - xp[pp], nyl = yp[qq + 1] - yp[qq], nzl = zp[rr + 1] - zp[rr];
    int64_t g = zp[rr] * nx * ny + yp[qq] * nx * nzl + xp[pp] * (nyl * nzl);
    g += ((iz - zp[rr]) * nyl + (iy - yp[qq])) * nxl + (ix - xp[pp]);
    return g;
  };
  const int nxl = (int)(xp[p + 1] - xp[p]), nyl = (int)(yp[q + 1] - yp[q]), nzl = (int)(zp[r + 1] - zp[r]);
  const int64_t nloc = (int64_t)nxl * nyl * nzl;
  if ((int64_t)nx * ny * nz > 0x7fffffffLL) throw std::runtime_error("global grid exceeds 2^31 rows");
  first_row = map(xp[p], yp[q], zp[r], p, q, r);
  A.resize_rows((int)nloc, (int)((int64_t)nx * ny * nz));
  std::vector<int> len(nloc);
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < nloc; ++t) {
    const int64_t ix = xp[p] + t % nxl, iy = yp[q] + (t / nxl) % nyl, iz = zp[r] + t / ((int64_t)nxl * nyl);
    len[t] = 1 + (iz > 0) + (iy > 0) + (ix > 0) + (ix + 1 < nx) + (iy + 1 < ny) + (iz + 1 < nz);
  }
  for (int64_t t = 0; t < nloc; ++t) A.i[t + 1] = A.i[t] + len[t];
  A.j.resize(A.i[nloc]);
  A.a.resize(A.i[nloc]);
  auto owner = [](const std::vector<int64_t>& part, int64_t c) {
    return (int)(std::upper_bound(part.begin(), part.end(), c) - part.begin()) - 1;
  };
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < nloc; ++t) {
    const int64_t ix = xp[p] + t % nxl, iy = yp[q] + (t / nxl) % nyl, iz = zp[r] + t / ((int64_t)nxl * nyl);
    int k = A.i[t];
    auto put = [&](int64_t x, int64_t y, int64_t z, double v) {
      A.j[k] = (int)map(x, y, z, owner(xp, x), owner(yp, y), owner(zp, z));
      A.a[k++] = v;
    };
    put(ix, iy, iz, value[0]);
    if (iz > 0) put(ix, iy, iz - 1, value[3]);
    if (iy > 0) put(ix, iy - 1, iz, value[2]);
    if (ix > 0) put(ix - 1, iy, iz, value[1]);
    if (ix + 1 < nx) put(ix + 1, iy, iz, value[1]);
    if (iy + 1 < ny) put(ix, iy + 1, iz, value[2]);
    if (iz + 1 < nz) put(ix, iy, iz + 1, value[3]);
  }
}

// GenerateLaplacian27pt's block (p, q, r) of a P x Q x R processor grid
// (par_laplace_27pt.c:15): hypre_GeneratePartitioning per axis and the
// processor-block-contiguous global numbering (global_part, par_laplace_27pt.c:78);
// entries in the single-process order (diagonal, then the 3x3x3 box z-major),
// global column indices.
void generate_laplacian_27pt_block(int nx, int ny, int nz, int P, int Q, int R, int p, int q, int r,
                                   const double* value, CSR& A, int64_t& first_row) {
  const auto xp = gen_part(nx, P), yp = gen_part(ny, Q), zp = gen_part(nz, R);
  auto owner = [](const std::vector<int64_t>& part, int64_t c) {
    return (int)(std::upper_bound(part.begin(), part.end(), c) - part.begin()) - 1;
  };
  auto map = [&](int64_t ix, int64_t iy, int64_t iz) -> int64_t {
    const int pp = owner(xp, ix), qq = owner(yp, iy), rr = owner(zp, iz);
    const int64_t nxl = xp[pp + 1] - xp[pp], nyl = yp[qq + 1] - yp[qq], nzl = zp[rr + 1] - zp[rr];
    int64_t g = zp[rr] * nx * ny + yp[qq] * nx * nzl + xp[pp] * (nyl * nzl);
    g += ((iz - zp[rr]) * nyl + (iy - yp[qq])) * nxl + (ix - xp[pp]);
    return g;
  };
  const int nxl = (int)(xp[p + 1] - xp[p]), nyl = (int)(yp[q + 1] - yp[q]), nzl = (int)(zp[r + 1] - zp[r]);
  const int64_t nloc = (int64_t)nxl * nyl * nzl;
  if ((int64_t)nx * ny * nz > 0x7fffffffLL) throw std::runtime_error("global grid exceeds 2^31 rows");
  first_row = map(xp[p], yp[q], zp[r]);
  A.resize_rows((int)nloc, (int)((int64_t)nx * ny * nz));
  auto coord = [&](int64_t t, int64_t& ix, int64_t& iy, int64_t& iz) {
    ix = xp[p] + t % nxl;
    iy = yp[q] + (t / nxl) % nyl;
    iz = zp[r] + t / ((int64_t)nxl * nyl);
  };
  std::vector<int> len(nloc);
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < nloc; ++t) {
    int64_t ix, iy, iz;
    coord(t, ix, iy, iz);
    const int cx = 1 + (ix > 0) + (ix + 1 < nx), cy = 1 + (iy > 0) + (iy + 1 < ny), cz = 1 + (iz > 0) + (iz + 1 < nz);
    len[t] = cx * cy * cz;
  }
  for (int64_t t = 0; t < nloc; ++t) {
    A.i[t + 1] = A.i[t] + len[t];
    if (A.i[t + 1] < 0) throw std::runtime_error("nnz overflow (use more GPUs)");
  }
  A.j.resize(A.i[nloc]);
  A.a.resize(A.i[nloc]);
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < nloc; ++t) {
    int64_t ix, iy, iz;
    coord(t, ix, iy, iz);
    int k = A.i[t];
    A.j[k] = (int)map(ix, iy, iz);
    A.a[k++] = value[0];
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy && !dz) continue;
          const int64_t x = ix + dx, y = iy + dy, z = iz + dz;
          if (x >= 0 && x < nx && y >= 0 && y < ny && z >= 0 && z < nz) {
            A.j[k] = (int)map(x, y, z);
            A.a[k++] = value[1];
          }
        }
  }
}

// parcsr_ls/par_laplace_27pt.c GenerateLaplacian27pt (P=Q=R=1): diagonal 26,
// every neighbour in the 3x3x3 box -1, neighbours visited z-major, then y, then x.
void generate_laplacian_27pt(int nx, int ny, int nz, CSR& A) {
  const int64_t n64 = (int64_t)nx * ny * nz;
  if (n64 > 0x7fffffff) throw std::runtime_error("grid too large for 32-bit rows");
  const int n = (int)n64;
  const int64_t nxny = (int64_t)nx * ny;
  A.resize_rows(n, n);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    int ix = r % nx, iy = (r / nx) % ny, iz = (int)(r / nxny);
    int c = 0;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          int x = ix + dx, y = iy + dy, z = iz + dz;
          if (x >= 0 && x < nx && y >= 0 && y < ny && z >= 0 && z < nz) ++c;
        }
    A.i[r + 1] = c;
  }
  for (int r = 0; r < n; ++r) A.i[r + 1] += A.i[r];
  if (A.i[n] < 0) throw std::runtime_error("nnz overflow (use more GPUs)");
  A.j.resize(A.i[n]);
  A.a.resize(A.i[n]);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    int ix = r % nx, iy = (r / nx) % ny, iz = (int)(r / nxny);
    int k = A.i[r];
    A.j[k] = r; A.a[k++] = 26.0;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy && !dz) continue;
          int x = ix + dx, y = iy + dy, z = iz + dz;
          if (x >= 0 && x < nx && y >= 0 && y < ny && z >= 0 && z < nz) {
            A.j[k] = (int)(((int64_t)z * ny + y) * nx + x);
            A.a[k++] = -1.0;
          }
        }
  }
}

// ---------------------------------------------------------------------------
// hypre_Rand: Park-Miller minimal standard, a = 16807, m = 2^31-1.
// utilities/random.c:40 (SeedRand), :56 (RandI via Schrage), :71 (Rand = RandI/m).
// The k-th draw after SeedRand(s) is a^(k+1) * s mod m; jump-ahead lets the
// measure initialisation run in parallel while producing the identical stream.
// ---------------------------------------------------------------------------
static const uint64_t kRandA = 16807ULL, kRandM = 2147483647ULL;
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
  uint64_t r = 1 % m;
  b %= m;
  while (e) {
    if (e & 1) r = (r * b) % m;
    b = (b * b) % m;
    e >>= 1;
  }
  return r;
}
double hypre_rand_at(int64_t k, int seed) {
  uint64_t s = (uint64_t)seed;
  if (seed < 1) s = 1; else if (s >= kRandM) s = kRandM - 1;
  uint64_t v = (powmod(kRandA, (uint64_t)k + 1, kRandM) * s) % kRandM;
  return (double)v / (double)kRandM;
}

// ---------------------------------------------------------------------------
// Strength of connection: par_strength.c:80 hypre_BoomerAMGCreateSHost,
// num_functions == 1, no offd part.  The first stored entry of each row is
// the diagonal and is never in S.
// ---------------------------------------------------------------------------
const int* hve_setup_dof = nullptr;

// num_functions > 1 (par_strength.c:254-294, :347-396): the row's scale and
// sum take the entries of its own function only, and only those can be strong
void create_strength(const CSR& A, double thr, double max_row_sum, Pattern& S) {
  const int* dof = hve_setup_dof;
  if (dof) {
    const int n = A.nrows;
    S.n = n;
    S.i.assign(n + 1, 0);
    std::vector<unsigned char> keep(A.nnz(), 0);
    std::vector<int> cnt(n, 0);
#pragma omp parallel for schedule(static)
    for (int r = 0; r < n; ++r) {
      const int b = A.i[r], e = A.i[r + 1];
      const double diag = A.a[b];
      double row_scale = 0.0, row_sum = diag;
      for (int k = b + 1; k < e; ++k) {
        if (dof[r] != dof[A.j[k]]) continue;
        row_scale = diag < 0 ? std::max(row_scale, A.a[k]) : std::min(row_scale, A.a[k]);
        row_sum += A.a[k];
      }
      int c = 0;
      if (!((std::fabs(row_sum) > std::fabs(diag) * max_row_sum) && (max_row_sum < 1.0))) {
        for (int k = b + 1; k < e; ++k) {
          if (dof[r] != dof[A.j[k]]) continue;
          if (diag < 0 ? !(A.a[k] <= thr * row_scale) : !(A.a[k] >= thr * row_scale)) { keep[k] = 1; ++c; }
        }
      }
      cnt[r] = c;
    }
    for (int r = 0; r < n; ++r) S.i[r + 1] = S.i[r] + cnt[r];
    S.j.resize(S.i[n]);
#pragma omp parallel for schedule(static)
    for (int r = 0; r < n; ++r) {
      int o = S.i[r];
      for (int k = A.i[r] + 1; k < A.i[r + 1]; ++k)
        if (keep[k]) S.j[o++] = A.j[k];
    }
    return;
  }
  const int n = A.nrows;
  S.n = n;
  S.i.assign(n + 1, 0);
  std::vector<int> cnt(n, 0);
  // first pass: count (row-parallel; the per-row decisions are independent)
  std::vector<unsigned char> keep(A.nnz(), 0);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    const int b = A.i[r], e = A.i[r + 1];
    const double diag = A.a[b];
    double row_scale = 0.0, row_sum = diag;
    if (diag < 0) {
      for (int k = b + 1; k < e; ++k) { row_scale = std::max(row_scale, A.a[k]); row_sum += A.a[k]; }
    } else {
      for (int k = b + 1; k < e; ++k) { row_scale = std::min(row_scale, A.a[k]); row_sum += A.a[k]; }
    }
    int c = 0;
    if ((std::fabs(row_sum) > std::fabs(diag) * max_row_sum) && (max_row_sum < 1.0)) {
      // all dependencies weak
    } else if (diag < 0) {
      for (int k = b + 1; k < e; ++k)
        if (!(A.a[k] <= thr * row_scale)) { keep[k] = 1; ++c; }
    } else {
      for (int k = b + 1; k < e; ++k)
        if (!(A.a[k] >= thr * row_scale)) { keep[k] = 1; ++c; }
    }
    cnt[r] = c;
  }
  for (int r = 0; r < n; ++r) S.i[r + 1] = S.i[r] + cnt[r];
  S.j.resize(S.i[n]);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    int o = S.i[r];
    for (int k = A.i[r] + 1; k < A.i[r + 1]; ++k)
      if (keep[k]) S.j[o++] = A.j[k];
  }
}

// ---------------------------------------------------------------------------
// PMIS coarsening: par_coarsen.c:2031 hypre_BoomerAMGCoarsenPMISHost, one
// process.  cf_init 0 (coarsen_type 8), 2 (type 9, sequential random stream),
// 1 (HMIS second stage: cf holds the first-pass C points), 3 / 4 (aggressive
// second pass of type 8 / 9: isolated points become C points).  In one
// process the sequential stream (2, 4) equals the per-rank one (0, 3).
// ---------------------------------------------------------------------------
// Owner rank of row i for row starts rs (rank r owns [rs[r], rs[r+1])).
static inline int owner_of(const std::vector<int>& rs, int i) {
  return (int)(std::upper_bound(rs.begin(), rs.end(), i) - rs.begin()) - 1;
}

void coarsen_pmis(const Pattern& S, int cf_init, std::vector<int>& cf, const std::vector<int>* rs) {
  const int n = S.n;
  std::vector<double> measure(n, 0.0);
  // column counts of S (number of points each point influences)
  {
    std::vector<int> mcount(n, 0);
    for (int64_t k = 0; k < (int64_t)S.j.size(); ++k) mcount[S.j[k]]++;
#pragma omp parallel for schedule(static)
    for (int r = 0; r < n; ++r) measure[r] = (double)mcount[r];
  }
  // hypre_BoomerAMGIndepSetInit (par_indepset.c:25): seed 2747 + my_id (0),
  // one hypre_Rand() per local row in row order (first_row_index = 0).
  // Emulating N ranks (rs): rank r seeds 2747 + r and draws over its own rows,
  // unless the stream is the sequential one (CF_init 2 / 4, seq_rand).
  if (rs && !(cf_init == 2 || cf_init == 4)) {
    const int nr = (int)rs->size() - 1;
#pragma omp parallel for schedule(static)
    for (int r = 0; r < nr; ++r) {
      uint64_t sd = (uint64_t)(2747 + r) % kRandM;
      for (int i = (*rs)[r]; i < (*rs)[r + 1]; ++i) {
        sd = (sd * kRandA) % kRandM;
        measure[i] += (double)sd / (double)kRandM;
      }
    }
  } else {
    const int seed = 2747;
#pragma omp parallel
    {
#ifdef _OPENMP
      int t = omp_get_thread_num(), nt = omp_get_num_threads();
#else
      int t = 0, nt = 1;
#endif
      int64_t chunk = (n + nt - 1) / nt;
      int64_t b = std::min<int64_t>((int64_t)t * chunk, n), e = std::min<int64_t>(b + chunk, n);
      if (b < e) {
        uint64_t s = (powmod(kRandA, (uint64_t)b + 1, kRandM) * (uint64_t)seed) % kRandM;
        for (int64_t r = b; r < e; ++r) {
          measure[r] += (double)s / (double)kRandM;
          s = (s * kRandA) % kRandM;
        }
      }
    }
  }
  // emulated ranks: whether row r has a strong connection owned by another rank
  // (hypre's S_offd row); such rows drop their first-pass marker (par_coarsen.c:2296)
  auto has_offd = [&](int r) {
    if (!rs) return false;
    const int o = owner_of(*rs, r);
    for (int k = S.i[r]; k < S.i[r + 1]; ++k)
      if (owner_of(*rs, S.j[k]) != o) return true;
    return false;
  };
  std::vector<int> graph;
  graph.reserve(n);
  if (cf_init == 1) {
    // CF from the first (Ruge) pass: C points keep 1, others reset to 0/F.
    for (int r = 0; r < n; ++r) {
      if (cf[r] != SF_PT) {
        if (cf[r] == -1 || has_offd(r)) cf[r] = 0;
        if (cf[r] == Z_PT) {
          if (measure[r] >= 1.0 || S.i[r + 1] - S.i[r] > 0) { cf[r] = 0; graph.push_back(r); }
          else cf[r] = F_PT;
        } else {
          graph.push_back(r);
        }
      } else {
        measure[r] = 0;
      }
    }
  } else {
    cf.assign(n, 0);
    for (int r = 0; r < n; ++r) {
      if (S.i[r + 1] - S.i[r] == 0) {
        cf[r] = (cf_init == 3 || cf_init == 4) ? C_PT : SF_PT;  // par_coarsen.c:2320-2326
        measure[r] = 0;
      } else {
        graph.push_back(r);
      }
    }
  }
  std::vector<int> graph2;
  graph2.reserve(n);
  int iter = 0;
  while (!graph.empty()) {
    const int gs = (int)graph.size();
    if (!cf_init || iter) {
#pragma omp parallel for schedule(static)
      for (int ig = 0; ig < gs; ++ig) {
        int i = graph[ig];
        if (measure[i] > 1) cf[i] = 1;
      }
      // remove nodes from the initial independent set (only writes 0: order-free)
#pragma omp parallel for schedule(static)
      for (int ig = 0; ig < gs; ++ig) {
        int i = graph[ig];
        if (measure[i] > 1) {
          for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
            int j = S.j[k];
            if (measure[j] > 1) {
              if (measure[i] > measure[j]) {
#pragma omp atomic write
                cf[j] = 0;
              } else if (measure[j] > measure[i]) {
#pragma omp atomic write
                cf[i] = 0;
              }
            }
          }
        }
      }
    }
    const bool first_seeded = cf_init && iter == 0;
    ++iter;
    if (first_seeded) {
      // The seeded C points (Ruge pass) can be demoted below (measure < 1)
      // while their neighbours test them; follow the reference's row order:
      // graph is ascending, so a neighbour j < i in the graph already holds
      // its new marker.  Emulated ranks: an off-rank neighbour reads
      // CF_marker_offd, still 0 in this first pass (par_coarsen.c:2348).
      for (int ig = 0; ig < gs; ++ig) {
        const int i = graph[ig];
        if (measure[i] < 1) cf[i] = F_PT;
        if (cf[i] > 0) {
          cf[i] = C_PT;
        } else {
          const int oi = rs ? owner_of(*rs, i) : 0;
          for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
            if (rs && owner_of(*rs, S.j[k]) != oi) continue;
            if (cf[S.j[k]] > 0) { cf[i] = F_PT; break; }
          }
        }
      }
    } else {
    // set C and F points (no marker > 0 is demoted here: order-free)
#pragma omp parallel for schedule(static)
    for (int ig = 0; ig < gs; ++ig) {
      int i = graph[ig];
      if (measure[i] < 1) cf[i] = F_PT;
      if (cf[i] > 0) {
        cf[i] = C_PT;
      } else {
        for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
          int j = S.j[k];
          if (cf[j] > 0) { cf[i] = F_PT; break; }
        }
      }
    }
    }
    graph2.clear();
    for (int ig = 0; ig < gs; ++ig) {
      int i = graph[ig];
      if (cf[i] != 0) measure[i] = 0;
      else graph2.push_back(i);
    }
    graph.swap(graph2);
  }
}

// ---------------------------------------------------------------------------
// Ruge-Stueben first pass, parcsr_ls/par_coarsen.c:874 hypre_BoomerAMGCoarsenRuge
// for one process (no offd part).  The point selection order is defined by the
// list-of-lists of utilities/amg_linklist.c: buckets of equal measure kept in
// decreasing measure order, each a FIFO threaded through lists[] / where[];
// the next C point is the head of the largest bucket.  The structure is
// restated as is (including how a point with measure 0, already marked, can
// re-enter the lists) because the coarse grid depends on it.
// ---------------------------------------------------------------------------
namespace {
constexpr int kListHead = -1, kListTail = -2;  // amg_linklist.c:16

struct MeasureLists {
  struct Elt { int data, head, tail, prev, next; };
  std::vector<Elt> pool;
  std::vector<int> free_;
  int head = -1, tail = -1;  // LoL_head / LoL_tail
  std::vector<int> lists, where;
  explicit MeasureLists(int n) : lists(n, 0), where(n, 0) {}

  int create(int item) {
    int e;
    if (!free_.empty()) { e = free_.back(); free_.pop_back(); }
    else { e = (int)pool.size(); pool.push_back({}); }
    pool[e] = {item, kListTail, kListHead, -1, -1};
    return e;
  }
  // amg_linklist.c:41 hypre_remove_point
  void remove(int measure, int index) {
    for (int lp = head; lp != -1; lp = pool[lp].next) {
      Elt& L = pool[lp];
      if (L.data != measure) continue;
      if (L.head == index && L.tail == index) {
        if (lp == head && lp == tail) { head = tail = -1; }
        else if (lp == head) { pool[L.next].prev = -1; head = L.next; }
        else if (lp == tail) { pool[L.prev].next = -1; tail = L.prev; }
        else { pool[L.next].prev = L.prev; pool[L.prev].next = L.next; }
        free_.push_back(lp);
      } else if (L.head == index) {
        L.head = lists[index];
        where[lists[index]] = kListHead;
      } else if (L.tail == index) {
        L.tail = where[index];
        lists[where[index]] = kListTail;
      } else {
        lists[where[index]] = lists[index];
        where[lists[index]] = where[index];
      }
      return;
    }
    throw std::runtime_error("Ruge coarsening: no such list");
  }
  // amg_linklist.c:168 hypre_enter_on_lists
  void enter(int measure, int index) {
    if (head == -1) {
      int e = create(measure);
      pool[e].head = pool[e].tail = index;
      lists[index] = kListTail;
      where[index] = kListHead;
      head = tail = e;
      return;
    }
    for (int lp = head; lp != -1; lp = pool[lp].next) {
      if (measure > pool[lp].data) {
        int e = create(measure);
        pool[e].head = pool[e].tail = index;
        lists[index] = kListTail;
        where[index] = kListHead;
        if (pool[lp].prev != -1) {
          pool[e].prev = pool[lp].prev;
          pool[pool[lp].prev].next = e;
          pool[lp].prev = e;
          pool[e].next = lp;
        } else {
          pool[e].next = lp;
          pool[lp].prev = e;
          pool[e].prev = -1;
          head = e;
        }
        return;
      } else if (measure == pool[lp].data) {
        const int old_tail = pool[lp].tail;
        lists[old_tail] = index;
        where[index] = old_tail;
        lists[index] = kListTail;
        pool[lp].tail = index;
        return;
      }
    }
    int e = create(measure);
    pool[e].head = pool[e].tail = index;
    lists[index] = kListTail;
    where[index] = kListHead;
    pool[tail].next = e;
    pool[e].prev = tail;
    pool[e].next = -1;
    tail = e;
  }
};
}  // namespace

// The first pass of par_coarsen.c:940 hypre_BoomerAMGCoarsenRuge, which is
// all of coarsen_type 11 (:1347-1354) and HMIS's first stage (coarsen_type 10
// -> 11 with f_pnt = Z_PT for measure-0 points, :1082-1086); coarsen_type 11
// itself leaves f_pnt = F_PT.
void coarsen_ruge_first_pass(const Pattern& S, const CSR* A, int measure_type, int cut_factor,
                             std::vector<int>& cf, const int* full_row_len, int f_pnt, const int* meas_add) {
  constexpr int UNDECIDED = 0, SC_PT = 3;
  const int n = S.n;
  const bool agg_2 = (measure_type == 3 || measure_type == 4);
  // ST = transpose of S (par_coarsen.c:1032-1057), counting sort
  std::vector<int> ST_i(n + 1, 0), ST_j(S.j.size());
  for (size_t k = 0; k < S.j.size(); ++k) ST_i[S.j[k] + 1]++;
  for (int i = 0; i < n; ++i) ST_i[i + 1] += ST_i[i];
  {
    std::vector<int> pos(ST_i.begin(), ST_i.end() - 1);
    for (int i = 0; i < n; ++i)
      for (int k = S.i[i]; k < S.i[i + 1]; ++k) ST_j[pos[S.j[k]]++] = i;
  }
  std::vector<int> measure(n);
  for (int i = 0; i < n; ++i) measure[i] = ST_i[i + 1] - ST_i[i] + (meas_add ? meas_add[i] : 0);

  cf.assign(n, 0);  // CF_marker allocated by the coarsening (all UNDECIDED)
  int num_left = 0;
  for (int j = 0; j < n; ++j) {
    if (cf[j] == 0) {
      // nnzrow counts the diag and offd parts (par_coarsen.c:1137)
      if ((full_row_len ? full_row_len[j] : S.i[j + 1] - S.i[j]) == 0) {
        cf[j] = agg_2 ? SC_PT : SF_PT;
        measure[j] = 0;
      } else {
        cf[j] = UNDECIDED;
        num_left++;
      }
    } else {
      measure[j] = 0;
    }
  }
  if (cut_factor > 0 && A && n > 0) {
    const int64_t avg = (int64_t)A->nnz() / n;
    const int64_t cut = cut_factor * avg;
    for (int j = 0; j < n; ++j) {
      if (A->i[j + 1] - A->i[j] > cut) {
        if (cf[j] == UNDECIDED) num_left--;
        cf[j] = SF_PT;
      }
    }
  }
  MeasureLists L(n);
  for (int j = 0; j < n; ++j) {
    const int m = measure[j];
    if (cf[j] != SF_PT && cf[j] != SC_PT) {
      if (m > 0) {
        L.enter(m, j);
      } else {
        if (m < 0) throw std::runtime_error("negative measure");
        cf[j] = f_pnt;
        for (int k = S.i[j]; k < S.i[j + 1]; ++k) {
          const int nb = S.j[k];
          if (cf[nb] != SF_PT && cf[nb] != SC_PT) {
            if (nb < j) {
              if (measure[nb] > 0) L.remove(measure[nb], nb);
              L.enter(++measure[nb], nb);
            } else {
              ++measure[nb];
            }
          }
        }
        --num_left;
      }
    }
  }
  while (num_left > 0) {
    if (L.head == -1) throw std::runtime_error("Ruge coarsening: lists exhausted with points left");
    const int index = L.pool[L.head].head;
    cf[index] = C_PT;
    const int m = measure[index];
    measure[index] = 0;
    --num_left;
    L.remove(m, index);
    for (int k = ST_i[index]; k < ST_i[index + 1]; ++k) {
      const int nb = ST_j[k];
      if (cf[nb] == UNDECIDED) {
        cf[nb] = F_PT;
        L.remove(measure[nb], nb);
        --num_left;
        for (int k2 = S.i[nb]; k2 < S.i[nb + 1]; ++k2) {
          const int nb2 = S.j[k2];
          if (cf[nb2] == UNDECIDED) {
            L.remove(measure[nb2], nb2);
            L.enter(++measure[nb2], nb2);
          }
        }
      }
    }
    for (int k = S.i[index]; k < S.i[index + 1]; ++k) {
      const int nb = S.j[k];
      if (cf[nb] == UNDECIDED) {
        int mm = measure[nb];
        L.remove(mm, nb);
        measure[nb] = --mm;
        if (mm > 0) {
          L.enter(mm, nb);
        } else {
          cf[nb] = F_PT;
          --num_left;
          for (int k2 = S.i[nb]; k2 < S.i[nb + 1]; ++k2) {
            const int nb2 = S.j[k2];
            if (cf[nb2] == UNDECIDED) {
              L.remove(measure[nb2], nb2);
              L.enter(++measure[nb2], nb2);
            }
          }
        }
      }
    }
  }
  for (int i = 0; i < n; ++i)
    if (cf[i] == SC_PT) cf[i] = C_PT;
}

// par_coarsen.c:2774 hypre_BoomerAMGCoarsenHMIS: Ruge first pass, then PMIS
// seeded with its C points (CF_init = 1).
// Emulated ranks (rs): every rank runs the first pass on its own rows with the
// strong connections it owns (S_diag, local measures, measure_type 0), then
// PMIS runs over the whole graph.
// Emulated ranks (rs): every rank runs the Ruge first pass on its own rows
// with the strong connections it owns (S_diag, local measures:
// par_coarsen.c:1088 builds no S_ext for measure_type 0), counting the whole
// row (diag and offd) for the isolated-point test.
// measure_type 1 (global measures, par_coarsen.c:1088-1108): a point's
// measure also counts the other ranks' points that strongly depend on it
// (S_ext); the pass itself still follows the rank's own connections.
static void ruge_first_pass_ranks(const Pattern& S, int measure_type, int f_pnt, std::vector<int>& cf,
                                  const std::vector<int>* rs) {
  const int nr = (int)rs->size() - 1;
  std::vector<int> ext;
  if (measure_type == 1) {
    auto owner = [&](int i) { return (int)(std::upper_bound(rs->begin(), rs->end(), i) - rs->begin()) - 1; };
    ext.assign(S.n, 0);
    for (int i = 0; i < S.n; ++i)
      for (int k = S.i[i]; k < S.i[i + 1]; ++k)
        if (owner(S.j[k]) != owner(i)) ext[S.j[k]]++;
  }
  cf.assign(S.n, 0);
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 0; r < nr; ++r) {
    const int a = (*rs)[r], b = (*rs)[r + 1];
    Pattern Sl;
    Sl.n = b - a;
    Sl.i.assign(Sl.n + 1, 0);
    std::vector<int> full(Sl.n);
    for (int i = a; i < b; ++i) {
      full[i - a] = S.i[i + 1] - S.i[i];
      for (int k = S.i[i]; k < S.i[i + 1]; ++k)
        if (S.j[k] >= a && S.j[k] < b) Sl.j.push_back(S.j[k] - a);
      Sl.i[i - a + 1] = (int)Sl.j.size();
    }
    std::vector<int> cl;
    coarsen_ruge_first_pass(Sl, nullptr, measure_type, 0, cl, full.data(), f_pnt, ext.empty() ? nullptr : ext.data() + a);
    std::copy(cl.begin(), cl.end(), cf.begin() + a);
  }
}

void coarsen_hmis(const Pattern& S, const CSR* A, int measure_type, int cut_factor, std::vector<int>& cf,
                  const std::vector<int>* rs) {
  if (!rs) {
    coarsen_ruge_first_pass(S, A, measure_type, cut_factor, cf);
  } else {
    if (cut_factor > 0) throw std::runtime_error("rank emulation: HMIS with a cut factor is not restated");
    // local measures: 0, or 3 (the aggressive second pass: local, agg_2)
    if (measure_type != 0 && measure_type != 3)
      throw std::runtime_error("rank emulation: HMIS needs local measures (measure_type 0 or 3)");
    ruge_first_pass_ranks(S, measure_type, Z_PT, cf, rs);
  }
  coarsen_pmis(S, 1, cf, rs);
}

// coarsen_type 11 (ij -ruge1p): the Ruge first pass alone, measure-0 points F
// (par_coarsen.c:1347); with emulated ranks, local (0) or global (1) measures.
void coarsen_ruge1p(const Pattern& S, const CSR* A, int measure_type, int cut_factor, std::vector<int>& cf,
                    const std::vector<int>* rs) {
  if (!rs) {
    coarsen_ruge_first_pass(S, A, measure_type, cut_factor, cf, nullptr, F_PT);
    return;
  }
  if (cut_factor > 0 || (measure_type != 0 && measure_type != 1))
    throw std::runtime_error("rank emulation: coarsen_type 11 needs measure_type 0 or 1 and no cut factor");
  ruge_first_pass_ranks(S, measure_type, F_PT, cf, rs);
}

// ---------------------------------------------------------------------------
// Truncation: parcsr_mv/par_csr_matrix.c:2671 hypre_ParCSRMatrixTruncate with
// rescale = 1, nrm_type = 0 (inf-norm), one thread, no offd.
// hypre_qsort2_abs (utilities/hypre_qsort.c:367) is reproduced exactly because
// the kept entries among equal magnitudes depend on its pivoting.
// ---------------------------------------------------------------------------
static void qsort2_abs(int* v, double* w, int left, int right) {
  if (left >= right) return;
  auto swap2 = [&](int a, int b) { std::swap(v[a], v[b]); std::swap(w[a], w[b]); };
  swap2(left, (left + right) / 2);
  int last = left;
  for (int i = left + 1; i <= right; ++i)
    if (std::fabs(w[i]) > std::fabs(w[left])) swap2(++last, i);
  swap2(left, last);
  qsort2_abs(v, w, left, last - 1);
  qsort2_abs(v, w, last + 1, right);
}

int truncate_row(CSR& P, int r, double tol, int max_elmts, std::vector<int>& rj, std::vector<double>& ra) {
  const int b = P.i[r], e = P.i[r + 1];
  rj.assign(P.j.begin() + b, P.j.begin() + e);
  ra.assign(P.a.begin() + b, P.a.begin() + e);
  if (tol > 0) {
    double row_nrm = 0;
    for (double x : ra) row_nrm = (row_nrm < std::fabs(x)) ? std::fabs(x) : row_nrm;
    const double drop = tol * row_nrm;
    double row_sum = 0, scale = 0;
    size_t o = 0;
    for (size_t k = 0; k < ra.size(); ++k) {
      row_sum += ra[k];
      if (!(std::fabs(ra[k]) < drop)) { scale += ra[k]; rj[o] = rj[k]; ra[o] = ra[k]; ++o; }
    }
    rj.resize(o);
    ra.resize(o);
    if (scale != 0. && scale != row_sum) {
      scale = row_sum / scale;
      for (double& x : ra) x *= scale;
    }
  }
  if (max_elmts > 0 && (int)ra.size() > max_elmts) {
    double row_sum = 0;
    for (double x : ra) row_sum += x;
    qsort2_abs(rj.data(), ra.data(), 0, (int)ra.size() - 1);
    double scale = 0;
    for (int k = 0; k < max_elmts; ++k) scale += ra[k];
    rj.resize(max_elmts);
    ra.resize(max_elmts);
    if (scale != 0. && scale != row_sum) {
      scale = row_sum / scale;
      for (double& x : ra) x *= scale;
    }
  }
  std::copy(rj.begin(), rj.end(), P.j.begin() + b);
  std::copy(ra.begin(), ra.end(), P.a.begin() + b);
  return (int)ra.size();
}

void truncate_rows(CSR& P, double tol, int max_elmts) {
  if (tol <= 0.0 && max_elmts == 0) return;
  const int n = P.nrows;
  std::vector<int> newlen(n, 0);
  // each row is truncated in place inside its own slots (rows are independent)
#pragma omp parallel
  {
    std::vector<int> rj;
    std::vector<double> ra;
#pragma omp for schedule(static)
    for (int r = 0; r < n; ++r) newlen[r] = truncate_row(P, r, tol, max_elmts, rj, ra);
  }
  std::vector<int> ni(n + 1, 0);
  for (int r = 0; r < n; ++r) ni[r + 1] = ni[r] + newlen[r];
  hvec<int> nj(ni[n]);
  hvec<double> na(ni[n]);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) {
    std::copy(P.j.begin() + P.i[r], P.j.begin() + P.i[r] + newlen[r], nj.begin() + ni[r]);
    std::copy(P.a.begin() + P.i[r], P.a.begin() + P.i[r] + newlen[r], na.begin() + ni[r]);
  }
  P.i.swap(ni);
  P.j.swap(nj);
  P.a.swap(na);
}

// ---------------------------------------------------------------------------
// Extended+i interpolation: par_lr_interp.c:1041
// hypre_BoomerAMGBuildExtPIInterpHost, single process, one thread.
// ---------------------------------------------------------------------------
// Ext+i rows [0, nrows) of P.  A and S are indexed in a "universe" of nuniv
// points (the whole matrix in one process; owned rows + ghost points in the
// distributed setup); cf and fine_to_coarse (global coarse index of C points)
// are given for every universe point; rows of A and S are needed for the
// computed rows and their strong F neighbours.  P's columns are global coarse
// indices (ncoarse in all).
// One row of extpi_core.  The reference's P_marker (one int per point) only
// ever tells, for the row being built, whether a point is in its C-hat set
// (marker = the entry's slot, >= jj_begin_row), one of its strong F
// neighbours (marker = strong_f_marker) or neither (a stale value of an
// earlier row); a per-row map (RowMap) answers the same three ways, so every
// row's entries, their order and their sums are unchanged.
static int64_t extpi_bound(const Pattern& S, int i) {
  int64_t b = 1 + (S.i[i + 1] - S.i[i]);
  for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) b += S.i[S.j[jj] + 1] - S.i[S.j[jj]];
  return b;
}
// first pass (par_lr_interp.c:1290-1370): |C-hat_i|
int extpi_row_count(const Pattern& S, const std::vector<int>& cf, int i, RowMap& M) {
  int cnt = 0;
  if (cf[i] >= 0) {
    cnt = 1;
  } else if (cf[i] != SF_PT) {
    M.begin(extpi_bound(S, i));
    bool fresh;
    for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {
      int i1 = S.j[jj];
      if (cf[i1] >= 0) {
        M.find_or_insert(i1, 0, &fresh);
        cnt += fresh;
      } else if (cf[i1] != SF_PT) {
        for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
          int k1 = S.j[kk];
          if (cf[k1] >= 0) {
            M.find_or_insert(k1, 0, &fresh);
            cnt += fresh;
          }
        }
      }
    }
  }
  return cnt;
}
// second pass: row i into P.j / P.a from P.i[i] on
// plus_i false: extended interpolation (interp_type 14, par_lr_interp.c:4686
// hypre_BoomerAMGBuildExtInterpHost, weight loop :5194-5262): a strong F
// neighbour's connection is distributed over C-hat_i only, i itself takes no
// share, so the sum and the distribution leave out a_{i1,i}.
void extpi_row_fill(const CSR& A, const Pattern& S, const std::vector<int>& cf, const std::vector<int>& fine_to_coarse,
                    int i, RowMap& M, CSR& P, bool plus_i) {
  constexpr int kNone = -1, kStrongF = -2;
  const int jj_begin_row = P.i[i];
  int jc = jj_begin_row;
  if (cf[i] >= 0) {
    P.j[jc] = fine_to_coarse[i];
    P.a[jc] = 1.0;
    return;
  }
  if (cf[i] == SF_PT) return;
  M.begin(extpi_bound(S, i));
  bool fresh;
  for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {
    int i1 = S.j[jj];
    if (cf[i1] >= 0) {
      M.find_or_insert(i1, jc, &fresh);
      if (fresh) { P.j[jc] = fine_to_coarse[i1]; P.a[jc] = 0.0; jc++; }
    } else if (cf[i1] != SF_PT) {
      *M.find_or_insert(i1, kStrongF, &fresh) = kStrongF;
      for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
        int k1 = S.j[kk];
        if (cf[k1] >= 0) {
          M.find_or_insert(k1, jc, &fresh);
          if (fresh) { P.j[jc] = fine_to_coarse[k1]; P.a[jc] = 0.0; jc++; }
        }
      }
    }
  }
  const int jj_end_row = jc;
  double diagonal = A.a[A.i[i]];
  for (int jj = A.i[i] + 1; jj < A.i[i + 1]; ++jj) {
    int i1 = A.j[jj];
    const int m1 = M.get(i1, kNone);
    if (m1 >= 0) {
      P.a[m1] += A.a[jj];
    } else if (m1 == kStrongF) {
      double sum = 0.0;
      int sgn = 1;
      if (A.a[A.i[i1]] < 0) sgn = -1;
      for (int jj1 = A.i[i1] + 1; jj1 < A.i[i1 + 1]; ++jj1) {
        int i2 = A.j[jj1];
        if ((M.get(i2, kNone) >= 0 || (plus_i && i2 == i)) && (sgn * A.a[jj1]) < 0) sum += A.a[jj1];
      }
      if (sum != 0) {
        double distribute = A.a[jj] / sum;
        for (int jj1 = A.i[i1] + 1; jj1 < A.i[i1 + 1]; ++jj1) {
          int i2 = A.j[jj1];
          const int m2 = M.get(i2, kNone);
          if (m2 >= 0 && (sgn * A.a[jj1]) < 0) P.a[m2] += distribute * A.a[jj1];
          if (plus_i && i2 == i && (sgn * A.a[jj1]) < 0) diagonal += distribute * A.a[jj1];
        }
      } else {
        diagonal += A.a[jj];
      }
    } else if (cf[i1] != SF_PT && (!hve_setup_dof || hve_setup_dof[i] == hve_setup_dof[i1])) {
      diagonal += A.a[jj];  // a weak neighbour of another function is dropped (par_lr_interp.c:1727)
    }
  }
  if (diagonal) {
    for (int jj = jj_begin_row; jj < jj_end_row; ++jj) P.a[jj] /= -diagonal;
  }
}

// Extended+i where no common C point (interp_type 7; par_lr_interp.c:1932
// hypre_BoomerAMGBuildExtPICCInterp): the interpolatory set is i's strong C
// neighbours, then, for every strong F neighbour i1 (marker -1) that shares
// no strong C neighbour with i, the strong C neighbours of i1; the weights
// are ext+i's (extpi_row_fill's second half, distribution over that set).
static void extpicc_chat(const Pattern& S, const std::vector<int>& cf, int i, RowMap& M, std::vector<int>& out) {
  out.clear();
  constexpr int kStrongF = -2;
  M.begin(extpi_bound(S, i));
  bool fresh;
  for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {  // the C neighbours first
    const int i1 = S.j[jj];
    if (cf[i1] > 0) {
      M.find_or_insert(i1, (int)out.size(), &fresh);
      if (fresh) out.push_back(i1);
    }
  }
  const int ndirect = (int)out.size();
  for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {
    const int i1 = S.j[jj];
    if (cf[i1] != -1) continue;
    *M.find_or_insert(i1, kStrongF, &fresh) = kStrongF;
    bool common = false;
    for (int kk = S.i[i1]; kk < S.i[i1 + 1] && !common; ++kk) {
      const int m = M.get(S.j[kk], -1);
      common = m >= 0 && m < ndirect;  // a strong C neighbour of i itself
    }
    if (common) continue;
    for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
      const int k1 = S.j[kk];
      if (cf[k1] > 0) {
        M.find_or_insert(k1, (int)out.size(), &fresh);
        if (fresh) out.push_back(k1);
      }
    }
  }
}

void build_extpicc_interp(const CSR& A, std::vector<int>& cf, const Pattern& S, double trunc_factor, int max_elmts,
                          CSR& P) {
  const int n = A.nrows;
  std::vector<int> f2c(n, -1);
  int nc = 0;
  for (int i = 0; i < n; ++i)
    if (cf[i] >= 0) f2c[i] = nc++;
  P.resize_rows(n, nc);
  std::vector<int> rowcnt(n, 0);
#pragma omp parallel
  {
    RowMap M;
    std::vector<int> ch;
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) {
      if (cf[i] >= 0) rowcnt[i] = 1;
      else if (cf[i] != SF_PT) {
        extpicc_chat(S, cf, i, M, ch);
        rowcnt[i] = (int)ch.size();
      }
    }
  }
  for (int i = 0; i < n; ++i) P.i[i + 1] = P.i[i] + rowcnt[i];
  P.j.assign(P.i[n], 0);
  P.a.assign(P.i[n], 0.0);
#pragma omp parallel
  {
    RowMap M;
    std::vector<int> ch;
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) {
      const int jb = P.i[i];
      if (cf[i] >= 0) {
        P.j[jb] = f2c[i];
        P.a[jb] = 1.0;
        continue;
      }
      if (cf[i] == SF_PT) continue;
      constexpr int kNone = -1, kStrongF = -2;
      extpicc_chat(S, cf, i, M, ch);  // M: C-hat point -> index, strong F (-1) -> kStrongF
      const int jc = jb + (int)ch.size();
      for (int k = 0; k < (int)ch.size(); ++k) { P.j[jb + k] = f2c[ch[k]]; P.a[jb + k] = 0.0; }
      auto pos = [&](int p) -> int { const int m = M.get(p, kNone); return m >= 0 ? jb + m : m; };
      double diagonal = A.a[A.i[i]];
      for (int jj = A.i[i] + 1; jj < A.i[i + 1]; ++jj) {
        const int i1 = A.j[jj];
        const int m1 = pos(i1);
        if (m1 >= jb) {
          P.a[m1] += A.a[jj];
        } else if (m1 == kStrongF) {
          double sum = 0.0;
          const int sgn = A.a[A.i[i1]] < 0 ? -1 : 1;
          for (int jj1 = A.i[i1] + 1; jj1 < A.i[i1 + 1]; ++jj1) {
            const int i2 = A.j[jj1];
            if ((pos(i2) >= jb || i2 == i) && (sgn * A.a[jj1]) < 0) sum += A.a[jj1];
          }
          if (sum != 0) {
            const double distribute = A.a[jj] / sum;
            for (int jj1 = A.i[i1]; jj1 < A.i[i1 + 1]; ++jj1) {
              const int i2 = A.j[jj1];
              const int m2 = pos(i2);
              if (m2 >= jb && (sgn * A.a[jj1]) < 0) P.a[m2] += distribute * A.a[jj1];
              if (i2 == i && (sgn * A.a[jj1]) < 0) diagonal += distribute * A.a[jj1];
            }
          } else {
            diagonal += A.a[jj];
          }
        } else if (cf[i1] != SF_PT && (!hve_setup_dof || hve_setup_dof[i] == hve_setup_dof[i1])) {
          diagonal += A.a[jj];
        }
      }
      if (diagonal)
        for (int jj = jb; jj < jc; ++jj) P.a[jj] /= -diagonal;
    }
  }
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
  for (int& v : cf)
    if (v == SF_PT) v = F_PT;
}

// Standard interpolation (interp_type 8, 9 = 8 with sep_weight 1;
// par_lr_interp.c:22 hypre_BoomerAMGBuildStdInterp, weight loop :600-910).
// The interpolatory set and its order are ext+i's (extpi_row_fill's first
// half).  The row of A is then "hatted": every strong F neighbour i1 is
// eliminated through its own equation (a_{i,i1} / a_{i1,i1} times row i1
// subtracted), the others added as they stand; each point met gets a slot in
// order of discovery (C-hat points: C slots; i itself first among the F
// slots; any other point an F slot, weak SF neighbours of i left out).  With
// sep_weight 0, alfa = (sum of all slots but the diagonal) / (sum of the C
// slots) / diagonal and w_ij = -alfa * ahat_j; with 1, positive and negative
// slots get their own factor (beta, alfa).  Under rank emulation the slots
// of other-rank points are summed after the own ones (the reference's
// ahat_offd), each group in discovery order.  A row whose factor cannot be
// formed (sum_C * diagonal == 0) keeps the previous row's, as the reference's
// function-scope alfa / beta do (per rank).  Rows of SF points stay empty;
// SF markers become F after (par_lr_interp.c:996).
namespace {
struct StdRow {  // one row's pre-scale data
  double alfa = 0, beta = 0;
  bool has_a = false, has_b = false;
};
}
void build_std_interp(const CSR& A, std::vector<int>& cf, const Pattern& S, double trunc_factor, int max_elmts,
                      int sep_weight, CSR& P, const std::vector<int>* rs, bool partial) {
  const int n = A.nrows;
  std::vector<int> f2c(n, -1);
  int nc = 0;
  for (int i = 0; i < n; ++i)
    if (partial ? cf[i] == 1 : cf[i] >= 0) f2c[i] = nc++;
  // the rows built: every point, or (partial) the first stage's C points
  auto built = [&](int i) { return !partial || cf[i] == 1 || cf[i] == -2; };
  auto rank_of = [&](int p) -> int {
    if (!rs) return 0;
    return (int)(std::upper_bound(rs->begin(), rs->end(), p) - rs->begin()) - 1;
  };
  P.resize_rows(n, nc);
  std::vector<int> rowcnt(n, 0);
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) rowcnt[i] = built(i) ? extpi_row_count(S, cf, i, M) : 0;
  }
  for (int i = 0; i < n; ++i) P.i[i + 1] = P.i[i] + rowcnt[i];
  P.j.assign(P.i[n], 0);
  P.a.assign(P.i[n], 0.0);
  std::vector<StdRow> rw(n);
  std::vector<int> pt(P.i[n], 0);  // interpolatory points (fine indices) of each row, in order
#pragma omp parallel
  {
    RowMap M, H;
    std::vector<int> spt;      // slot -> point
    std::vector<double> sv;    // slot values
    std::vector<char> sc, so;  // slot is a C-hat point / an own-rank point
#pragma omp for schedule(dynamic, 64)
    for (int i = 0; i < n; ++i) {
      if (!built(i)) continue;
      const int jb = P.i[i];
      if (cf[i] >= 0) {
        pt[jb] = i;
        P.a[jb] = 1.0;
        continue;
      }
      if (cf[i] == SF_PT) continue;
      constexpr int kNone = -1, kStrongF = -2;
      M.begin(extpi_bound(S, i));
      int jc = jb;
      bool fresh;
      for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {
        const int i1 = S.j[jj];
        if (cf[i1] >= 0) {
          M.find_or_insert(i1, jc, &fresh);
          if (fresh) pt[jc++] = i1;
        } else if (cf[i1] != SF_PT) {
          *M.find_or_insert(i1, kStrongF, &fresh) = kStrongF;
          for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
            const int k1 = S.j[kk];
            if (cf[k1] >= 0) {
              M.find_or_insert(k1, jc, &fresh);
              if (fresh) pt[jc++] = k1;
            }
          }
        }
      }
      // the hatted row
      int64_t hb = 1 + (A.i[i + 1] - A.i[i]);
      for (int jj = A.i[i] + 1; jj < A.i[i + 1]; ++jj) hb += A.i[A.j[jj] + 1] - A.i[A.j[jj]];
      H.begin(hb);
      spt.clear(); sv.clear(); sc.clear(); so.clear();
      const int ri = rank_of(i);
      auto slot = [&](int p, bool isc) -> int {
        int* v = H.find_or_insert(p, (int)spt.size(), &fresh);
        if (fresh) {
          spt.push_back(p);
          sv.push_back(0.0);
          sc.push_back(isc ? 1 : 0);
          so.push_back(rank_of(p) == ri ? 1 : 0);
        }
        return *v;
      };
      const int dslot = slot(i, false);
      sv[dslot] = A.a[A.i[i]];
      for (int jj = A.i[i] + 1; jj < A.i[i + 1]; ++jj) {
        const int i1 = A.j[jj];
        const int m1 = M.get(i1, kNone);
        if (m1 != kStrongF) {
          const int h = H.get(i1, -1);
          if (h >= 0) sv[h] += A.a[jj];
          else if (m1 >= 0) { const int q = slot(i1, true); sv[q] += A.a[jj]; }
          else if (cf[i1] != SF_PT) { const int q = slot(i1, false); sv[q] += A.a[jj]; }
        } else {
          const double distribute = A.a[jj] / A.a[A.i[i1]];
          for (int kk = A.i[i1] + 1; kk < A.i[i1 + 1]; ++kk) {
            const int k1 = A.j[kk];
            int h = H.get(k1, -1);
            if (h < 0) h = slot(k1, M.get(k1, kNone) >= 0);
            sv[h] -= A.a[kk] * distribute;
          }
        }
      }
      const double diagonal = sv[dslot];
      StdRow& r = rw[i];
      if (sep_weight == 1) {
        double spc = 0, snc = 0;
        for (int pass = 1; pass >= 0; --pass)  // own-rank slots, then the others
          for (size_t q = 0; q < spt.size(); ++q)
            if (sc[q] && so[q] == pass) {
              if (sv[q] > 0) spc += sv[q];
              else snc += sv[q];
            }
        double sp = spc, sn = snc;
        for (int pass = 1; pass >= 0; --pass)
          for (size_t q = 0; q < spt.size(); ++q)
            if (!sc[q] && so[q] == pass && (int)q != dslot) {
              if (sv[q] > 0) sp += sv[q];
              else sn += sv[q];
            }
        if (snc * diagonal != 0) { r.alfa = sn / snc / diagonal; r.has_a = true; }
        if (spc * diagonal != 0) { r.beta = sp / spc / diagonal; r.has_b = true; }
      } else {
        double sum_c = 0;
        for (int pass = 1; pass >= 0; --pass)
          for (size_t q = 0; q < spt.size(); ++q)
            if (sc[q] && so[q] == pass) sum_c += sv[q];
        double sum = sum_c;
        for (int pass = 1; pass >= 0; --pass)
          for (size_t q = 0; q < spt.size(); ++q)
            if (!sc[q] && so[q] == pass && (int)q != dslot) sum += sv[q];
        if (sum_c * diagonal != 0) { r.alfa = sum / sum_c / diagonal; r.has_a = true; }
      }
      for (int jj = jb; jj < jc; ++jj) P.a[jj] = sv[H.get(pt[jj], -1)];  // ahat, scaled below
    }
  }
  // the factors carried from row to row (per rank, in row order), then the weights
  {
    const int nr = rs ? (int)rs->size() - 1 : 1;
    for (int k = 0; k < nr; ++k) {
      const int r0 = rs ? (*rs)[k] : 0, r1 = rs ? (*rs)[k + 1] : n;
      double alfa = 1.0, beta = 1.0;
      for (int i = r0; i < r1; ++i) {
        if (!built(i) || cf[i] >= 0 || cf[i] == SF_PT) continue;
        if (rw[i].has_a) alfa = rw[i].alfa;
        if (rw[i].has_b) beta = rw[i].beta;
        rw[i].alfa = alfa;
        rw[i].beta = beta;
      }
    }
  }
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    for (int jj = P.i[i]; jj < P.i[i + 1]; ++jj) {
      if (cf[i] < 0) {
        const double ah = P.a[jj];
        P.a[jj] = (sep_weight == 1 && ah > 0) ? -rw[i].beta * ah : -rw[i].alfa * ah;
      }
      P.j[jj] = f2c[pt[jj]];
    }
  }
  if (partial) {  // rows of the first stage's C points only, in order
    CSR Pc;
    std::vector<int> old;
    for (int i = 0; i < n; ++i)
      if (built(i)) old.push_back(i);
    const int no = (int)old.size();
    Pc.resize_rows(no, nc);
    for (int k = 0; k < no; ++k) Pc.i[k + 1] = Pc.i[k] + rowcnt[old[k]];
    Pc.j.assign(Pc.i[no], 0);
    Pc.a.assign(Pc.i[no], 0.0);
#pragma omp parallel for schedule(static)
    for (int k = 0; k < no; ++k) {
      const int i = old[k];
      std::copy(P.j.begin() + P.i[i], P.j.begin() + P.i[i + 1], Pc.j.begin() + Pc.i[k]);
      std::copy(P.a.begin() + P.i[i], P.a.begin() + P.i[i + 1], Pc.a.begin() + Pc.i[k]);
    }
    P = std::move(Pc);
  }
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
  for (int& v : cf)  // par_lr_interp.c:996; the partial form: partial.c:1812
    if (partial ? v < -1 : v == SF_PT) v = F_PT;
}

// Row lists for the device setup's host fallback and its table bounds
// (OpenMP here; setup_dev.hip is compiled without it).
int64_t extpi_bound_max(const Pattern& S) {
  int64_t m = 1;
#pragma omp parallel for reduction(max : m) schedule(static)
  for (int i = 0; i < S.n; ++i) m = std::max(m, extpi_bound(S, i));
  return m;
}
void extpi_count_rows(const Pattern& S, const std::vector<int>& cf, const std::vector<int>& rows,
                      std::vector<int>& cnt) {
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(dynamic, 64)
    for (size_t k = 0; k < rows.size(); ++k) cnt[rows[k]] = extpi_row_count(S, cf, rows[k], M);
  }
}
void extpi_fill_rows(const CSR& A, const Pattern& S, const std::vector<int>& cf,
                     const std::vector<int>& fine_to_coarse, const std::vector<int>& rows, CSR& P) {
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(dynamic, 64)
    for (size_t k = 0; k < rows.size(); ++k) extpi_row_fill(A, S, cf, fine_to_coarse, rows[k], M, P);
  }
}
void truncate_row_list(CSR& P, const std::vector<int>& rows, double tol, int max_elmts, std::vector<int>& newlen) {
#pragma omp parallel
  {
    std::vector<int> rj;
    std::vector<double> ra;
#pragma omp for schedule(dynamic, 16)
    for (size_t k = 0; k < rows.size(); ++k) newlen[rows[k]] = truncate_row(P, rows[k], tol, max_elmts, rj, ra);
  }
}
int64_t rap_bound_max(const CSR& R, const CSR& A) {
  int64_t m = 1;
#pragma omp parallel for reduction(max : m) schedule(static)
  for (int q = 0; q < R.nrows; ++q) {
    int64_t b = 0;
    for (int jj = R.i[q]; jj < R.i[q + 1]; ++jj) b += A.i[R.j[jj] + 1] - A.i[R.j[jj]];
    m = std::max(m, b);
  }
  return m;
}
void rap_row_list(const CSR& R, const CSR& A, const CSR& P, const std::vector<int>& rows,
                  std::vector<std::vector<int>>& oj, std::vector<std::vector<double>>& oa) {
  oj.assign(rows.size(), {});
  oa.assign(rows.size(), {});
#pragma omp parallel
  {
    RapScratch W;
#pragma omp for schedule(dynamic, 16)
    for (size_t k = 0; k < rows.size(); ++k) {
      rap_row(R, A, P, rows[k], rows[k], W);
      oj[k] = W.tj;
      oa[k] = W.ta;
    }
  }
}

void extpi_core(const CSR& A, const Pattern& S, const std::vector<int>& cf, const std::vector<int>& fine_to_coarse,
                int nrows, int ncoarse, int nuniv, CSR& P, bool plus_i) {
  (void)nuniv;
  const int n = nrows;
  P.resize_rows(n, ncoarse);
  std::vector<int> rowcnt(n, 0);
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) rowcnt[i] = extpi_row_count(S, cf, i, M);
  }
  for (int i = 0; i < n; ++i) P.i[i + 1] = P.i[i] + rowcnt[i];
  const int64_t nnzP = P.i[n];
  P.j.assign(nnzP, 0);
  P.a.assign(nnzP, 0.0);
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) extpi_row_fill(A, S, cf, fine_to_coarse, i, M, P, plus_i);
  }
}

void build_extpi_interp(const CSR& A, std::vector<int>& cf, const Pattern& S,
                        double trunc_factor, int max_elmts, CSR& P, bool plus_i) {
  const int n = A.nrows;
  std::vector<int> fine_to_coarse(n, -1);
  int coarse_counter = 0;
  for (int i = 0; i < n; ++i)
    if (cf[i] >= 0) fine_to_coarse[i] = coarse_counter++;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double t0 = now();
  extpi_core(A, S, cf, fine_to_coarse, n, coarse_counter, n, P, plus_i);
  double t1 = now();
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
  if (getenv("HVE_SETUP_T")) fprintf(stderr, "extpi core %.3f trunc %.3f\n", t1 - t0, now() - t1);
  for (int i = 0; i < n; ++i)
    if (cf[i] == SF_PT) cf[i] = F_PT;
}

// ---------------------------------------------------------------------------
// Interpolation in matrix-matrix form (par_mod_lr_interp.c, par_2s_interp.c),
// one process.  The pieces:
// * fffc: As_FF / As_FC as gen_fffc.c:19 hypre_ParCSRMatrixGenerateFFFC
//   (partial = false: rows = F points, CF < 0) or gen_fffc.c:506
//   hypre_ParCSRMatrixGenerateFFFC3 (partial = true: As_FF rows = the -2
//   points only, As_FC rows = every F point).  An As_FF row is the diagonal,
//   then the strong non-C neighbours (columns: index among the non-C points);
//   an As_FC row the strong C neighbours (columns: coarse index); both in S's
//   order, values from A (the first match after the diagonal).
// * matmul_first_touch: hypre_ParMatmul (par_csr_matop.c:277), the CPU
//   build's product for W = As_FF As_FC and P = P1 P2.
// SF points (-3) count as F and keep their marker (these builders do not
// reset it, unlike ext+i).
// ---------------------------------------------------------------------------
static void fffc(const CSR& A, const std::vector<int>& cf, const Pattern& S, bool partial, CSR& FF, CSR& FC,
                 std::vector<int>& frow, std::vector<int>& ffrow) {
  const int n = A.nrows;
  std::vector<int> f2f(n, -1), f2c(n, -1);
  int nC = 0, nF = 0;
  frow.clear();
  ffrow.clear();
  for (int i = 0; i < n; ++i) {
    if (cf[i] > 0) f2c[i] = nC++;
    else f2f[i] = nF++;
    if (cf[i] < 0) frow.push_back(i);
    if (partial ? cf[i] == -2 : cf[i] < 0) ffrow.push_back(i);
  }
  const int nfr = (int)frow.size(), nff = (int)ffrow.size();
  FC.resize_rows(nfr, nC);
  FF.resize_rows(nff, nF);
  for (int r = 0; r < nfr; ++r) {
    const int i = frow[r];
    int c = 0;
    for (int q = S.i[i]; q < S.i[i + 1]; ++q) c += cf[S.j[q]] > 0;
    FC.i[r + 1] = FC.i[r] + c;
  }
  for (int r = 0; r < nff; ++r) {
    const int i = ffrow[r];
    int c = 1;
    for (int q = S.i[i]; q < S.i[i + 1]; ++q) c += cf[S.j[q]] <= 0;
    FF.i[r + 1] = FF.i[r] + c;
  }
  FC.j.resize(FC.i[nfr]);
  FC.a.resize(FC.i[nfr]);
  FF.j.resize(FF.i[nff]);
  FF.a.resize(FF.i[nff]);
  auto aval = [&](int i, int js) {
    int ja = A.i[i] + 1;
    while (A.j[ja] != js) ja++;
    return A.a[ja];
  };
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nfr; ++r) {
    const int i = frow[r];
    int c = FC.i[r];
    for (int q = S.i[i]; q < S.i[i + 1]; ++q)
      if (cf[S.j[q]] > 0) { FC.j[c] = f2c[S.j[q]]; FC.a[c++] = aval(i, S.j[q]); }
  }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nff; ++r) {
    const int i = ffrow[r];
    int c = FF.i[r];
    FF.j[c] = f2f[A.j[A.i[i]]];
    FF.a[c++] = A.a[A.i[i]];
    for (int q = S.i[i]; q < S.i[i + 1]; ++q)
      if (cf[S.j[q]] <= 0) { FF.j[c] = f2f[S.j[q]]; FF.a[c++] = aval(i, S.j[q]); }
  }
}

// Owners under N-rank emulation (hypre_BoomerAMGSetRankEmulation): the rank
// of each row of X, of each column of X (= row of Y) and of each column of Y.
struct MatmulRanks {
  std::vector<int> row, xcol, ycol;
  int nranks = 0;
};
// With ranks, the np > 1 order of hypre_ParMatmul (par_csr_matop.c:860-1000):
// a row's entries in other ranks' columns (A_offd) go first, each through its
// B row's other-rank columns (B_ext_offd) and then own ones (B_ext_diag); then
// the own-column entries (A_diag), through B_diag then B_offd; the product row
// is C_diag's first-touch list followed by C_offd's.
// square_mode: -1 the product's own sizes decide hypre_ParMatmul's allsquare
// (a zero diagonal entry first); 0 / 1 the caller's global sizes (the
// distributed setup multiplies a rank's universe, not the whole matrix).
static void matmul_first_touch(const CSR& X, const CSR& Y, CSR& C, const MatmulRanks* rk = nullptr,
                               int square_mode = -1) {
  const int nr = X.nrows, nc = Y.ncols;
  bool square = square_mode < 0 ? nr == nc : square_mode != 0;
  std::vector<int> lrows, lcols;  // emulated: rows / Y columns per rank (allsquare is local too)
  if (rk) {
    lrows.assign(rk->nranks, 0);
    lcols.assign(rk->nranks, 0);
    for (int r : rk->row) lrows[r]++;
    for (int c : rk->ycol) lcols[c]++;
  }
  std::vector<int> rfirst(lrows.size() + 1, 0), cfirst(lcols.size() + 1, 0);  // rows / columns owned by ranks < R
  for (size_t q = 0; q < lrows.size(); ++q) { rfirst[q + 1] = rfirst[q] + lrows[q]; cfirst[q + 1] = cfirst[q] + lcols[q]; }
  std::vector<std::vector<int>> cj(nr);
  std::vector<std::vector<double>> ca(nr);
#pragma omp parallel
  {
    std::vector<int> mark(std::max(nc, 1), -1);
    std::vector<int> touched;
    std::vector<int> oj;  // emulated: the C_offd list
    std::vector<double> oa;
#pragma omp for schedule(dynamic, 256)
    for (int r = 0; r < nr; ++r) {
      std::vector<int>& rj = cj[r];
      std::vector<double>& ra = ca[r];
      touched.clear();
      if (!rk) {
        if (square) { mark[r] = 0; rj.push_back(r); ra.push_back(0.0); touched.push_back(r); }
        for (int q = X.i[r]; q < X.i[r + 1]; ++q) {
          const double ae = X.a[q];
          const int k = X.j[q];
          for (int t = Y.i[k]; t < Y.i[k + 1]; ++t) {
            const int c = Y.j[t];
            if (mark[c] < 0) {
              mark[c] = (int)rj.size();
              touched.push_back(c);
              rj.push_back(c);
              ra.push_back(ae * Y.a[t]);
            } else {
              ra[mark[c]] += ae * Y.a[t];
            }
          }
        }
      } else {
        const int R = rk->row[r];
        oj.clear();
        oa.clear();
        if (square && lrows[R] == lcols[R]) {  // C_{i1,i1}: the rank's local diagonal
          const int c = cfirst[R] + (r - rfirst[R]);
          mark[c] = 0; rj.push_back(c); ra.push_back(0.0); touched.push_back(c);
        }
        auto add = [&](double ae, int c, double b) {
          const bool own = rk->ycol[c] == R;
          std::vector<int>& lj = own ? rj : oj;
          std::vector<double>& la = own ? ra : oa;
          if (mark[c] < 0) {
            mark[c] = (int)lj.size();
            touched.push_back(c);
            lj.push_back(c);
            la.push_back(ae * b);
          } else {
            la[mark[c]] += ae * b;
          }
        };
        for (int pass = 0; pass < 2; ++pass)  // 0: A_offd entries, 1: A_diag entries
          for (int q = X.i[r]; q < X.i[r + 1]; ++q) {
            const int k = X.j[q];
            if ((rk->xcol[k] == R) != (pass == 1)) continue;
            const double ae = X.a[q];
            for (int half = 0; half < 2; ++half)  // A_offd: B_ext_offd first; A_diag: B_diag first
              for (int t = Y.i[k]; t < Y.i[k + 1]; ++t) {
                const bool own = rk->ycol[Y.j[t]] == R;
                if (own != ((pass == 1) == (half == 0))) continue;
                add(ae, Y.j[t], Y.a[t]);
              }
          }
        rj.insert(rj.end(), oj.begin(), oj.end());
        ra.insert(ra.end(), oa.begin(), oa.end());
      }
      for (int c : touched) mark[c] = -1;
    }
  }
  C.resize_rows(nr, nc);
  for (int r = 0; r < nr; ++r) C.i[r + 1] = C.i[r] + (int)cj[r].size();
  C.j.resize(C.i[nr]);
  C.a.resize(C.i[nr]);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nr; ++r) {
    std::copy(cj[r].begin(), cj[r].end(), C.j.begin() + C.i[r]);
    std::copy(ca[r].begin(), ca[r].end(), C.a.begin() + C.i[r]);
  }
}

// Owners of W = As_FF As_FC's rows and columns under rank emulation (emul:
// fine row starts); nullptr without it.
static std::unique_ptr<MatmulRanks> mm_ranks(const std::vector<int>& cf, const std::vector<int>& ffrow,
                                             const std::vector<int>* emul) {
  if (!emul || emul->size() <= 2) return nullptr;
  auto owner = [&](int i) { return (int)(std::upper_bound(emul->begin(), emul->end(), i) - emul->begin()) - 1; };
  auto rk = std::make_unique<MatmulRanks>();
  rk->nranks = (int)emul->size() - 1;
  for (int i : ffrow) rk->row.push_back(owner(i));
  for (int i = 0; i < (int)cf.size(); ++i) (cf[i] > 0 ? rk->ycol : rk->xcol).push_back(owner(i));
  return rk;
}

// P's rows: `rows` (fine points, in order) are C points (cf > 0: injection at
// their coarse index) or take the next row of W.
static void assemble_mm_p(const std::vector<int>& cf, const std::vector<int>& rows, const CSR& W, int ncoarse,
                          CSR& P) {
  const int n = (int)rows.size();
  P.resize_rows(n, ncoarse);
  std::vector<int> wr(n, -1);
  int c = 0, w = 0;
  for (int r = 0; r < n; ++r) {
    if (cf[rows[r]] > 0) { P.i[r + 1] = P.i[r] + 1; ++c; }
    else { wr[r] = w; P.i[r + 1] = P.i[r] + (W.i[w + 1] - W.i[w]); ++w; }
  }
  P.j.resize(P.i[n]);
  P.a.resize(P.i[n]);
  c = 0;
  for (int r = 0; r < n; ++r) {
    const int b = P.i[r];
    if (wr[r] < 0) { P.j[b] = c++; P.a[b] = 1.0; continue; }
    std::copy(W.j.begin() + W.i[wr[r]], W.j.begin() + W.i[wr[r] + 1], P.j.begin() + b);
    std::copy(W.a.begin() + W.i[wr[r]], W.a.begin() + W.i[wr[r] + 1], P.a.begin() + b);
  }
}

// Extended+e (interp_type 18, agg_interp_type 7's first stage):
// par_mod_lr_interp.c:1040 hypre_BoomerAMGBuildModExtPEInterpHost, the
// diagonal scalings of :1204-1318.  Extended (agg_interp_type 5's first
// stage, pe = false): :16 hypre_BoomerAMGBuildModExtInterpHost, :170-245.
void build_modext_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                         int max_elmts, bool pe, CSR& P, const std::vector<int>* emul, int mm_square) {
  CSR FF, FC;
  std::vector<int> frow, ffrow;
  fffc(A, cf, S, false, FF, FC, frow, ffrow);
  const int nF = (int)frow.size();
  std::vector<double> lam(nF, 0.0), beta(nF, 0.0), tmp(nF, 0.0), dw(nF, 0.0), tau(nF, 0.0);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    for (int q = FC.i[r]; q < FC.i[r + 1]; ++q) beta[r] += FC.a[q];
    if (!pe) continue;
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) lam[r] += FF.a[q];
    const double number = (double)(FF.i[r + 1] - FF.i[r] - 1);
    if (number) lam[r] /= number;
    if (lam[r] + beta[r]) tmp[r] = lam[r] / (beta[r] + lam[r]);
  }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    const int i = frow[r];
    for (int q = A.i[i]; q < A.i[i + 1]; ++q) dw[r] += A.a[q];
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) dw[r] -= FF.a[q];
    dw[r] -= beta[r];
    if (pe)
      for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) tau[r] += FF.a[q] * tmp[FF.j[q]];
  }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    double fscale, cscale;
    if (pe) {
      double value = dw[r] + tau[r];
      if (value) value = -1.0 / value;
      double theta = beta[r] + lam[r];
      FF.a[FF.i[r]] = value * theta;
      if (theta) theta = 1.0 / theta;
      fscale = value;
      cscale = theta;
    } else {
      const double b = dw[r] ? 1.0 / dw[r] : 1.0;
      FF.a[FF.i[r]] = b * beta[r];
      fscale = b;
      cscale = beta[r] ? -1.0 / beta[r] : 1.0;
    }
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) FF.a[q] *= fscale;
    for (int q = FC.i[r]; q < FC.i[r + 1]; ++q) FC.a[q] *= cscale;
  }
  CSR W;
  const auto rk = mm_ranks(cf, ffrow, emul);
  matmul_first_touch(FF, FC, W, rk.get(), mm_square);
  std::vector<int> all(A.nrows);
  for (int i = 0; i < A.nrows; ++i) all[i] = i;
  assemble_mm_p(cf, all, W, FC.ncols, P);
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
}

void build_modextpe_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                           int max_elmts, CSR& P, const std::vector<int>* emul, int mm_square) {
  build_modext_interp(A, cf, S, trunc_factor, max_elmts, true, P, emul, mm_square);
}

// Extended+i in matrix-matrix form (interp_type 17): par_mod_lr_interp.c:474
// hypre_BoomerAMGBuildModExtPIInterpHost (:640-800).  As_FF's off-diagonal
// a_ij is divided by D_q[j] + a_ji (a_ji from an unmodified copy; D_q[j] alone
// when j has no strong connection back to i), those a_ji shares form D_theta,
// the diagonal is 1, and the row is scaled by -1 / (D_theta + D_w); As_FC is
// used as is.
void build_modextpi_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                           int max_elmts, CSR& P, const std::vector<int>* emul, int mm_square) {
  CSR FF, FC;
  std::vector<int> frow, ffrow;
  fffc(A, cf, S, false, FF, FC, frow, ffrow);
  const int nF = (int)frow.size();
  const hvec<double> orig = FF.a;
  std::vector<double> dq(nF, 0.0), dw(nF, 0.0), dth(nF, 0.0);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r)
    for (int q = FC.i[r]; q < FC.i[r + 1]; ++q) dq[r] += FC.a[q];
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    const int i = frow[r];
    for (int q = A.i[i]; q < A.i[i + 1]; ++q) dw[r] += A.a[q];
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) dw[r] -= FF.a[q];
    dw[r] -= dq[r];
  }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) {
      const int jj = FF.j[q];
      double value = dq[jj];
      for (int k = FF.i[jj] + 1; k < FF.i[jj + 1]; ++k)
        if (FF.j[k] == r) {
          const double value1 = orig[k];
          value += value1;
          dth[r] += FF.a[q] * value1 / value;
          break;
        }
      FF.a[q] /= value;
    }
    FF.a[FF.i[r]] = 1.0;
    double theta = dth[r] + dw[r];
    if (theta) {
      theta = -1.0 / theta;
      for (int q = FF.i[r]; q < FF.i[r + 1]; ++q) FF.a[q] *= theta;
    }
  }
  CSR W;
  const auto rk = mm_ranks(cf, ffrow, emul);
  matmul_first_touch(FF, FC, W, rk.get(), mm_square);
  std::vector<int> all(A.nrows);
  for (int i = 0; i < A.nrows; ++i) all[i] = i;
  assemble_mm_p(cf, all, W, FC.ncols, P);
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
}

// Second stage of the 2-stage aggressive interpolations (cf: 1 = C of both
// stages, -2 = C of the first stage only): P2 from the first stage's C
// points to the second's.  agg_interp_type 5: par_2s_interp.c:15
// hypre_BoomerAMGBuildModPartialExtInterpHost (:180-330); 7 (pe): :564
// hypre_BoomerAMGBuildModPartialExtPEInterpHost (:730-900), with D_lambda as
// gen_fffc.c:1056 hypre_ParCSRMatrixGenerateFFFCD3 forms it (every F row: the
// mean of its strong non-C connections).
void build_modpartialext_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                                int max_elmts, bool pe, CSR& P, const std::vector<int>* emul, int mm_square) {
  CSR FF, FC;
  std::vector<int> frow, ffrow;
  fffc(A, cf, S, true, FF, FC, frow, ffrow);
  const int nF = (int)frow.size(), nN = (int)ffrow.size();
  std::vector<int> f2f(A.nrows, -1);
  {
    int k = 0;
    for (int i = 0; i < A.nrows; ++i)
      if (cf[i] < 0) f2f[i] = k++;
  }
  std::vector<double> dq(nF, 0.0), dw(nN, 0.0), lam(nF, 0.0), dinv(nF, 0.0), tau(nN, 0.0);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    for (int q = FC.i[r]; q < FC.i[r + 1]; ++q) dq[r] += FC.a[q];
    if (!pe) continue;
    const int i = frow[r];
    double sum = 0;
    for (int q = S.i[i]; q < S.i[i + 1]; ++q) {
      const int js = S.j[q];
      if (cf[js] > 0) continue;
      int ja = A.i[i] + 1;
      while (A.j[ja] != js) ja++;
      sum += 1;
      lam[r] += A.a[ja];
    }
    if (sum) lam[r] = lam[r] / sum;
    if (dq[r] + lam[r]) dinv[r] = 1.0 / (dq[r] + lam[r]);
  }
  // As_FF's columns index the non-C points; with cf in {1, -1, -2, -3} they
  // are exactly the F rows (CF < 0), so dq is indexed by them directly
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nN; ++r) {
    const int i = ffrow[r];
    if (pe) {
      for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) tau[r] += FF.a[q] * lam[FF.j[q]] * dinv[FF.j[q]];
      for (int q = A.i[i]; q < A.i[i + 1]; ++q) dw[r] += A.a[q];
      for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q)
        if (dinv[FF.j[q]]) dw[r] -= FF.a[q];
      dw[r] += tau[r] - dq[f2f[i]];
      continue;
    }
    for (int q = A.i[i]; q < A.i[i + 1]; ++q) dw[r] += A.a[q];
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q)
      if (dq[FF.j[q]]) dw[r] -= FF.a[q];
    dw[r] -= dq[f2f[i]];
  }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nN; ++r) {
    if (!dw[r]) continue;  // the reference leaves such a row unscaled, diagonal included
    const int fi = f2f[ffrow[r]];
    const double b = pe ? -1.0 / dw[r] : 1.0 / dw[r];
    FF.a[FF.i[r]] = pe ? b * (dq[fi] + lam[fi]) : b * dq[fi];
    for (int q = FF.i[r] + 1; q < FF.i[r + 1]; ++q) FF.a[q] *= b;
  }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < nF; ++r) {
    const double g = pe ? dinv[r] : dq[r] ? -1.0 / dq[r] : 0.0;
    for (int q = FC.i[r]; q < FC.i[r + 1]; ++q) FC.a[q] *= g;
  }
  CSR W;
  const auto rk = mm_ranks(cf, ffrow, emul);
  matmul_first_touch(FF, FC, W, rk.get(), mm_square);
  std::vector<int> c1;  // rows of P2: the first stage's C points, in order
  for (int i = 0; i < A.nrows; ++i)
    if (cf[i] > 0 || cf[i] == -2) c1.push_back(i);
  assemble_mm_p(cf, c1, W, FC.ncols, P);
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
}

// Second stage of the classical 2-stage aggressive interpolations:
// agg_interp_type 1 / 6 (partial.c:16 hypre_BoomerAMGBuildPartialExtPIInterp)
// and 3 (partial.c:1855 hypre_BoomerAMGBuildPartialExtInterp, plus_i false).
// Rows are the first stage's C points in order (cf 1: the identity to the
// second stage's C point, cf -2: an interpolated row), columns the second
// stage's C points.  An interpolated row is extpi_row_fill's over the combined
// marker: C neighbours are cf >= 0, strong F neighbours any other point but
// an SF one (-3), the weight loop the same (partial.c:590-700 / :2360-2430).
// Truncated with the P12 parameters inside (partial.c:797 / :2552); then
// every marker below -1 becomes -1 (partial.c:818 / :2573).
void build_partial_extpi_interp(const CSR& A, std::vector<int>& cf, const Pattern& S, double trunc_factor,
                                int max_elmts, bool plus_i, CSR& P) {
  const int n = A.nrows;
  std::vector<int> fine_to_coarse(n, -1), old;
  int nc = 0;
  for (int i = 0; i < n; ++i) {
    if (cf[i] == 1) fine_to_coarse[i] = nc++;
    if (cf[i] == 1 || cf[i] == -2) old.push_back(i);
  }
  const int no = (int)old.size();
  CSR Pf;  // fine-row indexed: only the first stage's C points hold entries
  Pf.resize_rows(n, nc);
  std::vector<int> rowcnt(n, 0);
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(static)
    for (int k = 0; k < no; ++k) rowcnt[old[k]] = extpi_row_count(S, cf, old[k], M);
  }
  for (int i = 0; i < n; ++i) Pf.i[i + 1] = Pf.i[i] + rowcnt[i];
  Pf.j.assign(Pf.i[n], 0);
  Pf.a.assign(Pf.i[n], 0.0);
#pragma omp parallel
  {
    RowMap M;
#pragma omp for schedule(static)
    for (int k = 0; k < no; ++k) extpi_row_fill(A, S, cf, fine_to_coarse, old[k], M, Pf, plus_i);
  }
  P.resize_rows(no, nc);
  for (int k = 0; k < no; ++k) P.i[k + 1] = P.i[k] + rowcnt[old[k]];
  P.j.assign(P.i[no], 0);
  P.a.assign(P.i[no], 0.0);
#pragma omp parallel for schedule(static)
  for (int k = 0; k < no; ++k) {
    const int i = old[k];
    std::copy(Pf.j.begin() + Pf.i[i], Pf.j.begin() + Pf.i[i + 1], P.j.begin() + P.i[k]);
    std::copy(Pf.a.begin() + Pf.i[i], Pf.a.begin() + Pf.i[i + 1], P.a.begin() + P.i[k]);
  }
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
  for (int& v : cf)
    if (v < -1) v = -1;
}

// P = P1 P2 (par_amg_setup.c:1681 hypre_ParMatmul), then the aggressive
// truncation (:1685)
void multiply_interp(const CSR& P1, const CSR& P2, double trunc_factor, int max_elmts, CSR& P, int mm_square) {
  matmul_first_touch(P1, P2, P, nullptr, mm_square);
  truncate_rows(P, trunc_factor, max_elmts);
}

// Direct interpolation (interp_type 3): par_interp.c hypre_BoomerAMGBuildDirInterp
// host path, one process.  Weights from strong C neighbours, positive and
// negative off-diagonals distributed separately.
void build_direct_interp(const CSR& A, std::vector<int>& cf, const Pattern& S,
                         double trunc_factor, int max_elmts, CSR& P) {
  const int n = A.nrows;
  std::vector<int> fine_to_coarse(n, -1);
  P.resize_rows(n, 0);
  int cc = 0;
  for (int i = 0; i < n; ++i) {
    int c = 0;
    if (cf[i] >= 0) { c = 1; fine_to_coarse[i] = cc++; }
    else for (int k = S.i[i]; k < S.i[i + 1]; ++k) if (cf[S.j[k]] >= 0) ++c;
    P.i[i + 1] = P.i[i] + c;
  }
  P.ncols = cc;
  P.j.assign(P.i[n], 0);
  P.a.assign(P.i[n], 0.0);
  std::vector<int> P_marker(n, -1);
  // par_interp.c:2008: alfa/beta are initialised once and carried across rows
  // whose strong-C sums vanish (single-thread semantics).
  double alfa = 1.0, beta = 1.0;
  for (int i = 0; i < n; ++i) {
    int jc = P.i[i];
    if (cf[i] >= 0) { P.j[jc] = fine_to_coarse[i]; P.a[jc] = 1.0; continue; }
    const int begin = jc;
    for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
      int i1 = S.j[k];
      if (cf[i1] >= 0) { P_marker[i1] = jc; P.j[jc] = fine_to_coarse[i1]; P.a[jc] = 0.0; ++jc; }
    }
    const int end = jc;
    const double diagonal = A.a[A.i[i]];
    double sum_N_pos = 0, sum_N_neg = 0, sum_P_pos = 0, sum_P_neg = 0;
    for (int k = A.i[i] + 1; k < A.i[i + 1]; ++k) {
      int i1 = A.j[k];
      double v = A.a[k];
      if (v > 0) sum_N_pos += v; else sum_N_neg += v;
      if (P_marker[i1] >= begin) {
        P.a[P_marker[i1]] += v;
        if (v > 0) sum_P_pos += v; else sum_P_neg += v;
      }
    }
    if (sum_P_neg) alfa = sum_N_neg / sum_P_neg / diagonal;
    if (sum_P_pos) beta = sum_N_pos / sum_P_pos / diagonal;
    for (int k = begin; k < end; ++k) {
      if (P.a[k] > 0) P.a[k] *= -beta; else P.a[k] *= -alfa;
    }
  }
  if (trunc_factor != 0.0 || max_elmts > 0) truncate_rows(P, trunc_factor, max_elmts);
  for (int i = 0; i < n; ++i)
    if (cf[i] == SF_PT) cf[i] = F_PT;
}

// ---------------------------------------------------------------------------
// Transpose: seq_mv/csr_matop.c:578 (counting sort; rows of A^T list the
// original row indices in ascending order).
// ---------------------------------------------------------------------------
void transpose(const CSR& A, CSR& AT) {
  AT.resize_rows(A.ncols, A.nrows);
  for (int64_t k = 0; k < A.nnz(); ++k) AT.i[A.j[k] + 1]++;
  for (int r = 0; r < A.ncols; ++r) AT.i[r + 1] += AT.i[r];
  AT.j.resize(A.nnz());
  AT.a.resize(A.nnz());
  std::vector<int> pos(AT.i.begin(), AT.i.end() - 1);
  for (int r = 0; r < A.nrows; ++r)
    for (int k = A.i[r]; k < A.i[r + 1]; ++k) {
      int c = A.j[k];
      AT.j[pos[c]] = r;
      AT.a[pos[c]] = A.a[k];
      pos[c]++;
    }
}

// ---------------------------------------------------------------------------
// Galerkin product RAP = P^T A P: par_rap.c:27 hypre_BoomerAMGBuildCoarseOperatorKT,
// single process (the RA row is formed first, then RA*P, each with first-touch
// column order and the diagonal placed first).  Parallel over coarse rows with
// the row structure computed in a first pass.
// ---------------------------------------------------------------------------
// Rows of C for the coarse rows R holds.  Universe indexing as in
// extpi_core: R's columns and A's rows / columns are fine-universe indices,
// P's rows fine-universe and columns coarse-universe indices; row q of R is
// coarse-universe point row_ic[q]; C's columns are coarse_glob[] of the
// coarse-universe points (global coarse indices).
// One row q of rap_core: the touch list tj / sums ta of C's row.  The
// reference's A_marker / P_marker arrays (per point) answer "position of this
// column in the row's touch list, or none" for the row being formed: a per-row
// map (RowMap) gives the same answers, so the first-touch order and every sum
// are unchanged.
void rap_row(const CSR& R, const CSR& A, const CSR& P, int q, int ic, RapScratch& W) {
  W.ra_j.clear();
  W.ra_a.clear();
  int64_t ba = 0;
  for (int jj1 = R.i[q]; jj1 < R.i[q + 1]; ++jj1) ba += A.i[R.j[jj1] + 1] - A.i[R.j[jj1]];
  W.AM.begin(ba);
  bool fresh;
  for (int jj1 = R.i[q]; jj1 < R.i[q + 1]; ++jj1) {
    const int i1 = R.j[jj1];
    const double r_entry = R.a[jj1];
    for (int jj2 = A.i[i1]; jj2 < A.i[i1 + 1]; ++jj2) {
      const int i2 = A.j[jj2];
      int* m = W.AM.find_or_insert(i2, (int)W.ra_j.size(), &fresh);
      if (fresh) {
        W.ra_j.push_back(i2);
        W.ra_a.push_back(r_entry * A.a[jj2]);
      } else {
        W.ra_a[*m] += r_entry * A.a[jj2];
      }
    }
  }
  W.tj.clear();
  W.ta.clear();
  int64_t bp = 1;
  for (int i1 : W.ra_j) bp += P.i[i1 + 1] - P.i[i1];
  W.PM.begin(bp);
  W.PM.find_or_insert(ic, 0, &fresh);
  W.tj.push_back(ic);
  W.ta.push_back(0.0);
  for (size_t k = 0; k < W.ra_j.size(); ++k) {
    const int i1 = W.ra_j[k];
    const double rap_ = W.ra_a[k];
    for (int jj2 = P.i[i1]; jj2 < P.i[i1 + 1]; ++jj2) {
      const int i2 = P.j[jj2];
      int* m = W.PM.find_or_insert(i2, (int)W.tj.size(), &fresh);
      if (fresh) {
        W.tj.push_back(i2);
        W.ta.push_back(rap_ * P.a[jj2]);
      } else {
        W.ta[*m] += rap_ * P.a[jj2];
      }
    }
  }
}

void rap_core(const CSR& R, const CSR& A, const CSR& P, const std::vector<int>& row_ic,
              const std::vector<int>& coarse_glob, int nfine_univ, int ncoarse_univ, int ncoarse_glob, CSR& C) {
  (void)nfine_univ;
  (void)ncoarse_univ;
  const int nc = R.nrows;
  C.resize_rows(nc, ncoarse_glob);
  std::vector<int> rowlen(nc, 0);
  // Two passes: sizes, then values.
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      for (int r = 0; r < nc; ++r) C.i[r + 1] = C.i[r] + rowlen[r];
      C.j.assign(C.i[nc], 0);
      C.a.assign(C.i[nc], 0.0);
    }
#pragma omp parallel
    {
      RapScratch W;
#pragma omp for schedule(dynamic, 256)
      for (int q = 0; q < nc; ++q) {
        rap_row(R, A, P, q, row_ic[q], W);
        if (pass == 0) {
          rowlen[q] = (int)W.tj.size();
        } else {
          int o = C.i[q];
          for (size_t k = 0; k < W.tj.size(); ++k, ++o) {
            C.j[o] = coarse_glob.empty() ? W.tj[k] : coarse_glob[W.tj[k]];
            C.a[o] = W.ta[k];
          }
        }
      }
    }
  }
}

void rap(const CSR& P, const CSR& A, CSR& C) {
  CSR R;
  transpose(P, R);
  const int nc = P.ncols;
  std::vector<int> row_ic(nc);
  for (int q = 0; q < nc; ++q) row_ic[q] = q;
  rap_core(R, A, P, row_ic, {}, A.ncols, nc, nc, C);
}

// ---------------------------------------------------------------------------
// l1 norms: ams.c:571 (one thread) and ams.c:3398 (num_threads blocks).
// option 1: full row l1 norm; option 4: |a_ii| + 0.5 * sum over off-block
// entries, truncated to |a_ii| when <= 4/3 |a_ii|.  Negative-diagonal rows
// get a negative norm (ams.c:760).
// ---------------------------------------------------------------------------
void compute_l1_norms(const CSR& A, int option, const int* cf, int num_blocks, std::vector<double>& l1) {
  const int n = A.nrows;
  const int nb = std::max(1, num_blocks);
  std::vector<int> bs(nb + 1, 0);
  for (int k = 0; k < nb; ++k) {
    int size = n / nb, rest = n - size * nb;
    bs[k] = k < rest ? k * size + k : k * size + rest;
  }
  bs[nb] = n;
  compute_l1_norms_blocks(A, option, cf, bs, l1);
}

// The same over explicit row blocks (bs: nb + 1 ascending starts): with
// several ranks each rank's rows form hypre's per-process thread blocks.
void compute_l1_norms_blocks(const CSR& A, int option, const int* cf, const std::vector<int>& bs,
                             std::vector<double>& l1) {
  const int n = A.nrows;
  l1.assign(n, 0.0);
  const int nb = (int)bs.size() - 1;
#pragma omp parallel for schedule(static)
  for (int k = 0; k < nb; ++k) {
    const int ns = bs[k], ne = bs[k + 1];
    for (int i = ns; i < ne; ++i) {
      double s = 0.0;
      if (option == 1) {
        for (int q = A.i[i]; q < A.i[i + 1]; ++q)
          if (!cf || cf[i] == cf[A.j[q]]) s += std::fabs(A.a[q]);
      } else if (option == 4) {
        double diag = 0.0;
        for (int q = A.i[i]; q < A.i[i + 1]; ++q) {
          int c = A.j[q];
          if ((c == i || c < ns || c >= ne) && (!cf || cf[i] == cf[c])) {
            if (c == i) { diag = std::fabs(A.a[q]); s += std::fabs(A.a[q]); }
            else s += 0.5 * std::fabs(A.a[q]);
          }
        }
        if (s <= 4.0 / 3.0 * diag) s = diag;
      }
      l1[i] = s;
    }
  }
  for (int i = 0; i < n; ++i)
    if (A.a[A.i[i]] < 0.0) l1[i] = -l1[i];
}

// ---------------------------------------------------------------------------
// Chebyshev smoother setup (relax type 16).
// ---------------------------------------------------------------------------
// par_relax_more.c cgpthy: sqrt(a^2 + b^2) without destructive over/underflow
static double linpack_pythag(double a, double b) {
  double p = std::max(std::fabs(a), std::fabs(b));
  if (!p) return p;
  double d = std::min(std::fabs(a), std::fabs(b)) / p;
  double r = d * d;
  for (;;) {
    const double t = r + 4.;
    if (t == 4.) break;
    const double s = r / t;
    const double u = s * 2. + 1.;
    p = u * p;
    d = s / u;
    r = d * d * r;
  }
  return p;
}

// par_relax_more.c:753 hypre_LINPACKcgtql1, restated with the same 1-based
// indexing and statement order.
int linpack_tql1(int n_, double* d0, double* e0) {
  const int n = n_;
  double* d = d0 - 1;
  double* e = e0 - 1;
  int ierr = 0;
  double c, f, g, h, p, r, s, c2, c3 = 0.0, s2 = 0.0, dl1, el1, tst1, tst2, ds;
  int i, j, l, m, l1, l2, ii, mml;
  if (n == 1) return 0;
  for (i = 2; i <= n; ++i) e[i - 1] = e[i];
  f = 0.;
  tst1 = 0.;
  e[n] = 0.;
  for (l = 1; l <= n; ++l) {
    j = 0;
    h = std::fabs(d[l]) + std::fabs(e[l]);
    if (tst1 < h) tst1 = h;
    for (m = l; m <= n; ++m) {
      tst2 = tst1 + std::fabs(e[m]);
      if (tst2 == tst1) break;
    }
    if (m != l) {
      for (;;) {  // L130
        if (j == 30) return l;
        ++j;
        l1 = l + 1;
        l2 = l1 + 1;
        g = d[l];
        p = (d[l1] - g) / (e[l] * 2.);
        r = linpack_pythag(p, 1.0);
        ds = 1.0;
        if (p < 0.0) ds = -1.0;
        d[l] = e[l] / (p + ds * r);
        d[l1] = e[l] * (p + ds * r);
        dl1 = d[l1];
        h = g - d[l];
        if (l2 <= n)
          for (i = l2; i <= n; ++i) d[i] -= h;
        f += h;
        p = d[m];
        c = 1.;
        c2 = c;
        el1 = e[l1];
        s = 0.;
        mml = m - l;
        for (ii = 1; ii <= mml; ++ii) {
          c3 = c2;
          c2 = c;
          s2 = s;
          i = m - ii;
          g = c * e[i];
          h = c * p;
          r = linpack_pythag(p, e[i]);
          e[i + 1] = s * r;
          s = e[i] / r;
          c = p / r;
          p = c * d[i] - s * g;
          d[i + 1] = h + s * (c * g + s * d[i]);
        }
        p = -s * s2 * c3 * el1 * e[l] / dl1;
        e[l] = s * p;
        d[l] = c * p;
        tst2 = tst1 + std::fabs(e[l]);
        if (!(tst2 > tst1)) break;
      }
    }
    // L210
    p = d[l] + f;
    i = 1;
    if (l != 1) {
      bool placed = false;
      for (ii = 2; ii <= l; ++ii) {
        i = l + 2 - ii;
        if (p >= d[i - 1]) { placed = true; break; }
        d[i] = d[i - 1];
      }
      if (!placed) i = 1;
    }
    d[i] = p;
  }
  return ierr;
}

// y = A x (csr_matvec.c, alpha 1 beta 0), one thread
static void host_matvec(const CSR& A, const std::vector<double>& x, std::vector<double>& y) {
  for (int r = 0; r < A.nrows; ++r) {
    double t = 0.0;
    for (int k = A.i[r]; k < A.i[r + 1]; ++k) t += A.a[k] * x[A.j[k]];
    y[r] = t;
  }
}
static double host_dot(const std::vector<double>& x, const std::vector<double>& y) {
  double s = 0.0;
  for (size_t i = 0; i < x.size(); ++i) s += y[i] * x[i];  // hypre_SeqVectorInnerProd: y_i * x_i
  return s;
}

void max_eig_estimate_cg(const CSR& A, int scale, int max_iter, double* max_eig, double* min_eig,
                         const std::vector<int>* rs) {
  const int n = A.nrows;
  if (n < max_iter) max_iter = n;
  std::vector<double> r(n), p(n, 0.0), s(n, 0.0), ds(n), u(n, 0.0);
  std::vector<double> tridiag(max_iter + 1, 0.0), trioffd(max_iter + 1, 0.0);
  // hypre_ParVectorSetRandomValues(r, 1): seed 1 * (my_id + 1), 2*rand - 1
  // (par_vector.c:337), every rank from its own first row
  if (rs) {
    for (size_t k = 0; k + 1 < rs->size(); ++k)
      for (int i = (*rs)[k]; i < (*rs)[k + 1]; ++i) r[i] = 2.0 * hypre_rand_at(i - (*rs)[k], (int)k + 1) - 1.0;
  } else {
    for (int i = 0; i < n; ++i) r[i] = 2.0 * hypre_rand_at(i, 1) - 1.0;
  }
  if (scale) {
    for (int i = 0; i < n; ++i) ds[i] = 1 / std::sqrt(A.a[A.i[i]]);
  } else {
    for (int i = 0; i < n; ++i) ds[i] = 1.0;
  }
  double gamma = host_dot(r, p), gamma_old, beta, alpha, sdotp, alphainv;
  int i = 0;
  while (i < max_iter) {
    s = r;
    gamma_old = gamma;
    gamma = host_dot(r, s);
    if (i == 0) {
      beta = 1.0;
      p = s;
    } else {
      beta = gamma / gamma_old;
      for (int k = 0; k < n; ++k) p[k] = s[k] + beta * p[k];
    }
    if (scale) {
      for (int k = 0; k < n; ++k) u[k] = ds[k] * p[k];
      host_matvec(A, u, s);
      for (int k = 0; k < n; ++k) s[k] = ds[k] * s[k];
    } else {
      host_matvec(A, p, s);
    }
    sdotp = host_dot(s, p);
    alpha = gamma / sdotp;
    alphainv = 1.0 / alpha;
    tridiag[i + 1] = alphainv;
    tridiag[i] *= beta;
    tridiag[i] += alphainv;
    trioffd[i + 1] = alphainv;
    trioffd[i] *= std::sqrt(beta);
    for (int k = 0; k < n; ++k) r[k] += (-alpha) * s[k];  // hypre_ParVectorAxpy(-alpha, s, r)
    i++;
  }
  linpack_tql1(i, tridiag.data(), trioffd.data());
  *max_eig = tridiag[i - 1];
  *min_eig = tridiag[0];
}

void max_eig_estimate_norm(const CSR& A, int scale, double* max_eig) {
  double max_norm = 0.0;
  int pos_diag = 0, neg_diag = 0;
  for (int i = 0; i < A.nrows; ++i) {
    const int start = A.i[i];
    double diag_value = A.a[start];
    if (diag_value > 0) pos_diag++;
    if (diag_value < 0) { neg_diag++; diag_value = -diag_value; }
    double row_sum = diag_value;
    for (int j = start + 1; j < A.i[i + 1]; ++j) row_sum += std::fabs(A.a[j]);
    if (scale && diag_value != 0.0) row_sum = row_sum / diag_value;
    if (row_sum > max_norm) max_norm = row_sum;
  }
  if (pos_diag == 0 && neg_diag > 0) max_norm = -max_norm;
  *max_eig = max_norm;
}

void cheby_setup(const CSR& A, double max_eig, double min_eig, double fraction, int order, int scale, int variant,
                 std::vector<double>& coefs, std::vector<double>& ds) {
  if (order > 4) order = 4;
  if (order < 1) order = 1;
  coefs.assign(order + 1, 0.0);
  const int cheby_order = order - 1;
  const double upper_bound = max_eig * 1.1;
  const double lower_bound = (upper_bound - min_eig) * fraction + min_eig;
  const double theta = (upper_bound + lower_bound) / 2;
  const double delta = (upper_bound - lower_bound) / 2;
  double den;
  if (variant == 1) {
    switch (cheby_order) {
      case 0: coefs[0] = 1.0 / theta; break;
      case 1:
        den = (theta * theta + delta * theta);
        coefs[0] = (delta + 2 * theta) / den;
        coefs[1] = -1.0 / den;
        break;
      case 2:
        den = 2 * delta * theta * theta - delta * delta * theta - std::pow(delta, 3) + 2 * std::pow(theta, 3);
        coefs[0] = (4 * delta * theta - std::pow(delta, 2) + 6 * std::pow(theta, 2)) / den;
        coefs[1] = -(2 * delta + 6 * theta) / den;
        coefs[2] = 2 / den;
        break;
      case 3:
        den = -(4 * delta * std::pow(theta, 3) - 3 * std::pow(delta, 2) * std::pow(theta, 2) -
                3 * std::pow(delta, 3) * theta + 4 * std::pow(theta, 4));
        coefs[0] = (6 * std::pow(delta, 2) * theta - 12 * delta * std::pow(theta, 2) + 3 * std::pow(delta, 3) -
                    16 * std::pow(theta, 3)) / den;
        coefs[1] = (12 * delta * theta - 3 * std::pow(delta, 2) + 24 * std::pow(theta, 2)) / den;
        coefs[2] = -(4 * delta + 16 * theta) / den;
        coefs[3] = 4 / den;
        break;
    }
  } else {
    switch (cheby_order) {
      case 0: coefs[0] = 1.0 / theta; break;
      case 1:
        den = delta * delta - 2 * theta * theta;
        coefs[0] = -4 * theta / den;
        coefs[1] = 2 / den;
        break;
      case 2:
        den = 3 * (delta * delta) * theta - 4 * (theta * theta * theta);
        coefs[0] = (3 * delta * delta - 12 * theta * theta) / den;
        coefs[1] = 12 * theta / den;
        coefs[2] = -4 / den;
        break;
      case 3:
        den = std::pow(delta, 4) - 8 * delta * delta * theta * theta + 8 * std::pow(theta, 4);
        coefs[0] = (32 * std::pow(theta, 3) - 16 * delta * delta * theta) / den;
        coefs[1] = (8 * delta * delta - 48 * theta * theta) / den;
        coefs[2] = 32 * theta / den;
        coefs[3] = -8 / den;
        break;
    }
  }
  ds.clear();
  if (scale) {
    ds.resize(A.nrows);
    for (int j = 0; j < A.nrows; ++j) ds[j] = 1 / std::sqrt(A.a[A.i[j]]);
  }
}

// ---------------------------------------------------------------------------
// Setup driver: par_amg_setup.c:889-2880 (coarsening loop), :2990-3120 (l1 norms).
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// Automatic relaxation weights: par_cg_relax_wt.c hypre_BoomerAMGCGRelaxWt.
// CG on A preconditioned by one sweep of the level's down smoother (weights 1,
// from zero) starting at a random vector (seed 5128, per rank when emulating);
// the Lanczos tridiagonal's largest eigenvalue (hypre_Bisection, par_cg_relax_wt.c:362)
// gives the weight 1/lambda_max, stopping when it moves by less than 1e-3.
// ---------------------------------------------------------------------------
static void bisection(int n, const double* diag, const double* offd, double y, double z, double tol, int k,
                      double* ev) {
  while (std::fabs(y - z) > tol * (std::fabs(y) + std::fabs(z))) {
    const double x = (y + z) / 2;
    int sign_change = 0;
    double p0 = 1, p1 = diag[0] - x, p2;
    if (p0 * p1 <= 0) sign_change++;
    for (int i = 1; i < n; i++) {
      p2 = (diag[i] - x) * p1 - offd[i] * offd[i] * p0;
      p0 = p1;
      p1 = p2;
      if (p0 * p1 <= 0) sign_change++;
    }
    if (sign_change >= k) z = x;
    else y = x;
  }
  *ev = (y + z) / 2;
}

// One sweep of relax_type with weights 1 (par_relax.c), blocks bs (hybrid GS),
// relax_points 0; u is updated in place (tmp: scratch of A.nrows).
static void host_relax_w1(const CSR& A, const std::vector<double>& f, int relax_type, const std::vector<double>& l1,
                          const std::vector<int>& bs, std::vector<double>& u, std::vector<double>& tmp) {
  const int n = A.nrows;
  switch (relax_type) {
    case 0: {  // par_relax.c:139, weight 1
      tmp = u;
      for (int i = 0; i < n; ++i) {
        const double d = A.a[A.i[i]];
        if (d == 0.0) continue;
        double res = f[i];
        for (int k = A.i[i] + 1; k < A.i[i + 1]; ++k) res -= A.a[k] * tmp[A.j[k]];
        u[i] *= 0.0;
        u[i] += 1.0 * res / d;
      }
      return;
    }
    case 7: case 18: {  // u += (f - A u)/l1 (ams.c:41 with the l1 norms; 7: the diagonal)
      tmp = f;
      for (int i = 0; i < n; ++i) {
        double t = tmp[i];
        for (int k = A.i[i]; k < A.i[i + 1]; ++k) t -= A.a[k] * u[A.j[k]];
        tmp[i] = t;
      }
      for (int i = 0; i < n; ++i) u[i] += tmp[i] / l1[i];
      return;
    }
    case 3: case 4: case 6: case 8: case 13: case 14: {
      const bool fwd = relax_type == 3 || relax_type == 6 || relax_type == 8 || relax_type == 13;
      const bool bwd = relax_type == 4 || relax_type == 6 || relax_type == 8 || relax_type == 14;
      const bool use_l1 = relax_type == 8 || relax_type == 13 || relax_type == 14;
      const int nb = (int)bs.size() - 1;
      tmp = u;
      for (int b = 0; b < nb; ++b) {
        const int ns = bs[b], ne = bs[b + 1];
        for (int pass = 0; pass < 2; ++pass) {
          if ((pass == 0 && !fwd) || (pass == 1 && !bwd)) continue;
          for (int q = 0; q < ne - ns; ++q) {
            const int i = pass == 0 ? ns + q : ne - 1 - q;
            if (use_l1) {
              if (l1[i] == 0.0) continue;
              double res = f[i];
              for (int k = A.i[i]; k < A.i[i + 1]; ++k) {
                const int c = A.j[k];
                res -= A.a[k] * ((nb == 1 || (c >= ns && c < ne)) ? u[c] : tmp[c]);
              }
              u[i] += res / l1[i];
            } else {
              const double d = A.a[A.i[i]];
              if (d == 0.0) continue;
              double res = f[i];
              for (int k = A.i[i] + 1; k < A.i[i + 1]; ++k) {
                const int c = A.j[k];
                res -= A.a[k] * ((nb == 1 || (c >= ns && c < ne)) ? u[c] : tmp[c]);
              }
              u[i] = res / d;
            }
          }
        }
      }
      return;
    }
    default:
      throw std::runtime_error("automatic relaxation weight (negative weight) with relax type " +
                               std::to_string(relax_type) + " is not available");
  }
}

static double cg_relax_weight(const CSR& A, int relax_type, const std::vector<double>& l1, const std::vector<int>& bs,
                              int num_cg_sweeps, const std::vector<int>* rs) {
  const int n = A.nrows;
  auto dot = [&](const std::vector<double>& x, const std::vector<double>& y) {
    if (!rs) return host_dot(x, y);
    double t = 0.0;  // per-rank sums (hypre_SeqVectorInnerProd), then the sum over ranks
    for (size_t r = 0; r + 1 < rs->size(); ++r) {
      double sr = 0.0;
      for (int i = (*rs)[r]; i < (*rs)[r + 1]; ++i) sr += y[i] * x[i];
      t += sr;
    }
    return t;
  };
  std::vector<double> R(n), Z(n), P(n, 0.0), V(n), tmp(n);
  // hypre_ParVectorSetRandomValues(Rtemp, 5128): 2 rand - 1, seed 5128 (my_id + 1)
  if (rs) {
    for (size_t r = 0; r + 1 < rs->size(); ++r)
      for (int i = (*rs)[r]; i < (*rs)[r + 1]; ++i) R[i] = 2.0 * hypre_rand_at(i - (*rs)[r], 5128 * ((int)r + 1)) - 1.0;
  } else {
    for (int i = 0; i < n; ++i) R[i] = 2.0 * hypre_rand_at(i, 5128) - 1.0;
  }
  std::vector<double> tridiag(num_cg_sweeps + 1, 0.0), trioffd(num_cg_sweeps + 1, 0.0);
  double gamma = 1.0, gammaold, alpha, beta, alphinv, row_sum, max_row_sum = 0.0;
  double rlx_wt = 0.0, rlx_wt_old = 0.0, lambda_max = 0.0, lambda_max_old;
  for (int jj = 0; jj < num_cg_sweeps; ++jj) {
    std::fill(Z.begin(), Z.end(), 0.0);
    host_relax_w1(A, R, relax_type, l1, bs, Z, tmp);
    gammaold = gamma;
    gamma = dot(R, Z);
    if (jj == 0) {
      P = Z;
      beta = 1.0;
    } else {
      beta = gamma / gammaold;
      for (int i = 0; i < n; ++i) P[i] = Z[i] + beta * P[i];
    }
    host_matvec(A, P, V);
    alpha = gamma / dot(P, V);
    alphinv = 1.0 / alpha;
    tridiag[jj + 1] = alphinv;
    tridiag[jj] *= beta;
    tridiag[jj] += alphinv;
    trioffd[jj] *= std::sqrt(beta);
    trioffd[jj + 1] = -alphinv;
    row_sum = std::fabs(tridiag[jj]) + std::fabs(trioffd[jj]);
    if (row_sum > max_row_sum) max_row_sum = row_sum;
    if (jj > 0) {
      row_sum = std::fabs(tridiag[jj - 1]) + std::fabs(trioffd[jj - 1]) + std::fabs(trioffd[jj]);
      if (row_sum > max_row_sum) max_row_sum = row_sum;
      lambda_max_old = lambda_max;
      rlx_wt_old = rlx_wt;
      bisection(jj + 1, tridiag.data(), trioffd.data(), lambda_max_old, max_row_sum, 1.e-3, jj + 1, &lambda_max);
      rlx_wt = 1.0 / lambda_max;
      if (std::fabs(rlx_wt - rlx_wt_old) < 1.e-3) break;
    } else {
      lambda_max = tridiag[0];
    }
    for (int i = 0; i < n; ++i) R[i] += (-alpha) * V[i];  // hypre_ParVectorAxpy(-alpha, Vtemp, Rtemp)
  }
  return rlx_wt;
}

static bool uses_l1_gs(int t) { return t == 8 || t == 13 || t == 14; }

// l1 norm option the setup computes on level j of nl (0 none, 1 full row
// sums for relax 18, 4 hybrid-GS norms for relax 8/13/14); *cf_restricted:
// whether it uses the C/F marker (relax_order, not on the coarsest level).
int l1_option_for_level(const AMGParams& prm, int j, int nl, bool* cf_restricted) {
  int opt = 0;
  bool cfr = false;
  if (j < nl - 1 && (uses_l1_gs(prm.relax_type[1]) || uses_l1_gs(prm.relax_type[2]))) { opt = 4; cfr = true; }
  else if (j == nl - 1 && uses_l1_gs(prm.relax_type[3])) { opt = 4; cfr = false; }
  if (j < nl - 1 && (prm.relax_type[1] == 18 || prm.relax_type[2] == 18)) { opt = 1; cfr = true; }
  else if (j == nl - 1 && prm.relax_type[3] == 18) { opt = 1; cfr = false; }
  if (cf_restricted) *cf_restricted = cfr && prm.relax_order;
  return opt;
}

// Rows of an N-rank run (hypre's ParCSR: each row = its diag part, then its
// offd part, both in their own entry order): stable partition of every row of
// M by whether the column's owner is the row's owner.
static void rank_order_rows(CSR& M, const std::vector<int>& rs, const std::vector<int>& cs) {
  auto owner = [](const std::vector<int>& st, int i) {
    return (int)(std::upper_bound(st.begin(), st.end(), i) - st.begin()) - 1;
  };
#pragma omp parallel
  {
    std::vector<int> tj;
    std::vector<double> ta;
#pragma omp for schedule(static)
    for (int r = 0; r < M.nrows; ++r) {
      const int o = owner(rs, r);
      const int c0 = cs[o], c1 = cs[o + 1];  // the owner's columns
      tj.clear();
      ta.clear();
      for (int pass = 0; pass < 2; ++pass)
        for (int k = M.i[r]; k < M.i[r + 1]; ++k)
          if ((M.j[k] >= c0 && M.j[k] < c1) == (pass == 0)) { tj.push_back(M.j[k]); ta.push_back(M.a[k]); }
      std::copy(tj.begin(), tj.end(), M.j.begin() + M.i[r]);
      std::copy(ta.begin(), ta.end(), M.a.begin() + M.i[r]);
    }
  }
}

int amg_setup(const CSR& A0, const AMGParams& prm_in, Hierarchy& H, const std::vector<int>* rank_starts,
              const std::vector<int>* coarsen_starts, const std::vector<int>* dof0) {
  H = Hierarchy();
  H.prm = prm_in;
  AMGParams& prm = H.prm;
  // par_amg_setup.c:319: interp_type 9 is standard interpolation with separated weights
  if (prm.interp_type == 9) {
    prm.interp_type = 8;
    prm.sep_weight = 1;
  }
  const int at = prm.agg_interp_type;
  // systems AMG, unknown approach (par_amg_setup.c:668-689: function j of the
  // interleaved unknowns, dof = global row % num_functions; coarse levels keep
  // the functions of their C points, par_coarse_parms.c)
  std::vector<int> dof;
  struct DofGuard {
    const int* saved = hve_setup_dof;
    ~DofGuard() { hve_setup_dof = saved; }
  } dof_guard;
  hve_setup_dof = nullptr;
  if (prm.num_functions > 1) {
    // the matrix-matrix builders (16-18, agg 5 / 7) take no functions: only
    // their strength matrix is per function (par_mod_lr_interp.c, par_2s_interp.c)
    if (prm.interp_type != 6 && prm.interp_type != 14 && (prm.interp_type < 16 || prm.interp_type > 18))
      throw std::runtime_error("num_functions > 1: interp_type " + std::to_string(prm.interp_type) +
                               " is not restated for systems (6, 14, 16-18)");
    if (prm.agg_num_levels > 0 && at != 1 && at != 3 && at != 4 && at != 5 && at != 7)
      throw std::runtime_error("num_functions > 1: agg_interp_type " + std::to_string(at) +
                               " is not restated for systems (1, 3, 4, 5, 7)");
    if (dof0) {
      if ((int)dof0->size() != A0.nrows) throw std::runtime_error("dof_func: one function per row");
      dof = *dof0;
    } else {
      dof.resize(A0.nrows);
      for (int i = 0; i < A0.nrows; ++i) dof[i] = i % prm.num_functions;
    }
  }
  if (prm.agg_num_levels > 0 && (at < 1 || at > 7))
    throw std::runtime_error("aggressive coarsening: agg_interp_type " + std::to_string(at) +
                             " is not available in this build (1 / 2 / 3 2-stage extended+i / standard / extended,"
                             " 4 multipass, 5 / 6 / 7 2-stage extended / ext+i / ext+e MM)");
  if (prm.num_paths < 1) throw std::runtime_error("num_paths must be >= 1");
  int coarsen_type = prm.coarsen_type;
  H.lev.emplace_back();
  H.lev[0].A = A0;
  // N-rank emulation: the row starts of every level (rank r owns the C points
  // of its fine rows), and every row in hypre's ParCSR order (diag, offd)
  std::vector<int> emul;
  if (rank_starts && rank_starts->size() > 2) {
    emul = *rank_starts;
    if (emul.front() != 0 || emul.back() != A0.nrows) throw std::runtime_error("rank emulation: row starts do not cover A");
    if (prm.interp_type != 6 && prm.interp_type != 7 && prm.interp_type != 8 && prm.interp_type != 14 &&
        (prm.interp_type < 16 || prm.interp_type > 18))
      throw std::runtime_error("rank emulation: interp_type " + std::to_string(prm.interp_type) + " is not restated");
    rank_order_rows(H.lev[0].A, emul, emul);
  }
  const std::vector<int>* rs = emul.empty() ? nullptr : &emul;
  // HMIS per rank without the rest of the emulation (the distributed setup's
  // coarsening): this level's rank starts
  std::vector<int> crs;
  if (!rs && coarsen_starts && coarsen_starts->size() > 2 && coarsen_type == 10) {
    crs = *coarsen_starts;
    if (crs.front() != 0 || crs.back() != A0.nrows) throw std::runtime_error("coarsen_starts do not cover A");
  }
  std::vector<std::vector<int>> lev_starts;  // emulated ranks: row starts of every level
  if (rs) lev_starts.push_back(emul);
  char buf[256];
  int level = 0;
  bool finished = prm.max_levels <= 1;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double t_s = 0, t_c = 0, t_i = 0, t_r = 0, t_t = 0;
  // the device calls of a level share its device A, S and P (setup_dev.hip)
  struct CacheScope {
    bool on;
    ~CacheScope() { if (on) dev_setup_cache_clear(); }
  } cache_scope{prm.device_setup};
  while (!finished) {
    Level& L = H.lev[level];
    const int fine_size = L.A.nrows;
    if (prm.device_setup) dev_setup_cache_clear();
    Pattern S;
    double t0 = now();
    hve_setup_dof = dof.empty() ? nullptr : dof.data();
    // one process, PMIS (the one-process streams of coarsen_type 8 and 9
    // agree): strength and coarsening on the device, the same S and markers
    // (levels of 2^16 rows and more; knob 15 sets the bound: tests take 1)
    const bool dev_sc = prm.device_setup && dof.empty() && !rs && (coarsen_type == 8 || coarsen_type == 9) &&
                        fine_size >= (knob(15) > 0 ? knob(15) : (1 << 16));
    std::vector<int> cf;
    double ts_dev = 0.0;
    if (dev_sc) dev_strength_pmis(L.A, prm.strong_threshold, prm.max_row_sum, S, cf, &ts_dev);
    else create_strength(L.A, prm.strong_threshold, prm.max_row_sum, S);
    double t1 = dev_sc ? t0 + ts_dev : now();
    t_s += t1 - t0;
    if (dev_sc) {
      // done above
    } else if (coarsen_type == 8) coarsen_pmis(S, 0, cf, rs);
    else if (coarsen_type == 9) coarsen_pmis(S, 2, cf, rs);
    else if (coarsen_type == 10)
      coarsen_hmis(S, &L.A, prm.measure_type, prm.coarsen_cut_factor, cf, rs ? rs : (crs.empty() ? nullptr : &crs));
    else if (coarsen_type == 11) coarsen_ruge1p(S, &L.A, prm.measure_type, prm.coarsen_cut_factor, cf, rs);
    else throw std::runtime_error("unsupported coarsen_type " + std::to_string(coarsen_type));
    double t2 = now();
    t_c += t2 - t1;
    // par_amg_setup.c:1239-1285: aggressive levels coarsen the C points
    // again on S*S + 2S, and the second marker refines the first
    const bool agg = level < prm.agg_num_levels;
    std::vector<int> cf1;
    if (agg) {
      Pattern S2;
      create_2nd_strength(S, cf, prm.num_paths, S2);
      // emulated ranks: S2's rows (the first pass's C points) split as the fine rows
      std::vector<int> rs2;
      const std::vector<int>* lrs = rs ? rs : (crs.empty() ? nullptr : &crs);
      if (lrs) {
        std::vector<int> pref(cf.size() + 1, 0);
        for (size_t i = 0; i < cf.size(); ++i) pref[i + 1] = pref[i] + (cf[i] > 0);
        for (int v : *lrs) rs2.push_back(pref[v]);
      }
      const std::vector<int>* rsc = lrs ? &rs2 : nullptr;
      std::vector<int> cfn;
      if (coarsen_type == 8) coarsen_pmis(S2, 3, cfn, rsc);
      else if (coarsen_type == 9) coarsen_pmis(S2, 4, cfn, rsc);
      else if (coarsen_type == 10) {
        CSR S2A;  // hypre passes S2 as the matrix too (only its row lengths, for cut_factor)
        S2A.resize_rows(S2.n, S2.n);
        S2A.i = S2.i;
        S2A.j.assign(S2.j.begin(), S2.j.end());
        S2A.a.assign(S2.j.size(), 1.0);
        coarsen_hmis(S2, &S2A, prm.measure_type + 3, prm.coarsen_cut_factor, cfn, rsc);
      } else {
        throw std::runtime_error("aggressive coarsening with coarsen_type " + std::to_string(coarsen_type));
      }
      if (prm.agg_interp_type == 4) {
        correct_cf_marker(cf, cfn);  // agg_interp_type 4: par_amg_setup.c:1590
      } else {
        cf1 = cf;  // the first stage's markers, for P1
        // P1 of types 1 / 3 (the classical ext+i / ext builders) turns the SF
        // markers into F ones before the markers are combined
        // (par_lr_interp.c:1890 / :5414, then par_amg_setup.c:1600)
        if (at == 1 || at == 2 || at == 3)
          for (int& v : cf)
            if (v == SF_PT) v = F_PT;
        correct_cf_marker2(cf, cfn);  // par_amg_setup.c:1600 (par_strength.c:2978)
      }
    }
    int coarse_size = 0;
    for (int v : cf) coarse_size += (v == 1);
    if (coarse_size == 0 || coarse_size == fine_size) {
      if (prm.relax_type[3] == 9 || prm.relax_type[3] == 99 || prm.relax_type[3] == 19 || prm.relax_type[3] == 98) {
        prm.relax_type[3] = prm.relax_type[0];
        prm.num_sweeps[3] = 1;
      }
      break;
    }
    if (coarse_size < prm.min_coarse_size) break;
    CSR P;
    if (agg && prm.agg_interp_type != 4) {
      // 2-stage: P1 to the first stage's C points, P2 from them to the
      // second's (par_amg_setup.c:1575-1689)
      CSR P1, P2;
      const bool pe = at == 7;
      // P1 (par_amg_setup.c:1553-1596): 1 ext+i, 3 ext, 5 MM ext, 6 MM ext+i,
      // 7 MM ext+e; P2 (:1620-1672): 1 / 6 partial ext+i, 3 partial ext,
      // 5 / 7 the MM partial forms
      auto stage1 = [&](double tf, int mx, const std::vector<int>* em) {
        if (at == 1 || at == 3) build_extpi_interp(L.A, cf1, S, tf, mx, P1, at == 1);
        else if (at == 2) build_std_interp(L.A, cf1, S, tf, mx, 0, P1, em);  // sep_weight 0 here (par_amg_setup.c:1562)
        else if (at == 6) build_modextpi_interp(L.A, cf1, S, tf, mx, P1, em);
        else build_modext_interp(L.A, cf1, S, tf, mx, pe, P1, em);
      };
      auto stage2 = [&](double tf, int mx, const std::vector<int>* em) {
        if (at == 1 || at == 3 || at == 6) build_partial_extpi_interp(L.A, cf, S, tf, mx, at != 3, P2);
        else if (at == 2) build_std_interp(L.A, cf, S, tf, mx, prm.sep_weight, P2, em, true);
        else build_modpartialext_interp(L.A, cf, S, tf, mx, pe, P2, em);
      };
      if (emul.empty()) {
        stage1(prm.agg_P12_trunc_factor, prm.agg_P12_max_elmts, nullptr);
        stage2(prm.agg_P12_trunc_factor, prm.agg_P12_max_elmts, nullptr);
        multiply_interp(P1, P2, prm.agg_trunc_factor, prm.agg_P_max_elmts, P);
      } else {
        // emulated ranks: every product in hypre_ParMatmul's np > 1 order and
        // every truncation over [P_diag | P_offd] (as for ext+i below)
        const int nfine = (int)cf.size();
        std::vector<int> c1pref(nfine + 1, 0), c2pref(nfine + 1, 0);
        for (int i = 0; i < nfine; ++i) {
          c1pref[i + 1] = c1pref[i] + (cf1[i] > 0);
          c2pref[i + 1] = c2pref[i] + (cf[i] > 0);
        }
        std::vector<int> cs1, cs2;
        for (int v : emul) { cs1.push_back(c1pref[v]); cs2.push_back(c2pref[v]); }
        auto trunc = [&](CSR& M, const std::vector<int>& rs, const std::vector<int>& cs, double tf, int mx) {
          rank_order_rows(M, rs, cs);
          if (tf != 0.0 || mx > 0) truncate_rows(M, tf, mx);
          rank_order_rows(M, rs, cs);
        };
        stage1(0.0, 0, &emul);
        trunc(P1, emul, cs1, prm.agg_P12_trunc_factor, prm.agg_P12_max_elmts);
        stage2(0.0, 0, &emul);
        trunc(P2, cs1, cs2, prm.agg_P12_trunc_factor, prm.agg_P12_max_elmts);
        MatmulRanks rk;
        rk.nranks = (int)emul.size() - 1;
        auto owner = [](const std::vector<int>& st, int i) {
          return (int)(std::upper_bound(st.begin(), st.end(), i) - st.begin()) - 1;
        };
        for (int i = 0; i < P1.nrows; ++i) rk.row.push_back(owner(emul, i));
        for (int c = 0; c < P1.ncols; ++c) rk.xcol.push_back(owner(cs1, c));
        for (int c = 0; c < P2.ncols; ++c) rk.ycol.push_back(owner(cs2, c));
        matmul_first_touch(P1, P2, P, &rk);
        trunc(P, emul, cs2, prm.agg_trunc_factor, prm.agg_P_max_elmts);
      }
    }
    else if (agg) {
      build_multipass_interp(L.A, cf, S, prm.agg_trunc_factor, prm.agg_P_max_elmts, P);
      if (!emul.empty()) {  // P_diag | P_offd
        std::vector<int> cs(emul.size(), 0), pref(cf.size() + 1, 0);
        for (size_t i = 0; i < cf.size(); ++i) pref[i + 1] = pref[i] + (cf[i] == 1);
        for (size_t r = 0; r < emul.size(); ++r) cs[r] = pref[emul[r]];
        rank_order_rows(P, emul, cs);
      }
    }
    else if ((prm.interp_type == 6 || prm.interp_type == 7 || prm.interp_type == 8 || prm.interp_type == 14 ||
              (prm.interp_type >= 16 && prm.interp_type <= 18)) &&
             !emul.empty()) {
      // par_csr_matrix.c:2671 truncates the row [P_diag | P_offd] and splits
      // the kept entries back into the two parts in their sorted order
      std::vector<int> cs(emul.size(), 0);
      {
        std::vector<int> pref(cf.size() + 1, 0);
        for (size_t i = 0; i < cf.size(); ++i) pref[i + 1] = pref[i] + (cf[i] == 1);
        for (size_t r = 0; r < emul.size(); ++r) cs[r] = pref[emul[r]];
      }
      if (prm.interp_type == 16) build_modext_interp(L.A, cf, S, 0.0, 0, false, P, &emul);
      else if (prm.interp_type == 17) build_modextpi_interp(L.A, cf, S, 0.0, 0, P, &emul);
      else if (prm.interp_type == 18) build_modextpe_interp(L.A, cf, S, 0.0, 0, P, &emul);
      else if (prm.interp_type == 8) build_std_interp(L.A, cf, S, 0.0, 0, prm.sep_weight, P, &emul);
      else if (prm.interp_type == 7) build_extpicc_interp(L.A, cf, S, 0.0, 0, P);
      else build_extpi_interp(L.A, cf, S, 0.0, 0, P, prm.interp_type == 6);
      rank_order_rows(P, emul, cs);
      if (prm.trunc_factor != 0.0 || prm.P_max_elmts > 0) truncate_rows(P, prm.trunc_factor, prm.P_max_elmts);
      rank_order_rows(P, emul, cs);
    }
    else if (prm.interp_type == 6 && prm.device_setup && dof.empty()) {
      std::vector<int> f2c(cf.size(), -1);
      int nc = 0;
      for (size_t i = 0; i < cf.size(); ++i)
        if (cf[i] >= 0) f2c[i] = nc++;
      dev_extpi_interp(L.A, S, cf, f2c, nc, prm.trunc_factor, prm.P_max_elmts, P);
      for (int& v : cf)
        if (v == SF_PT) v = F_PT;
      if (dev_setup_host_rows() > 0) {
        snprintf(buf, sizeof buf, "level %d: %lld interpolation rows on the host\n", level, dev_setup_host_rows());
        H.log += buf;
      }
    }
    else if (prm.interp_type == 6) build_extpi_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, P);
    else if (prm.interp_type == 18) build_modextpe_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, P);
    else if (prm.interp_type == 17) build_modextpi_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, P);
    else if (prm.interp_type == 16)
      build_modext_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, false, P);
    else if (prm.interp_type == 14) build_extpi_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, P, false);
    else if (prm.interp_type == 3) build_direct_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, P);
    else if (prm.interp_type == 8) build_std_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, prm.sep_weight, P);
    else if (prm.interp_type == 7) build_extpicc_interp(L.A, cf, S, prm.trunc_factor, prm.P_max_elmts, P);
    else throw std::runtime_error("unsupported interp_type " + std::to_string(prm.interp_type));
    double t3 = now();
    t_i += t3 - t2;
    CSR Ac, Rdev;
    if (prm.device_setup) {
      dev_rap(P, L.A, Rdev, Ac);
      if (dev_setup_host_rows() > 0) {
        snprintf(buf, sizeof buf, "level %d: %lld Galerkin rows on the host\n", level, dev_setup_host_rows());
        H.log += buf;
      }
    } else {
      rap(P, L.A, Ac);
    }
    std::vector<int> emul_c;
    if (!emul.empty()) {
      // hypre's RAP keeps each coarse row as diag then offd (par_rap.c)
      std::vector<int> pref(cf.size() + 1, 0);
      for (size_t i = 0; i < cf.size(); ++i) pref[i + 1] = pref[i] + (cf[i] == 1);
      emul_c.resize(emul.size());
      for (size_t r = 0; r < emul.size(); ++r) emul_c[r] = pref[emul[r]];
      rank_order_rows(Ac, emul_c, emul_c);
    }
    double t4 = now();
    t_r += t4 - t3;
    L.cf.swap(cf);
    L.P.swap(P);
    if (prm.device_setup) L.R.swap(Rdev);  // R = P^T came with the device RAP
    else transpose(L.P, L.R);
    t_t += now() - t4;
    snprintf(buf, sizeof buf, "level %d: rows %d nnz %lld -> coarse %d (P nnz %lld)\n", level, fine_size,
             (long long)L.A.nnz(), coarse_size, (long long)L.P.nnz());
    H.log += buf;
    if (!crs.empty()) {
      // rank r owns the C points of its rows on the next level
      std::vector<int> pref(L.cf.size() + 1, 0);
      for (size_t i = 0; i < L.cf.size(); ++i) pref[i + 1] = pref[i] + (L.cf[i] == 1);
      for (int& v : crs) v = pref[v];
    }
    if (!dof.empty()) {  // the next level's functions: those of the C points, in order
      std::vector<int> cdof;
      cdof.reserve(coarse_size);
      for (size_t i = 0; i < L.cf.size(); ++i)
        if (L.cf[i] == 1) cdof.push_back(dof[i]);
      dof.swap(cdof);
    }
    H.lev.emplace_back();
    H.lev[level + 1].A.swap(Ac);
    if (!emul.empty()) {
      emul.swap(emul_c);
      lev_starts.push_back(emul);
    }
    ++level;
    if (coarsen_type > 0 && coarse_size >= (int)(fine_size * 0.75)) {
      // par_amg_setup.c:2858 switches to CLJP; not available in this build.
      throw std::runtime_error("slow coarsening (coarse >= 0.75 fine) would switch to CLJP: unsupported");
    }
    // par_amg_setup.c:2880: the redundant coarse grid's threshold stops the
    // coarsening too (num_procs > 1 only: par_amg_setup.c:294)
    const int max_thresh = std::max(prm.max_coarse_size, rs ? prm.seq_threshold : 0);
    if (level == prm.max_levels - 1 || coarse_size <= max_thresh) finished = true;
  }
  // par_amg_setup.c:2893: the redundant coarse-grid AMG (gen_redcs_mat.c:18
  // hypre_seqAMGSetup): a one-process BoomerAMG on the last level, created with
  // the defaults plus the parameters hypre_seqAMGSetup copies, whose single
  // V-cycle (max_iter 1, tol 0, from the zero coarse-level guess) is the
  // coarse solve.  That cycle is the combined hierarchy's V-cycle below the
  // level, so its levels are appended; from the level on every rank holds the
  // rows whole and relaxes them in one process's blocks.
  if (rs && prm.seq_threshold > 0 && prm.seq_threshold >= prm.max_coarse_size &&
      H.lev.back().A.nrows > prm.max_coarse_size && level != prm.max_levels - 1) {
    AMGParams sub;  // HYPRE_BoomerAMGCreate defaults
    sub.max_row_sum = prm.max_row_sum;
    sub.strong_threshold = prm.strong_threshold;
    sub.coarsen_type = prm.coarsen_type;
    sub.interp_type = prm.interp_type;
    sub.sep_weight = prm.sep_weight;
    sub.trunc_factor = prm.trunc_factor;
    sub.P_max_elmts = prm.P_max_elmts;
    if (prm.user_relax_type > -1) {  // HYPRE_BoomerAMGSetRelaxType (par_amg.c:2100)
      for (int c = 0; c < 3; ++c) sub.relax_type[c] = prm.user_relax_type;
      sub.relax_type[3] = 9;
      sub.user_relax_type = prm.user_relax_type;
    }
    sub.relax_order = prm.relax_order;
    sub.relax_weight = prm.relax_weight;
    for (int c = 0; c < 4; ++c) sub.num_sweeps[c] = prm.num_sweeps[c];
    sub.num_blocks = prm.num_blocks;
    sub.auto_block_rows = prm.auto_block_rows;
    sub.auto_block_min = prm.auto_block_min;
    sub.max_iter = 1;
    sub.tol = 0.0;
    sub.num_functions = prm.num_functions;  // and the gathered functions (gen_redcs_mat.c:212)
    // the combined cycle relaxes every level alike: refuse what would differ
    for (int c = 0; c < 4; ++c)
      if (sub.relax_type[c] != prm.relax_type[c] || sub.num_sweeps[c] != prm.num_sweeps[c])
        throw std::runtime_error("seq_threshold: the coarse-grid AMG would relax otherwise than the hierarchy "
                                 "(set the relax type with SetRelaxType)");
    if (prm.lev_relax_wt_set || prm.lev_outer_wt_set || prm.outer_weight != 1.0)
      throw std::runtime_error("seq_threshold with per-level or outer weights");
    Hierarchy Hs;
    const int Lq = (int)H.lev.size() - 1;
    amg_setup(H.lev[Lq].A, sub, Hs, nullptr, nullptr, dof.empty() ? nullptr : &dof);
    if (Hs.lev.size() > 1) {
      Level& Lv = H.lev[Lq];
      Lv.cf.swap(Hs.lev[0].cf);
      Lv.P.swap(Hs.lev[0].P);
      Lv.R.swap(Hs.lev[0].R);
      for (size_t k = 1; k < Hs.lev.size(); ++k) {
        H.lev.emplace_back();
        Level& D = H.lev.back();
        D.A.swap(Hs.lev[k].A);
        D.P.swap(Hs.lev[k].P);
        D.R.swap(Hs.lev[k].R);
        D.cf.swap(Hs.lev[k].cf);
      }
      H.seq_level = Lq;
      for (int l = Lq; l < (int)H.lev.size(); ++l) {
        const std::vector<int> one = {0, H.lev[l].A.nrows};
        if (l < (int)lev_starts.size()) lev_starts[l] = one;
        else lev_starts.push_back(one);
      }
      snprintf(buf, sizeof buf, "seq_threshold: a one-process coarse-grid AMG from level %d (%d rows): %d levels\n", Lq,
               H.lev[Lq].A.nrows, (int)Hs.lev.size());
      H.log += buf;
    }
  }
  double rss_c, rss_p;
  host_rss_gb(&rss_c, &rss_p);
  snprintf(buf, sizeof buf,
           "setup phases: strength %.3fs coarsen %.3fs interp %.3fs rap %.3fs transpose %.3fs (host RSS %.1f GB, "
           "peak %.1f GB)\n",
           t_s, t_c, t_i, t_r, t_t, rss_c, rss_p);
  H.log += buf;
  const double t_l1 = now();
  const int nl = (int)H.lev.size();
  // l1 norms for the smoothers that need them
  for (int j = 0; j < nl; ++j) {
    Level& L = H.lev[j];
    const int* cfp = (prm.relax_order && !L.cf.empty()) ? L.cf.data() : nullptr;
    if (j < nl - 1 && (uses_l1_gs(prm.relax_type[1]) || uses_l1_gs(prm.relax_type[2])))
      compute_l1_norms(L.A, 4, cfp, prm.blocks_for(L.A.nrows), L.l1);
    else if (j == nl - 1 && uses_l1_gs(prm.relax_type[3]))
      compute_l1_norms(L.A, 4, nullptr, prm.blocks_for(L.A.nrows), L.l1);
    if (j < nl - 1 && (prm.relax_type[1] == 18 || prm.relax_type[2] == 18))
      compute_l1_norms(L.A, 1, cfp, 1, L.l1);
    else if (j == nl - 1 && prm.relax_type[3] == 18)
      compute_l1_norms(L.A, 1, nullptr, 1, L.l1);
    // par_amg_setup.c:3139: Chebyshev (relax 16) eigenvalue estimate and coefficients
    if (prm.relax_type[1] == 16 || prm.relax_type[2] == 16 || (prm.relax_type[3] == 16 && j == nl - 1)) {
      double max_eig = 0.0, min_eig = 0.0;
      if (prm.cheby_eig_est)
        max_eig_estimate_cg(L.A, prm.cheby_scale, prm.cheby_eig_est, &max_eig, &min_eig,
                            lev_starts.empty() ? nullptr : &lev_starts[j]);
      else max_eig_estimate_norm(L.A, prm.cheby_scale, &max_eig);
      L.max_eig = max_eig;
      L.min_eig = min_eig;
      cheby_setup(L.A, max_eig, min_eig, prm.cheby_fraction, prm.cheby_order, prm.cheby_scale, prm.cheby_variant,
                  L.cheby_coefs, L.cheby_ds);
    }
    // par_amg_setup.c:3122: relax type 7 scales by the diagonal (ams.c option 5)
    if (prm.relax_type[1] == 7 || prm.relax_type[2] == 7 || (prm.relax_type[3] == 7 && j == nl - 1)) {
      L.l1.resize(L.A.nrows);
      for (int r = 0; r < L.A.nrows; ++r) {
        double d = L.A.a[L.A.i[r]];
        L.l1[r] = (d == 0.0) ? 1.0 : d;
      }
    }
  }
  // par_amg_setup.c:3290-3305: a negative relax_weight[j] / omega[j] asks for
  // -w CG steps of hypre_BoomerAMGCGRelaxWt on that level (every level but a
  // Gaussian-elimination coarsest one, or one of at most 9 rows)
  for (int j = 0; j < nl; ++j) {
    const bool ge = prm.relax_type[3] == 9 || prm.relax_type[3] == 99 || prm.relax_type[3] == 19 ||
                    prm.relax_type[3] == 98;
    if (!(j < nl - 1 || (!ge && H.lev[j].A.nrows > 9))) continue;
    const double w0 = prm.wt(j), o0 = prm.omega(j);
    if (w0 >= 0 && o0 >= 0) continue;
    if (j >= AMGParams::kWeightLevels) throw std::runtime_error("automatic weights beyond level 63");
    const Level& L = H.lev[j];
    // the blocks of hypre's threads, or of every emulated rank (num_blocks each)
    std::vector<int> bs;
    std::vector<double> l1 = L.l1;
    if (!lev_starts.empty()) {
      const std::vector<int>& st = lev_starts[j];
      bs.push_back(0);
      for (size_t r = 0; r + 1 < st.size(); ++r) {
        const int nbk = prm.blocks_for(st[r + 1] - st[r]);
        const std::vector<int> loc = hypre_block_starts(st[r + 1] - st[r], nbk);
        for (int k = 1; k <= nbk; ++k) bs.push_back(st[r] + loc[k]);
      }
      bool cfr = false;
      if (!l1.empty() && l1_option_for_level(prm, j, nl, &cfr) == 4)
        compute_l1_norms_blocks(L.A, 4, (cfr && !L.cf.empty()) ? L.cf.data() : nullptr, bs, l1);
    } else {
      bs = hypre_block_starts(L.A.nrows, prm.blocks_for(L.A.nrows));
    }
    const int rt = prm.relax_type[1];
    if ((rt == 18 || rt == 7 || uses_l1_gs(rt)) && l1.empty()) throw std::runtime_error("l1 norms missing");
    const std::vector<int>* rsj = lev_starts.empty() ? nullptr : &lev_starts[j];
    if (w0 < 0) {
      prm.lev_relax_wt[j] = cg_relax_weight(L.A, rt, l1, bs, (int)(-w0), rsj);
      prm.lev_relax_wt_set |= (uint64_t)1 << j;
    }
    if (o0 < 0) {
      prm.lev_outer_wt[j] = cg_relax_weight(L.A, rt, l1, bs, (int)(-o0), rsj);
      prm.lev_outer_wt_set |= (uint64_t)1 << j;
    }
  }
  // par_amg_setup.c:3184: a relax weight of 0 on level j becomes 4/3 over the
  // scaled norm max_i sum_j |a_ij| d_i d_j, d = 1/sqrt(|a_ii|)
  // (par_scaled_matnorm.c:21; each row summed in stored order, diagonal part
  // first, then the max over all rows); a zero norm leaves the weight 0
  for (int j = 0; j < nl; ++j) {
    if (prm.wt(j) != 0.0) continue;
    if (j >= AMGParams::kWeightLevels) throw std::runtime_error("relax weight 0 beyond level 63");
    const CSR& M = H.lev[j].A;
    std::vector<double> dis(M.nrows);
    for (int i = 0; i < M.nrows; ++i) dis[i] = 1.0 / sqrt(fabs(M.a[M.i[i]]));
    double mx = 0.0;
#pragma omp parallel for reduction(max : mx) schedule(static)
    for (int i = 0; i < M.nrows; ++i) {
      double sum = 0.0;
      for (int q = M.i[i]; q < M.i[i + 1]; ++q) sum += fabs(M.a[q]) * dis[i] * dis[M.j[q]];
      if (mx < sum) mx = sum;
    }
    prm.lev_relax_wt[j] = mx != 0.0 ? 4.0 / 3.0 / mx : 0.0;
    prm.lev_relax_wt_set |= (uint64_t)1 << j;
  }
  // coarsest-level direct solve
  if (nl > 1 && (prm.relax_type[3] == 9 || prm.relax_type[3] == 99 || prm.relax_type[3] == 19 ||
                 prm.relax_type[3] == 98)) {
    const CSR& Ac = H.lev[nl - 1].A;
    if (Ac.nrows > 8192) throw std::runtime_error("coarsest level too large for the dense direct solve");
    H.coarse_n = Ac.nrows;
    csr_to_dense(Ac, H.coarse_dense);
  }
  snprintf(buf, sizeof buf, "setup: smoother data (l1 norms, weights, coarsest factor) %.3fs\n", now() - t_l1);
  H.log += buf;
  if (prm.print_level > 0) fputs(H.log.c_str(), stderr);
  double tot_rows = 0, tot_nnz = 0;
  const int ncx = H.seq_level >= 0 ? H.seq_level + 1 : (int)H.lev.size();  // the outer AMG's levels
  for (int l = 0; l < ncx; ++l) { tot_rows += H.lev[l].A.nrows; tot_nnz += (double)H.lev[l].A.nnz(); }
  H.grid_complexity = tot_rows / H.lev[0].A.nrows;
  H.operator_complexity = tot_nnz / (double)H.lev[0].A.nnz();
  return 0;
}

}  // namespace hve
