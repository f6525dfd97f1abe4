// Host-side data structures and BoomerAMG setup for hypre-ve_amd.
//
// The setup phase (strength, coarsening, interpolation, Galerkin product) runs
// on the host in C++ exactly as hypre's single-process CPU path does, so that
// the hierarchy handed to the GPU solve is the reference's hierarchy.  The solve
// phase (the hot path) lives in ../device and never falls back to the host.
//
// Reference anchors (SX-Aurora/hypre-ve, src/):
//   parcsr_ls/par_amg.c:141-229        hypre_BoomerAMGCreate defaults
//   parcsr_ls/par_amg_setup.c:889-2880 coarsening loop
//   parcsr_ls/par_strength.c:80        hypre_BoomerAMGCreateSHost
//   parcsr_ls/par_coarsen.c:2031       hypre_BoomerAMGCoarsenPMISHost
//   parcsr_ls/par_indepset.c:25        hypre_BoomerAMGIndepSetInit
//   parcsr_ls/par_lr_interp.c:1041     hypre_BoomerAMGBuildExtPIInterpHost
//   parcsr_mv/par_csr_matrix.c:2671    hypre_ParCSRMatrixTruncate
//   parcsr_ls/par_rap.c:27             hypre_BoomerAMGBuildCoarseOperatorKT
//   parcsr_ls/ams.c:571,3398           hypre_ParCSRComputeL1Norms(Threads)
#pragma once
#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <new>
#include <string>
#include <utility>
#include <vector>

namespace hve {

// Host staging arrays of the layouts (GBs at 512^3): allocated without the
// serial value-initialisation of std::vector, then first touched and filled by
// the builders' OpenMP loops (par_assign), which measured 3-8x faster on the
// 16 cores a GPU gets than std::vector::assign's single-threaded page faults.
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  // large arrays on 2 MiB pages where the kernel grants them (transparent huge
  // pages in madvise mode): 512x fewer first-touch faults
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < ((size_t)64 << 20)) return std::allocator<T>::allocate(n);
    const size_t huge = (size_t)2 << 20, len = (bytes + huge - 1) / huge * huge;
    void* p = std::aligned_alloc(huge, len);
    if (!p) throw std::bad_alloc();
    madvise(p, len, MADV_HUGEPAGE);
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) {
    if (n * sizeof(T) < ((size_t)64 << 20)) std::allocator<T>::deallocate(p, n);
    else std::free(p);
  }
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... Args>
  void construct(U* p, Args&&... args) {
    ::new ((void*)p) U(std::forward<Args>(args)...);
  }
};
template <class T>
using hvec = std::vector<T, NoInitAlloc<T>>;
template <class T>
void par_assign(hvec<T>& v, size_t n, T x) {
  v.clear();
  v.resize(n);
  T* p = v.data();
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) p[i] = x;
}


// Resident and peak host memory of this process in GB (/proc/self/status
// VmRSS / VmHWM; 0 where unavailable): the setup's stage logs.
inline void host_rss_gb(double* cur, double* peak) {
  *cur = *peak = 0.0;
  if (FILE* f = fopen("/proc/self/status", "r")) {
    char line[256];
    while (fgets(line, sizeof line, f)) {
      long long kb = 0;
      if (sscanf(line, "VmRSS: %lld kB", &kb) == 1) *cur = kb / 1048576.0;
      if (sscanf(line, "VmHWM: %lld kB", &kb) == 1) *peak = kb / 1048576.0;
    }
    fclose(f);
  }
}

// CSR matrix, 0-based, hypre convention: in square operators the diagonal
// entry is stored first in its row (parcsr_mv relies on A_diag_i[i] == diag).
struct CSR {
  int nrows = 0, ncols = 0;
  std::vector<int> i;     // nrows + 1
  hvec<int> j;     // nnz (resize leaves new entries uninitialised)
  hvec<double> a;  // nnz
  int64_t nnz() const { return i.empty() ? 0 : (int64_t)i[nrows]; }
  void resize_rows(int nr, int nc) { nrows = nr; ncols = nc; i.assign(nr + 1, 0); }
  void swap(CSR& o) {
    std::swap(nrows, o.nrows); std::swap(ncols, o.ncols);
    i.swap(o.i); j.swap(o.j); a.swap(o.a);
  }
};

// Strength pattern (hypre S): column indices only, no diagonal.
struct Pattern {
  int n = 0;
  std::vector<int> i;
  hvec<int> j;  // no zero fill: the device strength downloads into it
};

// Per-row marker map: the reference's P_marker / A_marker arrays (one int per
// point of the matrix, per thread) restricted to the points one row touches.
// Open addressing in a power-of-two table sized per row from an upper bound of
// its entries; a generation stamp per slot empties the table in O(1) between
// rows.  Lookups cost an L1 hit instead of a cache miss into an array of
// n ints, and a thread holds kilobytes instead of 4n bytes.
struct RowMap {
  std::vector<int> key, val;
  std::vector<unsigned> gen;
  unsigned cur = 0, mask = 0;
  int shift = 32;
  // start a row that inserts at most `bound` keys
  void begin(int64_t bound) {
    size_t cap = 16;
    while ((int64_t)cap < 2 * bound + 2) cap <<= 1;
    if (key.size() < cap) {
      key.assign(cap, 0);
      val.assign(cap, 0);
      gen.assign(cap, 0);
      cur = 0;
    }
    mask = (unsigned)cap - 1;
    shift = 32;
    for (size_t c = cap; c > 1; c >>= 1) --shift;
    if (++cur == 0) {  // stamp wrapped: clear once
      std::fill(gen.begin(), gen.end(), 0u);
      cur = 1;
    }
  }
  // slot of k (inserted with value v0 when absent; *fresh tells which)
  int* find_or_insert(int k, int v0, bool* fresh) {
    unsigned h = ((unsigned)k * 2654435761u) >> shift;
    for (;; h = (h + 1) & mask) {
      if (gen[h] != cur) {
        gen[h] = cur;
        key[h] = k;
        val[h] = v0;
        *fresh = true;
        return &val[h];
      }
      if (key[h] == k) {
        *fresh = false;
        return &val[h];
      }
    }
  }
  // value of k, or dflt when absent
  int get(int k, int dflt) const {
    unsigned h = ((unsigned)k * 2654435761u) >> shift;
    for (;; h = (h + 1) & mask) {
      if (gen[h] != cur) return dflt;
      if (key[h] == k) return val[h];
    }
  }
};

// Working storage of one thread's Galerkin rows (rap_row).
struct RapScratch {
  RowMap AM, PM;
  std::vector<int> ra_j, tj;
  std::vector<double> ra_a, ta;
};

// Point types (hypre: C_PT 1, F_PT -1, Z_PT -2, SF_PT -3).
enum { C_PT = 1, F_PT = -1, Z_PT = -2, SF_PT = -3 };

// Relaxation types supported by this build (hypre numbering, par_relax.c:120).
//   0  weighted Jacobi           18 l1-Jacobi
//   3  hybrid GS forward         4  hybrid GS backward   6 hybrid symmetric GS
//   13 hybrid l1-GS forward      14 hybrid l1-GS backward 8 hybrid l1 symmetric GS
//   7  Jacobi via matvec         9  Gaussian elimination (coarsest level)
struct AMGParams {
  int max_levels = 25;
  int max_coarse_size = 9;
  int min_coarse_size = 0;
  double strong_threshold = 0.25;
  double max_row_sum = 0.9;
  int coarsen_type = 10;          // 8 PMIS, 9 PMIS(seq rand), 10 HMIS
  int measure_type = 0;
  int coarsen_cut_factor = 0;
  int interp_type = 6;            // 6 ext+i, 14 ext, 16/17/18 ext / ext+i / ext+e (MM), 3 direct, 8 standard
  int sep_weight = 0;             // standard interpolation: separate factors for positive / negative weights
  int P_max_elmts = 4;
  double trunc_factor = 0.0;
  // grid_relax_type (par_amg.c:218-220, 339-341: [0] keeps the 3 of the
  // first allocation, par_amg.c:2136); [1] down, [2] up, [3] coarsest
  int relax_type[4] = {3, 13, 14, 9};
  // hypre_ParAMGDataUserRelaxType: set by SetRelaxType only; a one-level
  // hierarchy relaxes with it, or with 6 when unset (par_cycle.c:296-300)
  int user_relax_type = -1;
  int num_sweeps[4] = {1, 1, 1, 1};
  double relax_weight = 1.0;
  double outer_weight = 1.0;
  // Per-level weights (hypre's relax_weight[level] / omega[level] arrays:
  // SetLevelRelaxWt / SetLevelOuterWt, par_amg.c); a level whose bit is clear
  // takes the global value.  SetRelaxWt / SetOuterWt clear every level's bit,
  // as hypre overwrites the whole array.
  static constexpr int kWeightLevels = 64;
  double lev_relax_wt[kWeightLevels] = {};
  double lev_outer_wt[kWeightLevels] = {};
  uint64_t lev_relax_wt_set = 0, lev_outer_wt_set = 0;
  double wt(int level) const {
    return (level >= 0 && level < kWeightLevels && (lev_relax_wt_set >> level & 1)) ? lev_relax_wt[level] : relax_weight;
  }
  double omega(int level) const {
    return (level >= 0 && level < kWeightLevels && (lev_outer_wt_set >> level & 1)) ? lev_outer_wt[level] : outer_weight;
  }
  int relax_order = 0;            // 1 = C/F relaxation
  int cycle_type = 1;             // 1 V, 2 W
  int max_iter = 20;
  int min_iter = 0;
  double tol = 1e-6;
  int converge_type = 0;
  int print_level = 0;
  int logging = 0;
  // Number of contiguous row blocks for the hybrid (block-Jacobi / in-block GS)
  // smoothers; hypre's CPU path uses num_threads for this (par_relax.c:4387).
  int num_blocks = 1;
  // > 0 (hypreve_BoomerAMGSetNumBlocks(0)): num_blocks is the level-0 count,
  // one block of about auto_block_rows rows (hypre's OMP_NUM_THREADS), used on
  // every level as hypre does, except that a coarse level never gets blocks of
  // fewer than auto_block_min rows (there hypre's blocks of 0-1 rows would turn
  // relax 3/4/6 into unweighted Jacobi and 8/13/14 into l1-Jacobi).
  int auto_block_rows = 0;
  int auto_block_min = 64;
  // 1: the ext+i interpolation, its truncation, R = P^T and RAP run on the GPU
  // (device/setup_dev.hip, byte for byte the host result); set by the device
  // setup path only
  int device_setup = 0;
  // hybrid-GS row blocks of a level (one rank's share) of `rows` rows
  int blocks_for(int rows) const {
    const int top = num_blocks < 1 ? 1 : num_blocks;
    if (auto_block_rows > 0) {
      const long long cap = ((long long)rows + auto_block_min - 1) / auto_block_min;
      return (int)std::max(1LL, std::min<long long>(top, cap));
    }
    return top;
  }
  // Aggressive coarsening (par_amg.c:153-173 defaults): the first
  // agg_num_levels levels coarsen twice (second pass on S*S + 2S over the C
  // points, num_paths paths needed) and interpolate with agg_interp_type 4
  // (multipass), truncated by agg_trunc_factor / agg_P_max_elmts.
  // Redundant coarse-grid AMG (par_amg_setup.c:2880-2897, gen_redcs_mat.c:18):
  // with more than one process the hierarchy stops at seq_threshold global
  // rows and a one-process BoomerAMG on that level does the coarse solve
  // (one V-cycle); redundant: every process solves it (same numbers)
  int num_functions = 1;          // systems AMG: functions per point, interleaved (dof = row % num_functions)
  int seq_threshold = 0;
  int redundant = 0;
  int agg_num_levels = 0;
  int agg_interp_type = 4;
  double agg_trunc_factor = 0.0;
  int agg_P_max_elmts = 0;
  double agg_P12_trunc_factor = 0.0;
  int agg_P12_max_elmts = 0;
  int num_paths = 1;
  // Device layout / loop of each SELL operator: 0 automatic (by size, row
  // length and padding), 1 padded lane-per-row, 2 jagged lane-per-row,
  // 3 padded workgroup-per-slice (wide), 4 jagged wave-product-parallel,
  // 5 jagged with a per-slice column dictionary (x-tile in LDS).
  // Every choice gives the same bits; 1-4 let the tests prove that.
  int sell_policy = 0;
  // Chebyshev smoother (relax type 16): par_amg.c:225-229 defaults
  int cheby_order = 2;      // order of the residual polynomial (1..4)
  int cheby_variant = 0;    // 0 standard, 1 modified
  int cheby_scale = 1;      // scale by D^{-1/2}
  int cheby_eig_est = 10;   // CG steps of the eigenvalue estimate (0: inf-norm bound)
  double cheby_fraction = 0.3;
  // Multi-rank: levels from the first one with at most agglo_rows global rows
  // down are replicated on every rank (0 = never); see partition.hpp.
  // -1 (default): automatic, kAggloRowsPerRank rows per rank.
  int agglo_rows = -1;
  static constexpr int kAggloRowsPerRank = 12288;
};

struct Level {
  CSR A;                        // operator on this level
  CSR P;                        // interpolation to this level from level+1 (nrows = A.nrows)
  CSR R;                        // R = P^T (kept explicitly for the GPU restriction)
  std::vector<int> cf;          // CF marker (C_PT / F_PT), empty on coarsest
  std::vector<double> l1;       // row norms for the l1 smoothers (may be empty)
  std::vector<double> dinv;     // unused slot (Jacobi uses A's diagonal directly)
  // Chebyshev (relax 16): 1/sqrt(a_ii) when scaled, polynomial coefficients,
  // eigenvalue estimates (par_amg_setup.c:3139-3164)
  std::vector<double> cheby_ds, cheby_coefs;
  double max_eig = 0.0, min_eig = 0.0;
};

struct Hierarchy {
  AMGParams prm;
  std::vector<Level> lev;
  // Dense coarsest operator for relax type 9 (row-major, par_gauss_elim.c:84).
  int coarse_n = 0;
  std::vector<double> coarse_dense;
  double grid_complexity = 0, operator_complexity = 0;
  std::string log;
  // first level of a redundant coarse-grid AMG (seq_threshold under rank
  // emulation, gen_redcs_mat.c): from here on one process's hierarchy, whose
  // levels every rank holds whole; -1: none
  int seq_level = -1;
};

// ---- generators (parcsr_ls/par_laplace.c:15, par_laplace_27pt.c) ----
// 7-point Laplacian on nx*ny*nz with coefficients (cx,cy,cz), single partition,
// same row/entry ordering as GenerateLaplacian with P=Q=R=1.
void generate_laplacian_7pt(int nx, int ny, int nz, double cx, double cy, double cz, CSR& A);
void generate_laplacian_27pt_block(int nx, int ny, int nz, int P, int Q, int R, int p, int q, int r,
                                   const double* value, CSR& A, int64_t& first_row);
void generate_laplacian_27pt(int nx, int ny, int nz, CSR& A);
// Rank (p,q,r) of a P x Q x R process grid; global column indices, sets first_row.
void generate_laplacian_7pt_block(int nx, int ny, int nz, int P, int Q, int R, int p, int q, int r,
                                  const double* value, CSR& A, int64_t& first_row);

// ---- setup building blocks ----
void create_strength(const CSR& A, double thr, double max_row_sum, Pattern& S);
// Systems AMG ("unknown" approach, num_functions > 1, nodal 0): the function
// of every row of the level being set up (dof_func_array[level]), read by the
// strength, ext(+i), partial ext(+i) and multipass builders; null for one
// function.  Set by amg_setup for the duration of a level (not re-entrant
// across threads; the setup runs one hierarchy at a time).
extern const int* hve_setup_dof;
// rs (optional): emulate the coarsening of an N-rank run, rank r owning rows
// [rs[r], rs[r+1]) (per-rank random streams and first passes, hypre's
// CF_marker_offd semantics).
void coarsen_pmis(const Pattern& S, int cf_init, std::vector<int>& cf, const std::vector<int>* rs = nullptr);
// full_row_len (optional): strong connections of each row including those the
// pattern omits (another rank's columns), for the empty-row test.  f_pnt: the
// marker of measure-0 points (Z_PT under HMIS, F_PT for coarsen_type 11);
// meas_add (optional): measure counted from other ranks' rows (global measures).
void coarsen_ruge_first_pass(const Pattern& S, const CSR* A, int measure_type, int cut_factor,
                             std::vector<int>& cf, const int* full_row_len = nullptr, int f_pnt = Z_PT,
                             const int* meas_add = nullptr);
void coarsen_hmis(const Pattern& S, const CSR* A, int measure_type, int cut_factor, std::vector<int>& cf,
                  const std::vector<int>* rs = nullptr);
void coarsen_ruge1p(const Pattern& S, const CSR* A, int measure_type, int cut_factor, std::vector<int>& cf,
                    const std::vector<int>* rs = nullptr);
// plus_i false: extended interpolation (interp_type 14) instead of ext+i
void build_extpi_interp(const CSR& A, std::vector<int>& cf, const Pattern& S,
                        double trunc_factor, int max_elmts, CSR& P, bool plus_i = true);
// extended+i in matrix-matrix form (interp_type 17, par_mod_lr_interp.c:474)
// extended+i where no common C point (interp_type 7)
void build_extpicc_interp(const CSR& A, std::vector<int>& cf, const Pattern& S, double trunc_factor, int max_elmts,
                          CSR& P);
// standard interpolation (interp_type 8; 9 = 8 with sep_weight 1); rs: emulated rank starts
void build_std_interp(const CSR& A, std::vector<int>& cf, const Pattern& S, double trunc_factor, int max_elmts,
                      int sep_weight, CSR& P, const std::vector<int>* rs = nullptr, bool partial = false);
void build_modextpi_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                           int max_elmts, CSR& P, const std::vector<int>* emul = nullptr, int mm_square = -1);
// extended+e in matrix-matrix form (interp_type 18, par_mod_lr_interp.c:1040)
void build_modextpe_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                           int max_elmts, CSR& P, const std::vector<int>* emul = nullptr, int mm_square = -1);
void build_direct_interp(const CSR& A, std::vector<int>& cf, const Pattern& S,
                         double trunc_factor, int max_elmts, CSR& P);
void truncate_rows(CSR& P, double tol, int max_elmts);
// Aggressive coarsening (aggressive.cpp): par_strength.c:1729 Create2ndS,
// :2957 CorrectCFMarker, par_multi_interp.c:16 BuildMultipass.
void create_2nd_strength(const Pattern& S, std::vector<int>& cf, int num_paths, Pattern& S2);
void correct_cf_marker(std::vector<int>& cf, const std::vector<int>& new_cf);
void correct_cf_marker2(std::vector<int>& cf, const std::vector<int>& new_cf);
// matrix-matrix interpolations (setup.cpp): ModExt (pe false) / ModExtPE, the
// 2-stage second stage ModPartialExt, and P = P1 P2 with the aggressive truncation
// emul: fine row starts of an emulated N-rank run (hypre_ParMatmul's np > 1 order)
// mm_square: hypre_ParMatmul's allsquare decided by global sizes (0 / 1) rather
// than by the product's own (-1): the distributed setup multiplies a rank's
// ghost universe, whose sizes are not the matrix's
void build_modext_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                         int max_elmts, bool pe, CSR& P, const std::vector<int>* emul = nullptr, int mm_square = -1);
void build_modpartialext_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                                int max_elmts, bool pe, CSR& P, const std::vector<int>* emul = nullptr,
                                int mm_square = -1);
// partial ext+i / ext (agg_interp_type 1, 6 / 3): rows = the first stage's C
// points, columns = the second's; resets markers below -1 to -1
void build_partial_extpi_interp(const CSR& A, std::vector<int>& cf, const Pattern& S, double trunc_factor,
                                int max_elmts, bool plus_i, CSR& P);
void multiply_interp(const CSR& P1, const CSR& P2, double trunc_factor, int max_elmts, CSR& P, int mm_square = -1);
void build_multipass_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                            int max_elmts, CSR& P);
// Universe-indexed cores of ext+i and RAP shared by the one-process and the
// distributed setup (see setup.cpp).
void extpi_core(const CSR& A, const Pattern& S, const std::vector<int>& cf, const std::vector<int>& fine_to_coarse,
                int nrows, int ncoarse, int nuniv, CSR& P, bool plus_i = true);
void rap_core(const CSR& R, const CSR& A, const CSR& P, const std::vector<int>& row_ic,
              const std::vector<int>& coarse_glob, int nfine_univ, int ncoarse_univ, int ncoarse_glob, CSR& C);
// Their single rows (the device versions finish rows that overflow LDS here).
int extpi_row_count(const Pattern& S, const std::vector<int>& cf, int i, RowMap& M);
void extpi_row_fill(const CSR& A, const Pattern& S, const std::vector<int>& cf, const std::vector<int>& fine_to_coarse,
                    int i, RowMap& M, CSR& P, bool plus_i = true);
void rap_row(const CSR& R, const CSR& A, const CSR& P, int q, int ic, RapScratch& W);
// row lists of the device setup's host fallback, and its table bounds
int64_t extpi_bound_max(const Pattern& S);
void extpi_count_rows(const Pattern& S, const std::vector<int>& cf, const std::vector<int>& rows,
                      std::vector<int>& cnt);
void extpi_fill_rows(const CSR& A, const Pattern& S, const std::vector<int>& cf,
                     const std::vector<int>& fine_to_coarse, const std::vector<int>& rows, CSR& P);
void truncate_row_list(CSR& P, const std::vector<int>& rows, double tol, int max_elmts, std::vector<int>& newlen);
int64_t rap_bound_max(const CSR& R, const CSR& A);
void rap_row_list(const CSR& R, const CSR& A, const CSR& P, const std::vector<int>& rows,
                  std::vector<std::vector<int>>& oj, std::vector<std::vector<double>>& oa);
// one row of truncate_rows in its own slots; returns the new length
int truncate_row(CSR& P, int r, double tol, int max_elmts, std::vector<int>& rj, std::vector<double>& ra);
double hypre_rand_at(int64_t k, int seed);
// Chebyshev smoother setup (one process, one thread, as the reference's host
// path): par_relax_more.c:115 hypre_ParCSRMaxEigEstimateCG (random start
// vector of hypre_ParVectorSetRandomValues(r, 1), Lanczos tridiagonal from CG,
// eigenvalues by LINPACK tql1), par_relax_more.c:25 hypre_ParCSRMaxEigEstimate
// (inf-norm bound), par_cheby.c:36 hypre_ParCSRRelax_Cheby_Setup.
void max_eig_estimate_cg(const CSR& A, int scale, int max_iter, double* max_eig, double* min_eig,
                         const std::vector<int>* rs = nullptr);  // rs: emulated rank row starts
void max_eig_estimate_norm(const CSR& A, int scale, double* max_eig);
void cheby_setup(const CSR& A, double max_eig, double min_eig, double fraction, int order, int scale, int variant,
                 std::vector<double>& coefs, std::vector<double>& ds);
// EISPACK tql1 (par_relax_more.c:753): eigenvalues of the symmetric
// tridiagonal (d, e[1..n-1]) in ascending order into d; 0 or the failing index.
int linpack_tql1(int n, double* d, double* e);
void transpose(const CSR& A, CSR& AT);
void rap(const CSR& P, const CSR& A, CSR& RAP);
void compute_l1_norms(const CSR& A, int option, const int* cf, int num_blocks,
                      std::vector<double>& l1);
void compute_l1_norms_blocks(const CSR& A, int option, const int* cf, const std::vector<int>& block_starts,
                             std::vector<double>& l1);
// l1 norm option amg_setup computes on level j of nl (0, 1 or 4).
int l1_option_for_level(const AMGParams& prm, int j, int nl, bool* cf_restricted);

// Full setup; returns 0 on success.
// rank_starts (optional, N+1 level-0 row starts): build the hierarchy an N-rank
// hypre run builds (rows in ParCSR diag/offd order on every level, per-rank
// coarsening); the solve path is unchanged.
// coarsen_starts (optional, N+1 level-0 row starts): HMIS (coarsen_type 10)
// as an N-process run coarsens, each rank's Ruge first pass over the strong
// connections it owns and per-rank random streams in the PMIS stage, rank r
// owning the C points of its rows on the next level; nothing else changes
// (entry order, interpolation, RAP stay the one-process ones).  This is what
// the distributed setup computes (dsetup.cpp hmis_dist); PMIS ignores it.
// dof0 (num_functions > 1): the level-0 functions when given (the redundant
// coarse grid's gathered ones), else row % num_functions.
int amg_setup(const CSR& A, const AMGParams& prm, Hierarchy& H, const std::vector<int>* rank_starts = nullptr,
              const std::vector<int>* coarsen_starts = nullptr, const std::vector<int>* dof0 = nullptr);


}  // namespace hve
