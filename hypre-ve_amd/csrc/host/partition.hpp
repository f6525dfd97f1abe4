// Row partition of a BoomerAMG hierarchy over ranks (one GPU per rank).
//
// Level 0 rows are owned in the caller's contiguous blocks (the ParCSR row
// partition the user assembled, hypre's row_starts).  On every coarser level a
// rank owns the C points of its fine rows (hypre_BoomerAMGCoarseParms), which
// are again contiguous because fine_to_coarse is monotone.
//
// Each operator a rank applies is stored with columns in a [local | halo]
// index space of the input vector (the reference's diag/offd pair with
// col_map_offd, par_csr_matrix.h, folded into one column space), and its rows
// are split into interior rows (no halo column: computed while the halo is in
// flight) and boundary rows.  Entries keep their global row order, so every
// row sum equals the single-GPU one bit for bit.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "hve_host.hpp"

namespace hve {

struct RankOp {
  CSR interior, boundary;            // rows: subsets of the owned rows
  std::vector<int> map_int, map_bnd; // subset row -> local row
  int nrows_local = 0;               // owned rows of the output vector
};

// Halo of one vector: values this rank receives (placed after its n_loc owned
// entries, grouped by peer in ascending global index) and sends.
struct RankHalo {
  int n_loc = 0, n_halo = 0;
  std::vector<int> peers;      // ranks exchanged with (sorted)
  std::vector<int> recv_cnt;   // per peer, contiguous at n_loc + recv_off
  std::vector<int> send_cnt;   // per peer
  std::vector<int> send_idx;   // local indices, concatenated per peer
  std::vector<int> halo_glob;  // global indices of the halo entries (debug / tests)
};

struct RankLevel {
  int n_loc = 0, first = 0, n_glob = 0;
  RankOp A;          // A_l local rows; cols in u_l space
  RankOp P;          // P_l local fine rows; cols in u_{l+1} space (not on coarsest)
  RankOp R;          // R_l = P_l^T local coarse rows (level l+1); cols in V_l space
  RankHalo hu;       // halo of u_l (union of A_l and P_{l-1} needs)
  RankHalo hv;       // halo of V_l (R_l needs)
  std::vector<double> l1;
  std::vector<int> cf;
  std::vector<double> cheby_ds;     // Chebyshev: 1/sqrt(a_ii) of the owned rows (scaled variant)
  std::vector<double> cheby_coefs;  // Chebyshev polynomial coefficients (replicated)
  // Hybrid Gauss-Seidel row blocks over the held rows (local numbering, nb+1
  // starts); empty: hypre_block_starts(n_loc, num_blocks).  Several ranks:
  // num_blocks blocks of each rank's rows, as hypre's threads per process.
  std::vector<int> gs_blocks;
};

struct RankHierarchy {
  int rank = 0, size = 1;
  AMGParams prm;
  std::vector<RankLevel> lev;
  int coarse_n = 0;
  std::vector<double> coarse_dense;  // replicated coarsest operator
  double grid_complexity = 0, operator_complexity = 0;
  std::vector<int64_t> nnz_A, rows;  // global per-level statistics
  // Coarse-level agglomeration: levels >= agg_level are held whole by every
  // rank (first 0, n_loc = n_glob, no halos) and cycled redundantly, without
  // communication; the restriction into agg_level writes this rank's rows
  // agg_starts[rank] .. agg_starts[rank+1] and an all-gather completes the
  // vector.  P of level agg_level-1 reads the replicated vector directly.
  // -1: no agglomeration (one rank, or agglo_rows 0).
  int agg_level = -1;
  std::vector<int> agg_starts;
};
// First replicated level for `size` ranks (rank-independent): the first level
// l >= 1 with rows[l] <= prm.agglo_rows (automatic when negative: 12288 rows
// per rank), or -1.
int agglomeration_level(const AMGParams& prm, const std::vector<int64_t>& rows, int size);

// starts0: level-0 row starts (size+1 entries).
void partition_hierarchy(const Hierarchy& H, const std::vector<int>& starts0, int rank, int size,
                         RankHierarchy& out);
// Rows [r0, r1) of M (global columns) as a rank's operator whose input vector
// is owned on [a, b) with the sorted off-rank reads `halo`: columns in the
// [local | halo] space, rows split into interior and boundary.
void make_rank_op(const CSR& M, int r0, int r1, int a, int b, const std::vector<int>& halo, RankOp& op);
// Every rank's part in one pass (O(global) work; partition_hierarchy
// partitions all ranks to return one).
void partition_hierarchy_all(const Hierarchy& H, const std::vector<int>& starts0, int size,
                             std::vector<RankHierarchy>& out);
// Whole hierarchy as one rank (no halo), used for the single-GPU path.
// gs_rank_starts (optional, N+1 level-0 row starts): run the hybrid
// Gauss-Seidel smoothers with the row blocks an N-rank partition would use
// on every level (num_blocks per rank, l1 norms to match), so that one GPU
// reproduces the N-rank iterates.
void single_rank_hierarchy(const Hierarchy& H, RankHierarchy& out, const std::vector<int>* gs_rank_starts = nullptr);
// One rank without copies: every row of a one-rank partition is an interior
// row and every column local, so the rank's operators are the hierarchy's own
// matrices.  lend moves them into `out` (the rest as single_rank_hierarchy
// builds it) and leaves H's level matrices empty until give_back returns them
// (call it after the device build, also when the build throws).  Returns
// false (nothing moved) where a matrix's shape does not allow it; the caller
// then uses single_rank_hierarchy.
bool lend_single_rank(Hierarchy& H, RankHierarchy& out, const std::vector<int>* gs_rank_starts = nullptr);
void give_back_single_rank(Hierarchy& H, RankHierarchy& out);
// The hybrid-GS row blocks and option-4 l1 norms of every level that
// single_rank_hierarchy gives the device for gs_rank_starts (empty when the
// emulation is off): exported so the CPU oracle sweeps the same blocks.
void gs_rank_blocks_host(const Hierarchy& H, const std::vector<int>& gs_rank_starts,
                         std::vector<std::vector<int>>& blocks, std::vector<std::vector<double>>& l1);
// Per level: global hybrid-GS block starts of an N-rank partition with level-0
// starts starts0 (num_blocks blocks of every rank's rows; replicated levels
// num_blocks blocks of the whole level).
std::vector<std::vector<int>> rank_gs_blocks(const Hierarchy& H, const std::vector<int>& starts0, int size);

int partition_self_check(const Hierarchy& H, int size, std::string& msg);

void serialize(const RankHierarchy& R, std::vector<char>& buf);
void deserialize(const std::vector<char>& buf, RankHierarchy& R);

}  // namespace hve
