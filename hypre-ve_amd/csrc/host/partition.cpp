// Row partition of the hierarchy (see partition.hpp).
#include "layout.hpp"
#include "partition.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace hve {

namespace {

int owner_of(const std::vector<int>& starts, int g) {
  // starts: size+1 ascending; returns r with starts[r] <= g < starts[r+1]
  auto it = std::upper_bound(starts.begin(), starts.end(), g);
  return (int)(it - starts.begin()) - 1;
}

// Collect the sorted, unique global columns outside [a,b) referenced by rows
// [r0,r1) of M.
void halo_cols(const CSR& M, int r0, int r1, int a, int b, std::vector<int>& out) {
  if (a <= 0 && b >= M.ncols) return;  // every column is local (one rank, or a replicated level)
  for (int r = r0; r < r1; ++r)
    for (int k = M.i[r]; k < M.i[r + 1]; ++k) {
      const int c = M.j[k];
      if (c < a || c >= b) out.push_back(c);
    }
}
void sort_unique(std::vector<int>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

// Build the local operator for rows [r0,r1) of M whose input vector is owned
// on [a,b) with halo list `halo` (sorted global indices).
void make_op(const CSR& M, int r0, int r1, int a, int b, const std::vector<int>& halo, RankOp& op) {
  const int nloc_in = b - a;
  const int nrows = r1 - r0;
  op.nrows_local = nrows;
  std::vector<char> bnd(nrows, 0);
#pragma omp parallel for schedule(static)
  for (int r = r0; r < r1; ++r)
    for (int k = M.i[r]; k < M.i[r + 1]; ++k) {
      const int c = M.j[k];
      if (c < a || c >= b) { bnd[r - r0] = 1; break; }
    }
  // row copies in parallel (one rank's operators are the whole hierarchy)
  auto build = [&](bool want_bnd, CSR& out, std::vector<int>& map) {
    map.clear();
    for (int r = 0; r < nrows; ++r)
      if ((bool)bnd[r] == want_bnd) map.push_back(r);
    const int m = (int)map.size();
    out.resize_rows(m, nloc_in + (int)halo.size());
    for (int q = 0; q < m; ++q) {
      const int r = map[q] + r0;
      out.i[q + 1] = out.i[q] + (M.i[r + 1] - M.i[r]);
    }
    out.j.resize(out.i[m]);
    out.a.resize(out.i[m]);
#pragma omp parallel for schedule(static)
    for (int q = 0; q < m; ++q) {
      const int r = map[q] + r0;
      int o = out.i[q];
      for (int k = M.i[r]; k < M.i[r + 1]; ++k, ++o) {
        const int c = M.j[k];
        int lc;
        if (c >= a && c < b) lc = c - a;
        else lc = nloc_in + (int)(std::lower_bound(halo.begin(), halo.end(), c) - halo.begin());
        out.j[o] = lc;
        out.a[o] = M.a[k];
      }
    }
  };
  build(false, op.interior, op.map_int);
  build(true, op.boundary, op.map_bnd);
}

}  // namespace

void make_rank_op(const CSR& M, int r0, int r1, int a, int b, const std::vector<int>& halo, RankOp& op) {
  make_op(M, r0, r1, a, b, halo, op);
}

// Row starts of every level: a rank owns the C points of its fine rows.
static std::vector<std::vector<int>> level_starts(const Hierarchy& H, const std::vector<int>& starts0, int size) {
  const int nl = (int)H.lev.size();
  if ((int)starts0.size() != size + 1 || starts0[size] != H.lev[0].A.nrows)
    throw std::runtime_error("partition: level-0 row starts do not cover the matrix");
  std::vector<std::vector<int>> starts(nl, std::vector<int>(size + 1, 0));
  starts[0] = starts0;
  for (int l = 0; l + 1 < nl; ++l) {
    const std::vector<int>& cf = H.lev[l].cf;
    std::vector<int> pref(cf.size() + 1, 0);
    for (size_t i = 0; i < cf.size(); ++i) pref[i + 1] = pref[i] + (cf[i] == 1);
    for (int r = 0; r <= size; ++r) starts[l + 1][r] = pref[starts[l][r]];
  }
  return starts;
}

static int hierarchy_agg_level(const Hierarchy& H, int size) {
  std::vector<int64_t> grows(H.lev.size());
  for (size_t l = 0; l < H.lev.size(); ++l) grows[l] = H.lev[l].A.nrows;
  int a = agglomeration_level(H.prm, grows, size);
  if (H.seq_level >= 0 && (a < 0 || H.seq_level < a)) a = H.seq_level;  // a redundant coarse-grid AMG
  return a;
}

static bool uses_hybrid_gs(const AMGParams& prm) {
  for (int c = 0; c < 4; ++c) {
    const int t = prm.relax_type[c];
    if (t == 3 || t == 4 || t == 6 || t == 8 || t == 13 || t == 14) return true;
  }
  return false;
}

// Hybrid-GS row blocks of every level in an N-rank run: each rank's rows in
// num_blocks blocks (hypre's threads per process).  Agglomerated levels keep
// them (every rank sweeps the whole level redundantly, in its owners' blocks,
// which is hypre's per-process sweep); the levels of the redundant coarse-grid
// AMG (seq_threshold) are one process's (gen_redcs_mat.c).
std::vector<std::vector<int>> rank_gs_blocks(const Hierarchy& H, const std::vector<int>& starts0, int size) {
  const int nl = (int)H.lev.size();
  const auto starts = level_starts(H, starts0, size);
  std::vector<std::vector<int>> out(nl);
  for (int l = 0; l < nl; ++l) {
    const int n = H.lev[l].A.nrows;
    if (H.seq_level >= 0 && l >= H.seq_level) {
      out[l] = hypre_block_starts(n, H.prm.blocks_for(n));
      continue;
    }
    out[l].assign(1, 0);
    for (int r = 0; r < size; ++r) {
      const int a = starts[l][r], b = starts[l][r + 1];
      const int nb = H.prm.blocks_for(b - a);
      const std::vector<int> loc = hypre_block_starts(b - a, nb);
      for (int k = 1; k <= nb; ++k) out[l].push_back(a + loc[k]);
    }
  }
  return out;
}

// l1 norms of every level as the hybrid-GS row blocks `blocks` give them
// (option 4 levels only; other levels keep the setup's norms).
static std::vector<std::vector<double>> l1_for_blocks(const Hierarchy& H, const std::vector<std::vector<int>>& blocks) {
  const int nl = (int)H.lev.size();
  std::vector<std::vector<double>> out(nl);
  for (int l = 0; l < nl; ++l) {
    const Level& L = H.lev[l];
    bool cfr = false;
    if (L.l1.empty() || l1_option_for_level(H.prm, l, nl, &cfr) != 4) {
      out[l] = L.l1;
      continue;
    }
    const int* cfp = (cfr && !L.cf.empty()) ? L.cf.data() : nullptr;
    compute_l1_norms_blocks(L.A, 4, cfp, blocks[l], out[l]);
  }
  return out;
}

static void partition_all(const Hierarchy& H, const std::vector<int>& starts0, int size,
                          std::vector<RankHierarchy>& out) {
  const int nl = (int)H.lev.size();
  const std::vector<std::vector<int>> starts = level_starts(H, starts0, size);
  const int agg = hierarchy_agg_level(H, size);
  // hybrid GS across ranks: every rank's rows form num_blocks blocks (hypre's
  // threads per process), and the option-4 l1 norms follow those blocks
  const bool gs_ranks = size > 1 && uses_hybrid_gs(H.prm);
  std::vector<std::vector<double>> l1_ranks;
  std::vector<std::vector<int>> gs_blocks;
  if (gs_ranks) {
    gs_blocks = rank_gs_blocks(H, starts0, size);
    l1_ranks = l1_for_blocks(H, gs_blocks);
  }
  // rows of level l this rank holds: its block, or all of a replicated level
  auto lo = [&](int l, int r) { return (agg >= 0 && l >= agg) ? 0 : starts[l][r]; };
  auto hi = [&](int l, int r) { return (agg >= 0 && l >= agg) ? H.lev[l].A.nrows : starts[l][r + 1]; };
  out.assign(size, RankHierarchy());
  for (int r = 0; r < size; ++r) {
    RankHierarchy& R = out[r];
    R.rank = r;
    R.size = size;
    R.prm = H.prm;
    R.lev.resize(nl);
    R.coarse_n = H.coarse_n;
    R.coarse_dense = H.coarse_dense;
    R.grid_complexity = H.grid_complexity;
    R.operator_complexity = H.operator_complexity;
    for (int l = 0; l < nl; ++l) {
      R.nnz_A.push_back(H.lev[l].A.nnz());
      R.rows.push_back(H.lev[l].A.nrows);
    }
    R.agg_level = agg;
    if (agg >= 0) R.agg_starts = starts[agg];
  }
  // halo sets per rank per level: u_l (A_l and P_{l-1}) and V_l (R_l)
  std::vector<std::vector<std::vector<int>>> hu(nl, std::vector<std::vector<int>>(size)),
      hv(nl, std::vector<std::vector<int>>(size));
  for (int l = 0; l < nl; ++l) {
    const Level& L = H.lev[l];
#pragma omp parallel for schedule(dynamic) if (size > 1)
    for (int r = 0; r < size; ++r) {
      const int a = lo(l, r), b = hi(l, r);
      std::vector<int> u;
      halo_cols(L.A, a, b, a, b, u);
      if (l > 0) halo_cols(H.lev[l - 1].P, lo(l - 1, r), hi(l - 1, r), a, b, u);
      sort_unique(u);
      hu[l][r].swap(u);
      if (l + 1 < nl) {
        // R_l rows: this rank's rows of level l+1 in the distributed sense
        // (its share of the restriction into a replicated level too)
        std::vector<int> v;
        const int ra = (agg >= 0 && l >= agg) ? 0 : starts[l + 1][r];
        const int rb = (agg >= 0 && l >= agg) ? H.lev[l + 1].A.nrows : starts[l + 1][r + 1];
        halo_cols(L.R, ra, rb, a, b, v);
        sort_unique(v);
        hv[l][r].swap(v);
      }
    }
  }
  for (int l = 0; l < nl; ++l) {
    const Level& L = H.lev[l];
    // one rank: the rank loop stays serial and make_op's row copies run in parallel
#pragma omp parallel for schedule(dynamic) if (size > 1)
    for (int r = 0; r < size; ++r) {
      RankLevel& RL = out[r].lev[l];
      const int a = lo(l, r), b = hi(l, r);
      RL.n_loc = b - a;
      RL.first = a;
      RL.n_glob = L.A.nrows;
      make_op(L.A, a, b, a, b, hu[l][r], RL.A);
      if (l + 1 < nl) {
        const int ca = lo(l + 1, r), cb = hi(l + 1, r);
        make_op(L.P, a, b, ca, cb, hu[l + 1][r], RL.P);
        const int ra = (agg >= 0 && l >= agg) ? 0 : starts[l + 1][r];
        const int rb = (agg >= 0 && l >= agg) ? H.lev[l + 1].A.nrows : starts[l + 1][r + 1];
        make_op(L.R, ra, rb, a, b, hv[l][r], RL.R);
      }
      if (gs_ranks) {
        if (!l1_ranks[l].empty()) RL.l1.assign(l1_ranks[l].begin() + a, l1_ranks[l].begin() + b);
        // a replicated level: every rank sweeps it whole in its owners' blocks
        RL.gs_blocks = (agg >= 0 && l >= agg) ? gs_blocks[l] : hypre_block_starts(b - a, H.prm.blocks_for(b - a));
      } else if (!L.l1.empty()) {
        RL.l1.assign(L.l1.begin() + a, L.l1.begin() + b);
      }
      if (!L.cf.empty()) RL.cf.assign(L.cf.begin() + a, L.cf.begin() + b);
      if (!L.cheby_ds.empty()) RL.cheby_ds.assign(L.cheby_ds.begin() + a, L.cheby_ds.begin() + b);
      RL.cheby_coefs = L.cheby_coefs;
      // halo plans
      for (int which = 0; which < 2; ++which) {
        if (which == 1 && l + 1 >= nl) break;
        RankHalo& h = which == 0 ? RL.hu : RL.hv;
        const std::vector<int>& mine = which == 0 ? hu[l][r] : hv[l][r];
        h.n_loc = b - a;
        h.n_halo = (int)mine.size();
        h.halo_glob = mine;
        // receive side: group my halo by owner
        std::vector<int> rc(size, 0), sc(size, 0);
        for (int g : mine) rc[owner_of(starts[l], g)]++;
        // send side: every peer's halo entries that I own
        std::vector<std::vector<int>> sidx(size);
        for (int p = 0; p < size; ++p) {
          if (p == r) continue;
          const std::vector<int>& theirs = which == 0 ? hu[l][p] : hv[l][p];
          auto lo_it = std::lower_bound(theirs.begin(), theirs.end(), a);
          auto hi_it = std::lower_bound(theirs.begin(), theirs.end(), b);
          for (auto it = lo_it; it != hi_it; ++it) sidx[p].push_back(*it - a);
          sc[p] = (int)sidx[p].size();
        }
        for (int p = 0; p < size; ++p) {
          if (p == r || (rc[p] == 0 && sc[p] == 0)) continue;
          h.peers.push_back(p);
          h.recv_cnt.push_back(rc[p]);
          h.send_cnt.push_back(sc[p]);
          h.send_idx.insert(h.send_idx.end(), sidx[p].begin(), sidx[p].end());
        }
      }
    }
  }
}

int agglomeration_level(const AMGParams& prm, const std::vector<int64_t>& rows, int size) {
  if (size <= 1 || prm.agglo_rows == 0) return -1;
  // automatic (-1): a level is replicated once each rank's share is below
  // kAggloRowsPerRank rows; its operators then take a few microseconds per
  // application on one GPU, less than one halo exchange's latency
  const int64_t lim = prm.agglo_rows > 0 ? prm.agglo_rows : (int64_t)AMGParams::kAggloRowsPerRank * size;
  for (size_t l = 1; l < rows.size(); ++l)
    if (rows[l] <= lim) return (int)l;
  return -1;
}

// Self-check used by the CPU test-suite: reassembles every rank's operators,
// checks halo plans pairwise and emulates the distributed apply (interior +
// boundary rows over [local | halo] vectors) against the global operator.
int partition_self_check(const Hierarchy& H, int size, std::string& msg) {
  const int n0 = H.lev[0].A.nrows;
  std::vector<int> s0(size + 1);
  for (int r = 0; r <= size; ++r) s0[r] = (int)((int64_t)n0 * r / size);
  std::vector<RankHierarchy> all;
  partition_all(H, s0, size, all);
  int errs = 0;
  auto fail = [&](const std::string& m) { if (errs++ < 5) msg += m + "\n"; };
  // serialization round trip
  for (int r = 0; r < size; ++r) {
    std::vector<char> b1, b2;
    serialize(all[r], b1);
    RankHierarchy back;
    deserialize(b1, back);
    serialize(back, b2);
    if (b1 != b2) fail("serialize round trip differs on rank " + std::to_string(r));
  }
  const int nl = (int)H.lev.size();
  uint64_t seed = 12345;
  auto rnd = [&]() { seed = seed * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(seed >> 11) / 9007199254740992.0 - 0.5; };
  for (int l = 0; l < nl; ++l) {
    for (int which = 0; which < 3; ++which) {  // A, P, R
      if (which > 0 && l + 1 >= nl) continue;
      const CSR& G = which == 0 ? H.lev[l].A : (which == 1 ? H.lev[l].P : H.lev[l].R);
      std::vector<double> x(G.ncols), yg(G.nrows, 0.0), yd(G.nrows, 0.0);
      for (auto& v : x) v = rnd();
      for (int i = 0; i < G.nrows; ++i) {
        double t = 0.0;
        for (int k = G.i[i]; k < G.i[i + 1]; ++k) t += G.a[k] * x[G.j[k]];
        yg[i] = t;
      }
      for (int r = 0; r < size; ++r) {
        const RankLevel& L = all[r].lev[l];
        // input vector ownership and halo for this operator
        const RankLevel& Lin = which == 1 ? all[r].lev[l + 1] : L;
        const RankHalo& h = which == 2 ? L.hv : Lin.hu;
        const int in_first = Lin.first, in_loc = Lin.n_loc;
        std::vector<double> xl(in_loc + h.n_halo);
        for (int i = 0; i < in_loc; ++i) xl[i] = x[in_first + i];
        for (int k = 0; k < h.n_halo; ++k) xl[in_loc + k] = x[h.halo_glob[k]];
        const RankOp& op = which == 0 ? L.A : (which == 1 ? L.P : L.R);
        // the restriction into the first replicated level writes this rank's
        // share of its rows (agg_starts); everything else its held rows
        const int agg = all[r].agg_level;
        const int out_first = which == 2 ? ((agg >= 0 && l + 1 == agg) ? all[r].agg_starts[r] : all[r].lev[l + 1].first)
                                         : L.first;
        for (int part = 0; part < 2; ++part) {
          const CSR& M = part == 0 ? op.interior : op.boundary;
          const std::vector<int>& mp = part == 0 ? op.map_int : op.map_bnd;
          for (int q = 0; q < M.nrows; ++q) {
            double t = 0.0;
            for (int k = M.i[q]; k < M.i[q + 1]; ++k) {
              if (part == 0 && M.j[k] >= in_loc) fail("interior row reads a halo column");
              t += M.a[k] * xl[M.j[k]];
            }
            yd[out_first + mp[q]] = t;
          }
        }
      }
      for (int i = 0; i < G.nrows; ++i)
        if (yg[i] != yd[i]) { fail("level " + std::to_string(l) + " op " + std::to_string(which) + " row " + std::to_string(i) + " differs"); break; }
    }
    // pairwise halo plans: what p sends to r == r's halo entries owned by p
    for (int which = 0; which < 2; ++which) {
      if (which == 1 && l + 1 >= nl) continue;
      for (int r = 0; r < size; ++r) {
        const RankHalo& hr = which == 0 ? all[r].lev[l].hu : all[r].lev[l].hv;
        int roff = 0;
        for (size_t q = 0; q < hr.peers.size(); ++q) {
          const int p = hr.peers[q];
          const RankHalo& hp = which == 0 ? all[p].lev[l].hu : all[p].lev[l].hv;
          auto it = std::find(hp.peers.begin(), hp.peers.end(), r);
          if (it == hp.peers.end()) { fail("asymmetric peer lists"); continue; }
          const size_t pq = it - hp.peers.begin();
          int soff = 0;
          for (size_t z = 0; z < pq; ++z) soff += hp.send_cnt[z];
          if (hp.send_cnt[pq] != hr.recv_cnt[q]) fail("send/recv count mismatch");
          else
            for (int k = 0; k < hr.recv_cnt[q]; ++k)
              if (all[p].lev[l].first + hp.send_idx[soff + k] != hr.halo_glob[roff + k]) { fail("halo order mismatch"); break; }
          roff += hr.recv_cnt[q];
        }
        if (roff != hr.n_halo) fail("halo not fully received");
      }
    }
  }
  return errs;
}

void partition_hierarchy_all(const Hierarchy& H, const std::vector<int>& starts0, int size,
                             std::vector<RankHierarchy>& out) {
  partition_all(H, starts0, size, out);
}

void partition_hierarchy(const Hierarchy& H, const std::vector<int>& starts0, int rank, int size,
                         RankHierarchy& out) {
  std::vector<RankHierarchy> all;
  partition_all(H, starts0, size, all);
  out = std::move(all[rank]);
}

void gs_rank_blocks_host(const Hierarchy& H, const std::vector<int>& gs_rank_starts,
                         std::vector<std::vector<int>>& blocks, std::vector<std::vector<double>>& l1) {
  blocks.clear();
  l1.clear();
  if (gs_rank_starts.size() <= 2 || !uses_hybrid_gs(H.prm)) return;
  blocks = rank_gs_blocks(H, gs_rank_starts, (int)gs_rank_starts.size() - 1);
  l1 = l1_for_blocks(H, blocks);
}

void single_rank_hierarchy(const Hierarchy& H, RankHierarchy& out, const std::vector<int>* gs_rank_starts) {
  std::vector<int> s0 = {0, H.lev[0].A.nrows};
  partition_hierarchy(H, s0, 0, 1, out);
  if (gs_rank_starts && gs_rank_starts->size() > 2 && uses_hybrid_gs(H.prm)) {
    const int size = (int)gs_rank_starts->size() - 1;
    const auto blocks = rank_gs_blocks(H, *gs_rank_starts, size);
    const auto l1 = l1_for_blocks(H, blocks);
    for (size_t l = 0; l < out.lev.size(); ++l) {
      out.lev[l].gs_blocks = blocks[l];
      out.lev[l].l1 = l1[l];
    }
  }
}

bool lend_single_rank(Hierarchy& H, RankHierarchy& out, const std::vector<int>* gs_rank_starts) {
  const int nl = (int)H.lev.size();
  if (nl == 0) return false;
  for (int l = 0; l < nl; ++l) {  // make_op's shapes: columns local to the one rank
    const Level& L = H.lev[l];
    if (L.A.ncols != L.A.nrows) return false;
    if (l + 1 < nl && (L.P.nrows != L.A.nrows || L.P.ncols != H.lev[l + 1].A.nrows ||
                       L.R.nrows != H.lev[l + 1].A.nrows || L.R.ncols != L.A.nrows))
      return false;
  }
  out = RankHierarchy();
  out.rank = 0;
  out.size = 1;
  out.prm = H.prm;
  out.lev.resize(nl);
  out.coarse_n = H.coarse_n;
  out.coarse_dense = H.coarse_dense;
  out.grid_complexity = H.grid_complexity;
  out.operator_complexity = H.operator_complexity;
  for (int l = 0; l < nl; ++l) {
    out.nnz_A.push_back(H.lev[l].A.nnz());
    out.rows.push_back(H.lev[l].A.nrows);
  }
  out.agg_level = -1;
  // the GS emulation reads H's matrices: before they move
  std::vector<std::vector<int>> blocks;
  std::vector<std::vector<double>> l1b;
  if (gs_rank_starts && gs_rank_starts->size() > 2 && uses_hybrid_gs(H.prm)) {
    blocks = rank_gs_blocks(H, *gs_rank_starts, (int)gs_rank_starts->size() - 1);
    l1b = l1_for_blocks(H, blocks);
  }
  auto lend = [](CSR& M, RankOp& op) {
    op.nrows_local = M.nrows;
    op.map_int.resize(M.nrows);
    for (int r = 0; r < M.nrows; ++r) op.map_int[r] = r;
    op.map_bnd.clear();
    op.boundary = CSR();
    op.boundary.resize_rows(0, M.ncols);
    op.interior.swap(M);
  };
  for (int l = 0; l < nl; ++l) {
    Level& L = H.lev[l];
    RankLevel& RL = out.lev[l];
    const int n = L.A.nrows;
    RL.n_loc = n;
    RL.first = 0;
    RL.n_glob = n;
    RL.l1 = blocks.empty() ? L.l1 : l1b[l];
    if (!blocks.empty()) RL.gs_blocks = blocks[l];
    RL.cf = L.cf;
    RL.cheby_ds = L.cheby_ds;
    RL.cheby_coefs = L.cheby_coefs;
    RL.hu = RankHalo();
    RL.hu.n_loc = n;
    RL.hv = RankHalo();
    if (l + 1 < nl) RL.hv.n_loc = n;
    lend(L.A, RL.A);
    if (l + 1 < nl) {
      lend(L.P, RL.P);
      lend(L.R, RL.R);
    }
  }
  return true;
}

void give_back_single_rank(Hierarchy& H, RankHierarchy& out) {
  const int nl = (int)std::min(H.lev.size(), out.lev.size());
  for (int l = 0; l < nl; ++l) {
    Level& L = H.lev[l];
    RankLevel& RL = out.lev[l];
    if (L.A.nrows == 0 && RL.A.interior.nrows > 0) L.A.swap(RL.A.interior);
    if (l + 1 < nl) {
      if (L.P.nrows == 0 && RL.P.interior.nrows > 0) L.P.swap(RL.P.interior);
      if (L.R.nrows == 0 && RL.R.interior.nrows > 0) L.R.swap(RL.R.interior);
    }
    for (RankOp* op : {&RL.A, &RL.P, &RL.R}) {
      op->interior = CSR();
      std::vector<int>().swap(op->map_int);
    }
  }
}

// ---------------------------------------------------------------------------
// serialization (flat little-endian bytes; both ends are this library)
// ---------------------------------------------------------------------------
namespace {
struct W {
  std::vector<char>& b;
  template <typename T> void pod(const T& v) {
    const char* p = (const char*)&v;
    b.insert(b.end(), p, p + sizeof(T));
  }
  template <typename T, typename Al> void vec(const std::vector<T, Al>& v) {
    pod<int64_t>((int64_t)v.size());
    const char* p = (const char*)v.data();
    b.insert(b.end(), p, p + v.size() * sizeof(T));
  }
  void csr(const CSR& m) { pod(m.nrows); pod(m.ncols); vec(m.i); vec(m.j); vec(m.a); }
  void op(const RankOp& o) { csr(o.interior); csr(o.boundary); vec(o.map_int); vec(o.map_bnd); pod(o.nrows_local); }
  void halo(const RankHalo& h) {
    pod(h.n_loc); pod(h.n_halo); vec(h.peers); vec(h.recv_cnt); vec(h.send_cnt); vec(h.send_idx); vec(h.halo_glob);
  }
};
struct Rd {
  const std::vector<char>& b;
  size_t o = 0;
  template <typename T> void pod(T& v) {
    if (o + sizeof(T) > b.size()) throw std::runtime_error("deserialize: truncated buffer");
    std::memcpy(&v, b.data() + o, sizeof(T));
    o += sizeof(T);
  }
  template <typename T, typename Al> void vec(std::vector<T, Al>& v) {
    int64_t n;
    pod(n);
    if (n < 0 || o + (size_t)n * sizeof(T) > b.size()) throw std::runtime_error("deserialize: bad length");
    v.resize(n);
    std::memcpy(v.data(), b.data() + o, n * sizeof(T));
    o += n * sizeof(T);
  }
  void csr(CSR& m) { pod(m.nrows); pod(m.ncols); vec(m.i); vec(m.j); vec(m.a); }
  void op(RankOp& x) { csr(x.interior); csr(x.boundary); vec(x.map_int); vec(x.map_bnd); pod(x.nrows_local); }
  void halo(RankHalo& h) {
    pod(h.n_loc); pod(h.n_halo); vec(h.peers); vec(h.recv_cnt); vec(h.send_cnt); vec(h.send_idx); vec(h.halo_glob);
  }
};
const int64_t kMagic = 0x48564533414d47LL;  // "HVE3AMG"
}  // namespace

void serialize(const RankHierarchy& R, std::vector<char>& buf) {
  buf.clear();
  W w{buf};
  w.pod(kMagic);
  w.pod(R.rank); w.pod(R.size); w.pod(R.prm);
  w.pod((int)R.lev.size());
  for (const RankLevel& L : R.lev) {
    w.pod(L.n_loc); w.pod(L.first); w.pod(L.n_glob);
    w.op(L.A); w.op(L.P); w.op(L.R);
    w.halo(L.hu); w.halo(L.hv);
    w.vec(L.l1); w.vec(L.cf);
    w.vec(L.cheby_ds); w.vec(L.cheby_coefs);
    w.vec(L.gs_blocks);
  }
  w.pod(R.coarse_n); w.vec(R.coarse_dense);
  w.pod(R.grid_complexity); w.pod(R.operator_complexity);
  w.vec(R.nnz_A); w.vec(R.rows);
  w.pod(R.agg_level); w.vec(R.agg_starts);
}

void deserialize(const std::vector<char>& buf, RankHierarchy& R) {
  Rd r{buf};
  int64_t magic;
  r.pod(magic);
  if (magic != kMagic) throw std::runtime_error("deserialize: bad magic");
  r.pod(R.rank); r.pod(R.size); r.pod(R.prm);
  int nl;
  r.pod(nl);
  R.lev.assign(nl, RankLevel());
  for (RankLevel& L : R.lev) {
    r.pod(L.n_loc); r.pod(L.first); r.pod(L.n_glob);
    r.op(L.A); r.op(L.P); r.op(L.R);
    r.halo(L.hu); r.halo(L.hv);
    r.vec(L.l1); r.vec(L.cf);
    r.vec(L.cheby_ds); r.vec(L.cheby_coefs);
    r.vec(L.gs_blocks);
  }
  r.pod(R.coarse_n); r.vec(R.coarse_dense);
  r.pod(R.grid_complexity); r.pod(R.operator_complexity);
  r.vec(R.nnz_A); r.vec(R.rows);
  r.pod(R.agg_level); r.vec(R.agg_starts);
}

}  // namespace hve
