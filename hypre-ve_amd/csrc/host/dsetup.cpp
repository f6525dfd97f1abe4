// Distributed BoomerAMG setup (see dsetup.hpp).
#include "dsetup.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "layout.hpp"

namespace hve {

namespace {

int owner_of(const std::vector<int>& starts, int g) {
  auto it = std::upper_bound(starts.begin(), starts.end(), g);
  return (int)(it - starts.begin()) - 1;
}

void sort_unique(std::vector<int>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

// Ghost values of a fixed list of off-rank points: who owns which, and which
// of my points each peer reads.  pull: owner values -> ghost copies; push:
// ghost-side contributions -> owners (combined by the caller's rule).
struct GhostPlan {
  int first = 0, nloc = 0;
  std::vector<int> want;                // sorted unique off-rank global indices
  std::vector<int> off;                 // size + 1: want[off[p] .. off[p+1]) owned by p
  std::vector<std::vector<int>> send;   // send[p]: my local indices p reads, in p's order

  void build(std::vector<int> w, int first_, int nloc_, const std::vector<int>& starts, HostComm& c) {
    first = first_;
    nloc = nloc_;
    sort_unique(w);
    want.swap(w);
    const int size = c.size();
    off.assign(size + 1, 0);
    for (int p = 0; p <= size; ++p)
      off[p] = (int)(std::lower_bound(want.begin(), want.end(), starts[p]) - want.begin());
    std::vector<std::vector<int>> req(size), got;
    for (int p = 0; p < size; ++p) req[p].assign(want.begin() + off[p], want.begin() + off[p + 1]);
    c.exchange(req, got);
    send.assign(size, {});
    for (int p = 0; p < size; ++p) {
      send[p].resize(got[p].size());
      for (size_t k = 0; k < got[p].size(); ++k) send[p][k] = got[p][k] - first;
    }
  }
  int find(int g) const {
    auto it = std::lower_bound(want.begin(), want.end(), g);
    return (it != want.end() && *it == g) ? (int)(it - want.begin()) : -1;
  }
  template <typename T>
  void pull(const T* owned, std::vector<T>& ghost, HostComm& c) const {
    const int size = c.size();
    std::vector<std::vector<T>> sv(size), rv;
    for (int p = 0; p < size; ++p) {
      sv[p].resize(send[p].size());
      for (size_t k = 0; k < send[p].size(); ++k) sv[p][k] = owned[send[p][k]];
    }
    c.exchange(sv, rv);
    ghost.assign(want.size(), T());
    for (int p = 0; p < size; ++p)
      for (size_t k = 0; k < rv[p].size(); ++k) ghost[off[p] + k] = rv[p][k];
  }
  template <typename T, typename F>
  void push(const std::vector<T>& ghost, T* owned, F combine, HostComm& c) const {
    const int size = c.size();
    std::vector<std::vector<T>> sv(size), rv;
    for (int p = 0; p < size; ++p) sv[p].assign(ghost.begin() + off[p], ghost.begin() + off[p + 1]);
    c.exchange(sv, rv);
    for (int p = 0; p < size; ++p)
      for (size_t k = 0; k < rv[p].size(); ++k) {
        T& o = owned[send[p][k]];
        o = combine(o, rv[p][k]);
      }
  }
};

// Rows `rows` (sorted unique, all off-rank) of the distributed matrix whose
// local rows are M (global columns), fetched from their owners; the result's
// rows follow `rows`, columns stay global.
CSR fetch_rows(const CSR& M, int first, const std::vector<int>& starts, const std::vector<int>& rows, HostComm& c) {
  const int size = c.size();
  std::vector<std::vector<int>> req(size), got;
  for (int g : rows) req[owner_of(starts, g)].push_back(g);
  c.exchange(req, got);
  std::vector<std::vector<int>> len(size), cols(size);
  std::vector<std::vector<double>> vals(size);
  for (int p = 0; p < size; ++p)
    for (int g : got[p]) {
      const int r = g - first;
      len[p].push_back(M.i[r + 1] - M.i[r]);
      cols[p].insert(cols[p].end(), M.j.begin() + M.i[r], M.j.begin() + M.i[r + 1]);
      vals[p].insert(vals[p].end(), M.a.begin() + M.i[r], M.a.begin() + M.i[r + 1]);
    }
  std::vector<std::vector<int>> rlen, rcols;
  std::vector<std::vector<double>> rvals;
  c.exchange(len, rlen);
  c.exchange(cols, rcols);
  c.exchange(vals, rvals);
  CSR G;
  G.resize_rows((int)rows.size(), M.ncols);
  int q = 0;
  for (int p = 0; p < size; ++p)
    for (int l : rlen[p]) { G.i[q + 1] = G.i[q] + l; ++q; }
  G.j.reserve(G.i[q]);
  G.a.reserve(G.i[q]);
  for (int p = 0; p < size; ++p) {
    G.j.insert(G.j.end(), rcols[p].begin(), rcols[p].end());
    G.a.insert(G.a.end(), rvals[p].begin(), rvals[p].end());
  }
  return G;
}

// Index of global point g in the universe [owned (first .. first+n) | ghosts
// (sorted)]; -1 when absent.
struct Universe {
  int first = 0, n = 0;
  std::vector<int> ghosts;  // sorted unique off-rank
  int size() const { return n + (int)ghosts.size(); }
  int loc(int g) const {
    if (g >= first && g < first + n) return g - first;
    auto it = std::lower_bound(ghosts.begin(), ghosts.end(), g);
    return (it != ghosts.end() && *it == g) ? n + (int)(it - ghosts.begin()) : -1;
  }
  int glob(int u) const { return u < n ? first + u : ghosts[u - n]; }
};

// rows of `M` (global columns) -> universe columns; absent columns throw
void map_cols(CSR& M, const Universe& U) {
  for (auto& c : M.j) {
    const int l = U.loc(c);
    if (l < 0) throw std::runtime_error("distributed setup: column outside the ghost universe");
    c = l;
  }
}

// ---------------------------------------------------------------------------
// PMIS (coarsen_type 8, cf_init 0; 9, cf_init 2), distributed as hypre runs
// it on N processes (setup.cpp coarsen_pmis with rank starts, the N-rank
// emulation pinned to the reference's np > 1 runs): the random measures from
// one stream per rank, seed 2747 + rank from the rank's first row
// (par_indepset.c:45, seq_rand 0), or the global stream for coarsen_type 9.
// ---------------------------------------------------------------------------
// cf_init 3 / 4 (the aggressive second pass of type 8 / 9, setup.cpp
// coarsen_pmis(S2, 3 | 4)): rows without strong connections become C points,
// and the first pass skips the independent-set selection; its F decisions
// read own-rank markers only (CF_marker_offd is 0 there).
// cf_init 1 (HMIS's second stage, hmis_dist): cf holds this rank's Ruge first
// pass; the random measures come from one stream per rank (seed 2747 + rank
// from the rank's first row, par_indepset.c:25 as hypre runs it on N
// processes), rows with an off-rank strong connection restart undecided
// (par_coarsen.c:2296), and the seeded first sweep reads only own-rank
// markers (CF_marker_offd is still 0 there, :2348): it runs in row order on
// each rank alone, as setup.cpp coarsen_pmis does with rank starts.
void pmis_dist(const Pattern& S, int first, int n, const std::vector<int>& starts, HostComm& comm,
               std::vector<int>& cf, int cf_init = 0) {
  const int size = comm.size(), rank = comm.rank();
  std::vector<int> mcount(n, 0);
  std::vector<std::vector<int>> contrib(size), got;
  for (int c : S.j) {
    if (c >= first && c < first + n) mcount[c - first]++;
    else contrib[owner_of(starts, c)].push_back(c);
  }
  comm.exchange(contrib, got);
  for (int p = 0; p < size; ++p)
    for (int g : got[p]) mcount[g - first]++;
  std::vector<double> measure(n);
  // par_indepset.c:45-57: seed 2747 + my_id, one hypre_Rand() per local row
  // from the rank's first row; seq_rand (CF_init 2 / 4: coarsen_type 9) seeds
  // 2747 and skips the rows of the ranks before, i.e. the global stream
  const bool seq_rand = cf_init == 2 || cf_init == 4;
  for (int r = 0; r < n; ++r) {
    measure[r] = (double)mcount[r];
    if (seq_rand) measure[r] += hypre_rand_at((int64_t)first + r, 2747);
    else measure[r] += hypre_rand_at(r, 2747 + rank);  // the rank's own stream
  }
  std::vector<int> off;
  for (int c : S.j)
    if (c < first || c >= first + n) off.push_back(c);
  GhostPlan gp;
  gp.build(off, first, n, starts, comm);
  // S entries as local (>= 0) or ghost (-1 - position) indices
  std::vector<int> sidx(S.j.size());
  for (size_t k = 0; k < S.j.size(); ++k) {
    const int c = S.j[k];
    sidx[k] = (c >= first && c < first + n) ? c - first : -1 - gp.find(c);
  }
  std::vector<int> graph, graph2;
  if (cf_init == 1) {
    // the first pass's C points keep 1, the others restart (setup.cpp coarsen_pmis)
    for (int r = 0; r < n; ++r) {
      if (cf[r] == SF_PT) {
        measure[r] = 0;
        continue;
      }
      bool offd = false;
      for (int k = S.i[r]; k < S.i[r + 1] && !offd; ++k) offd = sidx[k] < 0;
      if (cf[r] == F_PT || offd) cf[r] = 0;
      if (cf[r] == Z_PT) {
        if (measure[r] >= 1.0 || S.i[r + 1] - S.i[r] > 0) { cf[r] = 0; graph.push_back(r); }
        else cf[r] = F_PT;
      } else {
        graph.push_back(r);
      }
    }
  } else {
    cf.assign(n, 0);
    for (int r = 0; r < n; ++r) {
      if (S.i[r + 1] - S.i[r] == 0) {
        cf[r] = (cf_init == 3 || cf_init == 4) ? C_PT : SF_PT;
        measure[r] = 0;
      } else {
        graph.push_back(r);
      }
    }
  }
  std::vector<double> gmeas;
  std::vector<int> gcf, gdem;
  int iter = 0;
  while (comm.allreduce_sum((int64_t)graph.size()) > 0) {
    gp.pull(measure.data(), gmeas, comm);
    const int gs = (int)graph.size();
    const bool select = !cf_init || iter > 0;
    ++iter;
#pragma omp parallel for schedule(static)
    for (int ig = 0; ig < gs; ++ig) {
      const int i = graph[ig];
      if (select && measure[i] > 1) cf[i] = 1;
    }
    gdem.assign(gp.want.size(), 0);
#pragma omp parallel for schedule(static)
    for (int ig = 0; ig < gs; ++ig) {
      const int i = graph[ig];
      if (select && measure[i] > 1) {
        for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
          const int j = sidx[k];
          const double mj = j >= 0 ? measure[j] : gmeas[-1 - j];
          if (mj > 1) {
            if (measure[i] > mj) {
              if (j >= 0) {
#pragma omp atomic write
                cf[j] = 0;
              } else {
#pragma omp atomic write
                gdem[-1 - j] = 1;
              }
            } else if (mj > measure[i]) {
#pragma omp atomic write
              cf[i] = 0;
            }
          }
        }
      }
    }
    gp.push(gdem, cf.data(), [](int cur, int flag) { return flag ? 0 : cur; }, comm);
    gp.pull(cf.data(), gcf, comm);
    if (cf_init != 0 && iter == 1) {
      // the first sweep of a seeded / CF_init run (no selection before it):
      // row order, own-rank markers only, CF_marker_offd still 0
      // (par_coarsen.c:2348; a neighbour j < i already holds its new marker)
      for (int ig = 0; ig < gs; ++ig) {
        const int i = graph[ig];
        if (measure[i] < 1) cf[i] = F_PT;
        if (cf[i] > 0) {
          cf[i] = C_PT;
        } else {
          for (int k = S.i[i]; k < S.i[i + 1]; ++k)
            if (sidx[k] >= 0 && cf[sidx[k]] > 0) { cf[i] = F_PT; break; }
        }
      }
    } else
#pragma omp parallel for schedule(static)
    for (int ig = 0; ig < gs; ++ig) {
      const int i = graph[ig];
      if (measure[i] < 1) cf[i] = F_PT;
      if (cf[i] > 0) {
        cf[i] = C_PT;
      } else {
        for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
          const int j = sidx[k];
          int cj;
          if (j >= 0) {
#pragma omp atomic read
            cj = cf[j];
          } else {
            cj = gcf[-1 - j];
          }
          if (cj > 0) { cf[i] = F_PT; break; }
        }
      }
    }
    graph2.clear();
    for (int ig = 0; ig < gs; ++ig) {
      const int i = graph[ig];
      if (cf[i] != 0) measure[i] = 0;
      else graph2.push_back(i);
    }
    graph.swap(graph2);
  }
}

// ---------------------------------------------------------------------------
// HMIS (coarsen_type 10, hypre's default), distributed: par_coarsen.c:2774 as
// hypre runs it on N processes.  Each rank's Ruge first pass (par_coarsen.c:874)
// sees only the strong connections it owns (S_diag, local measures) with the
// empty-row test over the whole row, then PMIS seeded with those C points
// (pmis_dist cf_init 1).  setup.cpp coarsen_hmis with rank starts is the
// one-process statement of the same thing (amg_setup's coarsen_starts).
// measure_type 3: the aggressive second pass (agg_2: empty rows become C).
// ---------------------------------------------------------------------------
void hmis_dist(const Pattern& S, int first, int n, const std::vector<int>& starts, HostComm& comm, int measure_type,
               std::vector<int>& cf) {
  if (measure_type != 0 && measure_type != 3)
    throw std::runtime_error("distributed HMIS needs local measures (measure_type 0)");
  Pattern Sl;
  Sl.n = n;
  Sl.i.assign(n + 1, 0);
  std::vector<int> full(n);
  for (int i = 0; i < n; ++i) {
    full[i] = S.i[i + 1] - S.i[i];
    for (int k = S.i[i]; k < S.i[i + 1]; ++k)
      if (S.j[k] >= first && S.j[k] < first + n) Sl.j.push_back(S.j[k] - first);
    Sl.i[i + 1] = (int)Sl.j.size();
  }
  coarsen_ruge_first_pass(Sl, nullptr, measure_type, 0, cf, full.data());
  pmis_dist(S, first, n, starts, comm, cf, 1);
}

// ---------------------------------------------------------------------------
// Aggressive levels, distributed (par_amg_setup.c:1239-1285 as setup.cpp runs
// it in one process): second strength over the first pass's C points,
// PMIS on it, CorrectCFMarker, multipass interpolation.  Every row is built
// from the same global rows in the same order, so the result is the
// one-process hierarchy's rows.
// ---------------------------------------------------------------------------
Pattern fetch_pattern_rows(const Pattern& S, int first, const std::vector<int>& starts, const std::vector<int>& rows,
                           HostComm& c) {
  CSR M;
  M.resize_rows(S.n, 0);
  M.i = S.i;
  M.j.assign(S.j.begin(), S.j.end());
  M.a.assign(S.j.size(), 1.0);
  CSR G = fetch_rows(M, first, starts, rows, c);
  Pattern P;
  P.n = G.nrows;
  P.i = G.i;
  P.j.assign(G.j.begin(), G.j.end());
  return P;
}

// setup.cpp create_2nd_strength for the owned rows: S2 rows of the owned
// first-pass C points (cf > 0) in the global numbering of those points
// (c1starts); cf of an owned point whose S2 row is empty becomes 2.
void second_strength_dist(const Pattern& S, std::vector<int>& cf, int first, int n, const std::vector<int>& starts,
                          int num_paths, HostComm& comm, std::vector<int>& c1starts, Pattern& S2) {
  const int rank = comm.rank(), size = comm.size();
  int64_t nc1 = 0;
  for (int v : cf) nc1 += (v > 0);
  const auto cnt = comm.allgather(nc1);
  c1starts.assign(size + 1, 0);
  for (int p = 0; p < size; ++p) c1starts[p + 1] = c1starts[p] + (int)cnt[p];
  std::vector<int> f2c(n, -1);
  int cc = c1starts[rank];
  for (int i = 0; i < n; ++i)
    if (cf[i] > 0) f2c[i] = cc++;
  // G1: off-rank strong neighbours (their S rows are read); G2: theirs
  std::vector<int> g1;
  for (int c : S.j)
    if (c < first || c >= first + n) g1.push_back(c);
  sort_unique(g1);
  const Pattern SG1 = fetch_pattern_rows(S, first, starts, g1, comm);
  std::vector<int> gh = g1;
  for (int c : SG1.j)
    if (c < first || c >= first + n) gh.push_back(c);
  sort_unique(gh);
  GhostPlan gp;
  gp.build(gh, first, n, starts, comm);
  std::vector<int> gcf, gf2c;
  gp.pull(cf.data(), gcf, comm);
  gp.pull(f2c.data(), gf2c, comm);
  auto cf_of = [&](int g) { return (g >= first && g < first + n) ? cf[g - first] : gcf[gp.find(g)]; };
  auto f2c_of = [&](int g) { return (g >= first && g < first + n) ? f2c[g - first] : gf2c[gp.find(g)]; };
  auto srow = [&](int g, const int*& b, const int*& e) {
    if (g >= first && g < first + n) {
      b = S.j.data() + S.i[g - first];
      e = S.j.data() + S.i[g - first + 1];
    } else {
      const int k = (int)(std::lower_bound(g1.begin(), g1.end(), g) - g1.begin());
      b = SG1.j.data() + SG1.i[k];
      e = SG1.j.data() + SG1.i[k + 1];
    }
  };
  const int nc_loc = (int)nc1;
  S2.n = nc_loc;
  S2.i.assign(nc_loc + 1, 0);
  S2.j.clear();
  std::vector<int> touch, count, mark_pos;
  std::vector<int> marker_keys;  // global C-space index -> position in touch (small per row)
  int ic = 0;
  for (int i = 0; i < n; ++i) {
    if (cf[i] <= 0) continue;
    const int myc = f2c[i];
    touch.clear();
    count.clear();
    auto add = [&](int index, int w) {
      for (size_t t = 0; t < touch.size(); ++t)
        if (touch[t] == index) { count[t] += w; return; }
      touch.push_back(index);
      count.push_back(w);
    };
    for (int k1 = S.i[i]; k1 < S.i[i + 1]; ++k1) {
      const int i2 = S.j[k1];
      if (cf_of(i2) > 0) add(f2c_of(i2), 2);
      const int *b, *e;
      srow(i2, b, e);
      for (const int* q = b; q < e; ++q) {
        const int i3 = *q;
        if (cf_of(i3) > 0 && f2c_of(i3) != myc) add(f2c_of(i3), 1);
      }
    }
    int kept = 0;
    for (size_t t = 0; t < touch.size(); ++t)
      if (count[t] >= num_paths) {
        S2.j.push_back(touch[t]);
        ++kept;
      }
    S2.i[ic + 1] = S2.i[ic] + kept;
    if (kept == 0) cf[i] = 2;
    ++ic;
  }
}

// setup.cpp build_multipass_interp for the owned rows (global coarse columns
// from cstarts).  Passes are global (every rank runs the same count); a pass
// reads the assignment of ghost neighbours and, for its weights, the P rows of
// the ghost neighbours of the previous pass.  A row whose sum_C * a_ii is 0
// would reuse the previous row's weight factor in the reference's sequential
// loop; that has no distributed counterpart and is refused.
void multipass_dist(const CSR& A, const Pattern& S, const std::vector<int>& cf, int first, int n,
                    const std::vector<int>& starts, const std::vector<int>& cstarts, double trunc_factor,
                    int max_elmts, HostComm& comm, CSR& P) {
  const int rank = comm.rank();
  constexpr int max_num_passes = 10;
  std::vector<int> f2c(n, -1);
  int cc = cstarts[rank];
  for (int i = 0; i < n; ++i)
    if (cf[i] == 1) f2c[i] = cc++;
  std::vector<int> g1;
  for (int c : A.j)
    if (c < first || c >= first + n) g1.push_back(c);
  sort_unique(g1);
  GhostPlan gp;
  gp.build(g1, first, n, starts, comm);
  std::vector<int> gcf, gf2c, gassigned;
  gp.pull(cf.data(), gcf, comm);
  gp.pull(f2c.data(), gf2c, comm);
  auto gidx = [&](int g) { return gp.find(g); };
  auto cf_of = [&](int g) { return (g >= first && g < first + n) ? cf[g - first] : gcf[gidx(g)]; };
  auto f2c_of = [&](int g) { return (g >= first && g < first + n) ? f2c[g - first] : gf2c[gidx(g)]; };
  std::vector<int> assigned(n, -1);
  std::vector<std::vector<int>> rows_of_pass(max_num_passes + 1);
  for (int i = 0; i < n; ++i)
    if (cf[i] == 1) assigned[i] = 0;
  // pass 1: F points with a strong C neighbour
  for (int i = 0; i < n; ++i) {
    if (cf[i] != -1) continue;
    for (int k = S.i[i]; k < S.i[i + 1]; ++k)
      if (cf_of(S.j[k]) == 1) { assigned[i] = 1; break; }
    if (assigned[i] == 1) rows_of_pass[1].push_back(i);
  }
  auto unassigned = [&]() {
    int64_t u = 0;
    for (int i = 0; i < n; ++i) u += (cf[i] == -1 && assigned[i] < 0);
    return u;
  };
  int pass = 2;
  while (comm.allreduce_sum(unassigned()) > 0 && pass < max_num_passes) {
    gp.pull(assigned.data(), gassigned, comm);
    auto asg_of = [&](int g) { return (g >= first && g < first + n) ? assigned[g - first] : gassigned[gidx(g)]; };
    std::vector<int> now;
    for (int i = 0; i < n; ++i) {
      if (cf[i] != -1 || assigned[i] >= 0) continue;
      for (int k = S.i[i]; k < S.i[i + 1]; ++k)
        if (asg_of(S.j[k]) == pass - 1) { now.push_back(i); break; }
    }
    for (int i : now) assigned[i] = pass;
    rows_of_pass[pass].swap(now);
    ++pass;
  }
  const int num_passes = pass;
  gp.pull(assigned.data(), gassigned, comm);
  auto asg_of = [&](int g) { return (g >= first && g < first + n) ? assigned[g - first] : gassigned[gidx(g)]; };
  // rows: C points (the point itself), then pass by pass
  std::vector<std::vector<int>> pj(n);
  std::vector<std::vector<double>> pa(n);
  for (int i = 0; i < n; ++i)
    if (cf[i] == 1) { pj[i] = {f2c[i]}; pa[i] = {1.0}; }
  auto refuse = []() {
    throw std::runtime_error("distributed multipass: a row with sum_C * a_ii == 0 (sequential weight reuse)");
  };
  // pass 1: direct weights from the strong C neighbours, in A-row order
  for (int i : rows_of_pass[1]) {
    std::vector<int> strong;
    for (int k = S.i[i]; k < S.i[i + 1]; ++k)
      if (cf_of(S.j[k]) == 1) strong.push_back(S.j[k]);
    double sum_C = 0, sum_N = 0;
    for (int k = A.i[i] + 1; k < A.i[i + 1]; ++k) {
      const int j1 = A.j[k];
      if (cf_of(j1) != -3) sum_N += A.a[k];
      if (std::find(strong.begin(), strong.end(), j1) != strong.end()) {
        pa[i].push_back(A.a[k]);
        pj[i].push_back(f2c_of(j1));
        sum_C += A.a[k];
      }
    }
    const double diagonal = A.a[A.i[i]];
    if (!(sum_C * diagonal != 0)) refuse();
    const double alfa = -sum_N / (sum_C * diagonal);
    for (double& v : pa[i]) v *= alfa;
  }
  // passes >= 2: through the P rows of the previous pass (ghost rows fetched)
  for (pass = 2; pass < num_passes; ++pass) {
    // P rows of the previous pass, owned -> CSR with global columns, ghosts fetched
    std::vector<int> want;
    for (int i : rows_of_pass[pass]) {
      for (int k = S.i[i]; k < S.i[i + 1]; ++k) {
        const int j = S.j[k];
        if ((j < first || j >= first + n) && asg_of(j) == pass - 1) want.push_back(j);
      }
    }
    sort_unique(want);
    CSR Pown;
    Pown.resize_rows(n, 0);
    for (int i = 0; i < n; ++i) Pown.i[i + 1] = Pown.i[i] + (assigned[i] == pass - 1 ? (int)pj[i].size() : 0);
    for (int i = 0; i < n; ++i)
      if (assigned[i] == pass - 1) {
        Pown.j.insert(Pown.j.end(), pj[i].begin(), pj[i].end());
        Pown.a.insert(Pown.a.end(), pa[i].begin(), pa[i].end());
      }
    const CSR PG = fetch_rows(Pown, first, starts, want, comm);
    auto prow = [&](int g, const int*& cb, const double*& ab, int& len) {
      if (g >= first && g < first + n) {
        cb = pj[g - first].data();
        ab = pa[g - first].data();
        len = (int)pj[g - first].size();
      } else {
        const int k = (int)(std::lower_bound(want.begin(), want.end(), g) - want.begin());
        cb = PG.j.data() + PG.i[k];
        ab = PG.a.data() + PG.i[k];
        len = PG.i[k + 1] - PG.i[k];
      }
    };
    for (int i : rows_of_pass[pass]) {
      std::vector<int>& cols = pj[i];
      std::vector<double>& vals = pa[i];
      // columns: the previous-pass rows of the strong neighbours, first touch
      std::vector<int> nb;
      for (int k = S.i[i]; k < S.i[i + 1]; ++k)
        if (asg_of(S.j[k]) == pass - 1) nb.push_back(S.j[k]);
      for (int j1 : nb) {
        const int* cb;
        const double* ab;
        int len;
        prow(j1, cb, ab, len);
        for (int q = 0; q < len; ++q)
          if (std::find(cols.begin(), cols.end(), cb[q]) == cols.end()) cols.push_back(cb[q]);
      }
      vals.assign(cols.size(), 0.0);
      double sum_C = 0, sum_N = 0;
      for (int k = A.i[i] + 1; k < A.i[i + 1]; ++k) {
        const int j1 = A.j[k];
        if (std::find(nb.begin(), nb.end(), j1) != nb.end()) {
          const int* cb;
          const double* ab;
          int len;
          prow(j1, cb, ab, len);
          for (int q = 0; q < len; ++q) {
            const double alfa = A.a[k] * ab[q];
            const size_t pos = std::find(cols.begin(), cols.end(), cb[q]) - cols.begin();
            vals[pos] += alfa;
            sum_C += alfa;
            sum_N += alfa;
          }
        } else if (cf_of(j1) != -3) {
          sum_N += A.a[k];
        }
      }
      const double diagonal = A.a[A.i[i]];
      if (!(sum_C * diagonal != 0)) refuse();
      const double alfa = -sum_N / (sum_C * diagonal);
      for (double& v : vals) v *= alfa;
    }
  }
  P.resize_rows(n, cstarts.back());
  for (int i = 0; i < n; ++i) P.i[i + 1] = P.i[i] + (int)pj[i].size();
  P.j.reserve(P.i[n]);
  P.a.reserve(P.i[n]);
  for (int i = 0; i < n; ++i) {
    P.j.insert(P.j.end(), pj[i].begin(), pj[i].end());
    P.a.insert(P.a.end(), pa[i].begin(), pa[i].end());
  }
  if (trunc_factor != 0.0 || max_elmts != 0) truncate_rows(P, trunc_factor, max_elmts);
}

// ---------------------------------------------------------------------------
// A rank's ghost universe for the interpolations: its owned points, their
// off-rank neighbours G1 (A rows fetched, S rows recomputed from them:
// strength is row-local) and the points the G1 rows reach (G2: markers
// only).  The rows of owned and G1 points are complete, so a row function of
// an owned point, and of a G1 point it reads, sees exactly what it sees in
// one process (ext+i, ext, and the matrix-matrix forms 16-18 / 2-stage).
// ---------------------------------------------------------------------------
struct GhostUniverse {
  Universe U;
  CSR A;      // universe rows (G2-only points empty), universe columns
  Pattern S;
  GhostPlan gp;  // owned values -> the ghost part (gp.want == U.ghosts)
  // owned values followed by the pulled ghost values: universe-indexed
  std::vector<int> extend(const std::vector<int>& owned, HostComm& c) const {
    std::vector<int> g, out(owned);
    gp.pull(owned.data(), g, c);
    out.insert(out.end(), g.begin(), g.end());
    return out;
  }
};

// diag_rows: G2-only points get a row holding a unit diagonal (the
// whole-matrix builders read every F row's diagonal; no owned row reads them).
void build_ghost_universe(const CSR& A, const Pattern& S, int first, int n, const std::vector<int>& starts,
                          double strong_threshold, double max_row_sum, HostComm& comm, GhostUniverse& G,
                          bool diag_rows = false) {
  std::vector<int> g1;
  for (int c : A.j)
    if (c < first || c >= first + n) g1.push_back(c);
  sort_unique(g1);
  CSR AG1 = fetch_rows(A, first, starts, g1, comm);
  Pattern SG1;
  create_strength(AG1, strong_threshold, max_row_sum, SG1);
  std::vector<int> gh = g1;
  for (int c : AG1.j)
    if (c < first || c >= first + n) gh.push_back(c);
  sort_unique(gh);
  G.U.first = first;
  G.U.n = n;
  G.U.ghosts = gh;
  G.gp.build(gh, first, n, starts, comm);
  const int nU = G.U.size();
  CSR& AU = G.A;
  Pattern& SU = G.S;
  AU.resize_rows(nU, nU);
  SU.n = nU;
  SU.i.assign(nU + 1, 0);
  std::vector<int> g1pos(g1.size());
  for (size_t k = 0; k < g1.size(); ++k) g1pos[k] = G.U.loc(g1[k]);
  std::vector<int> rowlenA(nU, diag_rows ? 1 : 0), rowlenS(nU, 0);
  for (int i = 0; i < n; ++i) { rowlenA[i] = A.i[i + 1] - A.i[i]; rowlenS[i] = S.i[i + 1] - S.i[i]; }
  for (size_t k = 0; k < g1.size(); ++k) {
    rowlenA[g1pos[k]] = AG1.i[k + 1] - AG1.i[k];
    rowlenS[g1pos[k]] = SG1.i[k + 1] - SG1.i[k];
  }
  for (int u = 0; u < nU; ++u) { AU.i[u + 1] = AU.i[u] + rowlenA[u]; SU.i[u + 1] = SU.i[u] + rowlenS[u]; }
  AU.j.resize(AU.i[nU]);
  AU.a.resize(AU.i[nU]);
  SU.j.resize(SU.i[nU]);
  for (int i = 0; i < n; ++i) {
    std::copy(A.j.begin() + A.i[i], A.j.begin() + A.i[i + 1], AU.j.begin() + AU.i[i]);
    std::copy(A.a.begin() + A.i[i], A.a.begin() + A.i[i + 1], AU.a.begin() + AU.i[i]);
    std::copy(S.j.begin() + S.i[i], S.j.begin() + S.i[i + 1], SU.j.begin() + SU.i[i]);
  }
  std::vector<char> filled(nU, 0);
  for (size_t k = 0; k < g1.size(); ++k) {
    const int u = g1pos[k];
    filled[u] = 1;
    std::copy(AG1.j.begin() + AG1.i[k], AG1.j.begin() + AG1.i[k + 1], AU.j.begin() + AU.i[u]);
    std::copy(AG1.a.begin() + AG1.i[k], AG1.a.begin() + AG1.i[k + 1], AU.a.begin() + AU.i[u]);
    std::copy(SG1.j.begin() + SG1.i[k], SG1.j.begin() + SG1.i[k + 1], SU.j.begin() + SU.i[u]);
  }
  if (diag_rows)
    for (int u = n; u < nU; ++u)
      if (!filled[u]) { AU.j[AU.i[u]] = G.U.glob(u); AU.a[AU.i[u]] = 1.0; }
  map_cols(AU, G.U);
  for (auto& c : SU.j) {
    const int l = G.U.loc(c);
    if (l < 0) throw std::runtime_error("distributed setup: strength column outside the ghost universe");
    c = l;
  }
}

// ---------------------------------------------------------------------------
// Ext+i (plus_i) or ext (interp_type 14, par_lr_interp.c:4686) rows of the
// owned fine points (extpi_core over the ghost universe).
// ---------------------------------------------------------------------------
void extpi_dist(const CSR& A, const Pattern& S, const std::vector<int>& cf, int first, int n,
                const std::vector<int>& starts, const std::vector<int>& cstarts, double strong_threshold,
                double max_row_sum, HostComm& comm, CSR& P, bool plus_i) {
  const int rank = comm.rank(), size = comm.size();
  std::vector<int> f2c(n, -1);
  int cc = cstarts[rank];
  for (int i = 0; i < n; ++i)
    if (cf[i] >= 0) f2c[i] = cc++;
  GhostUniverse G;
  build_ghost_universe(A, S, first, n, starts, strong_threshold, max_row_sum, comm, G);
  const std::vector<int> cfU = G.extend(cf, comm), f2cU = G.extend(f2c, comm);
  extpi_core(G.A, G.S, cfU, f2cU, n, (int)cstarts[size], G.U.size(), P, plus_i);
}

// ---------------------------------------------------------------------------
// R = P^T rows of the owned coarse points: every P entry goes to the owner of
// its coarse column; rows list fine indices ascending (csr_matop.c:578).
// ---------------------------------------------------------------------------
void transpose_dist(const CSR& P, int first, int nfine_glob, const std::vector<int>& cstarts, HostComm& comm,
                    CSR& R) {
  const int rank = comm.rank(), size = comm.size();
  std::vector<std::vector<int>> sic(size), sfi(size), ric, rfi;
  std::vector<std::vector<double>> sva(size), rva;
  for (int i = 0; i < P.nrows; ++i)
    for (int k = P.i[i]; k < P.i[i + 1]; ++k) {
      const int q = owner_of(cstarts, P.j[k]);
      sic[q].push_back(P.j[k]);
      sfi[q].push_back(first + i);
      sva[q].push_back(P.a[k]);
    }
  comm.exchange(sic, ric);
  comm.exchange(sfi, rfi);
  comm.exchange(sva, rva);
  const int c0 = cstarts[rank], nc = cstarts[rank + 1] - c0;
  R.resize_rows(nc, nfine_glob);
  for (int p = 0; p < size; ++p)
    for (int ic : ric[p]) R.i[ic - c0 + 1]++;
  for (int r = 0; r < nc; ++r) R.i[r + 1] += R.i[r];
  R.j.resize(R.i[nc]);
  R.a.resize(R.i[nc]);
  std::vector<int> pos(R.i.begin(), R.i.end() - 1);
  // senders in rank order hold ascending fine rows, each in row order
  for (int p = 0; p < size; ++p)
    for (size_t k = 0; k < ric[p].size(); ++k) {
      const int r = ric[p][k] - c0;
      R.j[pos[r]] = rfi[p][k];
      R.a[pos[r]] = rva[p][k];
      pos[r]++;
    }
}

// ---------------------------------------------------------------------------
// Coarse operator rows of the owned coarse points (rap_core).
// ---------------------------------------------------------------------------
void rap_dist(const CSR& R, const CSR& A, const CSR& P, int first, const std::vector<int>& starts,
              const std::vector<int>& cstarts, HostComm& comm, CSR& Ac) {
  const int rank = comm.rank(), size = comm.size();
  const int n = A.nrows;
  // F1: off-rank fine rows R reads (their A rows are needed)
  std::vector<int> f1;
  for (int c : R.j)
    if (c < first || c >= first + n) f1.push_back(c);
  sort_unique(f1);
  CSR AF1 = fetch_rows(A, first, starts, f1, comm);
  // F2: off-rank columns of the A rows of owned and F1 points (their P rows)
  std::vector<int> f2;
  for (int c : A.j)
    if (c < first || c >= first + n) f2.push_back(c);
  for (int c : AF1.j)
    if (c < first || c >= first + n) f2.push_back(c);
  sort_unique(f2);
  CSR PF2 = fetch_rows(P, first, starts, f2, comm);
  Universe UF;
  UF.first = first;
  UF.n = n;
  UF.ghosts = f1;
  UF.ghosts.insert(UF.ghosts.end(), f2.begin(), f2.end());
  sort_unique(UF.ghosts);
  const int nUF = UF.size();
  // coarse universe: owned coarse points, then the off-rank ones P rows reach
  Universe UC;
  UC.first = cstarts[rank];
  UC.n = cstarts[rank + 1] - cstarts[rank];
  for (int c : P.j)
    if (c < UC.first || c >= UC.first + UC.n) UC.ghosts.push_back(c);
  for (int c : PF2.j)
    if (c < UC.first || c >= UC.first + UC.n) UC.ghosts.push_back(c);
  sort_unique(UC.ghosts);
  const int nUC = UC.size();
  std::vector<int> coarse_glob(nUC);
  for (int u = 0; u < nUC; ++u) coarse_glob[u] = UC.glob(u);
  // fine-universe A (owned + F1 rows) and P (owned + F2 rows)
  auto assemble = [&](const CSR& own, const CSR& ghost, const std::vector<int>& grows, CSR& out) {
    out.resize_rows(nUF, own.ncols);
    std::vector<int> gpos(grows.size());
    std::vector<int> len(nUF, 0);
    for (int i = 0; i < n; ++i) len[i] = own.i[i + 1] - own.i[i];
    for (size_t k = 0; k < grows.size(); ++k) {
      gpos[k] = UF.loc(grows[k]);
      len[gpos[k]] = ghost.i[k + 1] - ghost.i[k];
    }
    for (int u = 0; u < nUF; ++u) out.i[u + 1] = out.i[u] + len[u];
    out.j.resize(out.i[nUF]);
    out.a.resize(out.i[nUF]);
    for (int i = 0; i < n; ++i) {
      std::copy(own.j.begin() + own.i[i], own.j.begin() + own.i[i + 1], out.j.begin() + out.i[i]);
      std::copy(own.a.begin() + own.i[i], own.a.begin() + own.i[i + 1], out.a.begin() + out.i[i]);
    }
    for (size_t k = 0; k < grows.size(); ++k) {
      std::copy(ghost.j.begin() + ghost.i[k], ghost.j.begin() + ghost.i[k + 1], out.j.begin() + out.i[gpos[k]]);
      std::copy(ghost.a.begin() + ghost.i[k], ghost.a.begin() + ghost.i[k + 1], out.a.begin() + out.i[gpos[k]]);
    }
  };
  CSR AU, PU;
  assemble(A, AF1, f1, AU);
  assemble(P, PF2, f2, PU);
  // A rows of F2-only points are empty; their columns never get visited.
  map_cols(AU, UF);
  for (auto& c : PU.j) {
    const int l = UC.loc(c);
    if (l < 0) throw std::runtime_error("distributed setup: coarse column outside the ghost universe");
    c = l;
  }
  CSR RU = R;
  map_cols(RU, UF);
  std::vector<int> row_ic(R.nrows);
  for (int q = 0; q < R.nrows; ++q) row_ic[q] = q;
  rap_core(RU, AU, PU, row_ic, coarse_glob, nUF, nUC, cstarts[size], Ac);
}

// l1 norms of the owned rows (setup.cpp compute_l1_norms with global indices).
// Option 4's blocks are num_blocks blocks of this rank's rows (hypre's
// threads per process; partition.cpp rank_gs_blocks): columns of other ranks
// are off-block.
void l1_dist(const CSR& A, int first, int nglob, int option, const std::vector<int>* cf, const GhostPlan* gp,
             const std::vector<int>* gcf, int num_blocks, std::vector<double>& l1) {
  (void)nglob;
  const int n = A.nrows;
  l1.assign(n, 0.0);
  const std::vector<int> bs = hypre_block_starts(n, std::max(1, num_blocks));
  auto cf_of = [&](int c) -> int {
    if (c >= first && c < first + n) return (*cf)[c - first];
    return (*gcf)[gp->find(c)];
  };
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    const int gi = first + i;
    const int k = (int)(std::upper_bound(bs.begin(), bs.end(), i) - bs.begin()) - 1;
    const int ns = first + bs[k], ne = first + bs[k + 1];
    double s = 0.0;
    if (option == 1) {
      for (int q = A.i[i]; q < A.i[i + 1]; ++q)
        if (!cf || (*cf)[i] == cf_of(A.j[q])) s += std::fabs(A.a[q]);
    } else if (option == 4) {
      double diag = 0.0;
      for (int q = A.i[i]; q < A.i[i + 1]; ++q) {
        const int c = A.j[q];
        if ((c == gi || c < ns || c >= ne) && (!cf || (*cf)[i] == cf_of(c))) {
          if (c == gi) { diag = std::fabs(A.a[q]); s += std::fabs(A.a[q]); }
          else s += 0.5 * std::fabs(A.a[q]);
        }
      }
      if (s <= 4.0 / 3.0 * diag) s = diag;
    }
    l1[i] = s;
  }
  for (int i = 0; i < n; ++i)
    if (A.a[A.i[i]] < 0.0) l1[i] = -l1[i];
}

// ---------------------------------------------------------------------------
// Chebyshev smoother data (relax 16), distributed as the N-rank emulation
// (setup.cpp max_eig_estimate_cg with rank starts) states it:
// par_relax_more.c:115 hypre_ParCSRMaxEigEstimateCG's start vector takes each
// rank's own random stream (seed my_id + 1, par_vector.c:337), the matvec
// reads the ghost values of its vector, and every inner product is formed as
// that loop forms it: a running sum handed from rank to rank in rank order,
// each rank adding its rows to it.  The Lanczos tridiagonal, its eigenvalues
// and the coefficients (par_cheby.c:36) are then the emulation's bit for bit.
// par_relax_more.c:25's inf-norm bound is a max over rows.
// ---------------------------------------------------------------------------
double chain_dot(const std::vector<double>& x, const std::vector<double>& y, HostComm& comm) {
  const int size = comm.size(), rank = comm.rank();
  double s = 0.0;
  for (int q = 0; q < size; ++q) {
    int64_t bits = 0;
    if (rank == q) {
      for (size_t i = 0; i < x.size(); ++i) s += y[i] * x[i];  // hypre_SeqVectorInnerProd: y_i * x_i
      std::memcpy(&bits, &s, sizeof bits);
    }
    const auto all = comm.allgather(bits);
    std::memcpy(&s, &all[q], sizeof s);
  }
  return s;
}

void max_eig_cg_dist(const CSR& A, int first, int n, const std::vector<int>& starts, int scale, int max_iter,
                     HostComm& comm, double* max_eig, double* min_eig) {
  const int nglob = starts.back();
  if (nglob < max_iter) max_iter = nglob;
  std::vector<int> off;
  for (int c : A.j)
    if (c < first || c >= first + n) off.push_back(c);
  GhostPlan gp;
  gp.build(off, first, n, starts, comm);
  std::vector<int> lc(A.j.size());
  for (size_t k = 0; k < A.j.size(); ++k) {
    const int c = A.j[k];
    lc[k] = (c >= first && c < first + n) ? c - first : n + gp.find(c);
  }
  std::vector<double> r(n), p(n, 0.0), s(n, 0.0), ds(n), u(n, 0.0), xg, xfull;
  std::vector<double> tridiag(max_iter + 1, 0.0), trioffd(max_iter + 1, 0.0);
  // hypre_ParVectorSetRandomValues(r, 1) (par_vector.c:337): seed 1 * (my_id + 1),
  // every rank from its own first row
  for (int i = 0; i < n; ++i) r[i] = 2.0 * hypre_rand_at(i, comm.rank() + 1) - 1.0;
  for (int i = 0; i < n; ++i) ds[i] = scale ? 1 / std::sqrt(A.a[A.i[i]]) : 1.0;
  auto matvec = [&](const std::vector<double>& x, std::vector<double>& y) {
    gp.pull(x.data(), xg, comm);
    xfull = x;
    xfull.insert(xfull.end(), xg.begin(), xg.end());
    for (int row = 0; row < n; ++row) {
      double t = 0.0;
      for (int k = A.i[row]; k < A.i[row + 1]; ++k) t += A.a[k] * xfull[lc[k]];
      y[row] = t;
    }
  };
  double gamma = chain_dot(r, p, comm), gamma_old, beta = 1.0, alpha, alphainv;
  int i = 0;
  while (i < max_iter) {
    s = r;
    gamma_old = gamma;
    gamma = chain_dot(r, s, comm);
    if (i == 0) {
      beta = 1.0;
      p = s;
    } else {
      beta = gamma / gamma_old;
      for (int k = 0; k < n; ++k) p[k] = s[k] + beta * p[k];
    }
    if (scale) {
      for (int k = 0; k < n; ++k) u[k] = ds[k] * p[k];
      matvec(u, s);
      for (int k = 0; k < n; ++k) s[k] = ds[k] * s[k];
    } else {
      matvec(p, s);
    }
    const double sdotp = chain_dot(s, p, comm);
    alpha = gamma / sdotp;
    alphainv = 1.0 / alpha;
    tridiag[i + 1] = alphainv;
    tridiag[i] *= beta;
    tridiag[i] += alphainv;
    trioffd[i + 1] = alphainv;
    trioffd[i] *= std::sqrt(beta);
    for (int k = 0; k < n; ++k) r[k] += (-alpha) * s[k];
    i++;
  }
  linpack_tql1(i, tridiag.data(), trioffd.data());
  *max_eig = tridiag[i - 1];
  *min_eig = tridiag[0];
}

void max_eig_norm_dist(const CSR& A, int scale, HostComm& comm, double* max_eig) {
  double max_norm = 0.0;
  int64_t pos_diag = 0, neg_diag = 0;
  for (int i = 0; i < A.nrows; ++i) {
    double diag_value = A.a[A.i[i]];
    if (diag_value > 0) pos_diag++;
    if (diag_value < 0) { neg_diag++; diag_value = -diag_value; }
    double row_sum = diag_value;
    for (int j = A.i[i] + 1; j < A.i[i + 1]; ++j) row_sum += std::fabs(A.a[j]);
    if (scale && diag_value != 0.0) row_sum = row_sum / diag_value;
    if (row_sum > max_norm) max_norm = row_sum;
  }
  int64_t bits;
  std::memcpy(&bits, &max_norm, sizeof bits);
  double m = 0.0;
  for (int64_t b : comm.allgather(bits)) {
    double v;
    std::memcpy(&v, &b, sizeof v);
    if (v > m) m = v;
  }
  pos_diag = comm.allreduce_sum(pos_diag);
  neg_diag = comm.allreduce_sum(neg_diag);
  if (pos_diag == 0 && neg_diag > 0) m = -m;
  *max_eig = m;
}

bool uses_l1_gs(int t) { return t == 8 || t == 13 || t == 14; }
bool uses_hybrid_gs_any(const AMGParams& prm) {
  for (int c = 0; c < 4; ++c) {
    const int t = prm.relax_type[c];
    if (t == 3 || t == 4 || t == 6 || uses_l1_gs(t)) return true;
  }
  return false;
}

struct DLevel {
  CSR A, P, R;  // owned rows, global columns
  std::vector<int> cf;
  std::vector<double> l1;
  std::vector<double> cheby_ds, cheby_coefs;  // relax 16 (owned rows; coefficients replicated)
  std::vector<int> starts;  // row starts of this level over the ranks
  int first = 0, nloc = 0, nglob = 0;
  int64_t nnz_glob = 0;
};

// Halo of a vector owned in `starts` with the given off-rank reads: the
// RankHalo partition_all builds (peers ascending, per-peer counts, the local
// indices each peer reads).
RankHalo make_halo(const std::vector<int>& halo, int first, int nloc, const std::vector<int>& starts, HostComm& comm) {
  const int rank = comm.rank(), size = comm.size();
  RankHalo h;
  h.n_loc = nloc;
  h.n_halo = (int)halo.size();
  h.halo_glob = halo;
  std::vector<std::vector<int>> req(size), got;
  for (int g : halo) req[owner_of(starts, g)].push_back(g);
  comm.exchange(req, got);
  for (int p = 0; p < size; ++p) {
    if (p == rank) continue;
    const int rc = (int)req[p].size(), sc = (int)got[p].size();
    if (rc == 0 && sc == 0) continue;
    h.peers.push_back(p);
    h.recv_cnt.push_back(rc);
    h.send_cnt.push_back(sc);
    for (int g : got[p]) h.send_idx.push_back(g - first);
  }
  return h;
}

// Rows of a rank in hypre's ParCSR order (diag, then offd, each in its own
// entry order): a stable partition of every row by whether its column lies in
// the rank's own column range [c0, c1) (setup.cpp rank_order_rows for one rank).
void rank_order_local(CSR& M, int c0, int c1) {
#pragma omp parallel
  {
    std::vector<int> tj;
    std::vector<double> ta;
#pragma omp for schedule(static)
    for (int r = 0; r < M.nrows; ++r) {
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

void offrank_cols(const CSR& M, int a, int b, std::vector<int>& out) {
  for (int c : M.j)
    if (c < a || c >= b) out.push_back(c);
}

}  // namespace

bool dist_setup_supported(const AMGParams& prm, std::string* why) {
  auto no = [&](const char* w) { if (why) *why = w; return false; };
  if (prm.coarsen_type != 8 && prm.coarsen_type != 9 && prm.coarsen_type != 10)
    return no("coarsen_type not 8 / 9 (PMIS) or 10 (HMIS)");
  if (prm.coarsen_type == 10 && (prm.measure_type != 0 || prm.coarsen_cut_factor != 0))
    return no("HMIS with global measures or a cut factor");
  if (prm.interp_type != 6 && prm.interp_type != 14)
    return no("interp_type not 6 or 14 (the matrix-matrix forms follow hypre_ParMatmul's N-rank order: "
              "set up on rank 0 under the rank emulation)");
  if (prm.agg_num_levels > 0 && prm.agg_interp_type != 4)
    return no("aggressive coarsening with agg_interp_type not 4 (the 2-stage forms are set up on rank 0 under "
              "the rank emulation)");
  if (prm.num_functions > 1) return no("num_functions > 1 (systems AMG is set up in one process)");
  if (prm.seq_threshold > 0) return no("seq_threshold (the redundant coarse-grid AMG is set up in one process)");
  for (int j = 0; j < std::min(prm.max_levels, (int)AMGParams::kWeightLevels); ++j)
    if (prm.wt(j) == 0.0) return no("relax weight 0 (the scaled-norm weight of the one-process setup)");
  return true;
}

int amg_setup_dist(const CSR& A0, int first_row, const AMGParams& prm_in, HostComm& comm, RankHierarchy& out,
                   std::string* log) {
  if (!dist_setup_supported(prm_in)) return 1;
  const int rank = comm.rank(), size = comm.size();
  AMGParams prm = prm_in;
  std::vector<DLevel> L(1);
  L[0].A = A0;
  {
    auto cnt = comm.allgather(A0.nrows);
    L[0].starts.assign(size + 1, 0);
    for (int p = 0; p < size; ++p) L[0].starts[p + 1] = L[0].starts[p] + (int)cnt[p];
    if (L[0].starts[rank] != first_row) throw std::runtime_error("distributed setup: row blocks out of rank order");
    L[0].first = first_row;
    L[0].nloc = A0.nrows;
    L[0].nglob = L[0].starts[size];
  }
  // hypre's ParCSR rows: the diagonal block's entries, then the off-diagonal
  // block's (every operator of the hierarchy keeps that order: the input here,
  // P around its truncation and every Galerkin product below)
  rank_order_local(L[0].A, L[0].starts[rank], L[0].starts[rank + 1]);
  int level = 0;
  bool finished = prm.max_levels <= 1;
  char buf[256];
  while (!finished) {
    const int n = L[level].nloc, first = L[level].first, fine_size = L[level].nglob;
    Pattern S;
    create_strength(L[level].A, prm.strong_threshold, prm.max_row_sum, S);
    std::vector<int> cf;
    if (prm.coarsen_type == 10) hmis_dist(S, first, n, L[level].starts, comm, prm.measure_type, cf);
    else pmis_dist(S, first, n, L[level].starts, comm, cf, prm.coarsen_type == 9 ? 2 : 0);
    // aggressive level: PMIS again on S*S + 2S of the C points, and the second
    // marker refines the first (setup.cpp amg_setup, par_amg_setup.c:1239)
    const bool agg_lvl = level < prm.agg_num_levels;
    std::vector<int> c1starts, cf1;
    if (agg_lvl) {
      Pattern S2;
      std::vector<int> cfn;
      second_strength_dist(S, cf, first, n, L[level].starts, prm.num_paths, comm, c1starts, S2);
      if (prm.coarsen_type == 10) hmis_dist(S2, c1starts[rank], S2.n, c1starts, comm, prm.measure_type + 3, cfn);
      else pmis_dist(S2, c1starts[rank], S2.n, c1starts, comm, cfn, prm.coarsen_type == 9 ? 4 : 3);
      if (prm.agg_interp_type == 4) {
        correct_cf_marker(cf, cfn);
      } else {
        cf1 = cf;  // the first stage's markers, for P1
        correct_cf_marker2(cf, cfn);
      }
    }
    int64_t nc_loc = 0;
    for (int v : cf) nc_loc += (v == C_PT);
    const auto ncs = comm.allgather(nc_loc);
    int64_t coarse_size = 0;
    for (auto v : ncs) coarse_size += v;
    if (coarse_size == 0 || coarse_size == fine_size) {
      if (prm.relax_type[3] == 9 || prm.relax_type[3] == 99 || prm.relax_type[3] == 19 || prm.relax_type[3] == 98) {
        prm.relax_type[3] = prm.relax_type[0];
        prm.num_sweeps[3] = 1;
      }
      break;
    }
    if (coarse_size < prm.min_coarse_size) break;
    std::vector<int> cstarts(size + 1, 0);
    for (int p = 0; p < size; ++p) cstarts[p + 1] = cstarts[p] + (int)ncs[p];
    CSR P;
    const int cc0 = cstarts[rank], cc1 = cstarts[rank + 1];  // this rank's coarse columns
    if (agg_lvl) {
      // multipass rows as P_diag | P_offd (setup.cpp amg_setup, emulated ranks)
      multipass_dist(L[level].A, S, cf, first, n, L[level].starts, cstarts, prm.agg_trunc_factor, prm.agg_P_max_elmts,
                     comm, P);
      rank_order_local(P, cc0, cc1);
    } else {
      extpi_dist(L[level].A, S, cf, first, n, L[level].starts, cstarts, prm.strong_threshold, prm.max_row_sum, comm,
                 P, prm.interp_type == 6);
      // par_csr_matrix.c:2671 truncates the row [P_diag | P_offd] and splits the
      // kept entries back into the two parts in their sorted order
      rank_order_local(P, cc0, cc1);
      if (prm.trunc_factor != 0.0 || prm.P_max_elmts > 0) truncate_rows(P, prm.trunc_factor, prm.P_max_elmts);
      rank_order_local(P, cc0, cc1);
      for (int i = 0; i < n; ++i)
        if (cf[i] == SF_PT) cf[i] = F_PT;
    }
    CSR R;
    transpose_dist(P, first, fine_size, cstarts, comm, R);
    CSR Ac;
    rap_dist(R, L[level].A, P, first, L[level].starts, cstarts, comm, Ac);
    rank_order_local(Ac, cc0, cc1);  // hypre's RAP keeps each coarse row as diag then offd (par_rap.c)
    snprintf(buf, sizeof buf, "rank %d level %d: rows %d/%d -> coarse %d/%lld\n", rank, level, n, fine_size,
             (int)ncs[rank], (long long)coarse_size);
    if (log) *log += buf;
    L[level].cf.swap(cf);
    L[level].P.swap(P);
    L[level].R.swap(R);
    L.emplace_back();
    DLevel& C = L[level + 1];
    C.A.swap(Ac);
    C.starts = cstarts;
    C.first = cstarts[rank];
    C.nloc = (int)ncs[rank];
    C.nglob = (int)coarse_size;
    ++level;
    if (prm.coarsen_type > 0 && coarse_size >= (int64_t)(fine_size * 0.75))
      throw std::runtime_error("slow coarsening (coarse >= 0.75 fine) would switch to CLJP: unsupported");
    if (level == prm.max_levels - 1 || coarse_size <= prm.max_coarse_size) finished = true;
  }
  const int nl = (int)L.size();
  for (auto& D : L) D.nnz_glob = comm.allreduce_sum(D.A.nnz());
  // l1 norms (amg_setup's sequence, global indices)
  for (int j = 0; j < nl; ++j) {
    DLevel& D = L[j];
    // rank-uniform condition (a rank may own no rows of a level, hence an
    // empty cf): every rank must take part in the same exchanges
    const bool use_cf = prm.relax_order && j < nl - 1;
    GhostPlan gp;
    std::vector<int> gcf;
    if (use_cf) {
      std::vector<int> off;
      offrank_cols(D.A, D.first, D.first + D.nloc, off);
      gp.build(off, D.first, D.nloc, D.starts, comm);
      gp.pull(D.cf.data(), gcf, comm);
    }
    const std::vector<int>* cfp = use_cf ? &D.cf : nullptr;
    if (j < nl - 1 && (uses_l1_gs(prm.relax_type[1]) || uses_l1_gs(prm.relax_type[2])))
      l1_dist(D.A, D.first, D.nglob, 4, cfp, &gp, &gcf, prm.blocks_for(D.A.nrows), D.l1);
    else if (j == nl - 1 && uses_l1_gs(prm.relax_type[3]))
      l1_dist(D.A, D.first, D.nglob, 4, nullptr, nullptr, nullptr, prm.blocks_for(D.A.nrows), D.l1);
    if (j < nl - 1 && (prm.relax_type[1] == 18 || prm.relax_type[2] == 18))
      l1_dist(D.A, D.first, D.nglob, 1, cfp, &gp, &gcf, 1, D.l1);
    else if (j == nl - 1 && prm.relax_type[3] == 18)
      l1_dist(D.A, D.first, D.nglob, 1, nullptr, nullptr, nullptr, 1, D.l1);
    // par_amg_setup.c:3139: Chebyshev (relax 16) eigenvalue estimate and coefficients
    if (prm.relax_type[1] == 16 || prm.relax_type[2] == 16 || (prm.relax_type[3] == 16 && j == nl - 1)) {
      double max_eig = 0.0, min_eig = 0.0;
      if (prm.cheby_eig_est)
        max_eig_cg_dist(D.A, D.first, D.nloc, D.starts, prm.cheby_scale, prm.cheby_eig_est, comm, &max_eig, &min_eig);
      else
        max_eig_norm_dist(D.A, prm.cheby_scale, comm, &max_eig);
      cheby_setup(D.A, max_eig, min_eig, prm.cheby_fraction, prm.cheby_order, prm.cheby_scale, prm.cheby_variant,
                  D.cheby_coefs, D.cheby_ds);
    }
    if (prm.relax_type[1] == 7 || prm.relax_type[2] == 7 || (prm.relax_type[3] == 7 && j == nl - 1)) {
      D.l1.resize(D.nloc);
      for (int r = 0; r < D.nloc; ++r) {
        const double d = D.A.a[D.A.i[r]];
        D.l1[r] = (d == 0.0) ? 1.0 : d;
      }
    }
  }
  out = RankHierarchy();
  out.rank = rank;
  out.size = size;
  out.prm = prm;
  // rows of every rank, in rank order (= global row order), on every rank
  auto gather_rows = [&](const CSR& M, int nglob_rows) {
    std::vector<int> len(M.nrows);
    for (int r = 0; r < M.nrows; ++r) len[r] = M.i[r + 1] - M.i[r];
    auto alen = comm.allgatherv(len);
    auto acol = comm.allgatherv(M.j);
    auto aval = comm.allgatherv(M.a);
    CSR G;
    G.resize_rows(nglob_rows, M.ncols);
    for (int r = 0; r < nglob_rows; ++r) G.i[r + 1] = G.i[r] + alen[r];
    G.j.assign(acol.begin(), acol.end());
    G.a.assign(aval.begin(), aval.end());
    return G;
  };
  // coarsest-level direct solve: the coarsest operator gathered on every rank
  if (nl > 1 && (prm.relax_type[3] == 9 || prm.relax_type[3] == 99 || prm.relax_type[3] == 19 ||
                 prm.relax_type[3] == 98)) {
    const DLevel& D = L[nl - 1];
    if (D.nglob > 8192) throw std::runtime_error("coarsest level too large for the dense direct solve");
    CSR G = gather_rows(D.A, D.nglob);
    G.ncols = D.nglob;
    out.coarse_n = D.nglob;
    csr_to_dense(G, out.coarse_dense);
  }
  // coarse-level agglomeration (partition.hpp): levels >= agg held whole
  std::vector<int64_t> grows(nl);
  for (int l = 0; l < nl; ++l) grows[l] = L[l].nglob;
  const int agg = agglomeration_level(prm, grows, size);
  // the hybrid-GS blocks of a level over all its rows: num_blocks blocks of
  // every rank's rows (D.starts: the distributed owners)
  auto owner_blocks = [&](const DLevel& D) {
    std::vector<int> b(1, 0);
    for (int r = 0; r < size; ++r) {
      const int a0 = D.starts[r], n0 = D.starts[r + 1] - a0;
      const int nb = prm.blocks_for(n0);
      const std::vector<int> loc = hypre_block_starts(n0, nb);
      for (int k = 1; k <= nb; ++k) b.push_back(a0 + loc[k]);
    }
    return b;
  };
  int agg_share = 0;  // this rank's rows of level agg (the restriction's output)
  out.agg_level = agg;
  if (agg >= 0) {
    out.agg_starts = L[agg].starts;
    agg_share = L[agg].nloc;
    for (int l = agg; l < nl; ++l) {
      DLevel& D = L[l];
      D.A = gather_rows(D.A, D.nglob);
      if (l + 1 < nl) {
        D.P = gather_rows(D.P, D.nglob);
        D.R = gather_rows(D.R, L[l + 1].nglob);
      }
      D.cf = comm.allgatherv(D.cf);
      D.l1 = comm.allgatherv(D.l1);
      D.cheby_ds = comm.allgatherv(D.cheby_ds);
      // a replicated level is swept by every rank whole, in its owners'
      // blocks (partition.cpp rank_gs_blocks): its hybrid-GS l1 norms over them
      bool cfr = false;
      if (!D.l1.empty() && l1_option_for_level(prm, l, nl, &cfr) == 4)
        compute_l1_norms_blocks(D.A, 4, (cfr && !D.cf.empty()) ? D.cf.data() : nullptr, owner_blocks(D), D.l1);
    }
    for (int l = agg; l < nl; ++l) {
      DLevel& D = L[l];
      D.first = 0;
      D.nloc = D.nglob;
    }
  }
  double tot_rows = 0, tot_nnz = 0;
  for (auto& D : L) { tot_rows += D.nglob; tot_nnz += (double)D.nnz_glob; }
  out.grid_complexity = tot_rows / L[0].nglob;
  out.operator_complexity = tot_nnz / (double)L[0].nnz_glob;
  for (auto& D : L) {
    out.nnz_A.push_back(D.nnz_glob);
    out.rows.push_back(D.nglob);
  }
  // this rank's operators with [local | halo] columns and halo plans
  std::vector<std::vector<int>> hu(nl), hv(nl);
  for (int l = 0; l < nl; ++l) {
    const DLevel& D = L[l];
    if (agg >= 0 && l >= agg) continue;  // replicated: no halos
    std::vector<int> u;
    offrank_cols(D.A, D.first, D.first + D.nloc, u);
    if (l > 0) offrank_cols(L[l - 1].P, D.first, D.first + D.nloc, u);
    sort_unique(u);
    hu[l].swap(u);
    if (l + 1 < nl) {
      std::vector<int> v;
      offrank_cols(D.R, D.first, D.first + D.nloc, v);
      sort_unique(v);
      hv[l].swap(v);
    }
  }
  out.lev.resize(nl);
  for (int l = 0; l < nl; ++l) {
    const DLevel& D = L[l];
    RankLevel& RL = out.lev[l];
    RL.n_loc = D.nloc;
    RL.first = D.first;
    RL.n_glob = D.nglob;
    make_rank_op(D.A, 0, D.nloc, D.first, D.first + D.nloc, hu[l], RL.A);
    if (l + 1 < nl) {
      const DLevel& C = L[l + 1];
      make_rank_op(D.P, 0, D.nloc, C.first, C.first + C.nloc, hu[l + 1], RL.P);
      const int rrows = (agg >= 0 && l + 1 == agg) ? agg_share : C.nloc;
      make_rank_op(D.R, 0, rrows, D.first, D.first + D.nloc, hv[l], RL.R);
    }
    RL.l1 = D.l1;
    RL.cf = D.cf;
    RL.cheby_ds = D.cheby_ds;
    RL.cheby_coefs = D.cheby_coefs;
    if (size > 1 && uses_hybrid_gs_any(prm))
      RL.gs_blocks = (agg >= 0 && l >= agg) ? owner_blocks(D) : hypre_block_starts(D.nloc, prm.blocks_for(D.nloc));
    if (agg >= 0 && l >= agg) {
      RL.hu.n_loc = D.nloc;
      if (l + 1 < nl) RL.hv.n_loc = D.nloc;
    } else {
      RL.hu = make_halo(hu[l], D.first, D.nloc, D.starts, comm);
      if (l + 1 < nl) RL.hv = make_halo(hv[l], D.first, D.nloc, D.starts, comm);
    }
  }
  return 0;
}

int dist_setup_self_check(const CSR& A, const AMGParams& prm, int size, std::string& msg) {
  Hierarchy H;
  const int n0 = A.nrows;
  std::vector<int> s0(size + 1);
  for (int r = 0; r <= size; ++r) s0[r] = (int)((int64_t)n0 * r / size);
  // the one-process statement of the same N-rank setup: the rank emulation
  amg_setup(A, prm, H, size > 1 ? &s0 : nullptr, nullptr);
  std::vector<RankHierarchy> ref;
  partition_hierarchy_all(H, s0, size, ref);
  auto comms = make_thread_host_comms(size);
  std::vector<RankHierarchy> got(size);
  std::vector<std::string> err(size);
  std::vector<std::thread> th;
  for (int r = 0; r < size; ++r) {
    th.emplace_back([&, r] {
      try {
        CSR Ar;
        Ar.resize_rows(s0[r + 1] - s0[r], A.ncols);
        for (int i = s0[r]; i < s0[r + 1]; ++i) Ar.i[i - s0[r] + 1] = Ar.i[i - s0[r]] + (A.i[i + 1] - A.i[i]);
        Ar.j.assign(A.j.begin() + A.i[s0[r]], A.j.begin() + A.i[s0[r + 1]]);
        Ar.a.assign(A.a.begin() + A.i[s0[r]], A.a.begin() + A.i[s0[r + 1]]);
        if (amg_setup_dist(Ar, s0[r], prm, *comms[r], got[r]) != 0) err[r] = "unsupported parameters";
      } catch (const std::exception& e) {
        err[r] = e.what();
      }
    });
  }
  for (auto& t : th) t.join();
  int bad = 0;
  for (int r = 0; r < size; ++r) {
    if (!err[r].empty()) {
      msg += "rank " + std::to_string(r) + ": " + err[r] + "\n";
      ++bad;
      continue;
    }
    std::vector<char> b1, b2;
    serialize(ref[r], b1);
    serialize(got[r], b2);
    if (b1 != b2) {
      ++bad;
      msg += "rank " + std::to_string(r) + ": distributed hierarchy differs (levels " +
             std::to_string(got[r].lev.size()) + " vs " + std::to_string(ref[r].lev.size()) + ")\n";
      // first differing level / part
      const size_t nl = std::min(got[r].lev.size(), ref[r].lev.size());
      for (size_t l = 0; l < nl && msg.size() < 2000; ++l) {
        const RankLevel &x = got[r].lev[l], &y = ref[r].lev[l];
        auto cmp = [&](const CSR& p, const CSR& q, const char* what) {
          if (p.i != q.i || p.j != q.j || p.a != q.a || p.nrows != q.nrows || p.ncols != q.ncols)
            msg += "  level " + std::to_string(l) + " " + what + " differs\n";
        };
        cmp(x.A.interior, y.A.interior, "A.interior");
        cmp(x.A.boundary, y.A.boundary, "A.boundary");
        cmp(x.P.interior, y.P.interior, "P.interior");
        cmp(x.P.boundary, y.P.boundary, "P.boundary");
        cmp(x.R.interior, y.R.interior, "R.interior");
        cmp(x.R.boundary, y.R.boundary, "R.boundary");
        if (x.cf != y.cf) msg += "  level " + std::to_string(l) + " cf differs\n";
        if (x.l1 != y.l1) msg += "  level " + std::to_string(l) + " l1 differs\n";
        if (x.hu.send_idx != y.hu.send_idx || x.hu.peers != y.hu.peers || x.hu.halo_glob != y.hu.halo_glob)
          msg += "  level " + std::to_string(l) + " hu differs\n";
        if (x.hv.send_idx != y.hv.send_idx || x.hv.peers != y.hv.peers || x.hv.halo_glob != y.hv.halo_glob)
          msg += "  level " + std::to_string(l) + " hv differs\n";
      }
      if (got[r].coarse_dense != ref[r].coarse_dense) msg += "  coarse_dense differs\n";
      if (got[r].nnz_A != ref[r].nnz_A) msg += "  nnz_A differs\n";
    }
  }
  return bad;
}

}  // namespace hve
