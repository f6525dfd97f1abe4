// Aggressive coarsening (BoomerAMG agg_num_levels), one process:
//   * second strength graph on the C points of a first coarsening, S*S + 2S
//     with a path count (par_strength.c:1729 hypre_BoomerAMGCreate2ndSHost);
//   * the second-pass marker merged into the first (par_strength.c:2957
//     hypre_BoomerAMGCorrectCFMarker);
//   * multipass interpolation (par_multi_interp.c:16 hypre_BoomerAMGBuildMultipass,
//     weight_option 0), the reference's default agg_interp_type 4.
// Restated for num_procs == 1 and one thread: every list order and every
// floating-point accumulation follows the reference's statement order, since
// the coarse grid and the weights (and so the solve's bits) depend on them.
#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "hve_host.hpp"

namespace hve {

// S2 over the C points of cf (coarse numbering by ascending fine index).  Row
// ic lists, in first-touch order, the coarse points reached from C point i1
// directly (a strong C neighbour i2: 2 paths) or through one strong neighbour
// i2 (i2's strong C neighbours i3 != i1: 1 path each); a column is kept with
// at least num_paths paths.  A C point whose row stays empty gets cf = 2, as
// the reference marks it (its CorrectCFMarker then keeps it a C point).
void create_2nd_strength(const Pattern& S, std::vector<int>& cf, int num_paths, Pattern& S2) {
  const int n = S.n;
  std::vector<int> fine_to_coarse(n, -1), coarse_to_fine;
  coarse_to_fine.reserve(n / 2);
  for (int i = 0; i < n; ++i)
    if (cf[i] > 0) {
      fine_to_coarse[i] = (int)coarse_to_fine.size();
      coarse_to_fine.push_back(i);
    }
  const int nc = (int)coarse_to_fine.size();
  S2.n = nc;
  S2.i.assign(nc + 1, 0);
  S2.j.clear();
  std::vector<int> marker(nc, -1);  // position of a column in the current row's touch list
  std::vector<int> touch, count;
  for (int ic = 0; ic < nc; ++ic) {
    const int i1 = coarse_to_fine[ic];
    touch.clear();
    count.clear();
    auto add = [&](int index, int w) {
      if (marker[index] < 0) {
        marker[index] = (int)touch.size();
        touch.push_back(index);
        count.push_back(w);
      } else {
        count[marker[index]] += w;
      }
    };
    for (int k1 = S.i[i1]; k1 < S.i[i1 + 1]; ++k1) {
      const int i2 = S.j[k1];
      if (cf[i2] > 0) add(fine_to_coarse[i2], 2);
      for (int k2 = S.i[i2]; k2 < S.i[i2 + 1]; ++k2) {
        const int i3 = S.j[k2];
        if (cf[i3] > 0 && fine_to_coarse[i3] != ic) add(fine_to_coarse[i3], 1);
      }
    }
    int kept = 0;
    for (size_t t = 0; t < touch.size(); ++t) {
      if (count[t] >= num_paths) {
        S2.j.push_back(touch[t]);
        ++kept;
      }
      marker[touch[t]] = -1;
    }
    S2.i[ic + 1] = S2.i[ic] + kept;
    if (kept == 0) cf[i1] = 2;
  }
}

// par_strength.c:2957: the first pass's C points take the second pass's
// marker (cf == 2, an isolated C point of S2, stays C).
void correct_cf_marker(std::vector<int>& cf, const std::vector<int>& new_cf) {
  int cnt = 0;
  for (size_t i = 0; i < cf.size(); ++i) {
    if (cf[i] > 0) {
      if (cf[i] == 1) cf[i] = new_cf[cnt++];
      else { cf[i] = 1; cnt++; }
    }
  }
}

// par_strength.c:2978 (2-stage interpolations): a first-pass C point the
// second pass makes F becomes -2, every other one 1.
void correct_cf_marker2(std::vector<int>& cf, const std::vector<int>& new_cf) {
  int cnt = 0;
  for (size_t i = 0; i < cf.size(); ++i) {
    if (cf[i] > 0) cf[i] = new_cf[cnt++] == -1 ? -2 : 1;
  }
}

// par_multi_interp.c:16 hypre_BoomerAMGBuildMultipass, num_procs 1, one
// thread, num_functions 1, weight_option 0.
//   * pass 0: C points (P row: the point itself, weight 1);
//   * pass 1: F points with a strong C neighbour;
//   * pass p > 1: F points with a strong neighbour of pass p-1, up to 10 passes.
// pass_array holds the F points in descending index order and the passes are
// peeled off it by the reference's in-place swap, which fixes the order in
// which the rows of a pass are built (and so every row's column order).
void build_multipass_interp(const CSR& A, const std::vector<int>& cf, const Pattern& S, double trunc_factor,
                            int max_elmts, CSR& P) {
  const int n = A.nrows;
  const int max_num_passes = 10;
  int n_coarse = 0, n_SF = 0;
  for (int i = 0; i < n; ++i) {
    if (cf[i] == 1) ++n_coarse;
    else if (cf[i] == -3) ++n_SF;
  }
  const int pass_array_size = n - n_coarse - n_SF;
  std::vector<int> pass_array(std::max(1, pass_array_size), 0), pass_pointer(max_num_passes + 1, 0);
  std::vector<int> assigned(n, -1), fine_to_coarse(n, -1), C_array(n_coarse);
  std::vector<int> Pi(n + 1, 0);  // row lengths, then row starts
  int cnt = 0, p_cnt = pass_array_size - 1;
  for (int i = 0; i < n; ++i) {
    if (cf[i] == 1) {
      fine_to_coarse[i] = cnt;
      C_array[cnt++] = i;
      assigned[i] = 0;
      Pi[i + 1] = 1;
    } else if (cf[i] == -1) {
      pass_array[p_cnt--] = i;
    }
  }
  // pass 1: neighbours of C points
  pass_pointer[0] = 0;
  pass_pointer[1] = 0;
  cnt = 0;
  int64_t total_nz = n_coarse;
  int cnt_nz = 0;
  for (int i = pass_array_size - 1; i > cnt - 1; i--) {
    const int i1 = pass_array[i];
    for (int k = S.i[i1]; k < S.i[i1 + 1]; ++k) {
      if (cf[S.j[k]] == 1) {
        Pi[i1 + 1]++;
        cnt_nz++;
        assigned[i1] = 1;
      }
    }
    if (assigned[i1] == 1) {
      pass_array[i++] = pass_array[cnt];
      pass_array[cnt++] = i1;
    }
  }
  pass_pointer[2] = cnt;
  // later passes: strong neighbours of the previous pass
  int pass = 2;
  while (pass_array_size - cnt > 0 && pass < max_num_passes) {
    for (int i = pass_array_size - 1; i > cnt - 1; i--) {
      const int i1 = pass_array[i];
      for (int k = S.i[i1]; k < S.i[i1 + 1]; ++k) {
        if (assigned[S.j[k]] == pass - 1) {
          pass_array[i++] = pass_array[cnt];
          pass_array[cnt++] = i1;
          assigned[i1] = pass;
          break;
        }
      }
    }
    pass++;
    pass_pointer[pass] = cnt;
  }
  const int num_passes = pass;
  // column lists per pass (coarse indices), P_diag_start per point
  std::vector<std::vector<int>> pass_cols(num_passes);
  std::vector<int> start(n, 0);
  pass_cols[1].reserve(cnt_nz);
  for (int i = pass_pointer[1]; i < pass_pointer[2]; ++i) {
    const int i1 = pass_array[i];
    start[i1] = (int)pass_cols[1].size();
    for (int k = S.i[i1]; k < S.i[i1 + 1]; ++k)
      if (cf[S.j[k]] == 1) pass_cols[1].push_back(fine_to_coarse[S.j[k]]);
  }
  total_nz += (int64_t)pass_cols[1].size();
  std::vector<int> marker(std::max(1, n_coarse), -1);
  for (pass = 2; pass < num_passes; ++pass) {
    std::fill(marker.begin(), marker.end(), -1);
    const std::vector<int>& prev = pass_cols[pass - 1];
    std::vector<int>& cur = pass_cols[pass];
    // count (marker = i1), then set (marker = -i1-1), as the reference does
    for (int i = pass_pointer[pass]; i < pass_pointer[pass + 1]; ++i) {
      const int i1 = pass_array[i];
      for (int k = S.i[i1]; k < S.i[i1 + 1]; ++k) {
        const int j1 = S.j[k];
        if (assigned[j1] != pass - 1) continue;
        for (int q = start[j1]; q < start[j1] + Pi[j1 + 1]; ++q) {
          const int k1 = prev[q];
          if (marker[k1] != i1) {
            Pi[i1 + 1]++;
            marker[k1] = i1;
          }
        }
      }
    }
    for (int i = pass_pointer[pass]; i < pass_pointer[pass + 1]; ++i) {
      const int i1 = pass_array[i];
      start[i1] = (int)cur.size();
      for (int k = S.i[i1]; k < S.i[i1 + 1]; ++k) {
        const int j1 = S.j[k];
        if (assigned[j1] != pass - 1) continue;
        for (int q = start[j1]; q < start[j1] + Pi[j1 + 1]; ++q) {
          const int k1 = prev[q];
          if (marker[k1] != -i1 - 1) {
            cur.push_back(k1);
            marker[k1] = -i1 - 1;
          }
        }
      }
    }
    total_nz += (int64_t)cur.size();
  }
  if (total_nz > 0x7fffffffLL) throw std::runtime_error("multipass interpolation exceeds 2^31 entries");
  for (int i = 0; i < n; ++i) Pi[i + 1] += Pi[i];
  P.resize_rows(n, n_coarse);
  P.i = Pi;
  P.j.assign(Pi[n], 0);
  P.a.assign(Pi[n], 0.0);
  for (int c = 0; c < n_coarse; ++c) {
    const int i1 = C_array[c];
    P.j[Pi[i1]] = fine_to_coarse[i1];
    P.a[Pi[i1]] = 1.0;
  }
  // weights, pass 1: direct interpolation from the strong C neighbours
  double alfa = 1.0;  // carried from row to row (and used as a temporary), as in the reference
  std::vector<int> tmp_marker(n, -1);
  for (int i = pass_pointer[1]; i < pass_pointer[2]; ++i) {
    const int i1 = pass_array[i];
    double sum_C = 0, sum_N = 0;
    const int len = Pi[i1 + 1] - Pi[i1];
    for (int q = start[i1]; q < start[i1] + len; ++q) tmp_marker[C_array[pass_cols[1][q]]] = i1;
    int c = Pi[i1];
    for (int k = A.i[i1] + 1; k < A.i[i1 + 1]; ++k) {
      const int j1 = A.j[k];
      if (cf[j1] != -3 && (!hve_setup_dof || hve_setup_dof[i1] == hve_setup_dof[j1])) sum_N += A.a[k];
      if (j1 != -1 && tmp_marker[j1] == i1) {
        P.a[c] = A.a[k];
        P.j[c++] = fine_to_coarse[j1];
        sum_C += A.a[k];
      }
    }
    const double diagonal = A.a[A.i[i1]];
    if (sum_C * diagonal != 0) alfa = -sum_N / (sum_C * diagonal);
    for (int q = Pi[i1]; q < c; ++q) P.a[q] *= alfa;
  }
  // weights, passes >= 2: through the rows of the previous pass
  std::vector<int> tmp_array(std::max(1, n_coarse), 0);
  for (pass = 2; pass < num_passes; ++pass) {
    std::fill(tmp_marker.begin(), tmp_marker.end(), -1);
    for (int i = pass_pointer[pass]; i < pass_pointer[pass + 1]; ++i) {
      const int i1 = pass_array[i];
      double sum_C = 0, sum_N = 0;
      const int len = Pi[i1 + 1] - Pi[i1];
      int c = Pi[i1];
      for (int q = start[i1]; q < start[i1] + len; ++q) {
        const int k1 = pass_cols[pass][q];
        tmp_array[k1] = c;
        P.a[c] = 0;
        P.j[c++] = k1;
      }
      for (int k = S.i[i1]; k < S.i[i1 + 1]; ++k)
        if (assigned[S.j[k]] == pass - 1) tmp_marker[S.j[k]] = i1;
      for (int k = A.i[i1] + 1; k < A.i[i1 + 1]; ++k) {
        const int j1 = A.j[k];
        if (tmp_marker[j1] == i1) {
          for (int q = Pi[j1]; q < Pi[j1 + 1]; ++q) {
            const int k1 = P.j[q];
            alfa = A.a[k] * P.a[q];
            P.a[tmp_array[k1]] += alfa;
            sum_C += alfa;
            sum_N += alfa;
          }
        } else {
          if (cf[j1] != -3 && (!hve_setup_dof || hve_setup_dof[i1] == hve_setup_dof[j1])) sum_N += A.a[k];
        }
      }
      const double diagonal = A.a[A.i[i1]];
      if (sum_C * diagonal != 0) alfa = -sum_N / (sum_C * diagonal);
      for (int q = Pi[i1]; q < Pi[i1 + 1]; ++q) P.a[q] *= alfa;
    }
  }
  if (trunc_factor != 0.0 || max_elmts != 0) truncate_rows(P, trunc_factor, max_elmts);
}

}  // namespace hve
