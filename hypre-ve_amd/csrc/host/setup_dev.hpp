// Device restatements of the setup's heavy row kernels (device/setup_dev.hip).
// Each one produces the same entries, in the same order, with the same sums
// (same operations in the same order, no contraction) as the host function it
// replaces in setup.cpp, so the hierarchy is byte for byte the host one;
// tests/test_gpu_setup.py compares every level.  Rows whose marker tables do
// not fit the kernels' LDS are finished by the host functions' own row code.
#pragma once
#include <vector>

#include "hve_host.hpp"

namespace hve {

// Ext+i interpolation rows (extpi_core, one process): P with columns
// fine_to_coarse[] of the C-hat points, then truncate_rows(tol, max_elmts).
void dev_extpi_interp(const CSR& A, const Pattern& S, const std::vector<int>& cf,
                      const std::vector<int>& fine_to_coarse, int ncoarse, double trunc_factor, int max_elmts,
                      CSR& P);
// Galerkin product C = P^T A P (rap_core with R = P^T, coarse_glob empty) and
// R = P^T (transpose) itself.
void dev_rap(const CSR& P, const CSR& A, CSR& R, CSR& C);
// Strength (create_strength, one function) and PMIS (coarsen_pmis, CF_init 0
// or 2, one process): S and the CF marker as the host functions give them;
// *t_strength: the seconds of the strength part.
void dev_strength_pmis(const CSR& A, double thr, double max_row_sum, Pattern& S, std::vector<int>& cf,
                       double* t_strength);
// Frees the device copies of the current level's A, S and P that the dev_*
// calls share (amg_setup calls it at the start of every level and at the end).
void dev_setup_cache_clear();
// Rows of the last dev_* call finished on the host (tables too large for LDS).
long long dev_setup_host_rows();

}  // namespace hve
