#pragma once
#include <vector>

#include "hve_host.hpp"

namespace hve {
// SELL-64 layout (slices of 64 rows, entry k of a slice's lane at
// slice_ptr[s] + 64k + lane, padding col -1).  sigma > 0: rows are sorted by
// descending length inside windows of sigma rows (SELL-C-sigma) and perm[i]
// receives the CSR row stored at position i; sigma == 0 keeps the row order
// and leaves perm empty.
void build_sell_host(const CSR& A, int sigma, std::vector<int>& perm, std::vector<int>& slice_ptr,
                     std::vector<int>& col, std::vector<double>& val);
// Padded entry count of the SELL-64 layout for a given sigma (0 = no sort).
int64_t sell_padded_nnz(const CSR& A, int sigma);
void gselim_factor(int n, const std::vector<double>& dense, std::vector<double>& L, std::vector<unsigned char>& mask,
                   std::vector<double>& U);
void csr_to_dense(const CSR& A, std::vector<double>& dense);
}  // namespace hve
