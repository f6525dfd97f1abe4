#pragma once
#include <vector>

#include "hve_host.hpp"

namespace hve {
void build_sell_host(const CSR& A, std::vector<int>& slice_ptr, std::vector<int>& col, std::vector<double>& val);
void gselim_factor(int n, const std::vector<double>& dense, std::vector<double>& L, std::vector<unsigned char>& mask,
                   std::vector<double>& U);
void csr_to_dense(const CSR& A, std::vector<double>& dense);
}  // namespace hve
