#pragma once
#include <cstdint>
#include <string>
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
// SELL-64 with 16-bit column deltas (row order and entry order kept; padded
// slots may sit between a row's entries): entry k of the slice's lane r at
// slice_ptr[s] + 64k + r holds col - row - slot_base[slice_ptr[s]/64 + k], or
// kDeltaPad for padding.  false when some row does not fit (no layout built).
constexpr short kDeltaPad = -32768;
bool build_sell_delta_host(const CSR& A, std::vector<int>& slice_ptr, std::vector<int>& slot_base,
                           std::vector<short>& dcol, std::vector<double>& val);
// Slot-uniform SELL-64 for constant-coefficient stencils: no per-entry data.
// Slices with identical slot sequences share a pattern: slice s uses pattern
// slice_pat[s], whose `width` slots k (index pattern * width + k) hold column
// row + slot_off, value tab[slot_vi] for the lanes set in slot_mask (0 for
// unused slots).  slice_pat covers 8 slices past the last, the slot arrays 16
// slots of tail.  false when a slice needs more than max_width slots or more
// than 256 distinct values occur (layout.cpp).
bool build_sell_stencil_host(const CSR& A, int max_width, int& width, std::vector<int>& slice_pat,
                             std::vector<int>& slot_off, std::vector<int>& slot_vi, std::vector<uint64_t>& slot_mask,
                             std::vector<double>& tab);
// Lossless value table: idx[i] indexes tab (ascending by bit pattern) with
// tab[idx[i]] bitwise equal to val[i]; false when more than maxv (<= 256)
// distinct values occur.
bool build_value_table(const std::vector<double>& val, int maxv, std::vector<unsigned char>& idx,
                       std::vector<double>& tab);
// The same with 16-bit indices (maxv <= 65536).
bool build_value_table16(const std::vector<double>& val, int maxv, std::vector<unsigned short>& idx,
                         std::vector<double>& tab);
// Offset-coded SELL-64 (P and R between two levels of a grid hierarchy).  Row
// i of A (local row g = rowmap[i], identity when empty) has the anchor
// a = anc[g] (g when anc is empty); column c has the position colpos[c] (c when
// empty).  Each entry stores one 16-bit code, (offset index << vbits) | value
// index, where otab[offset index] = position(c) - a and vtab[value index] is
// bitwise the entry's value; the device recovers the column as a + off, or
// cmap[a + off] when cmap is not empty.  Padded, natural row order, padding
// code 0xFFFF.  false (nothing built) when more than 256 distinct offsets or
// 4096 distinct values occur, the codes do not fit 16 bits, or some column is
// not recovered exactly.
bool build_sell_coded_host(const CSR& A, const std::vector<int>& rowmap, const std::vector<int>& anc,
                           const std::vector<int>& colpos, const std::vector<int>& cmap, std::vector<int>& slice_ptr,
                           std::vector<unsigned short>& code, std::vector<int>& otab, std::vector<double>& vtab,
                           int& vbits);
// Jagged SELL-64 (no stored padding): perm[i] = CSR row at stored position i
// (rows sorted by descending length inside each slice), rowlen[i] its length
// (nslices*64 entries, 0 past the last row), entry k of the slice's lane r at
// slice_ptr[s] + sum_{k'<k} #{lanes with rowlen > k'} + r.
void build_sell_jagged_host(const CSR& A, std::vector<int>& perm, std::vector<int>& slice_ptr,
                            std::vector<int>& rowlen, std::vector<int>& col, std::vector<double>& val);
// Jagged SELL-64 with a per-slice column dictionary (16-bit local column
// indices into the slice's ascending list of distinct columns).  false when
// a slice has more than dmax distinct columns; max_distinct is set either way.
// group: slices sharing one dictionary (one workgroup of `group` waves).
// pre: the order rows are cut into slices in (a permutation of the rows;
// nullptr = natural order), before each slice is sorted by row length.
// max_ranges > 0: range dictionary instead.  The x-tile of a group is the
// union of at most max_ranges contiguous column ranges that cover its distinct
// columns (the largest holes between them left out), staged by coalesced
// copies; dict holds (start, offset) pairs, a terminal (-1, covered) after each
// group's ranges, dict_ptr indexes the pairs, and col16 is the column's
// position in the concatenated ranges.  false when a group covers more than
// dmax columns or the covered columns exceed max_cover x its distinct ones;
// max_distinct is then the largest covered count.
bool build_sell_dict_host(const CSR& A, int dmax, int group, std::vector<int>& perm, std::vector<int>& slice_ptr,
                          std::vector<int>& rowlen, std::vector<unsigned short>& col16, std::vector<double>& val,
                          std::vector<int>& dict_ptr, std::vector<int>& dict, int& max_distinct,
                          int max_ranges = 0, double max_cover = 1.5, const std::vector<int>* pre = nullptr);
// Padded entry count of the SELL-64 layout for a given sigma (0 = no sort).
int64_t sell_padded_nnz(const CSR& A, int sigma);
// Level schedule of one hybrid Gauss-Seidel sweep (par_relax.c cases 3/4/6/
// 8/13/14 with hypre's num_threads row blocks; the level scheduling of the
// reference's relax-6 path, par_relax.c:2340-2650).  Inside each block rows
// are grouped into levels: a row's level exceeds that of every in-block
// neighbour it must see updated (lower rows for a forward sweep), and every
// in-block neighbour it must see un-updated is pushed strictly above it, so the
// rows of one level never reference each other and a level is one parallel
// step.  Each level is stored SELL-64 (lane per row, entries in CSR order, so
// every row sum is formed in the reference's order).
struct GsSchedule {
  std::vector<int> block_start;  // nb + 1 row boundaries (hypre's ns / ne)
  std::vector<int> block_level;  // nb + 1: level range of each block
  std::vector<int> level_slice;  // nlevels + 1: slice range of each level
  std::vector<int> slice_ptr;    // nslices + 1 entry offsets
  std::vector<int> col;          // padded, -1 = padding
  std::vector<double> val;
  std::vector<int> rowmap;       // nslices * 64: row of each lane, -1 = none
  int max_levels = 0;            // longest block schedule
  double avg_rows_per_level = 0;
};
void build_gs_schedule(const CSR& A, const std::vector<int>& block_start, bool forward, GsSchedule& S);
// Host check of a schedule: the level-parallel sweep (every read of a level
// before any of its writes) against the sequential per-block sweep of the
// reference, on random f / u; returns 0 when bitwise equal.
int gs_schedule_self_check(const CSR& A, int num_blocks, bool forward, bool use_l1, const std::vector<double>& l1,
                           std::string& msg);
// hypre's thread partition of n rows into nb blocks (par_relax.c size / rest).
std::vector<int> hypre_block_starts(int n, int nb);

void gselim_factor(int n, const std::vector<double>& dense, std::vector<double>& L, std::vector<unsigned char>& mask,
                   std::vector<double>& U);
void csr_to_dense(const CSR& A, std::vector<double>& dense);
}  // namespace hve
