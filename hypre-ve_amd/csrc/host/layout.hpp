#pragma once
#include <cstdint>
#include <utility>
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
                     hvec<int>& col, hvec<double>& val);
// SELL-64 with 16-bit column deltas (row order and entry order kept; padded
// slots may sit between a row's entries): entry k of the slice's lane r at
// slice_ptr[s] + 64k + r holds col - row - slot_base[slice_ptr[s]/64 + k], or
// kDeltaPad for padding.  false when some row does not fit (no layout built).
constexpr short kDeltaPad = -32768;
bool build_sell_delta_host(const CSR& A, std::vector<int>& slice_ptr, std::vector<int>& slot_base,
                           hvec<short>& dcol, hvec<double>& val);
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
bool build_value_table(const double* val, size_t n, int maxv, hvec<unsigned char>& idx, std::vector<double>& tab);
// The same with 16-bit indices (maxv <= 65536).
bool build_value_table16(const double* val, size_t n, int maxv, hvec<unsigned short>& idx,
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
                           hvec<unsigned short>& code, std::vector<int>& otab, std::vector<double>& vtab,
                           int& vbits);
// Jagged SELL-64 (no stored padding): perm[i] = CSR row at stored position i
// (rows sorted by descending length inside each slice), rowlen[i] its length
// (nslices*64 entries, 0 past the last row), entry k of the slice's lane r at
// slice_ptr[s] + sum_{k'<k} #{lanes with rowlen > k'} + r.
void build_sell_jagged_host(const CSR& A, std::vector<int>& perm, std::vector<int>& slice_ptr,
                            std::vector<int>& rowlen, hvec<int>& col, hvec<double>& val);
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
// Rows 0..n-1 ordered by ascending key, ties by row (a stable sort by key).
void sort_rows_by_key(const std::vector<int64_t>& key, std::vector<int>& order);
bool build_sell_dict_host(const CSR& A, int dmax, int group, std::vector<int>& perm, std::vector<int>& slice_ptr,
                          std::vector<int>& rowlen, hvec<unsigned short>& col16, hvec<double>& val,
                          std::vector<int>& dict_ptr, std::vector<int>& dict, int& max_distinct,
                          int max_ranges = 0, double max_cover = 1.5, const std::vector<int>* pre = nullptr);
// Lane-packed streams of a jagged dictionary layout (k_sell_dictw): the same
// slices, rows and entry order, stored so that one 16-byte load of a lane
// fetches two consecutive values of its row, and one 16-byte load eight
// consecutive 16-bit local columns.  Per slice s, with cnt(k) = #{lanes whose
// row is longer than k}:
//   values: pair j (entries 2j, 2j+1) of lane l < cnt(2j) at
//           wptr[s] + 2 (cnt(0) + cnt(2) + ... + cnt(2j - 2)) + 2l (doubles);
//   columns: octet o (entries 8o .. 8o+7) of lane l < cnt(8o) at
//           wptr[ns + 1 + s] + 8 (cnt(0) + cnt(8) + ... + cnt(8o - 8)) + 8l;
// entries past a row's end are 0 (never summed).  wptr has 2 (ns + 1) ints;
// false when a stream exceeds 2^31 elements.
bool pack_dict_wide(const std::vector<int>& slice_ptr, const std::vector<int>& rowlen,
                    const hvec<unsigned short>& col16, const hvec<double>& val, std::vector<int>& wptr,
                    hvec<unsigned short>& colw, hvec<double>& valw);
// Jagged form of an offset-coded layout (k_code_pw): every slice's rows sorted
// by descending length (stable; perm[i] = CSR row at stored position i), entry
// k of stored lane l at slice_ptr[s] + cnt(0) + ... + cnt(k-1) + l with
// cnt(k) = #{lanes whose row is longer than k}; no padding stored.  From the
// padded codes of build_sell_coded_host (sp_pad, code_pad: entries in slots
// 0 .. len - 1 of their lane) and the rows' lengths.
void jag_codes_from_padded(const CSR& A, const std::vector<int>& sp_pad, const hvec<unsigned short>& code_pad,
                           std::vector<int>& perm, std::vector<int>& slice_ptr, std::vector<int>& rowlen,
                           hvec<unsigned short>& code);
// Packed SELL-64 entries (k_sell_code PK) from a padded layout (col, 16-bit
// value indices vi into nv values): code = ((col - base[slice]) << vbits) |
// value index, base = the slice's smallest column, padding 0xFFFFFFFF.  false
// when some slice's column span does not fit 32 - vbits bits.
bool pack_sell_codes(const std::vector<int>& sp, const hvec<int>& col, const hvec<unsigned short>& vi, int nv,
                     hvec<unsigned>& code, std::vector<int>& base, int& vbits);
// Largest column index of A (-1 when empty).
int csr_max_col(const CSR& A);
// True when every row's l1[map[i]] (map empty: i) equals, bit for bit, the sum
// of |a_ij| over its stored entries in order, negated for a negative first
// entry (the on-the-fly l1 norms of the device kernels).
bool l1_rows_match(const CSR& A, const std::vector<int>& map, const std::vector<double>& l1);
// Padded entry count of the SELL-64 layout for a given sigma (0 = no sort).
int64_t sell_padded_nnz(const CSR& A, int sigma);
// Packed, step-ordered schedule of one hybrid Gauss-Seidel sweep (par_relax.c
// cases 3/4/6/8/13/14 with hypre's num_threads row blocks; the level
// scheduling of the reference's relax-6 path, par_relax.c:2340-2650).
//  * Levels.  Inside each block a row's level exceeds that of every in-block
//    neighbour it must see updated (lower rows for a forward sweep), and every
//    in-block neighbour it must see un-updated is pushed strictly above it, so
//    the rows of one level never reference each other.
//  * Teams.  Blocks interact only through the pre-sweep copy tmp, so
//    consecutive blocks are swept together by one wavefront (a team): level l
//    of the team is level l of each of its blocks.  A team takes blocks while
//    its rows stay within team_rows x its level count.
//  * Steps.  A team level is cut into steps of at most ring_w rows (64; a
//    knob takes 16 for teams of at most 4 rows a level, whose kernel LDS ring
//    is then a quarter as wide).  Position k
//    of the sweep order (rowmap[k] = row) is step s's row offset + lane, and
//    the sweep works on vectors permuted into that order, so a step reads and
//    writes its rows contiguously.  They sit in one buffer G of 3n + nhalo
//    doubles: T = G[0, n) (the pre-sweep copy tmp; u itself unless a symmetric
//    sweep's second half runs), C = G[n, 2n) (u at the sweep's start),
//    U = G[2n, 3n) (the values this sweep wrote), then the off-rank halo of u
//    (multi-rank, natural order); F (the right-hand side) beside it, l1 / cf
//    permuted here.  Entry k of a step's row r sits at ent(s) + k * rows(s) + r.
//  * Sources.  Each entry stores a code for the value its product reads:
//      code >= 0   G[code]: T for an off-block column, C for an in-block one
//                  not updated yet (the row itself included), U for an
//                  in-block one updated at least kGsFence + 1 steps earlier
//                  (the kernel fences its U stores every kGsFence steps), or
//                  the halo for an off-rank column
//      -1          padding
//      <= -2       the team's LDS ring, slot -2 - code = (step % kGsRing) x
//                  ring_w + lane: a value an in-block row computed at most
//                  kGsFence steps earlier
//    Every row's products are summed in CSR order, so a sweep equals the
//    sequential per-block sweep bit for bit.
#ifndef HVE_GS_RING
#define HVE_GS_RING 16
#endif
constexpr int kGsRing = HVE_GS_RING;
constexpr int kGsFence = kGsRing - 1;
// U stores leave the ring in batches of kGsBatch steps (k_hybrid_gs): at the
// end of a batch the wave fences, which completes the previous batch's stores,
// then issues this batch's.  A value computed at step q is therefore visible
// in U from step (q / kGsBatch + 2) * kGsBatch on, at most 2 kGsBatch steps
// later.  The pipelined sweep (k_hybrid_gs_pipe) issues step j's U gathers
// during step j - 1, after the fence of step j - 2, so U codes need a distance
// of 2 kGsBatch + 1 <= kGsFence + 1 steps; gs_schedule_self_check emulates
// the stricter rule (a U read of step j sees fences of steps <= j - 2).
constexpr int kGsBatch = 4;
static_assert(2 * kGsBatch + 1 <= kGsFence + 1 && kGsFence < kGsRing, "ring reach");
struct GsSchedule {
  std::vector<int> block_start;  // nb + 1 row boundaries (hypre's ns / ne)
  std::vector<int> team_step;    // nteams + 1: step range of each team
  std::vector<int> step;         // 4 per step: entry offset (unsigned), position offset, rows, width
  hvec<int> code;                // per entry (see above)
  hvec<double> val;              // per entry, 0 for padding
  hvec<int> tcol;                // with_tcol: in-block entries' T offset in G (the weighted forms' Vtemp), else -1
  std::vector<int> rowmap;       // nrows: row of each position
  std::vector<double> l1;        // l1 norms by position (when given)
  std::vector<int> cf;           // CF marker by position (when given)
  int nteams = 0, max_steps = 0, max_width = 0;
  int ring_w = 64;               // rows a step holds at most = lanes of a ring slot (16 | 64)
  int64_t nnz = 0;               // the operator's entries (the stored ones minus padding)
  double rows_per_step = 0;
};
// A: the rows swept (columns >= A.nrows are off-rank, read from the halo).
void build_gs_schedule(const CSR& A, const std::vector<int>& block_start, bool forward, GsSchedule& S,
                       int team_rows = 64, bool with_tcol = false, const std::vector<double>* l1 = nullptr,
                       const std::vector<int>* cf = nullptr);
// Host check of a schedule: the team-parallel sweep emulated with the
// kernel's memory semantics (permuted C / T / U vectors; a step reads
// everything before writing; U stores become visible only at the kernel's
// fences; ring slots are reused after kGsRing steps) against the sequential
// per-block sweep of the reference, on random f / u and a different tmp (a
// symmetric sweep's second half); returns 0 when bitwise equal.  weighted: the
// w / omega form (par_relax.c:4544) with w = 0.7, omega = 1.3.
int gs_schedule_self_check(const CSR& A, int num_blocks, bool forward, bool use_l1, const std::vector<double>& l1,
                           std::string& msg, int team_rows = 64, bool weighted = false);
// hypre's thread partition of n rows into nb blocks (par_relax.c size / rest).
std::vector<int> hypre_block_starts(int n, int nb);

void gselim_factor(int n, const std::vector<double>& dense, std::vector<double>& L, std::vector<unsigned char>& mask,
                   std::vector<double>& U);
void csr_to_dense(const CSR& A, std::vector<double>& dense);
}  // namespace hve
