// Host-side construction of the HBM layouts consumed by the device runtime.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>
#include <parallel/algorithm>

#include "hve_host.hpp"
#include "layout.hpp"

namespace hve {

// SELL-64: slices of 64 consecutive rows, padded to the longest row of the
// slice; entry k of lane r at slice_ptr[s] + 64*k + r; padding col = -1.
static void sell_order(const CSR& A, int sigma, std::vector<int>& perm, const std::vector<int>* pre = nullptr) {
  const int n = A.nrows;
  perm.resize(n);
  for (int r = 0; r < n; ++r) perm[r] = pre ? (*pre)[r] : r;
  if (sigma <= 0) return;
#pragma omp parallel for schedule(static)
  for (int w0 = 0; w0 < n; w0 += sigma) {
    const int w1 = std::min(n, w0 + sigma);
    std::stable_sort(perm.begin() + w0, perm.begin() + w1, [&](int x, int y) {
      return A.i[x + 1] - A.i[x] > A.i[y + 1] - A.i[y];
    });
  }
}

int64_t sell_padded_nnz(const CSR& A, int sigma) {
  std::vector<int> perm;
  sell_order(A, sigma, perm);
  int64_t tot = 0;
  for (int s0 = 0; s0 < A.nrows; s0 += 64) {
    int w = 0;
    for (int r = s0; r < std::min(A.nrows, s0 + 64); ++r) w = std::max(w, A.i[perm[r] + 1] - A.i[perm[r]]);
    tot += (int64_t)w * 64;
  }
  return tot;
}

void build_sell_host(const CSR& A, int sigma, std::vector<int>& perm, std::vector<int>& slice_ptr,
                     hvec<int>& col, hvec<double>& val) {
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  sell_order(A, sigma, perm);
  slice_ptr.assign(ns + 1, 0);
  std::vector<int64_t> sp(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int w = 0;
    const int r1 = std::min(n, (s + 1) * 64);
    for (int r = s * 64; r < r1; ++r) w = std::max(w, A.i[perm[r] + 1] - A.i[perm[r]]);
    sp[s + 1] = sp[s] + (int64_t)w * 64;
  }
  if (sp[ns] > 0x7fffffffLL) throw std::runtime_error("padded operator exceeds 2^31 entries on one GPU");
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  col.clear();
  val.clear();
  col.resize((size_t)sp[ns]);
  val.resize((size_t)sp[ns]);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    const int r1 = std::min(n, (s + 1) * 64);
    std::fill(col.begin() + slice_ptr[s], col.begin() + slice_ptr[s + 1], -1);
    std::fill(val.begin() + slice_ptr[s], val.begin() + slice_ptr[s + 1], 0.0);
    for (int r = s * 64; r < r1; ++r) {
      const int lane = r & 63, src = perm[r];
      for (int k = A.i[src]; k < A.i[src + 1]; ++k) {
        const size_t pos = (size_t)slice_ptr[s] + (size_t)(k - A.i[src]) * 64 + lane;
        col[pos] = A.j[k];
        val[pos] = A.a[k];
      }
    }
  }
  if (sigma <= 0) perm.clear();
}

// SELL-64 with 16-bit column deltas.  Stencil-like operators reference, in
// entry slot k of a slice, columns at nearly the same offset from their row
// (the 7-point operator: slot k is the same neighbour for every interior lane).
// Each (slice, slot) stores one 32-bit base offset; each entry stores
// col - row - base as a signed 16-bit delta (kDeltaPad = padding).  Rows keep
// their entry order; a row shorter than the slice's longest is laid into the
// slots greedily (leftmost slot whose base reaches its next entry, which is
// optimal for an order-preserving match), so a missing stencil neighbour
// becomes an interior padding slot instead of shifting the ones after it.
// Bases come from the slice's first longest row; a slice that does not fit
// so takes one base for all its slots (entries in their natural slots) when
// its column offsets span less than 64K.  Returns false when some row
// does not fit its slice's slots (the operator then keeps 32-bit columns).
bool build_sell_delta_host(const CSR& A, std::vector<int>& slice_ptr, std::vector<int>& slot_base,
                           hvec<short>& dcol, hvec<double>& val) {
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  slice_ptr.assign(ns + 1, 0);
  std::vector<int64_t> sp(ns + 1, 0);
  std::vector<int> ref(ns, -1);
  for (int s = 0; s < ns; ++s) {
    int w = 0;
    for (int r = s * 64; r < std::min(n, (s + 1) * 64); ++r) {
      const int len = A.i[r + 1] - A.i[r];
      if (len > w) { w = len; ref[s] = r; }
    }
    sp[s + 1] = sp[s] + (int64_t)w * 64;
  }
  if (sp[ns] > 0x7fffffffLL) return false;
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  slot_base.assign((size_t)(sp[ns] / 64), 0);
  par_assign(dcol, (size_t)sp[ns], kDeltaPad);
  par_assign(val, (size_t)sp[ns], 0.0);
  int ok = 1;
#pragma omp parallel for schedule(static) reduction(min : ok)
  for (int s = 0; s < ns; ++s) {
    if (ref[s] < 0 || !ok) continue;
    const int w = (slice_ptr[s + 1] - slice_ptr[s]) / 64;
    int* base = slot_base.data() + slice_ptr[s] / 64;
    const int r0 = s * 64, r1 = std::min(n, (s + 1) * 64);
    // mode 0: per-slot bases from the first longest row, greedy slot match;
    // mode 1 (when 0 fails): one base for the whole slice (the middle of its
    // offset range) and every entry in its natural slot -- fits operators
    // whose offsets in a slice span < 64K columns (P: coarse neighbours of
    // 64 consecutive fine rows)
    bool fit = false;
    for (int mode = 0; mode < 2 && !fit; ++mode) {
      for (int r = r0; r < r1; ++r)
        for (int k = 0; k < w; ++k) {
          const size_t pos = (size_t)slice_ptr[s] + (size_t)k * 64 + (r & 63);
          dcol[pos] = kDeltaPad;
          val[pos] = 0.0;
        }
      if (mode == 0) {
        const int rr = ref[s];
        for (int k = 0; k < w; ++k) base[k] = A.j[A.i[rr] + k] - rr;
      } else {
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int r = r0; r < r1; ++r)
          for (int e = A.i[r]; e < A.i[r + 1]; ++e) {
            lo = std::min(lo, (int64_t)A.j[e] - r);
            hi = std::max(hi, (int64_t)A.j[e] - r);
          }
        if (hi - lo > 65534) break;
        for (int k = 0; k < w; ++k) base[k] = (int)(lo + (hi - lo) / 2);
      }
      fit = true;
      for (int r = r0; r < r1 && fit; ++r) {
        int k = 0;
        for (int e = A.i[r]; e < A.i[r + 1]; ++e, ++k) {
          const int64_t off = (int64_t)A.j[e] - r;
          while (k < w && (off - base[k] < -32767 || off - base[k] > 32767)) ++k;
          if (k == w) { fit = false; break; }
          const size_t pos = (size_t)slice_ptr[s] + (size_t)k * 64 + (r & 63);
          dcol[pos] = (short)(off - base[k]);
          val[pos] = A.a[e];
        }
      }
    }
    if (!fit) ok = 0;
  }
  // B = 16 slots of tail padding: the device issues a batch's loads unmasked
  slot_base.resize(slot_base.size() + 16, 0);
  dcol.resize(dcol.size() + 16 * 64, kDeltaPad);
  val.resize(val.size() + 16 * 64, 0.0);
  return ok != 0;
}

// Slot-uniform SELL-64 (the "stencil" layout).  A constant-coefficient stencil
// operator repeats one (column offset, value) pair in each slot of a slice: slot
// k holds, for every lane that has it, the neighbour at row + off_k with value
// val_k.  The slots of a slice are a shortest common supersequence of its rows'
// (offset, value) sequences, merged row by row through their longest common
// subsequence; each row is then matched greedily, in entry order, into the
// slots (a missing neighbour -- grid boundary -- leaves its lane's bit clear),
// with its first entry in slot 0.  Nothing is stored per entry: per (slice,
// slot) a 32-bit offset, an index into the table of the slot values (<= 256
// distinct) and the 64-bit lane mask, every slice padded to the operator's
// widest (empty slots: mask 0), so slot k of slice s sits at s * width + k.
// Each row still sums its entries in stored order.  false when the slots would
// exceed max_width or the values 256 (the operator then takes the per-entry
// delta layout).
namespace {
struct SlotKey {
  int64_t off;
  uint64_t bits;
  bool operator==(const SlotKey& o) const { return off == o.off && bits == o.bits; }
};
bool is_subseq(const std::vector<SlotKey>& s, const std::vector<SlotKey>& t) {
  size_t k = 0;
  for (const SlotKey& e : s) {
    while (k < t.size() && !(t[k] == e)) ++k;
    if (k == t.size()) return false;
    ++k;
  }
  return true;
}
// shortest common supersequence of a and b (through their LCS)
std::vector<SlotKey> scs(const std::vector<SlotKey>& a, const std::vector<SlotKey>& b) {
  const size_t m = a.size(), n = b.size();
  std::vector<int> L((m + 1) * (n + 1), 0);
  for (size_t i = m; i-- > 0;)
    for (size_t j = n; j-- > 0;)
      L[i * (n + 1) + j] = a[i] == b[j] ? L[(i + 1) * (n + 1) + j + 1] + 1
                                        : std::max(L[(i + 1) * (n + 1) + j], L[i * (n + 1) + j + 1]);
  std::vector<SlotKey> out;
  size_t i = 0, j = 0;
  while (i < m && j < n) {
    const int la = L[(i + 1) * (n + 1) + j], lb = L[i * (n + 1) + j + 1];
    if (a[i] == b[j]) { out.push_back(a[i]); ++i; ++j; }
    // ties go to the smaller (offset, value) first: rows stored in ascending
    // column order (after the diagonal) then merge into that same order
    else if (la > lb || (la == lb && (a[i].off < b[j].off || (a[i].off == b[j].off && a[i].bits < b[j].bits))))
      out.push_back(a[i++]);
    else out.push_back(b[j++]);
  }
  while (i < m) out.push_back(a[i++]);
  while (j < n) out.push_back(b[j++]);
  return out;
}
}  // namespace

bool build_sell_stencil_host(const CSR& A, int max_width, int& width, std::vector<int>& slice_pat,
                             std::vector<int>& slot_off, std::vector<int>& slot_vi, std::vector<uint64_t>& slot_mask,
                             std::vector<double>& tab) {
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  std::vector<std::vector<SlotKey>> T(ns);
  int ok = 1, wmax = 0;
#pragma omp parallel for schedule(static) reduction(min : ok) reduction(max : wmax)
  for (int s = 0; s < ns; ++s) {
    if (!ok) continue;
    std::vector<SlotKey> seq;
    for (int r = s * 64; r < std::min(n, (s + 1) * 64); ++r) {
      seq.clear();
      for (int e = A.i[r]; e < A.i[r + 1]; ++e) {
        SlotKey k{(int64_t)A.j[e] - r, 0};
        std::memcpy(&k.bits, &A.a[e], 8);
        seq.push_back(k);
      }
      if (!is_subseq(seq, T[s])) T[s] = scs(T[s], seq);
      if ((int)T[s].size() > max_width) { ok = 0; break; }
    }
    for (const SlotKey& k : T[s])
      if (k.off < INT_MIN || k.off > INT_MAX) ok = 0;
    wmax = std::max(wmax, (int)T[s].size());
  }
  if (!ok) return false;
  width = wmax;
  const size_t ns_pad = (size_t)ns + 8;  // a wave's last slices and batch past the end read padding
  const size_t nslots = ns_pad * (size_t)width;
  slot_off.assign(nslots + 16, 0);
  slot_mask.assign(nslots + 16, 0);
  std::vector<double> sval(nslots + 16, 0.0);
#pragma omp parallel for schedule(static) reduction(min : ok)
  for (int s = 0; s < ns; ++s) {
    if (!ok) continue;
    const size_t s0 = (size_t)s * width;
    for (size_t k = 0; k < T[s].size(); ++k) {
      slot_off[s0 + k] = (int)T[s][k].off;
      std::memcpy(&sval[s0 + k], &T[s][k].bits, 8);
    }
    const int w = (int)T[s].size();
    for (int r = s * 64; r < std::min(n, (s + 1) * 64) && ok; ++r) {
      int k = 0;
      for (int e = A.i[r]; e < A.i[r + 1]; ++e, ++k) {
        const int64_t off = (int64_t)A.j[e] - r;
        while (k < w && !(slot_off[s0 + k] == off && std::memcmp(&sval[s0 + k], &A.a[e], 8) == 0)) ++k;
        if (k == w || (e == A.i[r] && k != 0)) { ok = 0; break; }
        slot_mask[s0 + k] |= 1ull << (r & 63);
      }
    }
  }
  if (!ok) return false;
  hvec<unsigned char> vi;
  if (!build_value_table(sval.data(), sval.size(), 256, vi, tab)) return false;
  // Slices with the same slot sequence (offsets, values and lane masks: the
  // interior of a stencil, and each kind of boundary slice) share one
  // pattern; a slice keeps only its pattern's index, so the slot data of a
  // launch is a few KiB that stay in cache instead of a stream.
  const int W = width;
  std::vector<uint64_t> h(ns);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    uint64_t x = 1469598103934665603ull;
    for (int k = 0; k < W; ++k) {
      const size_t i = (size_t)s * W + k;
      for (uint64_t v : {(uint64_t)(uint32_t)slot_off[i], (uint64_t)vi[i], slot_mask[i]}) {
        x ^= v + 0x9e3779b97f4a7c15ull + (x << 6) + (x >> 2);
      }
    }
    h[s] = x;
  }
  std::unordered_map<uint64_t, std::vector<int>> seen;  // hash -> patterns
  std::vector<int> po, pv;
  std::vector<uint64_t> pm;
  slice_pat.assign((size_t)ns + 8, 0);
  auto same = [&](int s, int pt) {
    for (int k = 0; k < W; ++k) {
      const size_t i = (size_t)s * W + k, j = (size_t)pt * W + k;
      if (slot_off[i] != po[j] || (int)vi[i] != pv[j] || slot_mask[i] != pm[j]) return false;
    }
    return true;
  };
  for (int s = 0; s < ns; ++s) {
    std::vector<int>& cand = seen[h[s]];
    int found = -1;
    for (int pt : cand)
      if (same(s, pt)) { found = pt; break; }
    if (found < 0) {
      found = (int)(po.size() / (size_t)std::max(W, 1));
      for (int k = 0; k < W; ++k) {
        const size_t i = (size_t)s * W + k;
        po.push_back(slot_off[i]);
        pv.push_back(vi[i]);
        pm.push_back(slot_mask[i]);
      }
      cand.push_back(found);
    }
    slice_pat[s] = found;
  }
  // a batch reads up to 8 slots past a pattern's last: 16 slots of tail
  po.resize(po.size() + 16, 0);
  pv.resize(pv.size() + 16, 0);
  pm.resize(pm.size() + 16, 0);
  slot_off.swap(po);
  slot_vi.swap(pv);
  slot_mask.swap(pm);
  return true;
}

// Value table (value-indexed storage, lossless): when the stored values take
// at most maxv distinct bit patterns (constant-coefficient stencils: 2-4),
// each entry keeps an 8-bit index into the ascending-by-bits table instead of
// its 8-byte value.  Padding entries index their own (+0.0) pattern.
template <typename I>
static bool value_table_impl(const double* val, size_t n, int maxv, hvec<I>& idx, std::vector<double>& tab) {
  std::vector<uint64_t> all;
  bool over = false;
#pragma omp parallel
  {
    std::unordered_set<uint64_t> mine;
    uint64_t last = 0;
    bool have = false;
#pragma omp for schedule(static)
    for (size_t i = 0; i < n; ++i) {
      if (over) continue;
      uint64_t b;
      std::memcpy(&b, &val[i], 8);
      if (have && b == last) continue;  // runs of one value (padding, stencil slots)
      last = b;
      have = true;
      if (mine.insert(b).second && (int)mine.size() > maxv) over = true;
    }
#pragma omp critical
    all.insert(all.end(), mine.begin(), mine.end());
  }
  if (over) return false;
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end()), all.end());
  if ((int)all.size() > maxv) return false;
  tab.resize(all.size());
  for (size_t t = 0; t < all.size(); ++t) std::memcpy(&tab[t], &all[t], 8);
  idx.clear();
  idx.resize(n);
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) {
    uint64_t b;
    std::memcpy(&b, &val[i], 8);
    idx[i] = (I)(std::lower_bound(all.begin(), all.end(), b) - all.begin());
  }
  return true;
}
bool build_value_table(const double* val, size_t n, int maxv, hvec<unsigned char>& idx, std::vector<double>& tab) {
  return value_table_impl(val, n, std::min(maxv, 256), idx, tab);
}
bool build_value_table16(const double* val, size_t n, int maxv, hvec<unsigned short>& idx,
                         std::vector<double>& tab) {
  return value_table_impl(val, n, std::min(maxv, 65536), idx, tab);
}

// Offset-coded SELL-64.  Between two levels of a grid hierarchy the fine
// points an interpolation row or a restriction row touches lie at a few fixed
// offsets from the row's own grid point (the 7-point hierarchy's P_0 and R_0:
// the 25 points within distance 2), and their weights take ~1200 distinct
// values, so (offset, value) packs into 16 bits: 2 B an entry instead of 6
// (32-bit column + 16-bit value index) or 12.
bool build_sell_coded_host(const CSR& A, const std::vector<int>& rowmap, const std::vector<int>& anc,
                           const std::vector<int>& colpos, const std::vector<int>& cmap, std::vector<int>& slice_ptr,
                           hvec<unsigned short>& code, std::vector<int>& otab, std::vector<double>& vtab,
                           int& vbits) {
  const int n = A.nrows;
  if (n == 0 || A.nnz() == 0) return false;
  constexpr int kMaxOff = 256;
  auto anchor = [&](int i) -> int64_t {
    const int g = rowmap.empty() ? i : rowmap[i];
    if (anc.empty()) return g;
    return (g >= 0 && g < (int)anc.size()) ? anc[g] : INT64_MIN / 4;
  };
  auto position = [&](int c) -> int64_t {
    if (colpos.empty()) return c;
    return (c >= 0 && c < (int)colpos.size() && colpos[c] >= 0) ? colpos[c] : INT64_MIN / 4;
  };
  // distinct offsets, with the decode checked entry by entry
  std::vector<int64_t> offs;
  bool bad = false;
#pragma omp parallel
  {
    std::unordered_set<int64_t> mine;
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) {
      if (bad) continue;
      const int64_t a = anchor(i);
      for (int k = A.i[i]; k < A.i[i + 1]; ++k) {
        const int64_t pos = position(A.j[k]);
        const int64_t off = pos - a;
        const int64_t at = a + off;
        bool ok = pos > INT64_MIN / 8 && a > INT64_MIN / 8 && off >= INT_MIN && off <= INT_MAX;
        if (ok && !cmap.empty()) ok = at >= 0 && at < (int64_t)cmap.size() && cmap[at] == A.j[k];
        if (ok && cmap.empty()) ok = at == A.j[k];
        if (!ok || (mine.insert(off).second && (int)mine.size() > kMaxOff)) {
          bad = true;
          break;
        }
      }
    }
#pragma omp critical
    offs.insert(offs.end(), mine.begin(), mine.end());
  }
  if (bad) return false;
  std::sort(offs.begin(), offs.end());
  offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
  if ((int)offs.size() > kMaxOff) return false;
  hvec<unsigned short> vi;
  if (!build_value_table16(A.a.data(), A.a.size(), 4096, vi, vtab)) return false;
  vbits = 1;
  while ((1 << vbits) < (int)vtab.size()) ++vbits;
  const int obits = 16 - vbits;
  // the largest offset index stays below 2^obits - 1, so 0xFFFF is never a code
  if (obits <= 0 || (int64_t)offs.size() >= (1LL << obits)) return false;
  otab.assign(offs.begin(), offs.end());
  const int ns = (n + 63) / 64;
  std::vector<int64_t> sp(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int w = 0;
    for (int r = s * 64; r < std::min(n, (s + 1) * 64); ++r) w = std::max(w, A.i[r + 1] - A.i[r]);
    sp[s + 1] = sp[s] + (int64_t)w * 64;
  }
  if (sp[ns] > 0x7fffffffLL) return false;
  slice_ptr.assign(ns + 1, 0);
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  code.clear();
  code.resize((size_t)sp[ns]);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    std::fill(code.begin() + sp[s], code.begin() + sp[s + 1], (unsigned short)0xFFFF);
    for (int r = s * 64; r < std::min(n, (s + 1) * 64); ++r) {
      const int64_t a = anchor(r);
      for (int k = A.i[r]; k < A.i[r + 1]; ++k) {
        const int64_t off = position(A.j[k]) - a;
        const int oi = (int)(std::lower_bound(offs.begin(), offs.end(), off) - offs.begin());
        code[(size_t)sp[s] + (size_t)(k - A.i[r]) * 64 + (r & 63)] = (unsigned short)((oi << vbits) | vi[k]);
      }
    }
  }
  return true;
}

// Jagged SELL-64: rows sorted by descending length inside each 64-row slice
// (stable), entry k stored only for the cnt_k lanes whose row is longer than
// k, at slice_ptr[s] + (cnt_0 + ... + cnt_{k-1}) + lane.  No padding is
// stored; the device recovers each offset from a wave ballot of
// (k < rowlen[lane]).
void build_sell_jagged_host(const CSR& A, std::vector<int>& perm, std::vector<int>& slice_ptr,
                            std::vector<int>& rowlen, hvec<int>& col, hvec<double>& val) {
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  sell_order(A, 64, perm);
  slice_ptr.assign(ns + 1, 0);
  rowlen.assign((size_t)ns * 64, 0);
  std::vector<int64_t> sp(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int64_t t = 0;
    const int r1 = std::min(n, (s + 1) * 64);
    for (int r = s * 64; r < r1; ++r) t += A.i[perm[r] + 1] - A.i[perm[r]];
    sp[s + 1] = sp[s] + t;
  }
  if (sp[ns] > 0x7fffffffLL) throw std::runtime_error("operator exceeds 2^31 entries on one GPU");
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  col.clear();  // every entry is written below
  val.clear();
  col.resize((size_t)sp[ns]);
  val.resize((size_t)sp[ns]);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    const int r0 = s * 64, r1 = std::min(n, (s + 1) * 64);
    int len[64] = {0};
    for (int r = r0; r < r1; ++r) {
      len[r - r0] = A.i[perm[r] + 1] - A.i[perm[r]];
      rowlen[r] = len[r - r0];
    }
    size_t pos = (size_t)slice_ptr[s];
    for (int k = 0; k < len[0]; ++k) {
      int cnt = 0;
      while (cnt < r1 - r0 && len[cnt] > k) ++cnt;  // lanes sorted by descending length
      for (int l = 0; l < cnt; ++l) {
        const int src = perm[r0 + l];
        col[pos + l] = A.j[A.i[src] + k];
        val[pos + l] = A.a[A.i[src] + k];
      }
      pos += cnt;
    }
  }
}

// Jagged SELL-64 with a per-slice column dictionary: the distinct columns a
// slice references, ascending, are listed once (dict, dict_ptr per slice) and
// every entry stores the 16-bit position of its column in that list.  The
// device stages x[dict] of a slice in LDS (coalesced: the list is sorted and
// runs of consecutive columns share lines) and reads x from LDS in the row
// loop.  Entry order, row order (sorted inside the slice) and rowlen are those
// of build_sell_jagged_host.  Returns false (and builds nothing) when a slice
// references more than dmax distinct columns.
// Ranges covering the ascending distinct columns `cols` with at most
// max_ranges pieces: break at the max_ranges - 1 largest holes.  rs gets
// (start, offset) pairs and the terminal (-1, covered).
static void cover_ranges(const std::vector<int>& cols, int max_ranges, std::vector<int>& rs) {
  rs.clear();
  if (cols.empty()) {
    rs.push_back(-1);
    rs.push_back(0);
    return;
  }
  const int m = (int)cols.size();
  std::vector<int> brk;  // positions i where a new range starts at cols[i]
  {
    std::vector<std::pair<int, int>> holes;  // (hole size, position)
    for (int i = 1; i < m; ++i)
      if (cols[i] - cols[i - 1] > 1) holes.push_back({cols[i] - cols[i - 1] - 1, i});
    const size_t keep = std::min<size_t>(holes.size(), (size_t)std::max(0, max_ranges - 1));
    std::partial_sort(holes.begin(), holes.begin() + keep, holes.end(),
                      [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
                        return a.first != b.first ? a.first > b.first : a.second < b.second;
                      });
    for (size_t k = 0; k < keep; ++k) brk.push_back(holes[k].second);
    std::sort(brk.begin(), brk.end());
  }
  int off = 0, start = cols[0];
  size_t bi = 0;
  for (int i = 1; i <= m; ++i) {
    if (i == m || (bi < brk.size() && brk[bi] == i)) {
      rs.push_back(start);
      rs.push_back(off);
      off += cols[i - 1] - start + 1;
      if (i < m) {
        start = cols[i];
        ++bi;
      }
    }
  }
  rs.push_back(-1);
  rs.push_back(off);
}

void sort_rows_by_key(const std::vector<int64_t>& key, std::vector<int>& order) {
  // ties broken by row, so any correct sort gives the stable order: libstdc++'s
  // parallel sort on the OpenMP team (41M rows at 512^3: 3.0 s serial)
  const int n = (int)key.size();
  order.resize(n);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < n; ++r) order[r] = r;
  __gnu_parallel::sort(order.begin(), order.end(),
                       [&](int a, int b) { return key[a] < key[b] || (key[a] == key[b] && a < b); });
}

bool build_sell_dict_host(const CSR& A, int dmax, int group, std::vector<int>& perm, std::vector<int>& slice_ptr,
                          std::vector<int>& rowlen, hvec<unsigned short>& col16, hvec<double>& val,
                          std::vector<int>& dict_ptr, std::vector<int>& dict, int& max_distinct, int max_ranges,
                          double max_cover, const std::vector<int>* pre) {
  if (dmax > 65535) dmax = 65535;
  if (group < 1) group = 1;
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  const int ng = (ns + group - 1) / group;
  if (pre && (int)pre->size() != n) pre = nullptr;
  sell_order(A, 64, perm, pre);
  // distinct columns of each group of `group` slices (one workgroup), found
  // through a per-thread hash (RowMap) and kept for the fill pass
  std::vector<std::vector<int>> gcols(ng);
  auto group_cols = [&](int g, RowMap& M, std::vector<int>& cols) {
    cols.clear();
    const int r0 = g * group * 64, r1 = std::min(n, (g + 1) * group * 64);
    int64_t ent = 0;
    for (int r = r0; r < r1; ++r) ent += A.i[perm[r] + 1] - A.i[perm[r]];
    M.begin(std::min<int64_t>(ent, A.ncols));
    bool fresh;
    for (int r = r0; r < r1; ++r)
      for (int k = A.i[perm[r]]; k < A.i[perm[r] + 1]; ++k) {
        M.find_or_insert(A.j[k], 0, &fresh);
        if (fresh) cols.push_back(A.j[k]);
      }
    std::sort(cols.begin(), cols.end());
  };
  const bool ranges = max_ranges > 0;
  std::vector<int64_t> dcount(ng, 0);
  int mx = 0;
  int64_t tot_distinct = 0, tot_cover = 0;
#pragma omp parallel reduction(max : mx) reduction(+ : tot_distinct, tot_cover)
  {
    RowMap M;
    std::vector<int> rs;
#pragma omp for schedule(dynamic, 64)
    for (int g = 0; g < ng; ++g) {
      std::vector<int>& cols = gcols[g];
      group_cols(g, M, cols);
      int cover = (int)cols.size();
      if (ranges) {
        cover_ranges(cols, max_ranges, rs);
        cover = rs.back();
        dcount[g] = (int64_t)rs.size() / 2;  // pairs, terminal included
      } else {
        dcount[g] = (int64_t)cols.size();
      }
      tot_distinct += (int64_t)cols.size();
      tot_cover += cover;
      mx = std::max(mx, cover);
    }
  }
  max_distinct = mx;
  if (mx > dmax) return false;
  if (ranges && (double)tot_cover > max_cover * (double)std::max<int64_t>(1, tot_distinct)) return false;
  std::vector<int64_t> sp(ns + 1, 0), dp(ng + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int64_t t = 0;
    const int r1 = std::min(n, (s + 1) * 64);
    for (int r = s * 64; r < r1; ++r) t += A.i[perm[r] + 1] - A.i[perm[r]];
    sp[s + 1] = sp[s] + t;
  }
  for (int g = 0; g < ng; ++g) dp[g + 1] = dp[g] + dcount[g];
  if (sp[ns] > 0x7fffffffLL || dp[ng] > 0x7fffffffLL) throw std::runtime_error("operator exceeds 2^31 entries on one GPU");
  slice_ptr.assign(ns + 1, 0);
  dict_ptr.assign(ng + 1, 0);
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  for (int g = 0; g <= ng; ++g) dict_ptr[g] = (int)dp[g];
  rowlen.assign((size_t)ns * 64, 0);
  col16.clear();  // every entry is written below
  val.clear();
  col16.resize((size_t)sp[ns]);
  val.resize((size_t)sp[ns]);
  dict.assign((size_t)dp[ng] * (ranges ? 2 : 1), 0);
#pragma omp parallel
  {
    RowMap M;
    std::vector<int> rs;
#pragma omp for schedule(dynamic, 64)
    for (int g = 0; g < ng; ++g) {
      std::vector<int> cols;
      cols.swap(gcols[g]);
      if (ranges) {
        cover_ranges(cols, max_ranges, rs);
        std::copy(rs.begin(), rs.end(), dict.begin() + 2 * (size_t)dict_ptr[g]);
      } else {
        std::copy(cols.begin(), cols.end(), dict.begin() + dict_ptr[g]);
        M.begin((int64_t)cols.size());
        bool fresh;
        for (int t = 0; t < (int)cols.size(); ++t) *M.find_or_insert(cols[t], t, &fresh) = t;
      }
      const int nrg = (int)rs.size() / 2 - 1;
      // position of column c in the group's x-tile
      auto local = [&](int c) -> int {
        if (!ranges) return M.get(c, 0);
        int lo = 0, hi = nrg - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) / 2;
          if (rs[2 * mid] <= c) lo = mid;
          else hi = mid - 1;
        }
        return rs[2 * lo + 1] + (c - rs[2 * lo]);
      };
      for (int s = g * group; s < std::min(ns, (g + 1) * group); ++s) {
        const int r0 = s * 64, r1 = std::min(n, (s + 1) * 64);
        int len[64] = {0};
        for (int r = r0; r < r1; ++r) {
          len[r - r0] = A.i[perm[r] + 1] - A.i[perm[r]];
          rowlen[r] = len[r - r0];
        }
        size_t pos = (size_t)slice_ptr[s];
        for (int k = 0; k < len[0]; ++k) {
          int cnt = 0;
          while (cnt < r1 - r0 && len[cnt] > k) ++cnt;  // lanes sorted by descending length
          for (int l = 0; l < cnt; ++l) {
            const int src = perm[r0 + l];
            const int c = A.j[A.i[src] + k];
            col16[pos + l] = (unsigned short)local(c);
            val[pos + l] = A.a[A.i[src] + k];
          }
          pos += cnt;
        }
      }
    }
  }
  return true;
}

bool pack_dict_wide(const std::vector<int>& slice_ptr, const std::vector<int>& rowlen,
                    const hvec<unsigned short>& col16, const hvec<double>& val, std::vector<int>& wptr,
                    hvec<unsigned short>& colw, hvec<double>& valw) {
  const int ns = (int)slice_ptr.size() - 1;
  std::vector<int64_t> vs(ns + 1, 0), cs(ns + 1, 0);
  // cnt(k) of a slice: lanes are sorted by descending length
  auto cnt_at = [&](int s, int k) {
    int c = 0;
    while (c < 64 && rowlen[(size_t)s * 64 + c] > k) ++c;
    return c;
  };
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    const int w = rowlen[(size_t)s * 64];
    int64_t v = 0, c = 0;
    for (int k = 0; k < w; k += 2) v += 2 * cnt_at(s, k);
    for (int k = 0; k < w; k += 8) c += 8 * cnt_at(s, k);
    vs[s + 1] = v;
    cs[s + 1] = c;
  }
  for (int s = 0; s < ns; ++s) {
    vs[s + 1] += vs[s];
    cs[s + 1] += cs[s];
  }
  if (vs[ns] > 0x7fffffffLL || cs[ns] > 0x7fffffffLL) return false;
  wptr.assign(2 * (size_t)(ns + 1), 0);
  for (int s = 0; s <= ns; ++s) {
    wptr[s] = (int)vs[s];
    wptr[ns + 1 + s] = (int)cs[s];
  }
  valw.clear();
  colw.clear();
  valw.resize((size_t)vs[ns]);
  colw.resize((size_t)cs[ns]);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    const int w = rowlen[(size_t)s * 64];
    // jagged offset of entry k's first lane
    std::vector<int64_t> off(w + 1, slice_ptr[s]);
    std::vector<int> cnt(w + 1, 0);
    for (int k = 0; k < w; ++k) {
      cnt[k] = cnt_at(s, k);
      off[k + 1] = off[k] + cnt[k];
    }
    const int* len = &rowlen[(size_t)s * 64];
    int64_t pv = vs[s], pc = cs[s];
    for (int j = 0; 2 * j < w; ++j) {
      const int k = 2 * j, cl = cnt[k];
      for (int l = 0; l < cl; ++l) {
        valw[pv + 2 * l] = val[off[k] + l];
        valw[pv + 2 * l + 1] = len[l] > k + 1 ? val[off[k + 1] + l] : 0.0;
      }
      pv += 2 * cl;
    }
    for (int o = 0; 8 * o < w; ++o) {
      const int k0 = 8 * o, cl = cnt[k0];
      for (int l = 0; l < cl; ++l)
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + e;
          colw[pc + 8 * l + e] = len[l] > k ? col16[off[k] + l] : (unsigned short)0;
        }
      pc += 8 * cl;
    }
  }
  return true;
}

void jag_codes_from_padded(const CSR& A, const std::vector<int>& sp_pad, const hvec<unsigned short>& code_pad,
                           std::vector<int>& perm, std::vector<int>& slice_ptr, std::vector<int>& rowlen,
                           hvec<unsigned short>& code) {
  const int n = A.nrows;
  const int ns = (n + 63) / 64;
  sell_order(A, 64, perm);  // stable, descending length inside each slice
  slice_ptr.assign(ns + 1, 0);
  rowlen.assign((size_t)ns * 64, 0);
  std::vector<int64_t> sp(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int64_t t = 0;
    for (int r = s * 64; r < std::min(n, (s + 1) * 64); ++r) t += A.i[perm[r] + 1] - A.i[perm[r]];
    sp[s + 1] = sp[s] + t;
  }
  if (sp[ns] > 0x7fffffffLL) throw std::runtime_error("coded operator exceeds 2^31 entries on one GPU");
  for (int s = 0; s <= ns; ++s) slice_ptr[s] = (int)sp[s];
  code.clear();
  code.resize((size_t)sp[ns]);
#pragma omp parallel for schedule(static)
  for (int s = 0; s < ns; ++s) {
    const int r0 = s * 64, r1 = std::min(n, (s + 1) * 64);
    int len[64] = {0};
    for (int r = r0; r < r1; ++r) {
      len[r - r0] = A.i[perm[r] + 1] - A.i[perm[r]];
      rowlen[r] = len[r - r0];
    }
    size_t pos = (size_t)slice_ptr[s];
    for (int k = 0; k < len[0]; ++k) {
      int cnt = 0;
      while (cnt < r1 - r0 && len[cnt] > k) ++cnt;
      for (int l = 0; l < cnt; ++l) {
        const int src = perm[r0 + l];  // its lane in the padded slice: src & 63 (same slice)
        code[pos + l] = code_pad[(size_t)sp_pad[s] + (size_t)k * 64 + (src & 63)];
      }
      pos += cnt;
    }
  }
}

// Packed SELL-64 entries (k_sell_code PK): code = ((col - base[slice]) << vbits)
// | value index, base = the slice's smallest column, padding 0xFFFFFFFF.  false
// when some slice's column span does not fit 32 - vbits bits (all-ones span
// reserved, so no entry equals the padding code).
bool pack_sell_codes(const std::vector<int>& sp, const hvec<int>& col,
                            const hvec<unsigned short>& vi, int nv, hvec<unsigned>& code,
                            std::vector<int>& base, int& vbits) {
  int vb = 1;
  while ((1 << vb) < nv) ++vb;
  const int ns = (int)sp.size() - 1;
  const int64_t lim = (int64_t(1) << (32 - vb)) - 1;
  base.assign(ns + 1, 0);  // one past the last: the kernel's scalar load may run ahead
  code.clear();
  code.resize(col.size());
  int ok = 1;
#pragma omp parallel for schedule(static) reduction(min : ok)
  for (int s = 0; s < ns; ++s) {
    std::fill(code.begin() + sp[s], code.begin() + sp[s + 1], 0xFFFFFFFFu);
    int lo = INT32_MAX, hi = -1;
    for (int q = sp[s]; q < sp[s + 1]; ++q)
      if (col[q] >= 0) { lo = std::min(lo, col[q]); hi = std::max(hi, col[q]); }
    if (hi < 0) continue;
    if ((int64_t)hi - lo >= lim) { ok = 0; continue; }
    base[s] = lo;
    for (int q = sp[s]; q < sp[s + 1]; ++q)
      if (col[q] >= 0) code[q] = ((unsigned)(col[q] - lo) << vb) | vi[q];
  }
  if (!ok) return false;
  vbits = vb;
  return true;
}

int csr_max_col(const CSR& A) {
  int mx = -1;
  const int64_t nnz = A.nnz();
#pragma omp parallel for schedule(static) reduction(max : mx)
  for (int64_t k = 0; k < nnz; ++k) mx = std::max(mx, A.j[k]);
  return mx;
}

bool l1_rows_match(const CSR& A, const std::vector<int>& map, const std::vector<double>& l1) {
  int ok = 1;
#pragma omp parallel for schedule(static) reduction(min : ok)
  for (int i = 0; i < A.nrows; ++i) {
    double s = 0.0;
    for (int q = A.i[i]; q < A.i[i + 1]; ++q) s += std::fabs(A.a[q]);
    if (A.i[i + 1] > A.i[i] && A.a[A.i[i]] < 0.0) s = -s;
    const int g = map.empty() ? i : map[i];
    if (g < 0 || g >= (int)l1.size() || std::memcmp(&s, &l1[g], sizeof(double)) != 0) ok = 0;
  }
  return ok != 0;
}

std::vector<int> hypre_block_starts(int n, int nb) {
  if (nb < 1) nb = 1;
  std::vector<int> st(nb + 1);
  const int size = n / nb, rest = n - size * nb;
  for (int j = 0; j < nb; ++j) st[j] = j < rest ? j * size + j : j * size + rest;
  st[nb] = n;
  return st;
}

namespace {
// Rows of each block grouped by level (GsSchedule): byl[ns .. ne) holds block
// b's rows by ascending (level, row), lptr[b] its level boundaries.
struct GsLevels {
  std::vector<std::vector<int>> lptr;
  std::vector<int> byl, nlev;
};
void gs_levels(const CSR& A, const std::vector<int>& block_start, bool forward, GsLevels& G) {
  const int n = A.nrows, nb = (int)block_start.size() - 1;
  G.lptr.assign(nb, {});
  G.byl.assign(n, 0);
  G.nlev.assign(nb, 0);
  std::vector<int> level(n, 0), floor_(n, 0);
#pragma omp parallel for schedule(dynamic, 16)
  for (int b = 0; b < nb; ++b) {
    const int ns = block_start[b], ne = block_start[b + 1];
    int nlev = 0;
    for (int q = 0; q < ne - ns; ++q) {
      const int i = forward ? ns + q : ne - 1 - q;
      int m = -1;
      for (int k = A.i[i]; k < A.i[i + 1]; ++k) {
        const int c = A.j[k];
        if (c < ns || c >= ne || c == i) continue;
        if ((forward && c < i) || (!forward && c > i)) m = std::max(m, level[c]);
      }
      const int L = std::max(m + 1, floor_[i]);
      level[i] = L;
      nlev = std::max(nlev, L + 1);
      for (int k = A.i[i]; k < A.i[i + 1]; ++k) {
        const int c = A.j[k];
        if (c < ns || c >= ne || c == i) continue;
        if ((forward && c > i) || (!forward && c < i)) floor_[c] = std::max(floor_[c], L + 1);
      }
    }
    G.nlev[b] = nlev;
    auto& p = G.lptr[b];
    p.assign(nlev + 1, 0);
    for (int i = ns; i < ne; ++i) p[level[i] + 1]++;
    for (int l = 0; l < nlev; ++l) p[l + 1] += p[l];
    std::vector<int> pos(p.begin(), p.end() - 1);
    for (int i = ns; i < ne; ++i) G.byl[ns + pos[level[i]]++] = i;
  }
}
}  // namespace

int knob(int id);  // kernels.hip (tests' knobs)

// A step's stored entries: rows x width, padded to an even count so that every
// step (and every chunk of one, kernels.hip gs_kc) starts on an even entry,
// where the sweep's paired 8- / 16-byte loads are aligned
static int64_t gs_step_entries(int width, int rows) { return ((int64_t)width * rows + 1) & ~(int64_t)1; }

void build_gs_schedule(const CSR& A, const std::vector<int>& block_start, bool forward, GsSchedule& S,
                       int team_rows, bool with_tcol, const std::vector<double>* l1, const std::vector<int>* cf) {
  const int n = A.nrows, nb = (int)block_start.size() - 1;
  if (3 * (int64_t)n + std::max(0, A.ncols - n) >= INT_MAX)
    throw std::runtime_error("Gauss-Seidel schedule: too many rows or columns");
  S = GsSchedule();
  S.block_start = block_start;
  team_rows = std::max(1, team_rows);
  // rows a step, lanes a ring slot: 64.  Knob 14 = 16 takes 16 for the small
  // teams of wide operators (a quarter of the LDS ring: six workgroups a CU
  // instead of three, but steps of at most 16 rows): the cycle 6.99 against
  // 7.06 ms at 256^3, 47.5 against 44.3 ms at 512^3 (profiles/r06/17_gsring)
  const int rw = (team_rows <= 4 && knob(14) == 16) ? 16 : 64;
  S.ring_w = rw;
  // ring reach: values computed up to kGsFence steps earlier come from the LDS
  // ring, older ones from U.  Knob 11 (tests only) shortens it, which hands U
  // values out before the kernel's fences publish them: gs_schedule_self_check
  // must then refuse the schedule.
  const int reach = kGsFence - std::max(0, std::min(kGsFence - 1, knob(11)));
  GsLevels G;
  gs_levels(A, block_start, forward, G);
  // teams of consecutive blocks, about team_rows rows per team level
  std::vector<int> team_blk(1, 0);
  for (int b = 0; b < nb;) {
    int64_t rows = 0;
    int L = 0, e = b;
    for (; e < nb; ++e) {
      const int L2 = std::max(L, G.nlev[e]);
      const int64_t r2 = rows + (block_start[e + 1] - block_start[e]);
      if (e > b && r2 > (int64_t)team_rows * L2) break;
      rows = r2;
      L = L2;
    }
    team_blk.push_back(e);
    b = e;
  }
  const int nt = (int)team_blk.size() - 1;
  // the steps of team t in order: level by level, each level's rows in block
  // order, cut into chunks of at most 64
  auto for_each_step = [&](int t, const auto& fn) {
    int L = 0;
    for (int b = team_blk[t]; b < team_blk[t + 1]; ++b) L = std::max(L, G.nlev[b]);
    std::vector<int> rows;
    for (int l = 0; l < L; ++l) {
      rows.clear();
      for (int b = team_blk[t]; b < team_blk[t + 1]; ++b) {
        if (l >= G.nlev[b]) continue;
        const int ns = block_start[b];
        for (int q = G.lptr[b][l]; q < G.lptr[b][l + 1]; ++q) rows.push_back(G.byl[ns + q]);
      }
      for (size_t r0 = 0; r0 < rows.size(); r0 += rw) fn(rows.data() + r0, (int)std::min<size_t>(rw, rows.size() - r0));
    }
  };
  auto width_of = [&](const int* rows, int cnt) {
    int w = 0;
    for (int r = 0; r < cnt; ++r) w = std::max(w, A.i[rows[r] + 1] - A.i[rows[r]]);
    return w;
  };
  std::vector<int64_t> t_steps(nt + 1, 0), t_ent(nt + 1, 0);
#pragma omp parallel for schedule(dynamic, 4)
  for (int t = 0; t < nt; ++t) {
    int64_t ns = 0, ne = 0;
    for_each_step(t, [&](const int* rows, int cnt) {
      ++ns;
      ne += gs_step_entries(width_of(rows, cnt), cnt);
    });
    t_steps[t + 1] = ns;
    t_ent[t + 1] = ne;
  }
  for (int t = 0; t < nt; ++t) {
    S.max_steps = std::max(S.max_steps, (int)t_steps[t + 1]);
    t_steps[t + 1] += t_steps[t];
    t_ent[t + 1] += t_ent[t];
  }
  const int64_t nsteps = t_steps[nt], nent = t_ent[nt];
  if (nsteps > INT_MAX / 4) throw std::runtime_error("Gauss-Seidel schedule: too many steps");
  if (nent >= (int64_t)1 << 32) throw std::runtime_error("Gauss-Seidel schedule exceeds 2^32 entries");
  S.team_step.assign(nt + 1, 0);
  for (int t = 0; t <= nt; ++t) S.team_step[t] = (int)t_steps[t];
  S.step.assign((size_t)nsteps * 4, 0);
  par_assign(S.code, (size_t)nent, -1);
  par_assign(S.val, (size_t)nent, 0.0);
  if (with_tcol) par_assign(S.tcol, (size_t)nent, -1);
  S.rowmap.assign(n, 0);
  // per row: its position, step and lane
  std::vector<int> pos(n, 0), st_of(n, 0), ln_of(n, 0), blk_of(n, 0);
#pragma omp parallel for schedule(dynamic, 4)
  for (int t = 0; t < nt; ++t) {
    for (int b = team_blk[t]; b < team_blk[t + 1]; ++b)
      for (int i = block_start[b]; i < block_start[b + 1]; ++i) blk_of[i] = b;
    int64_t s = t_steps[t], e = t_ent[t];
    int r = block_start[team_blk[t]];  // a team's positions are its blocks' rows
    for_each_step(t, [&](const int* rows, int cnt) {
      const int w = width_of(rows, cnt);
      int* m = &S.step[(size_t)s * 4];
      m[0] = (int)(uint32_t)e;
      m[1] = r;
      m[2] = cnt;
      m[3] = w;
      for (int q = 0; q < cnt; ++q) {
        S.rowmap[r + q] = rows[q];
        pos[rows[q]] = r + q;
        st_of[rows[q]] = (int)s;
        ln_of[rows[q]] = q;
      }
      ++s;
      r += cnt;
      e += gs_step_entries(w, cnt);
    });
  }
#pragma omp parallel for schedule(dynamic, 4)
  for (int t = 0; t < nt; ++t) {
    const int s0 = (int)t_steps[t];
    for (int64_t sx = t_steps[t]; sx < t_steps[t + 1]; ++sx) {
      const int* m = &S.step[(size_t)sx * 4];
      const size_t base = (uint32_t)m[0];
      const int cnt = m[2];
      for (int q = 0; q < cnt; ++q) {
        const int i = S.rowmap[m[1] + q];
        const int ns = block_start[blk_of[i]], ne = block_start[blk_of[i] + 1];
        for (int k = A.i[i]; k < A.i[i + 1]; ++k) {
          const int c = A.j[k];
          const size_t p = base + (size_t)(k - A.i[i]) * cnt + q;
          S.val[p] = A.a[k];
          if (c >= n) {  // off-rank: the halo
            S.code[p] = 3 * n + (c - n);
            continue;
          }
          if (c < ns || c >= ne) {  // T
            S.code[p] = pos[c];
            continue;
          }
          if (with_tcol) S.tcol[p] = pos[c];
          const int d = (int)sx - st_of[c];
          if (c == i || d < 1) S.code[p] = n + pos[c];  // C
          else if (d <= reach) S.code[p] = -2 - (((st_of[c] - s0) % kGsRing) * rw + ln_of[c]);
          else S.code[p] = 2 * n + pos[c];  // U
        }
      }
    }
  }
  if (l1 && !l1->empty()) {
    S.l1.resize(n);
    for (int k = 0; k < n; ++k) S.l1[k] = (*l1)[S.rowmap[k]];
  }
  if (cf && !cf->empty()) {
    S.cf.resize(n);
    for (int k = 0; k < n; ++k) S.cf[k] = (*cf)[S.rowmap[k]];
  }
  for (int64_t s = 0; s < nsteps; ++s) S.max_width = std::max(S.max_width, S.step[(size_t)s * 4 + 3]);
  S.nteams = nt;
  S.nnz = A.i[n];
  S.rows_per_step = nsteps ? (double)n / nsteps : 0.0;
}

int gs_schedule_self_check(const CSR& A, int num_blocks, bool forward, bool use_l1, const std::vector<double>& l1,
                           std::string& msg, int team_rows, bool weighted) {
  const int n = A.nrows;
  const std::vector<int> bs = hypre_block_starts(n, num_blocks);
  GsSchedule S;
  build_gs_schedule(A, bs, forward, S, team_rows, weighted, &l1);
  const double w = 0.7, omega = 1.3;
  std::vector<double> f(n), u0(n), tmp(n);
  uint64_t st = 0x9e3779b97f4a7c15ULL;
  auto rnd = [&] { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (double)(st >> 11) / 9007199254740992.0 - 0.5; };
  for (int i = 0; i < n; ++i) { f[i] = rnd(); u0[i] = rnd(); tmp[i] = rnd(); }
  if (num_blocks == 1) tmp = u0;  // one block reads no tmp; keep the T and C vectors equal there
  // reference: sequential sweep per block (par_relax.c thread loops; weighted
  // forms par_relax.c:4544 / :1277): in-block columns read the iterate being
  // swept, off-block columns (and the weighted forms' Vtemp) the copy tmp
  std::vector<double> ref = u0;
  std::vector<int> blk(n);
  for (int b = 0; b < num_blocks; ++b)
    for (int i = bs[b]; i < bs[b + 1]; ++i) blk[i] = b;
  for (int b = 0; b < num_blocks; ++b) {
    const int ns = bs[b], ne = bs[b + 1];
    for (int q = 0; q < ne - ns; ++q) {
      const int i = forward ? ns + q : ne - 1 - q;
      const double scale = use_l1 ? l1[i] : A.a[A.i[i]];
      if (scale == 0.0) continue;
      double res = f[i], res0 = 0.0, res2 = 0.0;
      for (int k = A.i[i] + (use_l1 && !weighted ? 0 : 1); k < A.i[i + 1]; ++k) {
        const int c = A.j[k];
        const bool in = c >= ns && c < ne;
        if (weighted && in) {
          res0 -= A.a[k] * ref[c];
          res2 += A.a[k] * tmp[c];
        } else {
          res -= A.a[k] * (in ? ref[c] : tmp[c]);
        }
      }
      if (weighted) {
        double ui = ref[i];
        ui *= 1.0 - w * omega;
        ui += w * (omega * res + res0 + (1.0 - omega) * res2) / scale;
        ref[i] = ui;
      } else {
        ref[i] = use_l1 ? ref[i] + res / scale : res / scale;
      }
    }
  }
  // the kernel's view: C / T / F permuted into the sweep order, U stores
  // visible only as k_hybrid_gs makes them (a batch's stores are issued at its
  // last step and completed by the fence at the next batch's last step; the
  // pipelined sweep gathers step j's U values during step j - 1, so they must
  // have been fenced by the end of step j - 2), the LDS ring keeps the last
  // kGsRing steps
  std::vector<double> C(n), T(n), F(n), U(n, std::nan(""));
  std::vector<int> U_fenced(n, INT_MAX);  // the step whose end fence published U[k]
  std::vector<int> inv(n, -1);
  for (int k = 0; k < n; ++k) {
    if (S.rowmap[k] < 0 || S.rowmap[k] >= n || inv[S.rowmap[k]] >= 0) { msg = "rowmap is not a permutation"; return 1; }
    inv[S.rowmap[k]] = k;
    C[k] = u0[S.rowmap[k]];
    T[k] = tmp[S.rowmap[k]];
    F[k] = f[S.rowmap[k]];
  }
  std::vector<double> u = u0;  // the natural iterate (scattered stores)
  std::vector<int> seen(n, 0);
  const int k0 = use_l1 && !weighted ? 0 : 1;
  for (int t = 0; t < S.nteams; ++t) {
    const int s0 = S.team_step[t];
    const int rw = S.ring_w;
    if (rw != 16 && rw != 64) { msg = "ring width"; return 1; }
    std::vector<double> ring((size_t)kGsRing * rw, std::nan(""));
    std::vector<std::pair<int, double>> batch, issued;  // this batch's values; stores issued, not fenced
    for (int s = s0; s < S.team_step[t + 1]; ++s) {
      const int* m = &S.step[(size_t)s * 4];
      const size_t base = (uint32_t)m[0];
      const int cnt = m[2], width = m[3], j = s - s0;
      if (cnt < 1 || cnt > rw) { msg = "step rows out of range"; return 1; }
      if (base & 1) { msg = "step entries not on an even offset (paired loads)"; return 1; }
      std::vector<double> out(cnt);
      for (int q = 0; q < cnt; ++q) {
        const int kpos = m[1] + q, i = S.rowmap[kpos];
        if (i < 0 || i >= n) { msg = "row out of range"; return 1; }
        seen[i]++;
        const int ns = bs[blk[i]], ne = bs[blk[i] + 1];
        // the stored row must decode to the CSR row, entry for entry
        for (int k = 0; k < width; ++k) {
          const size_t p = base + (size_t)k * cnt + q;
          const int code = S.code[p];
          const int kk = A.i[i] + k;
          if (kk >= A.i[i + 1]) {
            if (code != -1) { msg = "padding slot holds a code"; return 1; }
            continue;
          }
          int c;
          bool in;
          if (code >= 3 * n) { msg = "halo code on a one-rank operator"; return 1; }
          else if (code >= n) c = S.rowmap[code % n], in = true;
          else if (code >= 0) c = S.rowmap[code], in = false;
          else if (code == -1) { msg = "padding inside a row"; return 1; }
          else {
            const int slot = -2 - code, rs = slot / rw, rl = slot % rw;
            int js = -1;
            for (int d = 1; d <= kGsFence; ++d)
              if (j - d >= 0 && (j - d) % kGsRing == rs) js = j - d;
            if (js < 0) { msg = "ring slot out of reach"; return 1; }
            const int* ms = &S.step[(size_t)(s0 + js) * 4];
            if (rl >= ms[2]) { msg = "ring lane out of range"; return 1; }
            c = S.rowmap[ms[1] + rl];
            in = true;
          }
          if (c != A.j[kk] || S.val[p] != A.a[kk]) { msg = "stored row differs from the CSR row"; return 1; }
          if (in != (c >= ns && c < ne)) { msg = "source kind disagrees with the block"; return 1; }
          if (weighted && S.tcol[p] != (in ? inv[c] : -1)) { msg = "tcol"; return 1; }
        }
        const double uo = C[kpos];
        const double scale = use_l1 ? S.l1[kpos] : S.val[base + q];
        out[q] = uo;
        if (scale == 0.0) continue;
        auto src = [&](int code) {
          if (code >= 2 * n) return U_fenced[code - 2 * n] <= j - 2 ? U[code - 2 * n] : std::nan("");
          if (code >= n) return C[code - n];
          if (code >= 0) return T[code];
          return ring[-2 - code];
        };
        double res = F[kpos], res0 = 0.0, res2 = 0.0;
        for (int k = k0; k < A.i[i + 1] - A.i[i]; ++k) {
          const size_t p = base + (size_t)k * cnt + q;
          const double a = S.val[p];
          if (weighted && S.tcol[p] >= 0) {
            res0 -= a * src(S.code[p]);
            res2 += a * T[S.tcol[p]];
          } else {
            res -= a * src(S.code[p]);
          }
        }
        if (weighted) {
          double ui = uo;
          ui *= 1.0 - w * omega;
          ui += w * (omega * res + res0 + (1.0 - omega) * res2) / scale;
          out[q] = ui;
        } else {
          out[q] = use_l1 ? uo + res / scale : res / scale;
        }
      }
      for (int q = 0; q < cnt; ++q) {
        batch.push_back({m[1] + q, out[q]});
        u[S.rowmap[m[1] + q]] = out[q];
        ring[(size_t)(j % kGsRing) * rw + q] = out[q];
      }
      if (j % kGsBatch == kGsBatch - 1 || s + 1 == S.team_step[t + 1]) {
        for (auto& pr : issued) {  // the fence completes the previous batch
          U[pr.first] = pr.second;
          U_fenced[pr.first] = j;
        }
        issued.swap(batch);                                // then this batch's stores are issued
        batch.clear();
      }
    }
  }
  for (int i = 0; i < n; ++i)
    if (seen[i] != 1) { msg = "row " + std::to_string(i) + " scheduled " + std::to_string(seen[i]) + " times"; return 1; }
  for (int i = 0; i < n; ++i)
    if (!(u[i] == ref[i])) {
      msg = "row " + std::to_string(i) + " differs from the sequential sweep";
      return 1;
    }
  msg = "ok: " + std::to_string(S.nteams) + " teams, " + std::to_string(S.team_step.back()) + " steps, max per team " +
        std::to_string(S.max_steps);
  return 0;
}

// hypre_gselim (sstruct_ls/gselim.h) forward elimination of the matrix alone:
// records each multiplier factor = A[j][k] * (1/A[k][k]) that the reference
// applies to x (mask = 1 where it applies one) and the eliminated matrix whose
// upper triangle the back substitution reads.
void gselim_factor(int n, const std::vector<double>& dense, std::vector<double>& L,
                   std::vector<unsigned char>& mask, std::vector<double>& U) {
  U = dense;
  L.assign((size_t)n * n, 0.0);
  mask.assign((size_t)n * n, 0);
  if (n <= 1) return;
  for (int k = 0; k < n - 1; ++k) {
    if (U[(size_t)k * n + k] != 0.0) {
      const double divA = 1.0 / U[(size_t)k * n + k];
      for (int j = k + 1; j < n; ++j) {
        if (U[(size_t)j * n + k] != 0.0) {
          const double factor = U[(size_t)j * n + k] * divA;
          for (int m = k + 1; m < n; ++m) U[(size_t)j * n + m] -= factor * U[(size_t)k * n + m];
          L[(size_t)j * n + k] = factor;
          mask[(size_t)j * n + k] = 1;
        }
      }
    }
  }
}

// Dense row-major copy of a (small) CSR operator, as hypre_GaussElimSetup
// (par_gauss_elim.c:84) assembles A_mat.
void csr_to_dense(const CSR& A, std::vector<double>& dense) {
  const int n = A.nrows;
  dense.assign((size_t)n * n, 0.0);
  for (int r = 0; r < n; ++r)
    for (int k = A.i[r]; k < A.i[r + 1]; ++k) dense[(size_t)r * n + A.j[k]] = A.a[k];
}

}  // namespace hve
