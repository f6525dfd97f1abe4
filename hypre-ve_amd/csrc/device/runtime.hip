// Device runtime: hierarchy upload, cycle driver, BoomerAMG solve loop and PCG.
// Control flow mirrors the reference routines cited per function; every
// arithmetic step runs in a HIP kernel (kernels.hip) -- there is no host path.
#include <hip/hip_runtime.h>

#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>


#include "../host/layout.hpp"
#include "runtime.hpp"

#include <cstdlib>

namespace hve {

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("HIP error '") + hipGetErrorString(e) + "' in " + what);
  }
}

template <typename T>
static T* dalloc(size_t n) {
  T* p = nullptr;
  if (n == 0) n = 1;
  // 256 B of slack past the end: the dictionary loop's clamped loads may read
  // one element past a stream's last slice (the value is never used)
  HVE_HIP(hipMalloc((void**)&p, n * sizeof(T) + 256));
  return p;
}
template <typename T>
static T* dupload(const T* h, size_t n) {
  T* p = dalloc<T>(n);
  if (n) HVE_HIP(hipMemcpy(p, h, n * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

// HVE_SELL_VALTAB=0 keeps 8-byte values in every layout (default 1).
static int sell_valtab_env() {
  static const int v = [] {
    const char* e = getenv("HVE_SELL_VALTAB");
    return e ? atoi(e) : 1;
  }();
  return v;
}

void DevSell::set_block_order(const std::vector<int>& stored_to_local, const std::vector<int64_t>& key) {
  if (key.empty() || nrows <= 0) return;
  // the row block one workgroup of the chosen loop runs (kernels.hip launch_sell)
  const int unit = col16 ? 64 * dict_group : slot_mask ? 256 * stencil_slices_per_wave() : (delta_like() || vidx16 || code16 || code32) ? 256 : (wide && !rowlen) ? 64 : 256;
  const int nb = (nrows + unit - 1) / unit;
  std::vector<int64_t> bk(nb);
  for (int b = 0; b < nb; ++b) {
    const int s = b * unit;
    const int loc = stored_to_local.empty() ? s : stored_to_local[s];
    bk[b] = (loc >= 0 && loc < (int)key.size()) ? key[loc] : (int64_t)loc;
  }
  std::vector<int> ord(nb);
  for (int b = 0; b < nb; ++b) ord[b] = b;
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return bk[a] < bk[b]; });
  bool ident = true;
  for (int b = 0; b < nb && ident; ++b) ident = ord[b] == b;
  if (ident) return;
  if (blk_map) (void)hipFree(blk_map);
  blk_map = dupload(ord.data(), ord.size());
  nblk = nb;
  blk_host = ord;
  build_wave_map();
}

// Stencil layout with one slice per wave: {stored slice, pattern} of every
// logical wave, in the traversal order of blk_map (kernels.hip k_sell_stencil).
void DevSell::build_wave_map() {
  if (wave_map) (void)hipFree(wave_map);
  wave_map = nullptr;
  nwave = 0;
  if (!slot_mask || stencil_slices_per_wave() != 1 || pat_host.empty()) return;
  const int nb = (nslices + 3) / 4;  // row blocks of 4 slices (256 rows)
  std::vector<int> m((size_t)nb * 4 * 2, 0);
  for (int lb = 0; lb < nb; ++lb) {
    const int b = (!blk_host.empty() && lb < (int)blk_host.size()) ? blk_host[lb] : lb;
    for (int w = 0; w < 4; ++w) {
      const int s = b * 4 + w;
      const size_t e = ((size_t)lb * 4 + w) * 2;
      m[e] = s < nslices ? s : -1;
      m[e + 1] = s < nslices ? pat_host[s] : 0;
    }
  }
  wave_map = dupload(m.data(), m.size());
  nwave = nb * 4;
}

static bool fine_grid(const CSR& A, int* nx, int* ny, int* nz, int shift = 0);

// Grid form of the stencil layout (k_grid_stencil) when the operator's rows
// are consecutive points of a grid in natural order with 64 | nx: stored row
// i is grid point i + shift (shift: whole planes; a rank's interior rows start
// one plane in), and the columns are the nlocal grid points.  Every used slot
// offset is shift + dz * nx * ny + dy * nx + dx with steps of at most one
// point, and no present lane's neighbour leaves the grid (so none wraps into
// another line or plane: the tile position of a point + offset is the
// neighbour's).  HVE_GRID_ZC (or knob 9, tests) sets the planes per workgroup
// (default: about 2048 workgroups).
bool DevSell::build_grid(const CSR& A, const std::vector<int>& so, const std::vector<int>& svi,
                         const std::vector<uint64_t>& sm, const std::vector<double>& tab, int shift, int nlocal) {
  int nx, ny, nzs;
  if (!fine_grid(A, &nx, &ny, &nzs, shift)) return false;
  const int64_t P = (int64_t)nx * ny;
  if (nx % 64 || ny < 3 || nlocal % P || shift % P || (int64_t)nx * ny * nzs != A.nrows) return false;
  const int nz = (int)(nlocal / P);
  if (nz < 3 || shift / P + nzs > nz) return false;
  if (!grid_stencil_addressable(nx, ny, nz)) return false;  // the per-slice loop takes it
  if (csr_max_col(A) >= nlocal) return false;  // a halo column
  const int W = stencil_w;
  std::vector<GSlot> gs((size_t)npat * W + 16);
  for (auto& g : gs) g = GSlot{0, 0.0, 0, 0, 0, 0};
  for (int pt = 0; pt < npat; ++pt)
    for (int k = 0; k < W; ++k) {
      const size_t e = (size_t)pt * W + k;
      if (!sm[e]) continue;
      bool found = false;
      for (int dz = -1; dz <= 1 && !found; ++dz)
        for (int dy = -1; dy <= 1 && !found; ++dy)
          for (int dx = -1; dx <= 1 && !found; ++dx)
            if (shift + dz * P + (int64_t)dy * nx + dx == so[e]) {
              gs[e] = GSlot{sm[e], tab[svi[e]], dz, dy * (64 + 2) + dx, 0, 0};
              found = true;
            }
      if (!found) return false;
    }
  int ok = 1;
#pragma omp parallel for schedule(static) reduction(min : ok)
  for (int s = 0; s < nslices; ++s) {
    const int64_t r0 = (int64_t)s * 64 + shift;
    const int x0 = (int)(r0 % nx), y = (int)((r0 / nx) % ny), z = (int)(r0 / P);
    const int pt = pat_host[s];
    for (int k = 0; k < W; ++k) {
      const GSlot& g = gs[(size_t)pt * W + k];
      if (!g.mask) continue;
      const int dx = ((g.dxy + 67) % 66) - 1, dy = (g.dxy - dx) / 66;
      if (z + g.dz < 0 || z + g.dz >= nz || y + dy < 0 || y + dy >= ny) ok = 0;
      if (dx < 0 && x0 == 0 && (g.mask & 1ull)) ok = 0;
      if (dx > 0 && x0 + 64 == nx && (g.mask >> 63)) ok = 0;
    }
  }
  if (!ok) return false;
  static const int zc_env = [] {
    const char* e = getenv("HVE_GRID_ZC");
    return e ? atoi(e) : 0;
  }();
  const int64_t txy = (int64_t)(nx / 64) * ((ny + grid_stencil_ty() - 1) / grid_stencil_ty());
  const int zc = knob(9) > 0 ? knob(9) : zc_env > 0 ? zc_env
               : (int)std::max<int64_t>(2, std::min<int64_t>(64, nzs * txy / 2048));
  gslot = dupload(gs.data(), gs.size());
  gnx = nx; gny = ny; gnz = nz; gzc = std::min(zc, nzs);
  gz0 = (int)(shift / P);
  gz1 = gz0 + nzs;
  if (getenv("HVE_LAYOUT_LOG"))
    fprintf(stderr, "[layout] grid stencil %dx%dx%d (planes %d..%d), %d planes a workgroup, %d workgroups\n", nx, ny,
            nz, gz0, gz1 - 1, gzc, grid_stencil_blocks(view()));
  return true;
}

// HVE_SETUP_T: host stages of an operator's layout construction and upload
namespace {
struct SetupLap {
  bool on = getenv("HVE_SETUP_T") != nullptr;
  double t = now();
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void operator()(const char* what) {
    if (!on) return;
    const double n = now();
    fprintf(stderr, "[upload]   %-32s %.3fs\n", what, n - t);
    t = n;
  }
};
}  // namespace

void DevSell::upload(const CSR& A, const std::vector<int>& rowmap_h, int policy, const std::vector<int64_t>* key,
                     const Coded* coded, const std::vector<int64_t>* tile) {
  SetupLap lap;
  release();
  // Offset-coded layout (P_0 / R_0 of a grid hierarchy: 25 offsets, ~1200
  // weights, so an entry is one 16-bit code, 2 B instead of 6) where the grid
  // context is given, the operator is large and the codes build.  Measured on
  // MI355X (k_sell_code against padded + 16-bit values): R_0 at 512^3 1.46 vs
  // 1.62 ms, at 256^3 0.160-0.176 vs 0.183; P_0 1.62 vs 1.29 ms and 0.19-0.23
  // vs 0.156 (its column needs a second dependent gather, through the fine ->
  // coarse map), so by default only restrictions take it.  Both are bound by
  // their scattered x gathers, not by the bytes.  HVE_SELL_CODED=0 turns it
  // off, 2 also on P; policy 12 forces it wherever it builds.
  static const int coded_env = [] {
    const char* e = getenv("HVE_SELL_CODED");
    return e ? atoi(e) : 1;
  }();
  const bool coded_auto = coded_env == 2 || (coded_env == 1 && coded && coded->anc);
  if (coded && A.nnz() > 0 && ((policy == 0 && coded_auto && A.nrows >= (1 << 18)) || policy == 12 || policy == 15)) {
    static const std::vector<int> none;
    std::vector<int> sp, ot;
    hvec<unsigned short> cd;
    std::vector<double> tab;
    int vb = 0;
    if (build_sell_coded_host(A, rowmap_h, coded->anc ? *coded->anc : none, coded->colpos ? *coded->colpos : none,
                              coded->cmap ? *coded->cmap : none, sp, cd, ot, tab, vb)) {
      nrows = A.nrows;
      ncols = A.ncols;
      nslices = (int)sp.size() - 1;
      nnz = A.nnz();
      nnz_pad = (int64_t)sp.back();
      batch = 8;
      pipe = 1;
      // Policy 15: restrictions (anchors, no position map) in the jagged,
      // product-parallel form (k_code_pw), no padding stored or gathered.  Not
      // the default: R_0 at 512^3 took 1.434-1.603 ms over its launch variants
      // against 1.405 ms for the padded loop on one box (profiles/r06/11_r0wpc).
      std::vector<int> jperm;
      if ((!coded->cmap || coded->cmap->empty()) && coded->anc && policy == 15) {
        std::vector<int> sp2, rl;
        hvec<unsigned short> cd2;
        jag_codes_from_padded(A, sp, cd, jperm, sp2, rl, cd2);
        sp.swap(sp2);
        cd.swap(cd2);
        nnz_pad = nnz;
        rowlen = dupload(rl.data(), rl.size());
      }
      slice_ptr = dupload(sp.data(), sp.size());
      code16 = dupload(cd.data(), cd.size());
      otab = dupload(ot.data(), ot.size());
      notab = (int)ot.size();
      vbits = vb;
      vtab = dupload(tab.data(), tab.size());
      nvtab = (int)tab.size();
      if (coded->anc && !coded->anc->empty()) {
        anc = dupload(coded->anc->data(), coded->anc->size());
        anc_n = (int64_t)coded->anc->size();
      }
      if (coded->cmap && !coded->cmap->empty()) {
        cmap = dupload(coded->cmap->data(), coded->cmap->size());
        cmap_n = (int64_t)coded->cmap->size();
      }
      if (getenv("HVE_LAYOUT_LOG"))
        fprintf(stderr, "[layout] coded rows=%d offsets=%d values=%d vbits=%d pad=%.2f\n", A.nrows, notab, nvtab, vbits,
                (double)nnz_pad / std::max<int64_t>(1, nnz));
      std::vector<int> map = rowmap_h;
      if (!jperm.empty()) {  // stored (sorted) row -> local row
        map.resize(A.nrows);
        for (int i = 0; i < A.nrows; ++i) map[i] = rowmap_h.empty() ? jperm[i] : rowmap_h[jperm[i]];
      }
      if (!map.empty()) {
        bool ident = true;
        for (int i = 0; i < A.nrows && ident; ++i) ident = map[i] == i;
        if (!ident) rowmap = dupload(map.data(), map.size());
      }
      stored_map = map;
      if (key) set_block_order(map, *key);
      return;
    }
  }
  std::vector<int> sp, perm;
  hvec<int> col;
  hvec<double> val;
  // Sort rows inside windows (SELL-C-sigma) only where the plain layout pads
  // noticeably: the Galerkin levels' rows range over 7..150 entries, the
  // finest 7-point operator is nearly uniform and keeps contiguous rows.
  // Measured on MI355X (256^3 Poisson, PMIS/ext+i): sorting a 1024-row window
  // cut level-1 padding from 1.40x to 1.03x but slowed its SpMV 745 -> 1073 us,
  // because a wave's 64 rows then gather x from a 16x wider range, so it is
  // off (build_sell_host keeps the sigma parameter).
  constexpr int sigma_env = 0;
  // Jagged layout (no stored padding) for large operators with long rows and
  // more than 10% padding: level-1/2 Galerkin A and R = P^T.  Measured on
  // MI355X (256^3, PMIS/ext+i): R_0 -16%, A_1 -15%, R_1 -14%, A_2 -4%; but
  // P (<= 4 entries a row: the 8 B/row of row map + length outweigh the
  // padding) +14..25%, and operators below ~2^18 rows, which are latency-bound,
  // +10..20%.  HVE_SELL_JAG=0|1 forces it off / on for experiments.
  static const int jag_env = [] {
    const char* e = getenv("HVE_SELL_JAG");
    return e ? atoi(e) : -1;
  }();
  const int64_t pad0 = A.nnz() > 0 ? sell_padded_nnz(A, 0) : 0;
  lap("padding count");
  // Small operators (coarse levels) run one workgroup per slice with the
  // products formed in parallel (k_sell_wide): in the lane-per-row loop they
  // are latency-bound.  Measured on MI355X (256^3): every operator below 2^18
  // rows 40-50% faster, level-2 A (700k rows, 70 entries a row) 186 -> 170 us;
  // level-1 R (700k rows, 26 a row) and everything larger is slower.
  // HVE_SELL_WIDE_ROWS moves the 2^18 bound (0 = never).
  static const int wide_rows = [] {
    const char* e = getenv("HVE_SELL_WIDE_ROWS");
    return e ? atoi(e) : (1 << 18);
  }();
  const double avg_len = A.nrows > 0 ? (double)A.nnz() / A.nrows : 0.0;
  wide = (A.nrows > 0 && avg_len >= 4.0 &&
          (A.nrows < wide_rows || (wide_rows == (1 << 18) && A.nrows < (1 << 20) && avg_len >= 40.0))) ? 1 : 0;
  bool jag = wide ? false : jag_env >= 0 ? (jag_env != 0 && A.nnz() > 0)
                                : (pad0 > A.nnz() + A.nnz() / 10 && A.nnz() >= 8LL * A.nrows && A.nrows >= (1 << 18));
  pw = (jag && sell_pw()) ? 1 : 0;
  // Dictionary layout (x-tile in LDS, one wave per slice) for large operators
  // with long rows: level-1 A and R, level-2 A.  Measured on MI355X (256^3):
  // A_1 516 -> 466 us, R_1 85 -> 76, A_2 177 (wide) -> 135; R_0 (10 entries
  // a row) 203 -> 211 and every operator below 2^18 rows 2-3x slower, so those
  // keep the jagged / wide loops.  HVE_SELL_DICT=0 turns it off, 1 forces it
  // wherever the jagged layout is chosen, 2 also in place of the wide loop.
  static const int dict_env = [] {
    const char* e = getenv("HVE_SELL_DICT");
    return e ? atoi(e) : -1;
  }();
  // configs[4] (anisotropic, aggressive coarsening, 256^3): A_1 has 15.9
  // entries a row, 0.093 ms as a dictionary against 0.105 jagged.
  bool use_dict = A.nnz() > 0 &&
                  (dict_env < 0 ? (A.nrows >= (1 << 18) && avg_len >= 12.0)
                                : ((dict_env >= 1 && jag) || (dict_env >= 2 && wide)));
  // With 16-bit value indices a padding slot costs 6 B instead of 12, and the
  // padded layout's natural row order gathers x better than the sorted jagged
  // one: R_0 at 256^3 187 us padded+vt16 against 197 jagged+vt16 (202 jagged).
  if (policy == 0 && jag && !pw && sell_valtab_env() != 0) {
    hvec<unsigned short> probe;
    std::vector<double> probe_tab;
    if (build_value_table16(A.a.data(), A.a.size(), 4096, probe, probe_tab)) jag = false;
    lap("value-table probe");
  }
  if (policy != 0) {  // forced (tests): every loop gives the same bits
    wide = policy == 3 ? 1 : 0;
    jag = (policy == 2 || policy == 4 || policy == 9) && A.nnz() > 0;
    pw = policy == 4 && jag;
    use_dict = (policy == 5 || policy == 10 || policy == 14) && A.nnz() > 0;
  }
  // 16-bit column deltas against per-(slice, slot) bases where the padded
  // layout stays and rows are stencil-long (the finest A): 10 B an entry
  // instead of 12.  Measured on MI355X (256^3): A_0 317 -> 302 us; P (<= 4
  // entries a row) no gain at level 0 and 59 -> 72 us at level 1, so P keeps
  // 32-bit columns.  HVE_SELL_DELTA=0 turns it off, 1 also on short rows.
  static const int delta_env = [] {
    const char* e = getenv("HVE_SELL_DELTA");
    return e ? atoi(e) : -1;
  }();
  // Short-row operators (P) take it only together with a value table.
  const bool short_rows = avg_len < 5.0 && delta_env != 1;
  // A long-row operator with few distinct values (the 27-point stencil: 27
  // slots, 2 values) takes delta + 8-bit value table (3 B an entry) ahead of
  // the dictionary (10 B an entry), when the table builds.
  const bool delta_before_dict = policy == 0 && use_dict && !jag && !wide && delta_env != 0 && sigma_env == 0 &&
                                 sell_valtab_env() != 0;
  bool use_delta = (A.nnz() > 0 && !wide && !jag && !use_dict && delta_env != 0 && sigma_env == 0) || delta_before_dict;
  if (policy != 0) use_delta = (policy == 6 || policy == 7 || policy == 11) && A.nnz() > 0;
  // A constant-coefficient stencil (every slot of a slice one neighbour offset
  // and one value for all its lanes) takes the slot-uniform layout: nothing
  // stored per entry, so an application streams only the vectors.
  // HVE_SELL_STENCIL=0 turns it off; policy 11 forces it where it builds.
  static const int stencil_env = [] {
    const char* e = getenv("HVE_SELL_STENCIL");
    return e ? atoi(e) : 1;
  }();
  if (use_delta && !short_rows && ((policy == 0 && stencil_env != 0) || policy == 11)) {
    std::vector<int> so, svi;
    std::vector<uint64_t> sm;
    std::vector<double> tab;
    std::vector<int> spat;
    int sw = 0;
    if (build_sell_stencil_host(A, 64, sw, spat, so, svi, sm, tab)) {
      nrows = A.nrows;
      ncols = A.ncols;
      nslices = (A.nrows + 63) / 64;
      nnz = A.nnz();
      nnz_pad = (int64_t)nslices * 64 * sw;
      stencil_w = sw;
      batch = 8;
      pipe = 0;
      wide = 0;
      pw = 0;
      slice_pat = dupload(spat.data(), spat.size());
      pat_host = spat;
      npat = (int)((so.size() - 16) / std::max(sw, 1));
      if (getenv("HVE_LAYOUT_LOG"))
        fprintf(stderr, "[layout] stencil rows=%d width=%d patterns=%d values=%zu\n", A.nrows, sw, npat, tab.size());
      slot_base = dupload(so.data(), so.size());
      slot_vi = dupload(svi.data(), svi.size());
      slot_mask = dupload(sm.data(), sm.size());
      vtab = dupload(tab.data(), tab.size());
      nvtab = (int)tab.size();
      // the grid form also where the rows are a run of whole planes (a
      // rank's interior rows): stored row i = local row i + shift
      int shift = 0;
      bool affine = true;
      if (!rowmap_h.empty()) {
        bool ident = true;
        for (int i = 0; i < A.nrows && ident; ++i) ident = rowmap_h[i] == i;
        if (!ident) rowmap = dupload(rowmap_h.data(), rowmap_h.size());
        shift = A.nrows > 0 ? rowmap_h[0] : 0;
        for (int i = 0; i < A.nrows && affine; ++i) affine = rowmap_h[i] == i + shift;
      }
      if (affine) build_grid(A, so, svi, sm, tab, shift, grid_nlocal > 0 ? grid_nlocal : A.nrows);
      stored_map = rowmap_h;
      if (key) set_block_order(rowmap_h, *key);
      if (!wave_map) build_wave_map();
      return;
    }
    sp.clear();
  }
  if (use_delta) {
    hvec<short> dc;
    std::vector<int> sb;
    hvec<unsigned char> vi_probe;
    std::vector<double> tab_probe;
    bool delta_ok = build_sell_delta_host(A, sp, sb, dc, val);
    if (delta_ok && delta_before_dict && !build_value_table(val.data(), val.size(), 256, vi_probe, tab_probe)) delta_ok = false;
    if (!delta_ok && delta_before_dict) {
      sp.clear();
      val.clear();
      goto dict;
    }
    if (delta_ok) {
      nrows = A.nrows;
      ncols = A.ncols;
      nslices = (int)sp.size() - 1;
      nnz = A.nnz();
      nnz_pad = (int64_t)sp.back();
      batch = (nslices > 0 && pad0 > (int64_t)nslices * 64 * 8) ? 16 : 8;
      pipe = 0;
      wide = 0;
      pw = 0;
      slice_ptr = dupload(sp.data(), sp.size());
      dcol = dupload(dc.data(), dc.size());
      slot_base = dupload(sb.data(), std::max<size_t>(1, sb.size()));
      // Few distinct values (a constant-coefficient stencil): 8-bit indices
      // into a table of them, 3 B an entry in all.  HVE_SELL_VALTAB=0 keeps
      // 8-byte values.
      const int vt_env = sell_valtab_env();
      // Up to 4096 distinct values (P of the 7-point hierarchy: ~1200): 16-bit
      // indices, the table (<= 32 KiB) in LDS.
      hvec<unsigned char> vi;
      hvec<unsigned short> vi16;
      std::vector<double> tab;
      const bool try_vt = (vt_env != 0 || policy == 7) && policy != 6;
      if (try_vt && build_value_table(val.data(), val.size(), 256, vi, tab)) {
        vidx = dupload(vi.data(), vi.size());
      } else if (try_vt && build_value_table16(val.data(), val.size(), 4096, vi16, tab)) {
        vidx16 = dupload(vi16.data(), vi16.size());
      } else if (short_rows && policy == 0) {
        release();  // no gain without a value table: plain layout
        goto plain;
      } else {
        this->val = dupload(val.data(), val.size());
      }
      if (!tab.empty()) {
        vtab = dupload(tab.data(), tab.size());
        nvtab = (int)tab.size();
      }
      if (nslices > 0 && pad0 <= (int64_t)nslices * 64 * 4) batch = 4;  // rows of <= 4 entries
      if (!rowmap_h.empty()) {
        bool ident = true;
        for (int i = 0; i < A.nrows && ident; ++i) ident = rowmap_h[i] == i;
        if (!ident) rowmap = dupload(rowmap_h.data(), rowmap_h.size());
      }
      stored_map = rowmap_h;
      if (key) set_block_order(rowmap_h, *key);
      return;
    }
  plain:
    sp.clear();
    val.clear();
  }
dict:
  if (use_dict) {
    // rows in compact grid tiles (DevAMG::build tile_keys): the groups of
    // consecutive slices share more of their columns
    std::vector<int> pre;
    if (tile && !tile->empty()) {
      std::vector<int64_t> tk(A.nrows);
#pragma omp parallel for schedule(static)
      for (int r = 0; r < A.nrows; ++r) {
        const int g = rowmap_h.empty() ? r : rowmap_h[r];
        tk[r] = g < (int)tile->size() ? (*tile)[g] : (int64_t)g;
      }
      sort_rows_by_key(tk, pre);
      lap("dict tile order");
    }
    const std::vector<int>* prep = pre.empty() ? nullptr : &pre;
    hvec<unsigned short> c16;
    std::vector<int> dp, dc, rl2;
    int mxd = 0;
    // Square operators: one dictionary per workgroup of 4 slices
    // (neighbouring slices share most of their columns; A1 at 256^3 419 vs
    // 472 us) where it fits 64 KiB of LDS, else per slice.  Restrictions keep
    // one per slice (R1 76 vs 83 us grouped).  HVE_SELL_DICT_GROUP=1|4 forces it.
    static const int group_env = [] {
      const char* e = getenv("HVE_SELL_DICT_GROUP");
      return e ? atoi(e) : 0;
    }();
    int group = (group_env == 1 || group_env == 2 || group_env == 4 || group_env == 8) ? group_env
                                                                                     : (A.nrows == A.ncols ? 4 : 1);
    // Range dictionary (square operators: the x-tile as at most 63 column
    // ranges, copied instead of gathered through a 4-byte index list) where
    // the ranges cover at most 1.5x the distinct columns.  Measured on MI355X:
    // A_1 at 256^3 411 vs 412 us, at 512^3 4.31 vs 3.66 ms (the larger tiles
    // cost occupancy), so only policy 10 takes it (tests).
    const bool try_ranges = policy == 10;
    bool built = false, ranges = false;
    if (try_ranges) {
      built = build_sell_dict_host(A, group > 1 ? 8192 : 4096, group, perm, sp, rl2, c16, val, dp, dc, mxd, 63,
                                   policy == 10 ? 1e30 : 1.5, prep);
      if (!built && group > 1 && group_env == 0) {
        group = 1;
        built = build_sell_dict_host(A, 4096, 1, perm, sp, rl2, c16, val, dp, dc, mxd, 63, policy == 10 ? 1e30 : 1.5,
                                     prep);
      }
      ranges = built;
      if (!built) group = (group_env == 1 || group_env == 2 || group_env == 4 || group_env == 8) ? group_env
                                                                                          : (A.nrows == A.ncols ? 4 : 1);
    }
    if (!built && policy != 10) {
      built = build_sell_dict_host(A, group > 1 ? 8192 : 4096, group, perm, sp, rl2, c16, val, dp, dc, mxd, 0, 1.5,
                                   prep);
      if (!built && group > 1 && group_env == 0) {
        group = 1;
        built = build_sell_dict_host(A, 4096, 1, perm, sp, rl2, c16, val, dp, dc, mxd, 0, 1.5, prep);
      }
    }
    if (built) {
      lap("dict build");
      dict_group = group;
      dict_ranges = ranges ? 1 : 0;
      nrows = A.nrows;
      ncols = A.ncols;
      nslices = (int)sp.size() - 1;
      nnz = A.nnz();
      nnz_pad = nnz;
      batch = (nslices > 0 && pad0 > (int64_t)nslices * 64 * 8) ? 16 : 8;
      pipe = 1;
      wide = 0;
      pw = 0;
      dmax = std::max(1, mxd);
      if (getenv("HVE_LAYOUT_LOG"))
        fprintf(stderr, "[layout] dict rows=%d group=%d dmax=%d mean dictionary=%.0f\n", A.nrows, group, dmax,
                (double)dc.size() / std::max<size_t>(1, dp.size() - 1));
      rowlen = dupload(rl2.data(), rl2.size());
      slice_ptr = dupload(sp.data(), sp.size());
      // one-slice dictionaries (restrictions) whose values take at most 4096
      // bit patterns: 16-bit indices into a table staged in LDS after the
      // x-tile, 4 B an entry instead of 10.  Measured on R_0 at 512^3 (its
      // 64-row slices hold 573 distinct fine columns, 9 a row): 3.73 ms
      // against 1.59 for the offset-coded layout, so it is taken only under
      // the forced dictionary policy (5, tested bitwise).
      constexpr int dict_vt_env = 0;
      hvec<unsigned short> vi16;
      std::vector<double> tab;
      if (group == 1 && !ranges && !relax_ops && (dict_vt_env != 0 || policy == 5) && sell_valtab_env() != 0 &&
          (size_t)(dmax + 4096) * sizeof(double) <= 64 * 1024 && build_value_table16(val.data(), val.size(), 4096, vi16, tab)) {
        vidx16 = dupload(vi16.data(), vi16.size());
        vtab = dupload(tab.data(), tab.size());
        nvtab = (int)tab.size();
        col16 = dupload(c16.data(), c16.size());
      } else {
        // Lane-packed streams (k_sell_dictw): one 16-B load brings a lane two
        // values or eight columns of its row, instead of one 8-B value load and
        // one 2-B column load per entry (the per-entry loop is address-bound:
        // TA busy 84 % on A_1, profiles/r05/02_opprof).  HVE_DICT_WIDE=0 keeps
        // the per-entry streams; range dictionaries keep them, and policy 14
        // forces them (tests).
        static const int wide_env = [] {
          const char* e = getenv("HVE_DICT_WIDE");
          return e ? atoi(e) : 1;
        }();
        std::vector<int> wp;
        hvec<unsigned short> cw;
        hvec<double> vw;
        if (!ranges && (group == 1 || group == 4) && wide_env != 0 && policy != 14 && pack_dict_wide(sp, rl2, c16, val, wp, cw, vw)) {
          wptr = dupload(wp.data(), wp.size());
          col16 = dupload(cw.data(), cw.size());
          this->val = dupload(vw.data(), vw.size());
          wval_n = (int64_t)vw.size();
          wcol_n = (int64_t)cw.size();
          lap("dict lane packing");
        } else {
          col16 = dupload(c16.data(), c16.size());
          this->val = dupload(val.data(), val.size());
        }
      }
      dict_ptr = dupload(dp.data(), dp.size());
      dict = dupload(dc.data(), std::max<size_t>(1, dc.size()));
      ndict = (int64_t)dc.size();  // ints: distinct columns, or 2 per range pair
      std::vector<int> map(A.nrows);
      for (int i = 0; i < A.nrows; ++i) map[i] = rowmap_h.empty() ? perm[i] : rowmap_h[perm[i]];
      bool ident = true;
      for (int i = 0; i < A.nrows && ident; ++i) ident = map[i] == i;
      if (!ident) rowmap = dupload(map.data(), map.size());
      if (!ident) stored_map = map;
      if (key) set_block_order(map, *key);
      lap("dict upload + row map");
      return;
    }
    perm.clear();  // a slice has too many distinct columns: fall back
  }
  std::vector<int> rl;
  if (jag) {
    build_sell_jagged_host(A, perm, sp, rl, col, val);
  } else {
    const int sigma = (sigma_env > 0 && A.nnz() > 0 && pad0 > A.nnz() + A.nnz() / 20) ? sigma_env : 0;
    build_sell_host(A, sigma, perm, sp, col, val);
  }
  lap(jag ? "jagged build" : "padded build");
  nrows = A.nrows;
  ncols = A.ncols;
  nslices = (int)sp.size() - 1;
  nnz = A.nnz();
  nnz_pad = (int64_t)col.size();
  // Long rows (Galerkin A, R = P^T) run 16 entries per load batch, short ones
  // (P: <= P_max_elmts, the finest 7-point A) 8: measured on MI355X, 16 was
  // 8% faster on level-1 A and R and 10% slower on P.
  batch = (nslices > 0 && pad0 > (int64_t)nslices * 64 * 8) ? 16 : 8;
  // Software pipelining (next batch's loads issued before this batch's adds)
  // measured 11% faster on level-1 A, 4-7% on R and P, ~2% slower on the
  // finest 7-point A (one batch per row): on except for mid-length short rows.
  // The jagged loop is always pipelined.
  const double avg_row = nrows > 0 ? (double)nnz / nrows : 0.0;
  pipe = (jag || batch == 16 || avg_row < 5.0) ? 1 : 0;
  if (jag) rowlen = dupload(rl.data(), rl.size());
  slice_ptr = dupload(sp.data(), sp.size());
  // 16-bit indices into the operator's distinct values where at most 4096
  // occur (P and R of the 7-point hierarchy at every size: ~1200), off for the
  // workgroup-per-slice loop of small operators.  HVE_SELL_VALTAB=0 turns it off.
  hvec<unsigned short> vi16;
  std::vector<double> tab;
  const bool try_vt16 = policy == 8 || policy == 9 || policy == 13 || (policy == 0 && !wide && sell_valtab_env() != 0);
  const bool vt_ok = try_vt16 && A.nnz() > 0 && build_value_table16(val.data(), val.size(), 4096, vi16, tab);
  lap("value table");
  if (vt_ok) {
    vtab = dupload(tab.data(), tab.size());
    nvtab = (int)tab.size();
    wide = 0;
    pipe = 1;
    // Packed 32-bit entries (column - slice base, value index): 4 B instead of
    // 6 where every slice's column span fits the bits the value index leaves
    // (P_0: ~1200 values, 21 bits of span).  Measured on MI355X at 512^3:
    // P_0 1.32 -> 0.99 ms; R_0 1.63 ms, no better than the offset-coded 1.62
    // (which it takes first).  Interpolation and restriction only (coded
    // given: the loop has no Jacobi epilogue).  HVE_SELL_PACK=0 turns it off;
    // policy 13 forces it.
    static const int pack_env = [] {
      const char* e = getenv("HVE_SELL_PACK");
      return e ? atoi(e) : 1;
    }();
    hvec<unsigned> c32;
    std::vector<int> sbase;
    if (!jag && coded && (policy == 13 || (policy == 0 && pack_env != 0)) && pack_sell_codes(sp, col, vi16, nvtab, c32, sbase, vbits)) {
      code32 = dupload(c32.data(), c32.size());
      slot_base = dupload(sbase.data(), sbase.size());
    } else {
      this->col = dupload(col.data(), col.size());
      vidx16 = dupload(vi16.data(), vi16.size());
    }
  } else {
    this->col = dupload(col.data(), col.size());
    this->val = dupload(val.data(), val.size());
  }
  // stored row i -> local output row: subset map composed with the sort order
  std::vector<int> map(A.nrows);
  for (int i = 0; i < A.nrows; ++i) {
    const int r = perm.empty() ? i : perm[i];
    map[i] = rowmap_h.empty() ? r : rowmap_h[r];
  }
  bool ident = true;
  for (int i = 0; i < A.nrows && ident; ++i) ident = map[i] == i;
  if (!ident) rowmap = dupload(map.data(), map.size());
  if (!ident) stored_map = map;
  if (key) set_block_order(map, *key);
  lap("pack / upload / row map");
}
// A rank operator's rows in local order (interior and boundary merged, each
// row's entries in stored order, columns in the [local | halo] space).
static CSR merged_rows(const RankOp& op, int n) {
  CSR M;
  M.resize_rows(n, std::max(op.interior.ncols, op.boundary.ncols));
  for (int part = 0; part < 2; ++part) {
    const CSR& A = part == 0 ? op.interior : op.boundary;
    const std::vector<int>& map = part == 0 ? op.map_int : op.map_bnd;
    for (int i = 0; i < A.nrows; ++i) M.i[(map.empty() ? i : map[i]) + 1] = A.i[i + 1] - A.i[i];
  }
  for (int i = 0; i < n; ++i) M.i[i + 1] += M.i[i];
  M.j.resize(M.i[n]);
  M.a.resize(M.i[n]);
  for (int part = 0; part < 2; ++part) {
    const CSR& A = part == 0 ? op.interior : op.boundary;
    const std::vector<int>& map = part == 0 ? op.map_int : op.map_bnd;
    for (int i = 0; i < A.nrows; ++i) {
      const int g = map.empty() ? i : map[i];
      std::copy(A.j.begin() + A.i[i], A.j.begin() + A.i[i + 1], M.j.begin() + M.i[g]);
      std::copy(A.a.begin() + A.i[i], A.a.begin() + A.i[i + 1], M.a.begin() + M.i[g]);
    }
  }
  return M;
}

// True when every row's stored l1 norm equals, bit for bit, the sum of |a_ij|
// over its stored entries in order, negated for a negative first entry
// (compute_l1_norms option 1 without C/F restriction): the device kernels can
// then form it on the fly instead of streaming it.
static bool l1_on_the_fly(const RankOp& op, const std::vector<double>& l1) {
  static const bool off = [] {
    const char* e = getenv("HVE_L1_FLY");
    return e && atoi(e) == 0;
  }();
  if (off) return false;
  return l1_rows_match(op.interior, op.map_int, l1) && l1_rows_match(op.boundary, op.map_bnd, l1);
}

void DevSell::release() {
  if (slice_ptr) (void)hipFree(slice_ptr);
  if (col) (void)hipFree(col);
  if (val) (void)hipFree(val);
  if (rowmap) (void)hipFree(rowmap);
  if (rowlen) (void)hipFree(rowlen);
  if (col16) (void)hipFree(col16);
  if (dict_ptr) (void)hipFree(dict_ptr);
  if (dict) (void)hipFree(dict);
  if (dcol) (void)hipFree(dcol);
  if (slot_base) (void)hipFree(slot_base);
  if (code32) (void)hipFree(code32);
  code32 = nullptr;
  if (vidx) (void)hipFree(vidx);
  if (vidx16) (void)hipFree(vidx16);
  if (vtab) (void)hipFree(vtab);
  if (slot_vi) (void)hipFree(slot_vi);
  if (slot_mask) (void)hipFree(slot_mask);
  if (slice_pat) (void)hipFree(slice_pat);
  if (blk_map) (void)hipFree(blk_map);
  blk_map = nullptr;
  nblk = 0;
  blk_host.clear();
  pat_host.clear();
  pat_host.shrink_to_fit();
  if (wave_map) (void)hipFree(wave_map);
  wave_map = nullptr;
  nwave = 0;
  stored_map.clear();
  stored_map.shrink_to_fit();
  dcol = nullptr; slot_base = nullptr; vidx = nullptr; vidx16 = nullptr; vtab = nullptr; nvtab = 0;
  slot_vi = nullptr; slot_mask = nullptr; stencil_w = 0; slice_pat = nullptr; npat = 0;
  slice_ptr = nullptr; col = nullptr; val = nullptr; rowmap = nullptr; rowlen = nullptr;
  col16 = nullptr; dict_ptr = nullptr; dict = nullptr; dmax = 0; dict_group = 1; dict_ranges = 0; ndict = 0;
  nrows = ncols = nslices = 0; nnz = nnz_pad = 0; wide = 0; pw = 0;
  for (void* q : {(void*)code16, (void*)otab, (void*)anc, (void*)cmap})
    if (q) (void)hipFree(q);
  code16 = nullptr; otab = nullptr; anc = nullptr; cmap = nullptr;
  notab = vbits = 0; anc_n = cmap_n = 0;
  if (wptr) (void)hipFree(wptr);
  wptr = nullptr;
  wval_n = wcol_n = 0;
  if (gslot) (void)hipFree(gslot);
  gslot = nullptr;
  gnx = gny = gnz = gzc = gz0 = gz1 = 0;
}

// Team size of the packed schedule: about this many rows per step.  A wide
// operator (Galerkin levels, rows of 20-100 entries) spends a step on its
// products, so its teams are small: more of them run at once and a step fits
// one LDS chunk.  Measured at 256^3 (relax 13/14): level 0 (7 entries a row)
// 0.70 ms a sweep with 64 rows against 1.01 with 16; level 1 (29 a row) 1.12
// ms with 16 against 2.34 with 64; the cycle 8.03 / 8.35 / 9.11 ms with wide
// teams of 4 / 8 / 16 rows (profiles/r04/gs_tune).
static int gs_team_rows(const CSR& A) {
  constexpr int narrow = 64, wide = 4;
  int w = 0;
  for (int i = 0; i < A.nrows; ++i) w = std::max(w, A.i[i + 1] - A.i[i]);
  return w > 8 ? wide : narrow;
}
void DevGs::upload(const CSR& A, const std::vector<int>& block_starts, bool forward, bool weighted,
                   const std::vector<double>& l1_rows, const std::vector<int>& cf_rows) {
  release();
  GsSchedule S;
  build_gs_schedule(A, block_starts, forward, S, gs_team_rows(A), weighted, &l1_rows, &cf_rows);
  nrows = A.nrows;
  nblocks = (int)S.block_start.size() - 1;
  nteams = S.nteams;
  max_steps = S.max_steps;
  max_width = S.max_width;
  ring_w = S.ring_w;
  one_chunk = true;  // k_hybrid_gs_pipe: every step's entries in one product chunk
  for (size_t q = 0; q + 3 < S.step.size() && one_chunk; q += 4)
    one_chunk = S.step[q + 3] <= ((gs_chunk_entries() / S.step[q + 2]) & ~1);  // kernels.hip gs_kc
  // the pipelined sweep's unit capacity: the power of two (128 to 512) at or
  // above the mean entries a step, so that a lane loads no more slots than a
  // typical step fills
  {
    const int64_t nst = (int64_t)S.step.size() / 4;
    const double mean = nst ? (double)S.code.size() / (double)nst : 0.0;
    cap = mean <= 128 ? 128 : mean <= 256 ? 256 : 512;
  }
  entries = (int64_t)S.code.size();
  nnz = S.nnz;
  team_step = dupload(S.team_step.data(), S.team_step.size());
  if (getenv("HVE_LAYOUT_LOG"))
    fprintf(stderr, "[layout] gs %s rows=%d teams=%d steps=%d one_chunk=%d\n", forward ? "fwd" : "bwd", A.nrows,
            S.nteams, S.team_step.empty() ? 0 : S.team_step.back(), (int)one_chunk);
  step = dupload(S.step.data(), std::max<size_t>(4, S.step.size()));
  code = dupload(S.code.data(), std::max<size_t>(1, S.code.size()));
  // At most 256 distinct values (level 0 of a constant-coefficient stencil):
  // 8-bit indices into a table, 1 B an entry instead of 8, read only by the
  // pipelined sweep.
  constexpr int vt_env = 1;
  {
    hvec<unsigned char> vi;
    std::vector<double> tab;
    if (vt_env != 0 && gs_uses_pipe(one_chunk) && !S.val.empty() &&
        build_value_table(S.val.data(), S.val.size(), 256, vi, tab)) {
      vidx8 = dupload(vi.data(), vi.size());
      vtab = dupload(tab.data(), tab.size());
      nvtab = (int)tab.size();
    } else {
      val = dupload(S.val.data(), std::max<size_t>(1, S.val.size()));
    }
  }
  if (weighted) tcol = dupload(S.tcol.data(), std::max<size_t>(1, S.tcol.size()));
  rowmap = dupload(S.rowmap.data(), std::max<size_t>(1, S.rowmap.size()));
  {
    std::vector<int> inv(S.rowmap.size());
    for (size_t k = 0; k < S.rowmap.size(); ++k) inv[S.rowmap[k]] = (int)k;
    pos = dupload(inv.data(), std::max<size_t>(1, inv.size()));
  }
  if (!S.l1.empty()) l1 = dupload(S.l1.data(), S.l1.size());
  if (!S.cf.empty()) cf = dupload(S.cf.data(), S.cf.size());
}
void DevGs::release() {
  for (void* p : {(void*)team_step, (void*)step, (void*)code, (void*)val, (void*)tcol, (void*)rowmap, (void*)pos,
                  (void*)l1, (void*)cf, (void*)vidx8, (void*)vtab})
    if (p) (void)hipFree(p);
  team_step = step = code = tcol = rowmap = pos = cf = nullptr;
  val = l1 = vtab = nullptr;
  vidx8 = nullptr;
  nvtab = 0;
  nrows = nteams = nblocks = max_steps = max_width = 0;
  one_chunk = false;
  cap = 512;
  ring_w = 64;
  entries = nnz = 0;
}

void DevOp::upload(const RankOp& op, int policy, const std::vector<int64_t>* key, const DevSell::Coded* coded,
                   const std::vector<int64_t>* tile) {
  static const bool tlog = getenv("HVE_SETUP_T") != nullptr;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = now();
  in.relax_ops = bd.relax_ops = relax_ops;
  in.grid_nlocal = bd.grid_nlocal = op.nrows_local;
  in.upload(op.interior, op.map_int, policy, key, coded, tile);
  if (tlog)
    fprintf(stderr, "[upload] %d rows %lld nnz: %s %.3fs\n", op.interior.nrows, (long long)op.interior.nnz(),
            in.code16 ? "coded" : in.code32 ? "packed" : in.slot_mask ? "stencil" : in.col16 ? "dict" : in.vidx16 ? "vt16" : in.rowlen ? "jagged"
            : in.wide ? "wide" : "padded", now() - t0);
  bd.upload(op.boundary, op.map_bnd, policy);
  nrows_local = op.nrows_local;
}

void DevHalo::upload(const RankHalo& h) {
  release();
  n_loc = h.n_loc;
  n_halo = h.n_halo;
  peers = h.peers;
  recv_cnt = h.recv_cnt;
  send_cnt = h.send_cnt;
  recv_off.assign(peers.size(), 0);
  send_off.assign(peers.size(), 0);
  int ro = 0, so = 0;
  for (size_t p = 0; p < peers.size(); ++p) {
    recv_off[p] = ro; ro += recv_cnt[p];
    send_off[p] = so; so += send_cnt[p];
  }
  n_send = so;
  if (n_send) {
    d_send_idx = dupload(h.send_idx.data(), h.send_idx.size());
    d_sendbuf = dalloc<double>(n_send);
  }
}
void DevHalo::release() {
  if (d_send_idx) (void)hipFree(d_send_idx);
  if (d_sendbuf) (void)hipFree(d_sendbuf);
  d_send_idx = nullptr; d_sendbuf = nullptr;
  peers.clear(); recv_cnt.clear(); recv_off.clear(); send_cnt.clear(); send_off.clear();
  n_loc = n_halo = n_send = 0;
}

DevAMG::~DevAMG() { release(); }

void DevAMG::release() {
  graphs_clear();
  for (auto& L : lev_) {
    L.A.release(); L.P.release(); L.R.release();
    L.hu.release(); L.hv.release();
    L.gs_fwd.release(); L.gs_bwd.release();
    for (void* p : {(void*)L.l1, (void*)L.cf, (void*)L.cf_l1, (void*)L.F, (void*)L.U[0], (void*)L.U[1], (void*)L.V,
                    (void*)L.gs_tmp, (void*)L.gs_G, (void*)L.gs_F, (void*)L.cheby_ds, (void*)L.cheby_r, (void*)L.cheby_t, (void*)L.cheby_o})
      if (p) (void)hipFree(p);
  }
  lev_.clear();
  for (void* p : {(void*)coarse_L_, (void*)coarse_mask_, (void*)coarse_U_, (void*)coarse_f_, (void*)coarse_u_,
                  (void*)u0_buf_[0], (void*)u0_buf_[1], (void*)x0_buf_, (void*)dot_part_, (void*)dscal_})
    if (p) (void)hipFree(p);
  coarse_L_ = nullptr; coarse_mask_ = nullptr; coarse_U_ = nullptr; coarse_f_ = nullptr; coarse_u_ = nullptr;
  u0_buf_[0] = u0_buf_[1] = nullptr; x0_buf_ = nullptr; dot_part_ = nullptr; dscal_ = nullptr;
  if (nrm_part_) (void)hipFree(nrm_part_);
  nrm_part_ = nullptr;
  nrm_cap_ = 0;
  if (hscal_) (void)hipHostFree(hscal_);
  hscal_ = nullptr;
  for (auto& s : scratch_) { if (s) (void)hipFree(s); s = nullptr; }
  if (ev_packed_) (void)hipEventDestroy(ev_packed_);
  if (ev_halo_) (void)hipEventDestroy(ev_halo_);
  ev_packed_ = ev_halo_ = nullptr;
  if (stream_) (void)hipStreamDestroy(stream_);
  if (comm_stream_) (void)hipStreamDestroy(comm_stream_);
  stream_ = comm_stream_ = nullptr;
  comm_ = nullptr;
  ws_n_ = 0;
}

static void init_common(hipStream_t* s, hipStream_t* cs, hipEvent_t* e1, hipEvent_t* e2) {
  HVE_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
  HVE_HIP(hipStreamCreateWithFlags(cs, hipStreamNonBlocking));
  HVE_HIP(hipEventCreateWithFlags(e1, hipEventDisableTiming));
  HVE_HIP(hipEventCreateWithFlags(e2, hipEventDisableTiming));
}

void DevAMG::init_workspace(int n, DevComm* comm) {
  release();
  comm_ = (comm && comm->size() > 1) ? comm : nullptr;
  init_common(&stream_, &comm_stream_, &ev_packed_, &ev_halo_);
  dot_part_ = dalloc<double>(1024);
  // fused norms / dots: one partial per row block (delta kernels), per wave
  // (stencil kernel) or per workgroup (PCG update)
  nrm_cap_ = std::max<size_t>(std::max<size_t>(4 * ((size_t)n / 256 + 32), 4096), (size_t)pcg_xr_parts());
  nrm_part_ = dalloc<double>(nrm_cap_);
  dscal_ = dalloc<double>(16);
  HVE_HIP(hipMemset(dscal_, 0, 16 * sizeof(double)));
  HVE_HIP(hipHostMalloc((void**)&hscal_, 16 * sizeof(double), hipHostMallocDefault));
  for (auto& s : scratch_) s = dalloc<double>(n);
  ws_n_ = n;
}

// The fused level-0 norms / dots (OP_RESID_L1JAC with a norm, the PCG
// matvec-dot) write sell_nrm_parts(in) + sell_nrm_parts(bd) partials: one per
// wave on the grid-stencil loop, which a thin grid (ny of a few points: every
// tile mostly empty rows) makes far more than the rows / 64 the workspace
// starts with.
void DevAMG::size_nrm_parts() {
  if (lev_.empty()) return;
  const DevLevel& L = lev_[0];
  size_t need = (size_t)pcg_xr_parts();
  if (L.A.in.nrows > 0 || L.A.bd.nrows > 0) {
    size_t np = L.A.in.nrows > 0 ? (size_t)sell_nrm_parts(L.A.in.view()) : 0;
    if (L.A.bd.nrows > 0) np += (size_t)sell_nrm_parts(L.A.bd.view());
    need = std::max(need, np);
  }
  if (need <= nrm_cap_) return;
  if (nrm_part_) (void)hipFree(nrm_part_);
  nrm_part_ = dalloc<double>(need);
  nrm_cap_ = need;
}

// Plane and line strides of a structured-grid operator, read off its column
// offsets: over a sample of rows, the most frequent largest offset (the plane,
// nx*ny) and smallest offset beyond 1 (the line, nx).  False when the operator
// shows no 3-D structure worth a locality order.
static bool grid_strides(const CSR& A, const std::vector<int>& map, int n_loc, int64_t* plane, int64_t* line) {
  const int n = A.nrows;
  if (n_loc < (1 << 20) || n < n_loc / 2) return false;
  std::map<int64_t, int> hmax, hmin;
  const int step = std::max(1, n / 20000);
  for (int i = 0; i < n; i += step) {
    const int64_t g = map.empty() ? i : map[i];  // local row
    int64_t mx = 0, mn = INT64_MAX;
    for (int k = A.i[i]; k < A.i[i + 1]; ++k) {
      if (A.j[k] >= n_loc) continue;  // halo column
      const int64_t d = (int64_t)A.j[k] - g;
      if (d > mx) mx = d;
      if (d > 1 && d < mn) mn = d;
    }
    if (mx > 0) ++hmax[mx];
    if (mn != INT64_MAX) ++hmin[mn];
  }
  auto mode = [](const std::map<int64_t, int>& h) {
    int64_t best = 0;
    int c = -1;
    for (const auto& kv : h)
      if (kv.second > c) { best = kv.first; c = kv.second; }
    return best;
  };
  *plane = mode(hmax);
  *line = mode(hmin);
  return *line > 1 && *plane >= 8 * *line && *plane >= (1 << 15) && (int64_t)n_loc >= 4 * *plane;
}

// Locality traversal keys per level (interior rows of every non-replicated
// level): a row's level-0 point f (C points map down through the CF markers)
// keyed as (XCD band of f's y coordinate, f).  Each XCD then streams one band
// of the grid through all its planes, so the x window that the neighbouring
// planes share stays in its 4 MiB L2 even when a whole plane does not (512^3:
// 2 MiB of x per plane).
static void locality_keys(const RankHierarchy& R, int agg_level, int nbands, std::vector<std::vector<int64_t>>& keys) {
  keys.assign(R.lev.size(), {});
  if (nbands <= 0 || R.lev.empty()) return;
  const RankLevel& L0 = R.lev[0];
  int64_t plane = 0, line = 0;
  if (!grid_strides(L0.A.interior, L0.A.map_int, L0.n_loc, &plane, &line)) return;
  const int64_t ny = std::max<int64_t>(1, plane / line);
  const int64_t n0 = L0.n_loc;
  std::vector<int64_t> f(n0);
  for (int64_t i = 0; i < n0; ++i) f[i] = i;
  for (size_t l = 0; l < R.lev.size(); ++l) {
    if (agg_level >= 0 && (int)l >= agg_level) break;
    const RankLevel& L = R.lev[l];
    if ((int64_t)f.size() != L.n_loc) break;
    std::vector<int64_t>& k = keys[l];
    k.resize(L.n_loc);
    for (int i = 0; i < L.n_loc; ++i) {
      const int64_t y = (f[i] % plane) / line;
      const int64_t band = std::min<int64_t>(nbands - 1, y * nbands / ny);
      k[i] = band * n0 + f[i];
    }
    if (L.cf.empty()) break;
    std::vector<int64_t> fc;
    fc.reserve(L.n_loc / 2);
    for (int i = 0; i < L.n_loc && i < (int)L.cf.size(); ++i)
      if (L.cf[i] == 1) fc.push_back(f[i]);
    f.swap(fc);
  }
}

// Compact 3-D tile keys of every coarse level's rows (dictionary layouts).
// A dictionary group is 4 slices = 256 consecutive rows; in natural order they
// are a thin strip of one grid line (512^3, level 1: 4095 distinct columns a
// group, 16 a row), in a compact tile about 3x their count.  The tile of a
// row is taken from its level-0 grid point f, with sides of about the cube
// root of the fine points 256 of the level's rows cover (powers of two), and
// rows are keyed (tile, f).  Only the row order of the layout changes, not any
// row's sum.
static void tile_keys(const RankHierarchy& R, int agg_level, std::vector<std::vector<int64_t>>& keys) {
  keys.assign(R.lev.size(), {});
  if (R.lev.empty()) return;
  const RankLevel& L0 = R.lev[0];
  int64_t plane = 0, line = 0;
  if (!grid_strides(L0.A.interior, L0.A.map_int, L0.n_loc, &plane, &line)) return;
  const int64_t n0 = L0.n_loc;
  const int64_t nx = line, ny = std::max<int64_t>(1, plane / line), nz = std::max<int64_t>(1, (n0 + plane - 1) / plane);
  std::vector<int64_t> f(n0);
  for (int64_t i = 0; i < n0; ++i) f[i] = i;
  auto pow2 = [](double v) {
    int64_t p = 1;
    while ((double)(p * 2) <= v * 1.41421356) p *= 2;
    return p;
  };
  for (size_t l = 0; l < R.lev.size(); ++l) {
    if (agg_level >= 0 && (int)l >= agg_level) break;
    const RankLevel& L = R.lev[l];
    if ((int64_t)f.size() != L.n_loc) break;
    if (l > 0 && L.n_loc > 0) {
      const double vol = 256.0 * (double)n0 / (double)L.n_loc;  // fine points under 256 rows
      // Tiles long in x: the per-row vectors (b, u, l1, y) of a slice stay in a
      // few cache lines while the dictionary shrinks.  Measured at 512^3
      // (profiles/r03/08_dict_tiles/tileshape*.log), level 1, A_1 residual /
      // l1 sweep: natural order 3.42 / -, cube-like 16x8x8 3.15 / 3.29,
      // 64x4x4 2.97 / 3.02, 128x4x2 2.88 / 2.94, 256x2x2 and longer slower;
      // the level-2 keys (R_1's rows) best at 64x4x4 (R_1 0.565 -> 0.486).
      int64_t tx, ty, tz;
      if (l == 1) {
        ty = std::min<int64_t>(ny, 4);
        tz = std::min<int64_t>(nz, 2);
        tx = std::min(nx, pow2(vol / (double)(ty * tz)));
      } else {
        tx = std::min<int64_t>(nx, 64);
        ty = std::min<int64_t>(ny, 4);
        tz = std::min<int64_t>(nz, 4);
      }
      const int64_t ntx = (nx + tx - 1) / tx, nty = (ny + ty - 1) / ty;
      std::vector<int64_t>& k = keys[l];
      k.resize(L.n_loc);
      for (int i = 0; i < L.n_loc; ++i) {
        const int64_t x = f[i] % line, y = (f[i] % plane) / line, z = f[i] / plane;
        k[i] = (((z / tz) * nty + y / ty) * ntx + x / tx) * n0 + f[i];
      }
    }
    if (L.cf.empty()) break;
    std::vector<int64_t> fc;
    fc.reserve(L.n_loc / 2);
    for (int i = 0; i < L.n_loc && i < (int)L.cf.size(); ++i)
      if (L.cf[i] == 1) fc.push_back(f[i]);
    f.swap(fc);
  }
}

// Tuning harness: one operator uploaded alone (layout policy, nbands of the
// traversal when the grid strides are found), op applied reps times on a
// private stream, timed with HIP events.  op: K_RESID, K_MATVEC, or the
// l1-Jacobi forms with the l1 norms formed on the fly (stencil / delta layouts).
double bench_operator(const CSR& A, int op, int policy, int nbands, int reps, double* stored_bytes, char* layout_msg,
                      int msg_len) {
  DevSell M;
  std::vector<int64_t> key;
  int64_t plane = 0, line = 0;
  if (nbands > 0 && grid_strides(A, {}, A.nrows, &plane, &line)) {
    const int64_t ny = std::max<int64_t>(1, plane / line);
    key.resize(A.nrows);
    for (int64_t i = 0; i < A.nrows; ++i)
      key[i] = std::min<int64_t>(nbands - 1, ((i % plane) / line) * nbands / ny) * A.nrows + i;
  }
  M.upload(A, {}, policy, key.empty() ? nullptr : &key);
  if (stored_bytes) *stored_bytes = (double)M.bytes() + 24.0 * A.nrows;
  if (layout_msg && msg_len > 0)
    snprintf(layout_msg, msg_len, "%s w=%d npat=%d wave_map=%d blk_map=%d", M.slot_mask ? "stencil" : M.dcol ? "delta" : "other",
             M.stencil_w, M.npat, M.wave_map != nullptr, M.blk_map != nullptr);
  const int n = A.nrows;
  double *x = dalloc<double>(n), *b = dalloc<double>(n), *y = dalloc<double>(n), *y2 = dalloc<double>(n);
  double* nrm = dalloc<double>(1 << 22);
  hipStream_t st;
  HVE_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  HVE_HIP(launch_set(n, 1.0, x, st));
  HVE_HIP(launch_set(n, 0.5, b, st));
  // the l1-Jacobi ops: the stencil and delta layouts form the norms from their
  // entries (as the cycle runs them); every other layout reads a norm vector
  const bool l1op = op == K_L1JAC || op == K_L1JAC_W || op == K_RESID_L1JAC;
  double* l1 = nullptr;
  if (l1op && !M.delta_like()) {
    l1 = dalloc<double>(n);
    HVE_HIP(launch_set(n, 8.0, l1, st));
  }
  auto one = [&]() {
    if (op == K_RESID_L1JAC)
      HVE_HIP(launch_sell(op, M.view(), x, b, l1, nullptr, 0, nullptr, 1.0, 0.0, st, y2, nrm));
    else
      HVE_HIP(launch_sell(op, M.view(), x, b, l1, nullptr, 0, y, op == K_RESID ? -1.0 : 1.0, 0.0, st));
  };
  for (int w = 0; w < 3; ++w) one();
  hipEvent_t e0, e1;
  HVE_HIP(hipEventCreate(&e0));
  HVE_HIP(hipEventCreate(&e1));
  HVE_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) one();
  HVE_HIP(hipEventRecord(e1, st));
  HVE_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  HVE_HIP(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(st);
  for (double* p : {x, b, y, y2, nrm, l1})
    if (p) (void)hipFree(p);
  M.release();
  return ms / reps;
}

// Fine grid of level 0 from its operator (row i is grid point i + shift),
// read off an interior row: line =
// its smallest column offset above 1 (plus one when that offset + 1 is also a
// neighbour: the diagonal neighbours of a 27-point stencil), plane = its
// largest offset (minus line + 1 for a 27-point stencil); nx = line,
// ny = plane / line.  Only a guess: DevSell::build_grid checks every slot
// offset against it, and any factorisation that passes gives the same sums.
static bool fine_grid(const CSR& A, int* nx, int* ny, int* nz, int shift) {
  const int n = A.nrows;
  if (n < 4096) return false;
  for (int i : {n / 2, n / 2 + 7, n / 3 + 11}) {
    std::vector<int64_t> off;
    for (int k = A.i[i]; k < A.i[i + 1]; ++k)
      if (A.j[k] > i + shift) off.push_back((int64_t)A.j[k] - i - shift);
    std::sort(off.begin(), off.end());
    auto has = [&](int64_t d) { return std::binary_search(off.begin(), off.end(), d); };
    int64_t line = 0;
    for (int64_t d : off)
      if (d > 1) { line = has(d + 1) ? d + 1 : d; break; }
    if (line < 2 || off.empty()) continue;
    int64_t plane = off.back();
    if (has(plane - 1)) plane -= line + 1;
    if (plane < 2 * line || plane % line || n % plane) continue;
    *nx = (int)line;
    *ny = (int)(plane / line);
    *nz = (int)(n / plane);
    return true;
  }
  return false;
}

void DevAMG::build(const RankHierarchy& R, DevComm* comm) {
  const int n0 = R.lev.empty() ? 0 : R.lev[0].n_loc;
  init_workspace(n0, comm);
  prm = R.prm;
  const int nl = (int)R.lev.size();
  lev_.resize(nl);
  agg_level_ = comm_ ? R.agg_level : -1;
  agg_starts_ = R.agg_starts;
  std::vector<std::vector<int64_t>> keys;
  constexpr int nbands_env = 8;  // bands of the grid's y extent (0 would be natural order)
  locality_keys(R, agg_level_, nbands_env, keys);
  // Restrictions gather from a window of ~10 fine planes per in-flight coarse
  // row range (R_0: the fine residual), wider than A's 3 planes, so they keep
  // it in L2 with narrower bands.  Measured on MI355X (512^3, R_0 alone):
  // 0 / 8 / 16 / 32 / 64 / 128 / 256 bands 1.92 / 1.81 / 1.67 / 1.63 / 1.61 /
  // 1.62 / 1.78 ms; A_0 and P_0 are best at 8.
  constexpr int nbands_r_env = 32;
  std::vector<std::vector<int64_t>> keys_r;
  if (nbands_r_env != nbands_env) locality_keys(R, agg_level_, nbands_r_env, keys_r);
  const std::vector<std::vector<int64_t>>& kr = nbands_r_env != nbands_env ? keys_r : keys;
  std::vector<std::vector<int64_t>> tiles;
  tile_keys(R, agg_level_, tiles);
  const bool tlog = getenv("HVE_SETUP_T") != nullptr;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  for (int l = 0; l < nl; ++l) {
    const double tl0 = now();
    const RankLevel& L = R.lev[l];
    DevLevel& D = lev_[l];
    D.n = L.n_loc;
    D.first = L.first;
    D.n_glob = L.n_glob;
    // A_l and P_l rows are level-l rows; R_l rows are level-(l+1) rows
    const std::vector<int64_t>* kl = keys[l].empty() ? nullptr : &keys[l];
    const std::vector<int64_t>* kc = (l + 1 < nl && !kr[l + 1].empty()) ? &kr[l + 1] : nullptr;
    // A on level 1 and the restrictions (measured at 512^3: A_1 3.42 -> 3.24 ms,
    // R_1 0.582 -> 0.560; A_2 0.873 -> 0.936, so A_2 keeps the natural order)
    // (tiling A_2 too, 64x4x4: 0.872 -> 0.932 ms at 512^3)
    const std::vector<int64_t>* tl = (l == 1 && !tiles[l].empty()) ? &tiles[l] : nullptr;
    const std::vector<int64_t>* tc = (l + 1 < nl && !tiles[l + 1].empty()) ? &tiles[l + 1] : nullptr;
    D.A.relax_ops = true;
    D.A.upload(L.A, prm.sell_policy, kl, nullptr, tl);
    D.hu.upload(L.hu);
    if (l < nl - 1) {
      // grid context of P_l / R_l for the offset-coded layout: the fine point
      // of each local coarse point (fc) and its inverse (cidx, -1 at F points)
      std::vector<int> fc, cidx;
      // (given without members where there is no grid context: the operator
      // is still known to be P / R, which the packed layout is limited to)
      DevSell::Coded cp, cr;
      const DevSell::Coded *pc = &cp, *rc = &cr;
      if (!L.cf.empty() && (int)L.cf.size() >= L.n_loc) {
        cidx.assign(L.n_loc, -1);
        for (int i = 0; i < L.n_loc; ++i)
          if (L.cf[i] == 1) {
            cidx[i] = (int)fc.size();
            fc.push_back(i);
          }
        if ((int)fc.size() == R.lev[l + 1].n_loc) {
          cp.colpos = &fc;
          cp.cmap = &cidx;
          cr.anc = &fc;
        }
      }
      D.P.upload(L.P, prm.sell_policy, kl, pc);
      D.R.upload(L.R, prm.sell_policy, kc, rc, tc);
      D.hv.upload(L.hv);
    }
    if (!L.l1.empty()) D.l1 = dupload(L.l1.data(), L.l1.size());
    D.l1_fly = !L.l1.empty() && l1_on_the_fly(L.A, L.l1) && D.A.in.delta_like() && (D.A.bd.nrows == 0 || D.A.bd.delta_like());
    if (!L.cf.empty()) D.cf = dupload(L.cf.data(), L.cf.size());
    if (!L.cf.empty() && prm.relax_order == 1 && (prm.relax_type[1] == 18 || prm.relax_type[2] == 18)) {
      std::vector<int> m(L.cf.begin(), L.cf.begin() + std::min<size_t>(L.cf.size(), (size_t)L.n_loc));
      for (int part = 0; part < 2; ++part) {
        const CSR& A = part == 0 ? L.A.interior : L.A.boundary;
        const std::vector<int>& map = part == 0 ? L.A.map_int : L.A.map_bnd;
        for (int i = 0; i < A.nrows; ++i) {
          const int g = map.empty() ? i : map[i];
          if (g < (int)m.size() && (A.i[i] == A.i[i + 1] || A.a[A.i[i]] == 0.0)) m[g] = 0;
        }
      }
      D.cf_l1 = dupload(m.data(), m.size());
    }
    D.F = dalloc<double>(D.n);
    D.U[0] = dalloc<double>(D.n + D.hu.n_halo);
    D.U[1] = dalloc<double>(D.n + D.hu.n_halo);
    D.V = dalloc<double>(D.n + D.hv.n_halo);
    HVE_HIP(hipMemset(D.F, 0, sizeof(double) * std::max(1, D.n)));
    HVE_HIP(hipMemset(D.U[0], 0, sizeof(double) * std::max(1, D.n + D.hu.n_halo)));
    HVE_HIP(hipMemset(D.U[1], 0, sizeof(double) * std::max(1, D.n + D.hu.n_halo)));
    HVE_HIP(hipMemset(D.V, 0, sizeof(double) * std::max(1, D.n + D.hv.n_halo)));
    if (!L.cheby_coefs.empty()) {
      D.cheby_coefs = L.cheby_coefs;
      if (!L.cheby_ds.empty()) D.cheby_ds = dupload(L.cheby_ds.data(), L.cheby_ds.size());
      D.cheby_r = dalloc<double>(D.n);
      D.cheby_t = dalloc<double>(D.n + D.hu.n_halo);
      D.cheby_o = dalloc<double>(D.n);
      HVE_HIP(hipMemset(D.cheby_t, 0, sizeof(double) * std::max(1, D.n + D.hu.n_halo)));
    }
    if (tlog) {
      double rc, rp;
      host_rss_gb(&rc, &rp);
      fprintf(stderr, "[build] level %d: %.3fs (A %s) host RSS %.1f GB, peak %.1f GB\n", l, now() - tl0,
              D.A.in.slot_mask ? "stencil" : "", rc, rp);
    }
  }
  // Hybrid Gauss-Seidel schedules for the relax types the cycle uses
  // (num_blocks = hypre's thread count: row blocks of each level).
  {
    bool fwd = false, bwd = false;
    for (int c = 0; c < 5; ++c) {
      // c == 4: the one-level smoother (par_cycle.c:296-300)
      const int rt = c < 4 ? prm.relax_type[c] : (nl == 1 ? (prm.user_relax_type >= 0 ? prm.user_relax_type : 6) : -1);
      fwd = fwd || rt == 3 || rt == 6 || rt == 8 || rt == 13;
      bwd = bwd || rt == 4 || rt == 6 || rt == 8 || rt == 14;
    }
    // Across ranks (par_relax.c with num_procs > 1): each rank sweeps its own
    // rows in num_blocks blocks (RankLevel::gs_blocks), off-rank columns read
    // the halo exchanged before the sweep, exactly as off-block columns read
    // the pre-sweep copy.
    for (int l = 0; l < nl && (fwd || bwd); ++l) {
      const RankLevel& L = R.lev[l];
      DevLevel& D = lev_[l];
      if (l == nl - 1 && R.coarse_n > 0) break;  // coarsest level: direct solve
      const CSR rows = merged_rows(L.A, L.n_loc);
      const std::vector<int> bs = L.gs_blocks.empty() ? hypre_block_starts(L.n_loc, prm.blocks_for(L.n_loc)) : L.gs_blocks;
      const bool weighted = prm.wt(l) != 1.0 || prm.omega(l) != 1.0;  // the w / omega forms also read tmp in-block
      // k_hybrid_gs addresses G (T | C | U | halo) with 32-bit buffer offsets
      if ((3 * (uint64_t)D.n + (uint64_t)D.hu.n_halo) * sizeof(double) > 0xffffffffull)
        throw std::runtime_error("hybrid Gauss-Seidel (relax 3/4/6/8/13/14): level " + std::to_string(l) + " has " +
                                 std::to_string(D.n) + " rows on this rank; the sweep's vectors (3 n + halo doubles) "
                                 "must stay below 4 GiB (about 178M rows a GPU): use more ranks or relax 18");
      if (fwd) D.gs_fwd.upload(rows, bs, true, weighted, L.l1, L.cf);
      if (bwd) D.gs_bwd.upload(rows, bs, false, weighted, L.l1, L.cf);
      D.gs_G = dalloc<double>(3 * (size_t)D.n + D.hu.n_halo + 1);
      D.gs_F = dalloc<double>((size_t)D.n + 1);
      if (fwd && bwd) D.gs_tmp = dalloc<double>((size_t)D.n + 1);
    }
  }
  size_nrm_parts();
  coarse_n_ = R.coarse_n;
  if (coarse_n_ > 0) {
    std::vector<double> Lf, U;
    std::vector<unsigned char> mask;
    gselim_factor(coarse_n_, R.coarse_dense, Lf, mask, U);
    coarse_L_ = dupload(Lf.data(), Lf.size());
    coarse_mask_ = dupload(mask.data(), mask.size());
    coarse_U_ = dupload(U.data(), U.size());
    coarse_f_ = dalloc<double>(coarse_n_);
    coarse_u_ = dalloc<double>(coarse_n_);
  }
  if (nl > 0 && lev_[0].hu.n_halo > 0) {
    const int m = lev_[0].n + lev_[0].hu.n_halo;
    u0_buf_[0] = dalloc<double>(m);
    u0_buf_[1] = dalloc<double>(m);
    x0_buf_ = dalloc<double>(m);
    HVE_HIP(hipMemset(u0_buf_[0], 0, sizeof(double) * m));
    HVE_HIP(hipMemset(u0_buf_[1], 0, sizeof(double) * m));
    HVE_HIP(hipMemset(x0_buf_, 0, sizeof(double) * m));
  }
  set_use_graph(use_graph_);
  HVE_HIP(hipDeviceSynchronize());
}

// Re-key the traversal of every interior operator with `nbands` bands (0:
// natural order) on the built hierarchy (tuning: the operators stay in place).
void DevAMG::set_block_bands(const RankHierarchy& R, int nbands, int which_mask) {
  std::vector<std::vector<int64_t>> keys;
  locality_keys(R, agg_level_, nbands, keys);
  const int nl = (int)lev_.size();
  for (int l = 0; l < nl; ++l) {
    DevLevel& D = lev_[l];
    const RankLevel& L = R.lev[l];
    const std::vector<int64_t> none;
    const std::vector<int64_t>& kl = keys[l];
    const std::vector<int64_t>& kc = l + 1 < nl ? keys[l + 1] : none;
    auto redo = [](DevSell& M, const std::vector<int64_t>& k, const std::vector<int>& map) {
      if (M.blk_map) (void)hipFree(M.blk_map);
      M.blk_map = nullptr;
      M.nblk = 0;
      M.blk_host.clear();
      if (!k.empty() && M.stored_map.size() == (size_t)M.nrows) M.set_block_order(M.stored_map, k);
      else if (!k.empty() && !M.rowmap) M.set_block_order(map, k);
      if (M.blk_host.empty()) M.build_wave_map();
    };
    if (which_mask & 1) redo(D.A.in, kl, {});
    if (l < nl - 1) {
      if (which_mask & 2) redo(D.P.in, kl, {});
      if (which_mask & 4) redo(D.R.in, kc, {});
    }
    (void)L;
  }
  graphs_clear();
}
void DevAMG::set_use_graph(bool g) {
  static const bool multi_ok = [] {
    const char* e = std::getenv("HVE_GRAPH_MULTI");
    return !e || std::atoi(e) != 0;
  }();
  use_graph_ = g && (!comm_ || (comm_->capturable() && multi_ok));
  if (!use_graph_) graphs_clear();
}
void DevAMG::graphs_clear() {
  for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
  graphs_.clear();
  eager_runs_.clear();  // a new hierarchy or communicator connects its peers again
}

void DevAMG::dot(int n, const double* x, const double* y, double* out, hipStream_t s) {
  HVE_HIP(launch_dot(n, x, y, dot_part_, out, s));
  if (comm_) comm_->allreduce_sum(out, 1, s);
}
double DevAMG::dot_host(int n, const double* x, const double* y, hipStream_t s) {
  dot(n, x, y, dscal_ + 15, s);
  HVE_HIP(hipMemcpyAsync(hscal_ + 15, dscal_ + 15, sizeof(double), hipMemcpyDeviceToHost, s));
  HVE_HIP(hipStreamSynchronize(s));
  return hscal_[15];
}

// ParCSR halo exchange (par_csr_communication.c hypre_ParCSRCommHandleCreate,
// job 1) as gather -> grouped RCCL send/recv on the side stream.
void DevAMG::halo_start(const DevHalo& h, double* x, hipStream_t s) {
  if (comm_level_ >= 0) {
    for (size_t l = 0; l < lev_.size(); ++l)
      if (&lev_[l].hu == &h || &lev_[l].hv == &h) {
        cycle_comm_[l].exchanges++;
        cycle_comm_[l].bytes += (int64_t)h.n_send * (int64_t)sizeof(double);
      }
  }
  HVE_HIP(launch_gather(h.n_send, h.d_send_idx, x, h.d_sendbuf, s));
  HVE_HIP(hipEventRecord(ev_packed_, s));
  HVE_HIP(hipStreamWaitEvent(comm_stream_, ev_packed_, 0));
  std::vector<P2PMsg> sends, recvs;
  for (size_t p = 0; p < h.peers.size(); ++p) {
    if (h.send_cnt[p]) sends.push_back({h.peers[p], h.d_sendbuf + h.send_off[p], sizeof(double) * h.send_cnt[p]});
    if (h.recv_cnt[p]) recvs.push_back({h.peers[p], x + h.n_loc + h.recv_off[p], sizeof(double) * h.recv_cnt[p]});
  }
  comm_->exchange(sends, recvs, comm_stream_);
  HVE_HIP(hipEventRecord(ev_halo_, comm_stream_));
}
void DevAMG::halo_finish(hipStream_t s) { HVE_HIP(hipStreamWaitEvent(s, ev_halo_, 0)); }

void DevAMG::apply(const DevOp& M, const DevHalo* hx, int op, double* x, const double* b, const double* l1,
                   const int* cf, int relax_points, double* y, double w, double temp, hipStream_t s, double* y2) {
  const bool ex = hx && hx->active() && comm_;
  if (ex) halo_start(*hx, x, s);
  HVE_HIP(launch_sell(op, M.in.view(), x, b, l1, cf, relax_points, y, w, temp, s, y2));
  if (ex) halo_finish(s);
  if (M.bd.nrows > 0) HVE_HIP(launch_sell(op, M.bd.view(), x, b, l1, cf, relax_points, y, w, temp, s, y2));
}

// The solve loop's residual r = f - A u forms, row for row, the same sum as
// the next cycle's first level-0 l1-Jacobi sweep (relax 7/18, weight 1,
// u + (f - A u)/l1), so one kernel can write both (OP_RESID_L1JAC) and the
// cycle starts after that sweep: one pass over A_0 fewer per iteration, same
// bits.
bool DevAMG::can_fuse_presmooth() const {
  if (lev_.size() < 2 || !lev_[0].l1) return false;
  const int rt = prm.relax_type[1];
  // with relax_order 1 the first down sweep is C/F-ordered (18) or one of two (7)
  return (rt == 18 || rt == 7) && prm.wt(0) == 1.0 && prm.num_sweeps[1] >= 1 && prm.relax_order != 1;
}
double* DevAMG::presmooth_buffer() { return u0_buf_[1] ? u0_buf_[1] : lev_[0].U[0]; }

void DevAMG::fine_apply(int op, const double* x, const double* b, double* y, double alpha, double temp,
                        hipStream_t s) {
  DevLevel& L = lev_[0];
  double* xin = const_cast<double*>(x);
  if (x0_buf_) {
    HVE_HIP(launch_copy(L.n, x, x0_buf_, s));
    xin = x0_buf_;
  }
  apply(L.A, &L.hu, op, xin, b, nullptr, nullptr, 0, y, alpha, temp, s);
}

// s = A p and <s, p> into the device scalar dot_out: one pass on the delta
// layout (partials summed afterwards), else the matvec and the dot kernel.
void DevAMG::fine_matvec_dot(const double* p, double* sv, double* dot_out, hipStream_t s) {
  DevLevel& L = lev_[0];
  const bool fused = L.A.in.delta_like() && (L.A.bd.nrows == 0 || L.A.bd.delta_like()) && nrm_fusion_ && !x0_buf_;
  if (!fused) {
    fine_apply(K_MATVEC, p, nullptr, sv, 1.0, 0.0, s);
    dot(L.n, sv, p, dot_out, s);
    return;
  }
  double* pin = const_cast<double*>(p);
  const bool ex = L.hu.active() && comm_;
  if (ex) halo_start(L.hu, pin, s);
  HVE_HIP(launch_sell(K_MATVEC, L.A.in.view(), pin, nullptr, nullptr, nullptr, 0, sv, 1.0, 0.0, s, nullptr,
                      nrm_part_));
  if (ex) halo_finish(s);
  int np = sell_nrm_parts(L.A.in.view());
  if (L.A.bd.nrows > 0) {
    HVE_HIP(launch_sell(K_MATVEC, L.A.bd.view(), pin, nullptr, nullptr, nullptr, 0, sv, 1.0, 0.0, s, nullptr,
                        nrm_part_ + np));
    np += sell_nrm_parts(L.A.bd.view());
  }
  HVE_HIP(launch_sum(np, nrm_part_, dot_part_, dot_out, s));
  if (comm_) comm_->allreduce_sum(dot_out, 1, s);
}

// PCG's x += alpha p; r -= alpha s, and (rr_out != null) <r, r> of the new r.
void DevAMG::pcg_update(int n, const double* alpha_p, const double* p, const double* sv, double* x, double* r,
                        double* rr_out, hipStream_t s) {
  HVE_HIP(launch_pcg_xr(n, alpha_p, p, sv, x, r, rr_out ? nrm_part_ : nullptr, s));
  if (rr_out) {
    HVE_HIP(launch_sum(pcg_xr_parts(), nrm_part_, dot_part_, rr_out, s));
    if (comm_) comm_->allreduce_sum(rr_out, 1, s);
  }
}

// v holds starts[r] .. starts[r+1] of every rank r; each rank fills in its own
// share and receives the others' (one grouped exchange).
void DevAMG::allgather_rows(double* v, const std::vector<int>& starts, hipStream_t s) {
  const int me = comm_->rank(), n = comm_->size();
  if (comm_level_ >= 0 && agg_level_ >= 0) {
    cycle_comm_[agg_level_].allgathers++;
    cycle_comm_[agg_level_].allgather_bytes += (int64_t)(starts[me + 1] - starts[me]) * (n - 1) * (int64_t)sizeof(double);
  }
  std::vector<P2PMsg> sends, recvs;
  const size_t mine = (size_t)(starts[me + 1] - starts[me]) * sizeof(double);
  for (int p = 0; p < n; ++p) {
    if (p == me) continue;
    if (mine) sends.push_back({p, v + starts[me], mine});
    const size_t theirs = (size_t)(starts[p + 1] - starts[p]) * sizeof(double);
    if (theirs) recvs.push_back({p, v + starts[p], theirs});
  }
  comm_->exchange(sends, recvs, s);
}

void DevAMG::coarse_solve(int level, const double* f, double* u, hipStream_t s) {
  DevLevel& L = lev_[level];
  if (coarse_n_ != L.n_glob) throw std::runtime_error("coarse solve size mismatch");
  if (!comm_ || agg_level_ >= 0) {  // one rank, or the coarsest level is replicated
    HVE_HIP(launch_coarse(coarse_n_, coarse_L_, coarse_mask_, coarse_U_, f, u, s));
    return;
  }
  // hypre_GaussElimSolve gathers f on every rank and solves redundantly
  HVE_HIP(launch_set(coarse_n_, 0.0, coarse_f_, s));
  HVE_HIP(launch_copy(L.n, f, coarse_f_ + L.first, s));
  if (comm_level_ >= 0) cycle_comm_[level].allreduces++;
  comm_->allreduce_sum(coarse_f_, coarse_n_, s);
  HVE_HIP(launch_coarse(coarse_n_, coarse_L_, coarse_mask_, coarse_U_, coarse_f_, coarse_u_, s));
  HVE_HIP(launch_copy(L.n, coarse_u_ + L.first, u, s));
}

// One smoothing step on `level` (par_cycle.c:333-505 dispatch).  u_cur holds the
// current iterate; out-of-place smoothers write u_alt and swap the two.
void DevAMG::relax(int level, int relax_type, int relax_points, const double* f, double*& u_cur,
                   double*& u_alt, bool zero_guess, hipStream_t s) {
  DevLevel& L = lev_[level];
  const double w = prm.wt(level), omega = prm.omega(level);  // relax_weight[level], omega[level]
  const int n = L.n;
  if (relax_type == 7) relax_points = 0;  // par_relax.c:3463: a C/F-ordered call is a full sweep
  if (zero_guess && relax_points != 0) {
    HVE_HIP(launch_set(n, 0.0, u_cur, s));
    zero_guess = false;
  }
  switch (relax_type) {
    case 18:
    case 7: {
      if (!L.l1) throw std::runtime_error("l1 norms missing for relax type 18/7");
      if (relax_points != 0) {
        // par_relax_more.c:991 hypre_ParCSRRelax_L1_Jacobi: rows of class
        // relax_points with a nonzero diagonal, u += (w (f - A u_old))/l1 with the
        // C/F-restricted norms; out of place, so every row reads the pre-sweep u
        // (its Vtemp copy), and the others are copied.  w (f - Au) equals the
        // weighted kernel's (-w)(-f + Au) bit for bit (negation is exact).
        if (!L.cf_l1) throw std::runtime_error("C/F marker missing for C/F-ordered l1-Jacobi");
        apply(L.A, &L.hu, w == 1.0 ? K_L1JAC : K_L1JAC_W, u_cur, f, L.l1, L.cf_l1, relax_points, u_alt, w, 0.0, s);
        std::swap(u_cur, u_alt);
        break;
      }
      if (zero_guess) {
        HVE_HIP(launch_zero_guess(n, w == 1.0 ? 0 : 1, w, f, L.l1, u_cur, s));
      } else {
        apply(L.A, &L.hu, w == 1.0 ? K_L1JAC : K_L1JAC_W, u_cur, f, L.l1_fly ? nullptr : L.l1, nullptr, 0, u_alt,
              w, 0.0, s);
        std::swap(u_cur, u_alt);
      }
      break;
    }
    case 0: {
      if (zero_guess) HVE_HIP(launch_set(n, 0.0, u_cur, s));
      apply(L.A, &L.hu, K_JAC, u_cur, f, nullptr, L.cf, relax_points, u_alt, w, 0.0, s);
      std::swap(u_cur, u_alt);
      break;
    }
    case 3: case 4: case 6: case 8: case 13: case 14: {
      // par_relax.c:354 (3), :1875 (4), :2266 (6), :3492 (8), :4340 (13), :4732 (14);
      // weighted forms (relax_weight or omega != 1): par_relax.c:1277, :2075, :3150, :3785, :4544, :4937
      const bool weighted = w != 1.0 || omega != 1.0;
      const bool use_l1 = relax_type == 8 || relax_type == 13 || relax_type == 14;
      const bool fw = relax_type == 3 || relax_type == 6 || relax_type == 8 || relax_type == 13;
      const bool bw = relax_type == 4 || relax_type == 6 || relax_type == 8 || relax_type == 14;
      if (use_l1 && !L.l1) throw std::runtime_error("l1 norms missing for l1 hybrid Gauss-Seidel");
      if ((fw && !L.gs_fwd.built()) || (bw && !L.gs_bwd.built()))
        throw std::runtime_error("hybrid Gauss-Seidel schedule missing on level " + std::to_string(level));
      if (weighted && ((fw && !L.gs_fwd.tcol) || (bw && !L.gs_bwd.tcol)))
        throw std::runtime_error("weighted hybrid Gauss-Seidel on level " + std::to_string(level) +
                                 ": the relaxation weight changed after the setup built the schedule");
      if (zero_guess) HVE_HIP(launch_set(n, 0.0, u_cur, s));
      // off-rank values of u before the sweep (par_relax.c: Vext_data)
      if (comm_ && L.hu.active()) {
        halo_start(L.hu, u_cur, s);
        halo_finish(s);
      }
      const bool cfsel = relax_points != 0 && L.cf != nullptr;
      // symmetric sweeps (6, 8): the second half's off-block columns (and the
      // weighted forms' Vtemp) read u from before the first half (tmp_data),
      // its in-block ones the first half's result
      if (fw && bw) HVE_HIP(launch_copy(n, u_cur, L.gs_tmp, s));
      if (fw) {
        HVE_HIP(launch_gs_gather(L.gs_fwd.view(), u_cur, nullptr, f, L.hu.n_halo, L.gs_G, L.gs_F, s));
        HVE_HIP(launch_hybrid_gs(L.gs_fwd.view(), use_l1, cfsel, relax_points, L.gs_G, L.hu.n_halo, L.gs_F, u_cur, w, omega,
                                 true, s));
      }
      if (bw) {
        HVE_HIP(launch_gs_gather(L.gs_bwd.view(), u_cur, fw ? L.gs_tmp : nullptr, f, L.hu.n_halo, L.gs_G, L.gs_F, s));
        HVE_HIP(launch_hybrid_gs(L.gs_bwd.view(), use_l1, cfsel, relax_points, L.gs_G, L.hu.n_halo, L.gs_F, u_cur, w, omega,
                                 !fw, s));
      }
      break;
    }
    case 16: {
      // par_cheby.c:166 hypre_ParCSRRelax_Cheby_Solve (par_cycle.c:445)
      if (L.cheby_coefs.empty()) throw std::runtime_error("Chebyshev coefficients missing on level " +
                                                          std::to_string(level));
      if (zero_guess) HVE_HIP(launch_set(n, 0.0, u_cur, s));
      int order = prm.cheby_order;
      if (order > 4) order = 4;
      if (order < 1) order = 1;
      const int co = order - 1;
      const int scale = prm.cheby_scale ? 1 : 0;
      if (scale && !L.cheby_ds) throw std::runtime_error("Chebyshev scaling vector missing");
      double* r = L.cheby_r;
      double* tmp = L.cheby_t;
      double* v = L.V;
      if (scale) {
        // tmp = -A u  (ParCSRMatrixMatvec(-1.0, A, u, 0.0, tmp))
        apply(L.A, &L.hu, K_GENERAL, u_cur, nullptr, nullptr, nullptr, 0, tmp, -1.0, 0.0, s);
      } else {
        // r = f - A u  (ParVectorCopy(f, r); Matvec(-1.0, A, u, 1.0, r))
        apply(L.A, &L.hu, K_RESID, u_cur, f, nullptr, nullptr, 0, r, -1.0, 0.0, s);
      }
      HVE_HIP(launch_cheby(n, 0, scale, L.cheby_coefs[co], L.cheby_ds, f, r, tmp, nullptr, L.cheby_o, u_cur, s));
      for (int i = co - 1; i >= 0; --i) {
        if (scale) {
          HVE_HIP(launch_cheby(n, 1, scale, 0.0, L.cheby_ds, nullptr, nullptr, tmp, nullptr, nullptr, u_cur, s));
          apply(L.A, &L.hu, K_MATVEC, tmp, nullptr, nullptr, nullptr, 0, v, 1.0, 0.0, s);
        } else {
          apply(L.A, &L.hu, K_MATVEC, u_cur, nullptr, nullptr, nullptr, 0, v, 1.0, 0.0, s);
        }
        HVE_HIP(launch_cheby(n, 2, scale, L.cheby_coefs[i], L.cheby_ds, nullptr, r, nullptr, v, nullptr, u_cur, s));
      }
      HVE_HIP(launch_cheby(n, 3, scale, 0.0, L.cheby_ds, nullptr, nullptr, nullptr, nullptr, L.cheby_o, u_cur, s));
      break;
    }
    default:
      throw std::runtime_error("relax_type " + std::to_string(relax_type) +
                               " is not available on the GPU path in this build");
  }
}

// par_cycle.c:22 hypre_BoomerAMGCycle, emitted as a kernel sequence.
// zero_u: u0 holds zeros on entry (PCG's cleared preconditioner output,
// pcg.c:434), so the first level-0 sweep takes the zero-guess form and u0 is
// neither cleared nor read.
void DevAMG::emit_cycle(const double* f0, double* u0, hipStream_t s, bool presmoothed, bool zero_u) {
  const int nl = (int)lev_.size();
  cycle_comm_.assign(nl, CycleComm());
  comm_level_ = 0;
  struct CountOff {
    int& l;
    ~CountOff() { l = -1; }
  } count_off{comm_level_};
  std::vector<int> lev_counter(nl, prm.cycle_type);
  std::vector<double*> ucur(nl), ualt(nl);
  std::vector<const double*> fl(nl);
  std::vector<char> zero(nl, 0), skip_sweep(nl, 0);
  lev_counter[0] = 1;
  if (zero_u) zero[0] = 1;
  if (u0_buf_[0]) {
    if (!presmoothed && !zero_u) HVE_HIP(launch_copy(lev_[0].n, u0, u0_buf_[0], s));
    ucur[0] = u0_buf_[0];
    ualt[0] = u0_buf_[1];
  } else {
    ucur[0] = u0;
    ualt[0] = lev_[0].U[0];
  }
  // the first level-0 sweep was formed by the fused residual into ualt[0]:
  // take the state the relax call would have left (its output, swapped in)
  bool skip_first = false;
  if (presmoothed) {
    if (!can_fuse_presmooth()) throw std::runtime_error("cycle: presmoothed iterate without a fusable smoother");
    std::swap(ucur[0], ualt[0]);
    skip_first = true;
  }
  fl[0] = f0;
  for (int l = 1; l < nl; ++l) {
    ucur[l] = lev_[l].U[0];
    ualt[l] = lev_[l].U[1];
    fl[l] = lev_[l].F;
  }
  int level = 0, cycle_param = 1;
  double ops = 0;
  bool done = false;
  while (!done) {
    int num_sweep, relax_type;
    if (nl > 1) {
      num_sweep = prm.num_sweeps[cycle_param];
      relax_type = prm.relax_type[cycle_param];
    } else {
      num_sweep = 1;
      relax_type = prm.user_relax_type >= 0 ? prm.user_relax_type : 6;  // par_cycle.c:296-300
    }
    for (int j = 0; j < num_sweep; ++j) {
      ops += (double)lev_[level].A.nnz();
      if (skip_first) {
        skip_first = false;
        continue;
      }
      if (skip_sweep[level]) {
        skip_sweep[level] = 0;
        continue;
      }
      if (relax_type == 9 || relax_type == 99 || relax_type == 19 || relax_type == 98) {
        coarse_solve(level, fl[level], ucur[level], s);
        zero[level] = 0;
      } else if (relax_type == 17) {
        // par_cycle.c:451 / par_relax_more.c:661 FCF-Jacobi: weighted Jacobi over
        // the F, C, F points whatever relax_order; one full sweep on the coarsest level
        const int pts[3] = {-1, 1, -1};
        for (int q = 0; q < (level == nl - 1 ? 1 : 3); ++q) {
          relax(level, 0, level == nl - 1 ? 0 : pts[q], fl[level], ucur[level], ualt[level], zero[level], s);
          zero[level] = 0;
        }
      } else if (relax_type == 18 && !(prm.relax_order == 1 && cycle_param < 3)) {
        relax(level, relax_type, 0, fl[level], ucur[level], ualt[level], zero[level], s);
        zero[level] = 0;
      } else {
        // relax 18 with relax_order 1: C/F-ordered L1_Jacobi twice (par_cycle.c:398-415);
        // the rest through hypre_BoomerAMGRelaxIF (par_relax_interface.c:35-76)
        if (prm.relax_order == 1 && cycle_param < 3) {
          int pts[2];
          if (cycle_param < 2) { pts[0] = 1; pts[1] = -1; } else { pts[0] = -1; pts[1] = 1; }
          for (int q = 0; q < 2; ++q) {
            relax(level, relax_type, pts[q], fl[level], ucur[level], ualt[level], zero[level], s);
            zero[level] = 0;
          }
        } else {
          relax(level, relax_type, 0, fl[level], ucur[level], ualt[level], zero[level], s);
          zero[level] = 0;
        }
      }
    }
    --lev_counter[level];
    if (lev_counter[level] >= 0 && level != nl - 1) {
      const int fine = level, coarse = level + 1;
      DevLevel& Lf = lev_[fine];
      // When the coarse level's first down sweep is l1-Jacobi (weight 1) from
      // the zero guess, u_c = 0 + F_c/l1 is formed by the restriction itself.
      const bool into_agg = agg_level_ >= 0 && coarse == agg_level_;
      const bool fuse_zg = !into_agg && coarse != nl - 1 && prm.num_sweeps[1] >= 1 && prm.relax_order != 1 &&
                           (prm.relax_type[1] == 18 || prm.relax_type[1] == 7) && prm.wt(coarse) == 1.0 &&
                           lev_[coarse].l1 != nullptr;
      // Vtemp = f - A u  (csr_matvec.c, alpha=-1 beta=1);  F_c = P^T Vtemp
      apply(Lf.A, &Lf.hu, K_RESID, ucur[fine], fl[fine], nullptr, nullptr, 0, Lf.V, -1.0, 0.0, s);
      if (fuse_zg) {
        apply(Lf.R, &Lf.hv, K_RESTRICT_ZG, Lf.V, nullptr, lev_[coarse].l1, nullptr, 0, lev_[coarse].F, 1.0, 0.0,
              s, ucur[coarse]);
      } else if (into_agg) {
        // this rank's share of the replicated level's rows, then everyone's
        const int r0 = agg_starts_[comm_->rank()];
        apply(Lf.R, &Lf.hv, K_RESTRICT, Lf.V, nullptr, nullptr, nullptr, 0, lev_[coarse].F + r0, 1.0, 0.0, s);
        allgather_rows(lev_[coarse].F, agg_starts_, s);
      } else {
        apply(Lf.R, &Lf.hv, K_RESTRICT, Lf.V, nullptr, nullptr, nullptr, 0, lev_[coarse].F, 1.0, 0.0, s);
      }
      ++level;
      lev_counter[level] = std::max(lev_counter[level], prm.cycle_type);
      cycle_param = (level == nl - 1) ? 3 : 1;
      zero[level] = 1;  // U_array[coarse] = 0 (par_cycle.c:556), folded into the next smoother
      if (fuse_zg) {
        zero[level] = 0;
        skip_sweep[level] = 1;  // that sweep is done
      }
    } else if (level != 0) {
      const int fine = level - 1, coarse = level;
      if (zero[coarse]) HVE_HIP(launch_set(lev_[coarse].n, 0.0, ucur[coarse], s));
      zero[coarse] = 0;
      // u_f = u_f + P u_c  (alpha=1, beta=1)
      apply(lev_[fine].P, &lev_[coarse].hu, K_PROLONG, ucur[coarse], nullptr, nullptr, nullptr, 0, ucur[fine], 1.0,
            0.0, s);
      --level;
      cycle_param = 2;
    } else {
      done = true;
    }
  }
  if (ucur[0] != u0) HVE_HIP(launch_copy(lev_[0].n, ucur[0], u0, s));
  cycle_ops_ = ops;
}

void DevAMG::capture_failed(const char* why) {
  fprintf(stderr, "[hypreve] rank %d: cycle capture over %s failed (%s); cycles run eagerly\n", comm_->rank(),
          comm_->kind(), why);
  use_graph_ = false;
  graphs_clear();
}

void DevAMG::cycle(const double* f, double* u, hipStream_t s, const double* presmoothed, bool zero_u) {
  const bool pre = presmoothed != nullptr;
  if (pre && presmoothed != presmooth_buffer()) throw std::runtime_error("cycle: unexpected presmoothed buffer");
  if (pre && zero_u) throw std::runtime_error("cycle: a presmoothed iterate is not zero");
  if (!use_graph_) {
    emit_cycle(f, u, s, pre, zero_u);
    return;
  }
  auto key = std::make_tuple((const void*)f, (const void*)u, (int)pre + 2 * (int)zero_u);
  auto it = graphs_.find(key);
  if (it == graphs_.end()) {
    if (comm_ && eager_runs_[key]++ == 0) {
      // first run of this shape on several ranks: eagerly (RCCL connects its
      // peers on first use, which must not happen inside a capture)
      emit_cycle(f, u, s, pre, zero_u);
      return;
    }
    hipGraph_t g = nullptr;
    HVE_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
      emit_cycle(f, u, s, pre, zero_u);
    } catch (...) {
      hipGraph_t tmp = nullptr;
      (void)hipStreamEndCapture(s, &tmp);
      if (tmp) (void)hipGraphDestroy(tmp);
      (void)hipGetLastError();
      if (!comm_) throw;
      // nothing captured has run: the cycle runs eagerly from here on (every
      // rank still issues the same sequence of transfers)
      capture_failed("emission");
      emit_cycle(f, u, s, pre, zero_u);
      return;
    }
    hipError_t ec = hipStreamEndCapture(s, &g);
    hipGraphExec_t ge = nullptr;
    if (ec == hipSuccess) ec = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (ec != hipSuccess) {
      if (!comm_) check_hip(ec, "cycle graph capture");
      (void)hipGetLastError();
      capture_failed(hipGetErrorString(ec));
      emit_cycle(f, u, s, pre, zero_u);
      return;
    }
    if (graphs_.size() > 16) {
      for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
      graphs_.clear();
    }
    if (comm_ && !graph_replay_matches(ge, f, u, s, pre, zero_u)) {
      (void)hipGraphExecDestroy(ge);
      capture_failed("the replayed graph's iterate differs from the eager cycle's");
      return;  // u holds the eager cycle's result
    }
    it = graphs_.emplace(key, ge).first;
    if (comm_) return;  // the validation ran this cycle
  }
  HVE_HIP(hipGraphLaunch(it->second, s));
}

// Several ranks: a captured cycle is trusted only after one replay has given
// the eager cycle's iterate bit for bit on every rank (the same inputs run
// both ways; u then holds that result).  A graph that captures but replays
// wrongly (a transport whose stream-ordered calls do not record faithfully)
// turns graphs off for the run.
bool DevAMG::graph_replay_matches(hipGraphExec_t ge, const double* f, double* u, hipStream_t s, bool pre,
                                  bool zero_u) {
  (void)f;
  const int n = lev_[0].n;
  double* pb = pre ? presmooth_buffer() : nullptr;
  const int np = pb ? n + lev_[0].hu.n_halo : 0;
  double* save = dalloc<double>((size_t)n + np + 1);
  HVE_HIP(launch_copy(n, u, save, s));
  if (pb) HVE_HIP(launch_copy(np, pb, save + n, s));
  HVE_HIP(hipGraphLaunch(ge, s));
  std::vector<double> hg(n), he(n);
  HVE_HIP(hipMemcpyAsync(hg.data(), u, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  HVE_HIP(launch_copy(n, save, u, s));
  if (pb) HVE_HIP(launch_copy(np, save + n, pb, s));
  emit_cycle(f, u, s, pre, zero_u);
  HVE_HIP(hipMemcpyAsync(he.data(), u, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  HVE_HIP(hipStreamSynchronize(s));
  const double bad = std::memcmp(hg.data(), he.data(), sizeof(double) * n) != 0 ? 1.0 : 0.0;
  HVE_HIP(hipMemcpyAsync(save, &bad, sizeof(double), hipMemcpyHostToDevice, s));
  comm_->allreduce_sum(save, 1, s);
  double any = 0.0;
  HVE_HIP(hipMemcpyAsync(&any, save, sizeof(double), hipMemcpyDeviceToHost, s));
  HVE_HIP(hipStreamSynchronize(s));
  (void)hipFree(save);
  return any == 0.0;
}

// par_amg_solve.c:22 hypre_BoomerAMGSolve
int DevAMG::solve(const double* f, double* u, hipStream_t s, int* iters, double* rel_res) {
  const int n = lev_[0].n;
  double* V = lev_[0].V;
  const double tol = prm.tol;
  double resid_nrm = 1.0, resid_nrm_init = 0.0, rhs_norm = 0.0, relative_resid = 1.0;
  int cycle_count = 0;
  const bool fuse = tol > 0. && can_fuse_presmooth();
  double* pre = fuse ? presmooth_buffer() : nullptr;
  // With the fused residual + first sweep on the delta layout the residual is
  // needed only for its norm: the kernel sums r_i^2 per workgroup and stores
  // no r (one write and one read of the fine vector fewer per iteration).
  // Norms then reduce in another order than the dot kernel's (as the oracle's
  // differs from both); iterates are unchanged.
  const DevLevel& L0 = lev_[0];
  const bool fuse_nrm = fuse && L0.A.in.delta_like() && (L0.A.bd.nrows == 0 || L0.A.bd.delta_like()) && nrm_fusion_;
  double resid_sq = 0.0;
  // r = f - A u, and with fusion the first sweep of the next cycle
  auto residual = [&](bool initial) {
    if (fuse_nrm) {
      DevLevel& L = lev_[0];
      double* xin = u;
      if (x0_buf_) {
        HVE_HIP(launch_copy(L.n, u, x0_buf_, s));
        xin = x0_buf_;
      }
      const double* l1 = L.l1_fly ? nullptr : L.l1;
      const bool ex = L.hu.active() && comm_;
      if (ex) halo_start(L.hu, xin, s);
      HVE_HIP(launch_sell(K_RESID_L1JAC, L.A.in.view(), xin, f, l1, nullptr, 0, nullptr, 1.0, 0.0, s, pre, nrm_part_));
      if (ex) halo_finish(s);
      int np = sell_nrm_parts(L.A.in.view());
      if (L.A.bd.nrows > 0) {
        HVE_HIP(launch_sell(K_RESID_L1JAC, L.A.bd.view(), xin, f, l1, nullptr, 0, nullptr, 1.0, 0.0, s, pre,
                            nrm_part_ + np));
        np += sell_nrm_parts(L.A.bd.view());
      }
      HVE_HIP(launch_sum(np, nrm_part_, dot_part_, dscal_ + 15, s));
      if (comm_) comm_->allreduce_sum(dscal_ + 15, 1, s);
      HVE_HIP(hipMemcpyAsync(hscal_ + 15, dscal_ + 15, sizeof(double), hipMemcpyDeviceToHost, s));
      HVE_HIP(hipStreamSynchronize(s));
      resid_sq = hscal_[15];
    } else if (fuse) {
      DevLevel& L = lev_[0];
      double* xin = u;
      if (x0_buf_) {
        HVE_HIP(launch_copy(L.n, u, x0_buf_, s));
        xin = x0_buf_;
      }
      apply(L.A, &L.hu, K_RESID_L1JAC, xin, f, L.l1_fly ? nullptr : L.l1, nullptr, 0, V, 1.0, 0.0, s, pre);
    } else if (initial) {
      // Vtemp = A u - f  (hypre copies f then Matvec(1, A, u, -1, Vtemp)); the
      // same numbers as f - A u up to the sign, so the norms agree bit for bit
      fine_apply(K_GENERAL, u, f, V, 1.0, -1.0, s);
    } else {
      fine_apply(K_RESID, u, f, V, -1.0, 0.0, s);
    }
  };
  bool pre_ready = false;
  if (tol > 0.) {
    residual(true);
    pre_ready = fuse;
    resid_nrm = std::sqrt(fuse_nrm ? resid_sq : dot_host(n, V, V, s));
    if (resid_nrm != 0.) {
      double ieee = resid_nrm / resid_nrm;
      if (ieee != ieee) return HYPRE_ERROR_GENERIC_CODE;
    }
    resid_nrm_init = resid_nrm;
    if (prm.converge_type == 0) {
      rhs_norm = std::sqrt(dot_host(n, f, f, s));
      relative_resid = rhs_norm ? resid_nrm_init / rhs_norm : resid_nrm_init;
    }
  }
  while ((relative_resid >= tol || cycle_count < prm.min_iter) && cycle_count < prm.max_iter) {
    cycle(f, u, s, pre_ready ? pre : nullptr);
    pre_ready = false;
    if (tol > 0.) {
      residual(false);
      pre_ready = fuse;
      resid_nrm = std::sqrt(fuse_nrm ? resid_sq : dot_host(n, V, V, s));
      if (prm.converge_type == 0) relative_resid = rhs_norm ? resid_nrm / rhs_norm : resid_nrm;
      else relative_resid = resid_nrm / resid_nrm_init;
      if (prm.print_level > 1)
        fprintf(stderr, "    Cycle %2d   %e          %e \n", cycle_count + 1, resid_nrm, relative_resid);
    }
    ++cycle_count;
  }
  if (iters) *iters = cycle_count;
  if (rel_res) *rel_res = relative_resid;
  if (cycle_count == prm.max_iter && tol > 0.) return HYPRE_ERROR_CONV_CODE;
  return 0;
}

// krylov/pcg.c:271 hypre_PCGSolve (two_norm selectable; stop_crit/rel_change
// off; no recompute) with one BoomerAMG cycle on a cleared vector as the
// preconditioner (HYPRE_BoomerAMGSolve with tol 0, max_iter 1).  Scalars stay
// on the device; one host read per iteration for the convergence test.
int pcg_solve(DevAMG* amg, int n, const MatvecFn& Aop, const PCGParams& prm, const Precond& user_precond,
              const double* b, double* x, hipStream_t s, int* iters, double* rel_res) {
  double* r = amg->scratch(0);
  double* p = amg->scratch(1);
  double* sv = amg->scratch(2);
  double* sc = nullptr;  // device scalars: 0 gamma,1 gamma_old,2 sdotp,3 alpha,4 beta,5 i_prod,6 flag
  double* hs = nullptr;
  HVE_HIP(hipMalloc((void**)&sc, 8 * sizeof(double)));
  HVE_HIP(hipHostMalloc((void**)&hs, 8 * sizeof(double), hipHostMallocDefault));
  HVE_HIP(hipMemsetAsync(sc, 0, 8 * sizeof(double), s));
  // ClearVector(z) (pcg.c:434) and the preconditioner: the callee knows z is
  // zero (a BoomerAMG cycle starts with the zero-guess sweep instead)
  auto precond = [&](const double* rr, double* zz) { user_precond(rr, zz, true); };
  auto read = [&]() {
    HVE_HIP(hipMemcpyAsync(hs, sc, 8 * sizeof(double), hipMemcpyDeviceToHost, s));
    HVE_HIP(hipStreamSynchronize(s));
  };
  double bi_prod;
  int i = 0, ret = 0;
  double i_prod = 0.0, i_prod_0 = 0.0;
  if (prm.two_norm) {
    amg->dot(n, b, b, sc + 7, s);
  } else {
    precond(b, p);
    amg->dot(n, p, b, sc + 7, s);
  }
  read();
  bi_prod = hs[7];
  double eps = prm.tol * prm.tol;
  if (bi_prod > 0.0) {
    eps = std::max(prm.tol * prm.tol, prm.atol * prm.atol / bi_prod);
  } else {
    HVE_HIP(launch_copy(n, b, x, s));
    HVE_HIP(hipStreamSynchronize(s));
    if (iters) *iters = 0;
    if (rel_res) *rel_res = 0.0;
    hipFree(sc); hipHostFree(hs);
    return 0;
  }
  // r = b - A x
  Aop(K_RESID, x, b, r, nullptr);
  precond(r, p);
  amg->dot(n, r, p, sc + 0, s);  // gamma
  if (prm.two_norm) amg->dot(n, r, r, sc + 5, s);
  read();
  i_prod_0 = prm.two_norm ? hs[5] : hs[0];
  while (i + 1 <= prm.max_iter) {
    ++i;
    Aop(K_MATVEC, p, nullptr, sv, sc + 2);                 // s = A p, sdotp = <s,p>
    HVE_HIP(launch_pcg_alpha(sc, s));
    // x += alpha p; r += -alpha s; i_prod = <r,r> (two-norm test)
    amg->pcg_update(n, sc + 3, p, sv, x, r, prm.two_norm ? sc + 5 : nullptr, s);
    precond(r, sv);
    amg->dot(n, r, sv, sc + 0, s);                         // gamma = <r,s>
    read();
    const double flag = hs[6];
    const double gamma = hs[0];
    if (flag != 0.0) {  // zero <s,p> or subnormal alpha: x, r untouched (alpha = 0)
      if (i == 1) i_prod = i_prod_0;
      ret = HYPRE_ERROR_CONV_CODE;  // pcg.c:516-526 hypre_error_w_msg(HYPRE_ERROR_CONV, ...)
      break;
    }
    i_prod = prm.two_norm ? hs[5] : gamma;
    if (prm.print_level > 1) fprintf(stderr, "% 5d    %e    %e\n", i, std::sqrt(i_prod), std::sqrt(i_prod / bi_prod));
    if (i_prod / bi_prod < eps) break;
    if (!(gamma > 2.2250738585072014e-308)) {  // pcg.c:680 "Subnormal gamma value"
      ret = HYPRE_ERROR_CONV_CODE;
      break;
    }
    HVE_HIP(launch_pcg_beta(sc, s));
    HVE_HIP(launch_pcg_p(n, sc + 4, sv, p, s));  // p = beta p + s
  }
  if (i >= prm.max_iter && (i_prod / bi_prod) >= eps && eps > 0) ret = HYPRE_ERROR_CONV_CODE;
  if (iters) *iters = i;
  if (rel_res) *rel_res = bi_prod > 0.0 ? std::sqrt(i_prod / bi_prod) : 0.0;
  HVE_HIP(hipStreamSynchronize(s));
  hipFree(sc);
  hipHostFree(hs);
  return ret;
}

}  // namespace hve
