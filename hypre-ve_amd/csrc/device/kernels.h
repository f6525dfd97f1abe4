// Launch interface of the hot-path kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace hve {

// Grid form of a stencil-layout slot (k_grid_stencil): lanes present, value,
// and the neighbour as a plane step dz in {-1, 0, 1} and an in-plane step
// dxy = dy * (64 + 2) + dx in the LDS tile.  32 B: one scalar load.
struct GSlot {
  uint64_t mask;
  double val;
  int dz, dxy, pad0, pad1;
};

// Device view of one SELL-64 operator, padded or jagged (see kernels.hip).
struct SellView {
  const int* slice_ptr = nullptr;  // nslices + 1 offsets (in entries)
  const int* col = nullptr;        // padded; -1 marks padding
  const double* val = nullptr;
  const int* rowmap = nullptr;     // subset row -> local row, nullptr = identity
  const int* rowlen = nullptr;     // jagged layout (no stored padding): stored row -> length
  int nrows = 0;
  int ncols = 0;
  int batch = 0;                   // entries per load batch (8 or 16), 0 = default
  int pipe = 0;                    // 1 = software-pipelined row loop
  int wide = 0;                    // 1 = one workgroup per slice (k_sell_wide), padded layout only
  int pw = 0;                      // 1 = wave product-parallel loop (k_sell_pw), jagged layout only
  const unsigned short* col16 = nullptr;  // dictionary layout (k_sell_dict): local columns
  const int* dict_ptr = nullptr;
  const int* dict = nullptr;
  int dmax = 0;                    // dictionary layout: largest dictionary (LDS doubles)
  int dict_group = 1;              // dictionary layout: slices per dictionary / workgroup (1 or 4)
  int dict_ranges = 0;             // dictionary layout: 1 = (start, offset) column ranges
  // dictionary layout, lane-packed streams (k_sell_dictw; host: pack_dict_wide):
  // val / col16 hold value pairs / column octets per lane, wptr the 2 (nslices + 1)
  // slice offsets (values, then columns); nullptr = the per-entry streams
  const int* wptr = nullptr;
  const short* dcol = nullptr;     // delta layout (k_sell_delta): col - row - slot base, padded
  const int* slot_base = nullptr;  // delta layout: base offset per (slice, slot)
  const unsigned char* vidx = nullptr;  // delta layout: 8-bit value indices (val unused)
  const unsigned short* vidx16 = nullptr;  // delta layout: 16-bit value indices (val unused)
  const double* vtab = nullptr;         // the operator's distinct values
  const int* slot_vi = nullptr;         // stencil layout (no per-entry data): value index,
  const uint64_t* slot_mask = nullptr;  // lanes present, offset (slot_base) per (slice, slot)
  int stencil_w = 0;                    // stencil layout: slots per pattern
  const int* slice_pat = nullptr;       // stencil layout: slot pattern of each slice
  int nvtab = 0;
  // Traversal order of the workgroup row blocks (logical block -> stored row
  // block, nullptr = identity): blocks are visited so that each XCD streams a
  // compact region of the grid whose x window stays in its L2.  Only the order
  // changes, not any row's arithmetic.
  const int* blk_map = nullptr;
  int nblk = 0;
  // stencil layout, one slice per wave: per logical wave (traversal order)
  // its stored slice and that slice's pattern, {slice, pattern} pairs (slice
  // -1: no rows), so a wave finds its slot data with one scalar load instead
  // of two dependent ones (traversal map, then pattern index)
  const int* wave_map = nullptr;
  int nwave = 0;
  // offset-coded layout (k_sell_code; host: build_sell_coded_host): per entry
  // one 16-bit code (offset index << vbits | value index into vtab); column =
  // a + otab[offset index], or cmap[a + otab[..]], a = anc[row] (the row itself
  // when anc is null)
  const unsigned short* code16 = nullptr;
  const int* otab = nullptr;
  int notab = 0;
  int vbits = 0;
  const int* anc = nullptr;
  const int* cmap = nullptr;
  // packed layout (k_sell_code PK; host: pack_sell_codes): per entry one 32-bit
  // code ((column - slot_base[slice]) << vbits | value index into vtab)
  const unsigned* code32 = nullptr;
  // stencil layout over the points of a gnx x gny x gnz grid in natural order
  // (k_grid_stencil: LDS x-tile, gzc planes per workgroup); gslot per
  // (pattern, slot), nullptr = the per-slice loop
  const GSlot* gslot = nullptr;
  int gnx = 0, gny = 0, gnz = 0, gzc = 0;
  int gz0 = 0, gz1 = 0;  // the stored rows: planes gz0 .. gz1 - 1 (row i = grid point i + gz0 * gnx * gny)
};

enum : int {
  K_RESID = 0, K_MATVEC = 1, K_L1JAC = 2, K_L1JAC_W = 3, K_JAC = 4,
  K_PROLONG = 5, K_RESTRICT = 6, K_GENERAL = 7, K_RESID_L1JAC = 8, K_RESTRICT_ZG = 9,
};

// nrm (K_RESID_L1JAC on the delta layout only): the residual's squares summed
// per workgroup into nrm[0 .. sell_nrm_parts(M)) (y may then be null: r not stored).
int sell_nrm_parts(const SellView& M);
// The grid-stencil loop's 32-bit byte offsets reach every point of an
// nx x ny x nz grid (DevSell::build_grid refuses the grid form otherwise).
bool grid_stencil_addressable(int64_t nx, int64_t ny, int64_t nz);
hipError_t launch_sell(int op, const SellView& M, const double* x, const double* b, const double* l1,
                       const int* cf, int relax_points, double* y, double w, double temp, hipStream_t s,
                       double* y2 = nullptr, double* nrm = nullptr);
// PCG: x += alpha p; r += (-alpha) s; part[0 .. pcg_xr_parts()) = per-workgroup
// sums of the new r_i^2 (part may be null)
hipError_t launch_pcg_xr(int n, const double* alpha_p, const double* p, const double* s, double* x, double* r,
                         double* part, hipStream_t st);
int pcg_xr_parts();
// *out = sum of part[0 .. nparts) in a fixed order (work: 1024 doubles)
hipError_t launch_sum(int nparts, const double* part, double* work, double* out, hipStream_t st);
// Chebyshev steps (kernels.hip k_cheby): 0 start, 1 tmp = ds*u, 2 update, 3 finish
hipError_t launch_cheby(int n, int step, int scale, double c, const double* ds, const double* f, double* r,
                        double* tmp, const double* v, double* orig, double* u, hipStream_t st);
// op: 0 l1-Jacobi w=1, 1 l1-Jacobi weighted, 2 Jacobi (s = diagonal)
hipError_t launch_zero_guess(int n, int op, double w, const double* f, const double* s, double* u,
                             hipStream_t st);
// Device view of a packed, step-ordered hybrid Gauss-Seidel schedule
// (host/layout.hpp GsSchedule).
struct GsView {
  const int* team_step = nullptr;  // nteams + 1 step ranges
  const int* step = nullptr;       // 4 per step: entry offset (unsigned), position offset, rows, width
  const int* code = nullptr;       // per entry: source code (layout.hpp)
  const double* val = nullptr;     // null when vidx8 is set
  const unsigned char* vidx8 = nullptr;  // 8-bit indices into vtab (k_hybrid_gs_pipe only)
  const double* vtab = nullptr;
  int nvtab = 0;
  const int* tcol = nullptr;       // weighted forms: in-block entries' T position (-1 otherwise)
  const int* rowmap = nullptr;     // position -> row
  const int* pos = nullptr;        // row -> position
  const double* l1 = nullptr;      // l1 norms by position
  const int* cf = nullptr;         // CF marker by position
  int nteams = 0, nrows = 0, max_width = 0;
  bool one_chunk = false;  // every step's rows x width fits one product chunk (k_hybrid_gs_pipe)
  int cap = 512;           // entries a unit of the pipelined sweep holds at most (128 | 256 | 512)
  int ring_w = 64;         // lanes of an LDS ring slot = most rows a step (GsSchedule::ring_w)
};
// entries of one product chunk of the hybrid-GS kernels (LDS per wave)
int gs_chunk_entries();
// whether launch_hybrid_gs takes the pipelined sweep for a schedule
bool gs_uses_pipe(bool one_chunk);
// The sweep's vectors in its order (layout.hpp GsSchedule): G[k] = tmp[rowmap[k]]
// (T; not written when tmp is null: the sweep then reads T from C, t_is_c),
// G[n + k] = u[rowmap[k]] (C), F[k] = f[rowmap[k]],
// and the off-rank halo of u, u[n .. n + nhalo), into G[3n ..).
hipError_t launch_gs_gather(const GsView& S, const double* u, const double* tmp, const double* f, int nhalo,
                            double* G, double* F, hipStream_t st);
// One hybrid Gauss-Seidel sweep over S: reads G's T, C and halo parts and F,
// writes G's U part, then scatters it into u (natural rows).  G (3n + nhalo
// doubles) must stay below 4 GiB.
hipError_t launch_hybrid_gs(const GsView& S, bool use_l1, bool cfsel, int relax_points, double* G, int nhalo,
                            const double* F, double* u, double w, double omega, bool t_is_c, hipStream_t st);
int sell_batch_override();
// Tuning knobs read at launch (0 = default): 0 offset-coded row blocks per
// step (1, 2, 4), 1 its codes per batch (4, 8, 16), 2 its workgroups per CU,
// 3 stream-mix access width (2: 16 B), 7 caps the device setup's LDS tables
// at 2^v slots (tests of its host fallback), 9 the planes a grid-stencil
// workgroup marches (k_grid_stencil) at the next Setup, 11 shortens the
// hybrid-GS ring reach (tests of gs_schedule_self_check).
void set_knob(int id, int v);
int knob(int id);
int stencil_slices_per_wave();
int stencil_grid(int nrows);
bool grid_stencil_on(const SellView& M);
int grid_stencil_blocks(const SellView& M);
int grid_stencil_waves();  // waves per workgroup (tiles of 64 x 4 waves lines)
int grid_stencil_ty();
bool stencil_wave_map();
int sell_pipe_override();
bool sell_nt();
bool sell_pw();
// y = sum of `reads` (1, 2 or 5) consecutive n-double streams of src: a
// read/write mix of reads*8 B in and 8 B out per element.
hipError_t launch_stream_mix(int64_t n, int reads, const double* src, double* y, hipStream_t st);
hipError_t launch_stream_read(int64_t n_bytes, int elem_bytes, const void* buf, double* out, hipStream_t st);
// n doubles read as per-wave 16 KiB segments (interleave: a workgroup's 4 waves
// alternate over 512-B chunks of its 64 KiB)
hipError_t launch_stream_seg(int64_t n, bool interleave, const double* buf, double* out, hipStream_t st);
hipError_t launch_gather(int n, const int* idx, const double* x, double* out, hipStream_t st);
hipError_t launch_axpy(int n, const double* alpha_p, double alpha, double sgn, const double* x, double* y,
                       hipStream_t st);
hipError_t launch_scale(int n, const double* alpha_p, double alpha, double* y, hipStream_t st);
hipError_t launch_set(int n, double v, double* y, hipStream_t st);
hipError_t launch_copy(int n, const double* x, double* y, hipStream_t st);
hipError_t launch_pcg_p(int n, const double* beta_p, const double* s, double* p, hipStream_t st);
int dot_num_parts(int n);
hipError_t launch_dot(int n, const double* x, const double* y, double* part, double* out, hipStream_t st);
hipError_t launch_pcg_alpha(double* sc, hipStream_t st);
hipError_t launch_pcg_beta(double* sc, hipStream_t st);
hipError_t launch_coarse(int n, const double* Lf, const unsigned char* Lmask, const double* U,
                         const double* f, double* u, hipStream_t st);

}  // namespace hve
