// Device-side runtime for the BoomerAMG solve path: operators resident in HBM,
// the cycle driver (hypre_BoomerAMGCycle control flow) launching HIP kernels on
// one stream, halo exchange over RCCL on a side stream, whole-cycle hipGraph
// capture, and the BoomerAMG / PCG loops.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <map>
#include <string>
#include <tuple>
#include <utility>
#include <cstdlib>
#include <vector>

#include "../host/hve_host.hpp"
#include "../host/partition.hpp"
#include "comm.hpp"
#include "kernels.h"

namespace hve {

enum { HYPRE_ERROR_GENERIC_CODE = 1, HYPRE_ERROR_CONV_CODE = 256 };

void check_hip(hipError_t e, const char* what);
#define HVE_HIP(x) ::hve::check_hip((x), #x)

struct DevSell {
  int nrows = 0, ncols = 0, nslices = 0;
  int64_t nnz = 0, nnz_pad = 0;
  int* slice_ptr = nullptr;
  int* col = nullptr;
  double* val = nullptr;
  int* rowmap = nullptr;
  int* rowlen = nullptr;  // jagged layout only
  unsigned short* col16 = nullptr;  // dictionary layout: local columns
  int* dict_ptr = nullptr;
  int* dict = nullptr;
  int dmax = 0;
  int dict_group = 1;
  int dict_ranges = 0;     // dictionary layout: the tile is a union of column ranges
  int* wptr = nullptr;     // dictionary layout, lane-packed streams (SellView::wptr)
  int64_t wval_n = 0, wcol_n = 0;  // their stored values / columns (padding included)
  short* dcol = nullptr;   // delta layout: 16-bit column deltas
  int* slot_base = nullptr;
  unsigned char* vidx = nullptr;  // delta layout with a value table
  int* slot_vi = nullptr;            // stencil layout: value index per (slice, slot)
  uint64_t* slot_mask = nullptr;     // stencil layout: lanes present per (slice, slot)
  int stencil_w = 0;                 // stencil layout: slots per pattern
  int* slice_pat = nullptr;          // stencil layout: pattern of each slice
  int npat = 0;
  unsigned short* vidx16 = nullptr;
  double* vtab = nullptr;
  int nvtab = 0;
  int batch = 8;
  int pipe = 0;
  int wide = 0;
  int pw = 0;
  int* blk_map = nullptr;  // locality traversal of the workgroup row blocks (SellView::blk_map)
  int nblk = 0;
  std::vector<int> blk_host;   // host copy of blk_map
  std::vector<int> pat_host;   // stencil layout: host copy of slice_pat
  int* wave_map = nullptr;     // stencil layout: SellView::wave_map
  int nwave = 0;
  void build_wave_map();
  std::vector<int> stored_map;  // host copy of the stored row -> local row map (empty: identity)
  // offset-coded layout (P_0 / R_0 of a grid hierarchy; SellView::code16)
  unsigned short* code16 = nullptr;
  int* otab = nullptr;
  int notab = 0, vbits = 0;
  int* anc = nullptr;
  int* cmap = nullptr;
  int64_t anc_n = 0, cmap_n = 0;
  // packed layout (SellView::code32): one 32-bit code per slot, the slice
  // bases in slot_base, the values in vtab
  unsigned* code32 = nullptr;
  // stencil layout over a grid in natural order (SellView::gslot, k_grid_stencil)
  GSlot* gslot = nullptr;
  int gnx = 0, gny = 0, gnz = 0, gzc = 0, gz0 = 0, gz1 = 0;
  int grid_nlocal = 0;  // the rank's local rows (columns below it are grid points); configuration
  bool build_grid(const CSR& A, const std::vector<int>& so, const std::vector<int>& svi,
                  const std::vector<uint64_t>& sm, const std::vector<double>& tab, int shift, int nlocal);
  // the operator is also applied by the residual and smoother ops (a level's
  // A), whose kernels do not take the 16-bit value-table dictionary layout;
  // configuration, kept across release()
  bool relax_ops = false;
  SellView view() const {
    SellView v;
    v.slice_ptr = slice_ptr; v.col = col; v.val = val; v.rowmap = rowmap; v.rowlen = rowlen; v.nrows = nrows; v.ncols = ncols; v.batch = batch; v.pipe = pipe; v.wide = wide; v.pw = pw;
    v.col16 = col16; v.dict_ptr = dict_ptr; v.dict = dict; v.dmax = dmax; v.dict_group = dict_group; v.dict_ranges = dict_ranges;
    v.wptr = wptr;
    v.dcol = dcol; v.slot_base = slot_base; v.vidx = vidx; v.vidx16 = vidx16; v.vtab = vtab; v.nvtab = nvtab;
    v.slot_vi = slot_vi; v.slot_mask = slot_mask; v.stencil_w = stencil_w; v.slice_pat = slice_pat;
    v.blk_map = blk_map; v.nblk = nblk; v.wave_map = wave_map; v.nwave = nwave;
    v.code16 = code16; v.otab = otab; v.notab = notab; v.vbits = vbits; v.anc = anc; v.cmap = cmap;
    v.code32 = code32;
    v.gslot = gslot; v.gnx = gnx; v.gny = gny; v.gnz = gnz; v.gzc = gzc; v.gz0 = gz0; v.gz1 = gz1;
    return v;
  }
  // Grid context of an interpolation / restriction operator for the
  // offset-coded layout (build_sell_coded_host): anchors per local row,
  // positions per column, position -> column map.
  struct Coded {
    const std::vector<int>* anc = nullptr;
    const std::vector<int>* colpos = nullptr;
    const std::vector<int>* cmap = nullptr;
  };
  // rowmap: subset row -> local row; empty or identity -> no map
  // policy: AMGParams::sell_policy
  // key: per local row, the sort key of the locality traversal (nullptr: natural order)
  // coded: grid context; the offset-coded layout is tried first where it is given
  // tile: per local row, a key of compact grid tiles; the dictionary layout
  // cuts its slices from rows in that order (fewer distinct columns per group)
  void upload(const CSR& A, const std::vector<int>& rowmap = {}, int policy = 0,
              const std::vector<int64_t>* key = nullptr, const Coded* coded = nullptr,
              const std::vector<int64_t>* tile = nullptr);
  // Workgroup row blocks visited in ascending key of their first row
  // (stored_to_local: stored row -> local row, empty = identity).
  void set_block_order(const std::vector<int>& stored_to_local, const std::vector<int64_t>& key);
  void release();
  int64_t ndict = 0;  // dictionary layout: stored distinct-column entries
  // Bytes one application streams from the stored operator (vectors excluded):
  // per stored slot its column (32-bit, 16-bit delta or 16-bit local column)
  // and value (8 B, or an 8/16-bit index into the LDS value table), plus slice
  // pointers, slot bases, dictionaries, row maps and row lengths.
  // delta or stencil layout: columns as offsets from the row, lane per row,
  // the finest-level fusions (residual norm, l1 on the fly) available
  bool delta_like() const { return dcol != nullptr || slot_mask != nullptr; }
  size_t bytes() const {
    if (slot_mask)  // stencil layout: per (slice, slot) offset, value index, lane mask
      return (size_t)nslices * 4 + (size_t)npat * stencil_w * 16 + (rowmap ? (size_t)nrows * 4 : 0);
    if (code16)  // offset-coded: 2 B a slot, the anchors, the position -> column map once
      return (size_t)(nslices + 1) * 4 + (size_t)nnz_pad * 2 + (size_t)(anc_n + cmap_n) * 4 +
             (rowmap ? (size_t)nrows * 4 : 0) + (rowlen ? (size_t)nrows * 4 : 0);
    if (code32)  // packed: 4 B a slot, a base per slice
      return (size_t)(nslices + 1) * 8 + (size_t)nnz_pad * 4 + (rowmap ? (size_t)nrows * 4 : 0);
    // (lane-packed dictionary streams, wptr: counted by their entries, as the
    // per-entry streams; the tails of odd pairs and short octets, about 3 % at
    // A_1, are overhead of the layout, not algorithmic bytes)
    const size_t colb = dcol || col16 ? 2 : 4;
    const size_t valb = vidx ? 1 : vidx16 ? 2 : 8;
    size_t b = (size_t)(nslices + 1) * 4 + (size_t)nnz_pad * (colb + valb);
    if (dcol) b += (size_t)nnz_pad / 16;  // 4 B base per (slice, slot)
    if (col16) b += (size_t)ndict * 4 + (size_t)((nslices + dict_group - 1) / dict_group + 1) * 4;
    if (wptr) b += (size_t)(nslices + 1) * 4;  // the second slice offset (columns)
    if (rowmap) b += (size_t)nrows * 4;
    if (rowlen) b += (size_t)nrows * 4;
    return b;
  }
};

// Rows of one operator a rank applies, split by whether they read halo values.
struct DevOp {
  DevSell in, bd;
  bool relax_ops = false;  // DevSell::relax_ops of both parts
  int nrows_local = 0;
  int64_t nnz() const { return in.nnz + bd.nnz; }
  // coded: grid context for the interior rows (DevSell::Coded)
  void upload(const RankOp& op, int policy = 0, const std::vector<int64_t>* key = nullptr,
              const DevSell::Coded* coded = nullptr, const std::vector<int64_t>* tile = nullptr);
  void release() { in.release(); bd.release(); }
};

// Packed, step-ordered schedule of one hybrid Gauss-Seidel sweep direction,
// in HBM (host/layout.hpp GsSchedule).
struct DevGs {
  int* team_step = nullptr;
  int* step = nullptr;
  int* code = nullptr;
  double* val = nullptr;          // null when vidx8 holds the values
  unsigned char* vidx8 = nullptr;  // 8-bit indices into vtab (<= 256 distinct values)
  double* vtab = nullptr;
  int nvtab = 0;
  int* tcol = nullptr;  // only when a weighted form may run
  int* rowmap = nullptr;
  int* pos = nullptr;    // rowmap^-1
  double* l1 = nullptr;  // by position
  int* cf = nullptr;     // by position
  int nrows = 0, nteams = 0, nblocks = 0, max_steps = 0, max_width = 0;
  bool one_chunk = false;
  int cap = 512;  // unit capacity of the pipelined sweep (GsView::cap)
  int ring_w = 64;
  int64_t entries = 0, nnz = 0;
  bool built() const { return nblocks > 0; }
  GsView view() const {
    GsView v;
    v.team_step = team_step; v.step = step; v.code = code; v.val = val; v.tcol = tcol; v.rowmap = rowmap;
    v.pos = pos; v.l1 = l1; v.cf = cf; v.nteams = nteams; v.nrows = nrows; v.max_width = max_width;
    v.one_chunk = one_chunk;
    v.cap = cap;
    v.ring_w = ring_w;
    v.vidx8 = vidx8; v.vtab = vtab; v.nvtab = nvtab;
    return v;
  }
  void upload(const CSR& A, const std::vector<int>& block_starts, bool forward, bool weighted,
              const std::vector<double>& l1_rows, const std::vector<int>& cf_rows);
  void release();
};

struct DevHalo {
  int n_loc = 0, n_halo = 0, n_send = 0;
  std::vector<int> peers, recv_cnt, recv_off, send_cnt, send_off;
  int* d_send_idx = nullptr;
  double* d_sendbuf = nullptr;
  bool active() const { return !peers.empty(); }
  void upload(const RankHalo& h);
  void release();
};

struct DevLevel {
  int n = 0;               // owned rows
  int first = 0, n_glob = 0;
  DevOp A, P, R;
  DevHalo hu, hv;
  double* l1 = nullptr;
  bool l1_fly = false;  // the l1-Jacobi kernels form the l1 norms from A's entries
  int* cf = nullptr;
  // C/F-ordered l1-Jacobi (relax 18, relax_order 1): the CF marker with rows
  // whose diagonal is zero set to 0, which no point class selects
  // (par_relax_more.c:1135 skips them)
  int* cf_l1 = nullptr;
  double* F = nullptr;
  double* U[2] = {nullptr, nullptr};  // n + hu.n_halo each
  double* V = nullptr;                // n + hv.n_halo
  DevGs gs_fwd, gs_bwd;               // hybrid Gauss-Seidel schedules (when a cycle uses them)
  double* gs_G = nullptr;             // the sweep's T | C | U | halo vectors (3n + hu.n_halo)
  double* gs_F = nullptr;             // the sweep's right-hand side (n)
  double* gs_tmp = nullptr;           // symmetric sweeps: u before the first half (n)
  // Chebyshev (relax 16): ds on the device, coefficients on the host (kernel
  // arguments), work vectors r, tmp (n + halo: A is applied to it), orig
  double* cheby_ds = nullptr;
  std::vector<double> cheby_coefs;
  double *cheby_r = nullptr, *cheby_t = nullptr, *cheby_o = nullptr;
};

class DevAMG {
 public:
  DevAMG() = default;
  ~DevAMG();
  // Build from a (rank-local) hierarchy; comm = nullptr for a single rank.
  void build(const RankHierarchy& R, DevComm* comm);
  // Scratch/dot workspace only (PCG without an AMG preconditioner).
  void init_workspace(int n, DevComm* comm);
  void release();
  bool built() const { return !lev_.empty(); }

  // One hypre_BoomerAMGCycle on device vectors f, u (owned rows, length n0).
  // presmoothed: level-0 iterate after the first down sweep, already formed by
  // a fused residual (OP_RESID_L1JAC); nullptr = run that sweep here.
  // zero_u: u holds zeros on entry (the first level-0 sweep takes the zero-guess form)
  void cycle(const double* f, double* u, hipStream_t s, const double* presmoothed = nullptr, bool zero_u = false);
  // PCG pieces: s = A p with <s,p> (fused on the delta layout); x/r update with <r,r>
  void fine_matvec_dot(const double* p, double* sv, double* dot_out, hipStream_t s);
  void pcg_update(int n, const double* alpha_p, const double* p, const double* sv, double* x, double* r,
                  double* rr_out, hipStream_t s);
  int solve(const double* f, double* u, hipStream_t s, int* iters, double* rel_res);
  // y = op(A_0) x on owned rows (halo exchanged through an internal buffer)
  void fine_apply(int op, const double* x, const double* b, double* y, double alpha, double temp, hipStream_t s);
  void dot(int n, const double* x, const double* y, double* out, hipStream_t s);  // global (allreduce)
  double dot_host(int n, const double* x, const double* y, hipStream_t s);
  int n0() const { return lev_.empty() ? ws_n_ : lev_[0].n; }
  int ws_n() const { return ws_n_; }
  int num_levels() const { return (int)lev_.size(); }
  const DevLevel& level(int l) const { return lev_[l]; }
  hipStream_t stream() const { return stream_; }
  double* scratch(int i) { return scratch_[i]; }
  // Whole-cycle hipGraphs: one rank always; several ranks when the transport
  // can be captured (RCCL), unless HVE_GRAPH_MULTI=0.
  void set_use_graph(bool g);
  double cycle_op_count() const { return cycle_ops_; }
  // This rank's communication in one V-cycle (the last one emitted), per level:
  // halo exchanges and the bytes they send, all-gathers into the replicated
  // levels, all-reduces (the coarsest right-hand side).
  struct CycleComm {
    int64_t exchanges = 0, bytes = 0, allgathers = 0, allgather_bytes = 0, allreduces = 0;
  };
  const std::vector<CycleComm>& cycle_comm() const { return cycle_comm_; }
  bool multi_rank() const { return comm_ != nullptr; }
  // Re-key the row-block traversal (tuning; see locality_keys in runtime.hip).
  // which_mask: bit 0 the A operators, bit 1 P, bit 2 R
  void set_block_bands(const RankHierarchy& R, int nbands, int which_mask = 7);
  void graphs_clear();

  AMGParams prm;

 private:
  void emit_cycle(const double* f0, double* u0, hipStream_t s, bool presmoothed, bool zero_u = false);
  bool can_fuse_presmooth() const;
  void capture_failed(const char* why);
  bool graph_replay_matches(hipGraphExec_t ge, const double* f, double* u, hipStream_t s, bool pre, bool zero_u);
  double* presmooth_buffer();
  void relax(int level, int relax_type, int relax_points, const double* f, double*& u_cur, double*& u_alt,
             bool zero_guess, hipStream_t s);
  // y = op(M) x with the halo of x exchanged first (interior rows overlap it)
  void apply(const DevOp& M, const DevHalo* hx, int op, double* x, const double* b, const double* l1,
             const int* cf, int relax_points, double* y, double w, double temp, hipStream_t s,
             double* y2 = nullptr);
  void halo_start(const DevHalo& h, double* x, hipStream_t s);
  void halo_finish(hipStream_t s);
  void coarse_solve(int level, const double* f, double* u, hipStream_t s);
  void allgather_rows(double* v, const std::vector<int>& starts, hipStream_t s);

  std::vector<DevLevel> lev_;
  int coarse_n_ = 0;
  double* coarse_L_ = nullptr;
  unsigned char* coarse_mask_ = nullptr;
  double* coarse_U_ = nullptr;
  double* coarse_f_ = nullptr;  // replicated rhs / solution of the coarsest level
  double* coarse_u_ = nullptr;
  double* u0_buf_[2] = {nullptr, nullptr};  // level-0 iterate with halo space (multi-rank)
  double* x0_buf_ = nullptr;                // fine_apply input with halo space
  double* dot_part_ = nullptr;
  double* nrm_part_ = nullptr;
  size_t nrm_cap_ = 0;  // doubles in nrm_part_
  // grow nrm_part_ to hold the partials of level 0's fused norms / dots
  void size_nrm_parts();
  double* dscal_ = nullptr;  // device scalars
  double* hscal_ = nullptr;  // pinned host scalars
  double* scratch_[4] = {nullptr, nullptr, nullptr, nullptr};
  hipStream_t stream_ = nullptr;
  hipStream_t comm_stream_ = nullptr;
  hipEvent_t ev_packed_ = nullptr, ev_halo_ = nullptr;
  DevComm* comm_ = nullptr;  // not owned
  bool use_graph_ = true;
  // multi-rank: a cycle shape runs eagerly once before it is captured (the
  // transport sets up its peer connections outside the capture)
  std::map<std::tuple<const void*, const void*, int>, int> eager_runs_;
  // the solve loop's residual norm summed inside the fused residual + sweep
  // kernel (no r stored); HVE_NRM_FUSE=0 stores r and runs the dot kernel
  bool nrm_fusion_ = [] {
    const char* e = std::getenv("HVE_NRM_FUSE");
    return !e || std::atoi(e) != 0;
  }();
  double cycle_ops_ = 0;
  std::vector<CycleComm> cycle_comm_;
  int comm_level_ = -1;  // level whose exchanges are being counted (emit_cycle), -1 = none
  int ws_n_ = 0;
  std::map<std::tuple<const void*, const void*, int>, hipGraphExec_t> graphs_;  // (f, u, presmoothed + 2 zero_u)
  int agg_level_ = -1;            // first replicated level (RankHierarchy::agg_level)
  std::vector<int> agg_starts_;   // its rows' distributed owners
};

// Tuning harness (hypreve_BenchOperator): average ms of op on A alone.
double bench_operator(const CSR& A, int op, int policy, int nbands, int reps, double* stored_bytes, char* layout_msg,
                      int msg_len);

// PCG (krylov/pcg.c:271).
struct PCGParams {
  double tol = 1e-6, atol = 0.0;
  int max_iter = 1000;
  int two_norm = 0;
  int print_level = 0;
};
// precond(r, z): z = M^{-1} r on stream s.
// precond(r, z, z_zero): z = C r; z_zero: z holds zeros on entry... or not yet:
// with z_zero the callee must treat z as cleared (it may skip the clearing)
using Precond = std::function<void(const double* r, double* z, bool z_zero)>;
// apply(op, x, b, y, dot): op K_MATVEC (y = A x; dot != null: <y, x> into that
// device scalar) or K_RESID (y = b - A x)
using MatvecFn = std::function<void(int op, const double* x, const double* b, double* y, double* dot)>;
int pcg_solve(DevAMG* ws, int n, const MatvecFn& A, const PCGParams& prm, const Precond& precond, const double* b,
              double* x, hipStream_t s, int* iters, double* rel_res);

}  // namespace hve
