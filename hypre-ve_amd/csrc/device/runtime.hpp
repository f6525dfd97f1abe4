// Device-side runtime for the BoomerAMG solve path: operators resident in HBM,
// the cycle driver (hypre_BoomerAMGCycle control flow) launching HIP kernels on
// one stream, whole-cycle hipGraph capture, and the BoomerAMG / PCG loops.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../host/hve_host.hpp"
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
  SellView view() const {
    SellView v;
    v.slice_ptr = slice_ptr; v.col = col; v.val = val; v.nrows = nrows; v.ncols = ncols;
    return v;
  }
  void upload(const CSR& A);
  void release();
  size_t bytes() const { return (size_t)(nslices + 1) * 4 + (size_t)nnz_pad * 12; }
};

struct DevLevel {
  int n = 0;
  DevSell A, P, R;        // P: n x n_{l+1}; R = P^T: n_{l+1} x n
  double* l1 = nullptr;   // smoother scaling (l1 norms or diagonal)
  int* cf = nullptr;
  double* F = nullptr;    // rhs of this level (level 0: internal copy slot unused)
  double* U[2] = {nullptr, nullptr};
  double* V = nullptr;    // Vtemp
  double* Z = nullptr;    // Ztemp (hybrid GS off-block copy)
};

struct KernelStats {
  double ms[8] = {0};
};

class DevAMG {
 public:
  DevAMG() = default;
  ~DevAMG();
  void build(const Hierarchy& H);
  // Scratch/dot workspace only (PCG without an AMG preconditioner).
  void init_workspace(int n);
  void release();
  bool built() const { return !lev_.empty(); }

  // One hypre_BoomerAMGCycle on device vectors f, u (natural order, length n0).
  void cycle(const double* f, double* u, hipStream_t s);
  // hypre_BoomerAMGSolve.  Returns 0 or HYPRE_ERROR_CONV-style flag.
  int solve(const double* f, double* u, hipStream_t s, int* iters, double* rel_res);
  // device dot product into a device scalar
  void dot(int n, const double* x, const double* y, double* out, hipStream_t s);
  double dot_host(int n, const double* x, const double* y, hipStream_t s);
  int n0() const { return lev_.empty() ? 0 : lev_[0].n; }
  int ws_n() const { return ws_n_; }
  int num_levels() const { return (int)lev_.size(); }
  const DevLevel& level(int l) const { return lev_[l]; }
  const DevSell& fineA() const { return lev_[0].A; }
  hipStream_t stream() const { return stream_; }
  double* scratch(int i) { return scratch_[i]; }
  void set_use_graph(bool g) { use_graph_ = g; }
  double cycle_op_count() const { return cycle_ops_; }

  AMGParams prm;

 private:
  void emit_cycle(const double* f, double* u, hipStream_t s);
  void relax(int level, int relax_type, int relax_points, const double* f, double*& u_cur, double*& u_alt,
             bool zero_guess, hipStream_t s);
  std::vector<DevLevel> lev_;
  int coarse_n_ = 0;
  double* coarse_L_ = nullptr;
  unsigned char* coarse_mask_ = nullptr;
  double* coarse_U_ = nullptr;
  double* dot_part_ = nullptr;
  double* dscal_ = nullptr;  // device scalars
  double* hscal_ = nullptr;  // pinned host scalars
  double* scratch_[4] = {nullptr, nullptr, nullptr, nullptr};
  hipStream_t stream_ = nullptr;
  bool use_graph_ = true;
  double cycle_ops_ = 0;
  int ws_n_ = 0;
  std::map<std::pair<const void*, const void*>, hipGraphExec_t> graphs_;
};

// PCG (krylov/pcg.c:262) with a BoomerAMG V-cycle as preconditioner.
struct PCGParams {
  double tol = 1e-6, atol = 0.0;
  int max_iter = 1000;
  int two_norm = 0;
  int print_level = 0;
};
// precond(r, z): z = M^{-1} r on stream s (z need not be cleared by the caller).
using Precond = std::function<void(const double* r, double* z)>;
int pcg_solve(DevAMG* ws, const DevSell& A, const PCGParams& prm, const Precond& precond, const double* b, double* x,
              hipStream_t s, int* iters, double* rel_res);

}  // namespace hve
