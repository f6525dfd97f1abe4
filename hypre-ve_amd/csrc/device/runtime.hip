// Device runtime: hierarchy upload, cycle driver, BoomerAMG solve loop and PCG.
// Control flow mirrors the reference routines cited per function; every
// arithmetic step runs in a HIP kernel (kernels.hip) -- there is no host path.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../host/layout.hpp"
#include "runtime.hpp"

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
  HVE_HIP(hipMalloc((void**)&p, n * sizeof(T)));
  return p;
}
template <typename T>
static T* dupload(const T* h, size_t n) {
  T* p = dalloc<T>(n);
  if (n) HVE_HIP(hipMemcpy(p, h, n * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

void DevSell::upload(const CSR& A) {
  release();
  std::vector<int> sp, col;
  std::vector<double> val;
  build_sell_host(A, sp, col, val);
  nrows = A.nrows;
  ncols = A.ncols;
  nslices = (int)sp.size() - 1;
  nnz = A.nnz();
  nnz_pad = (int64_t)col.size();
  slice_ptr = dupload(sp.data(), sp.size());
  this->col = dupload(col.data(), col.size());
  this->val = dupload(val.data(), val.size());
}
void DevSell::release() {
  if (slice_ptr) hipFree(slice_ptr);
  if (col) hipFree(col);
  if (val) hipFree(val);
  slice_ptr = nullptr; col = nullptr; val = nullptr;
  nrows = ncols = nslices = 0; nnz = nnz_pad = 0;
}

DevAMG::~DevAMG() { release(); }

void DevAMG::release() {
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  graphs_.clear();
  for (auto& L : lev_) {
    L.A.release(); L.P.release(); L.R.release();
    if (L.l1) hipFree(L.l1);
    if (L.cf) hipFree(L.cf);
    if (L.F) hipFree(L.F);
    if (L.U[0]) hipFree(L.U[0]);
    if (L.U[1]) hipFree(L.U[1]);
    if (L.V) hipFree(L.V);
    if (L.Z) hipFree(L.Z);
  }
  lev_.clear();
  if (coarse_L_) hipFree(coarse_L_);
  if (coarse_mask_) hipFree(coarse_mask_);
  if (coarse_U_) hipFree(coarse_U_);
  coarse_L_ = nullptr; coarse_mask_ = nullptr; coarse_U_ = nullptr;
  if (dot_part_) hipFree(dot_part_);
  if (dscal_) hipFree(dscal_);
  if (hscal_) hipHostFree(hscal_);
  for (auto& s : scratch_) { if (s) hipFree(s); s = nullptr; }
  dot_part_ = nullptr; dscal_ = nullptr; hscal_ = nullptr;
  if (stream_) hipStreamDestroy(stream_);
  stream_ = nullptr;
}

void DevAMG::build(const Hierarchy& H) {
  release();
  prm = H.prm;
  HVE_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  const int nl = (int)H.lev.size();
  lev_.resize(nl);
  for (int l = 0; l < nl; ++l) {
    const Level& L = H.lev[l];
    DevLevel& D = lev_[l];
    D.n = L.A.nrows;
    D.A.upload(L.A);
    if (l < nl - 1) {
      D.P.upload(L.P);
      D.R.upload(L.R);
    }
    if (!L.l1.empty()) D.l1 = dupload(L.l1.data(), L.l1.size());
    if (!L.cf.empty()) D.cf = dupload(L.cf.data(), L.cf.size());
    D.F = dalloc<double>(D.n);
    D.U[0] = dalloc<double>(D.n);
    D.U[1] = dalloc<double>(D.n);
    D.V = dalloc<double>(D.n);
    D.Z = dalloc<double>(D.n);
    HVE_HIP(hipMemset(D.F, 0, sizeof(double) * D.n));
    HVE_HIP(hipMemset(D.U[0], 0, sizeof(double) * D.n));
    HVE_HIP(hipMemset(D.U[1], 0, sizeof(double) * D.n));
  }
  coarse_n_ = H.coarse_n;
  if (coarse_n_ > 0) {
    std::vector<double> Lf, U;
    std::vector<unsigned char> mask;
    gselim_factor(coarse_n_, H.coarse_dense, Lf, mask, U);
    coarse_L_ = dupload(Lf.data(), Lf.size());
    coarse_mask_ = dupload(mask.data(), mask.size());
    coarse_U_ = dupload(U.data(), U.size());
  }
  dot_part_ = dalloc<double>(1024);
  dscal_ = dalloc<double>(16);
  HVE_HIP(hipMemset(dscal_, 0, 16 * sizeof(double)));
  HVE_HIP(hipHostMalloc((void**)&hscal_, 16 * sizeof(double), hipHostMallocDefault));
  for (auto& s : scratch_) s = dalloc<double>(lev_[0].n);
  ws_n_ = lev_[0].n;
  HVE_HIP(hipDeviceSynchronize());
}

void DevAMG::init_workspace(int n) {
  release();
  HVE_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  dot_part_ = dalloc<double>(1024);
  dscal_ = dalloc<double>(16);
  HVE_HIP(hipMemset(dscal_, 0, 16 * sizeof(double)));
  HVE_HIP(hipHostMalloc((void**)&hscal_, 16 * sizeof(double), hipHostMallocDefault));
  for (auto& s : scratch_) s = dalloc<double>(n);
  ws_n_ = n;
}

void DevAMG::dot(int n, const double* x, const double* y, double* out, hipStream_t s) {
  HVE_HIP(launch_dot(n, x, y, dot_part_, out, s));
}
double DevAMG::dot_host(int n, const double* x, const double* y, hipStream_t s) {
  dot(n, x, y, dscal_ + 15, s);
  HVE_HIP(hipMemcpyAsync(hscal_ + 15, dscal_ + 15, sizeof(double), hipMemcpyDeviceToHost, s));
  HVE_HIP(hipStreamSynchronize(s));
  return hscal_[15];
}

// One smoothing step on `level` (par_cycle.c:333-505 dispatch).  u_cur holds the
// current iterate; out-of-place smoothers write u_alt and swap the two.
void DevAMG::relax(int level, int relax_type, int relax_points, const double* f, double*& u_cur,
                   double*& u_alt, bool zero_guess, hipStream_t s) {
  DevLevel& L = lev_[level];
  const double w = prm.relax_weight;
  const int n = L.n;
  if (zero_guess && relax_points != 0) {
    HVE_HIP(launch_set(n, 0.0, u_cur, s));
    zero_guess = false;
  }
  switch (relax_type) {
    case 18:
    case 7: {
      if (!L.l1) throw std::runtime_error("l1 norms missing for relax type 18/7");
      if (relax_points != 0) throw std::runtime_error("C/F-ordered l1-Jacobi is not available on the GPU path");
      if (zero_guess) {
        HVE_HIP(launch_zero_guess(n, w == 1.0 ? 0 : 1, w, f, L.l1, u_cur, s));
      } else {
        HVE_HIP(launch_sell(w == 1.0 ? K_L1JAC : K_L1JAC_W, L.A.view(), u_cur, f, L.l1, nullptr, 0, u_alt, w,
                            0.0, s));
        std::swap(u_cur, u_alt);
      }
      break;
    }
    case 0: {
      if (zero_guess) HVE_HIP(launch_set(n, 0.0, u_cur, s));
      HVE_HIP(launch_sell(K_JAC, L.A.view(), u_cur, f, nullptr, L.cf, relax_points, u_alt, w, 0.0, s));
      std::swap(u_cur, u_alt);
      break;
    }
    default:
      throw std::runtime_error("relax_type " + std::to_string(relax_type) +
                               " is not available on the GPU path in this build");
  }
}

// par_cycle.c:22 hypre_BoomerAMGCycle, emitted as a kernel sequence.
void DevAMG::emit_cycle(const double* f0, double* u0, hipStream_t s) {
  const int nl = (int)lev_.size();
  std::vector<int> lev_counter(nl, prm.cycle_type);
  std::vector<double*> ucur(nl), ualt(nl);
  std::vector<const double*> fl(nl);
  std::vector<char> zero(nl, 0);
  lev_counter[0] = 1;
  ucur[0] = u0;
  ualt[0] = lev_[0].U[0];
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
      relax_type = prm.relax_type[0] >= 0 ? prm.relax_type[0] : 6;
    }
    for (int j = 0; j < num_sweep; ++j) {
      ops += (double)lev_[level].A.nnz;
      if (relax_type == 9 || relax_type == 99 || relax_type == 19 || relax_type == 98) {
        if (coarse_n_ != lev_[level].n) throw std::runtime_error("coarse solve size mismatch");
        HVE_HIP(launch_coarse(coarse_n_, coarse_L_, coarse_mask_, coarse_U_, fl[level], ucur[level], s));
        zero[level] = 0;
      } else if (relax_type == 18 || relax_type == 7) {
        relax(level, relax_type, 0, fl[level], ucur[level], ualt[level], zero[level], s);
        zero[level] = 0;
      } else {
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
      // Vtemp = f - A u  (csr_matvec.c, alpha=-1 beta=1);  F_c = P^T Vtemp
      HVE_HIP(launch_sell(K_RESID, Lf.A.view(), ucur[fine], fl[fine], nullptr, nullptr, 0, Lf.V, -1.0, 0.0, s));
      HVE_HIP(launch_sell(K_RESTRICT, Lf.R.view(), Lf.V, nullptr, nullptr, nullptr, 0, lev_[coarse].F, 1.0, 0.0,
                          s));
      ++level;
      lev_counter[level] = std::max(lev_counter[level], prm.cycle_type);
      cycle_param = (level == nl - 1) ? 3 : 1;
      zero[level] = 1;  // U_array[coarse] = 0 (par_cycle.c:556), folded into the next smoother
    } else if (level != 0) {
      const int fine = level - 1, coarse = level;
      if (zero[coarse]) HVE_HIP(launch_set(lev_[coarse].n, 0.0, ucur[coarse], s));
      zero[coarse] = 0;
      // u_f = u_f + P u_c  (alpha=1, beta=1)
      HVE_HIP(launch_sell(K_PROLONG, lev_[fine].P.view(), ucur[coarse], nullptr, nullptr, nullptr, 0, ucur[fine],
                          1.0, 0.0, s));
      --level;
      cycle_param = 2;
    } else {
      done = true;
    }
  }
  if (ucur[0] != u0) HVE_HIP(launch_copy(lev_[0].n, ucur[0], u0, s));
  cycle_ops_ = ops;
}

void DevAMG::cycle(const double* f, double* u, hipStream_t s) {
  if (!use_graph_) {
    emit_cycle(f, u, s);
    return;
  }
  auto key = std::make_pair((const void*)f, (const void*)u);
  auto it = graphs_.find(key);
  if (it == graphs_.end()) {
    hipGraph_t g;
    HVE_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
      emit_cycle(f, u, s);
    } catch (...) {
      hipGraph_t tmp;
      hipStreamEndCapture(s, &tmp);
      if (tmp) hipGraphDestroy(tmp);
      throw;
    }
    HVE_HIP(hipStreamEndCapture(s, &g));
    hipGraphExec_t ge;
    HVE_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HVE_HIP(hipGraphDestroy(g));
    if (graphs_.size() > 16) {
      for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
      graphs_.clear();
    }
    it = graphs_.emplace(key, ge).first;
  }
  HVE_HIP(hipGraphLaunch(it->second, s));
}

// par_amg_solve.c:22 hypre_BoomerAMGSolve
int DevAMG::solve(const double* f, double* u, hipStream_t s, int* iters, double* rel_res) {
  const int n = lev_[0].n;
  double* V = lev_[0].V;
  const double tol = prm.tol;
  double resid_nrm = 1.0, resid_nrm_init = 0.0, rhs_norm = 0.0, relative_resid = 1.0;
  int cycle_count = 0;
  if (tol > 0.) {
    // Vtemp = A u - f  (hypre copies f then Matvec(1, A, u, -1, Vtemp))
    HVE_HIP(launch_sell(K_GENERAL, lev_[0].A.view(), u, f, nullptr, nullptr, 0, V, 1.0, -1.0, s));
    resid_nrm = std::sqrt(dot_host(n, V, V, s));
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
    cycle(f, u, s);
    if (tol > 0.) {
      HVE_HIP(launch_sell(K_RESID, lev_[0].A.view(), u, f, nullptr, nullptr, 0, V, -1.0, 0.0, s));
      resid_nrm = std::sqrt(dot_host(n, V, V, s));
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

// krylov/pcg.c:262 hypre_PCGSolve (two_norm selectable; stop_crit/rel_change
// off; no recompute) with one BoomerAMG cycle on a cleared vector as the
// preconditioner (HYPRE_BoomerAMGSolve with tol 0, max_iter 1).  Scalars stay
// on the device; one host read per iteration for the convergence test.
int pcg_solve(DevAMG* amg, const DevSell& A, const PCGParams& prm, const Precond& user_precond, const double* b,
              double* x, hipStream_t s, int* iters, double* rel_res) {
  const int n = A.nrows;
  double* r = amg->scratch(0);
  double* p = amg->scratch(1);
  double* sv = amg->scratch(2);
  double* sc = nullptr;  // device scalars: 0 gamma,1 gamma_old,2 sdotp,3 alpha,4 beta,5 i_prod,6 flag
  double* hs = nullptr;
  HVE_HIP(hipMalloc((void**)&sc, 8 * sizeof(double)));
  HVE_HIP(hipHostMalloc((void**)&hs, 8 * sizeof(double), hipHostMallocDefault));
  HVE_HIP(hipMemsetAsync(sc, 0, 8 * sizeof(double), s));
  auto precond = [&](const double* rr, double* zz) {
    HVE_HIP(launch_set(n, 0.0, zz, s));  // ClearVector (pcg.c:434)
    user_precond(rr, zz);
  };
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
  HVE_HIP(launch_sell(K_RESID, A.view(), x, b, nullptr, nullptr, 0, r, -1.0, 0.0, s));
  precond(r, p);
  amg->dot(n, r, p, sc + 0, s);  // gamma
  if (prm.two_norm) amg->dot(n, r, r, sc + 5, s);
  read();
  i_prod_0 = prm.two_norm ? hs[5] : hs[0];
  while (i + 1 <= prm.max_iter) {
    ++i;
    HVE_HIP(launch_sell(K_MATVEC, A.view(), p, nullptr, nullptr, nullptr, 0, sv, 1.0, 0.0, s));
    amg->dot(n, sv, p, sc + 2, s);
    HVE_HIP(launch_pcg_alpha(sc, s));
    HVE_HIP(launch_axpy(n, sc + 3, 0.0, 1.0, p, x, s));    // x += alpha p
    HVE_HIP(launch_axpy(n, sc + 3, 0.0, -1.0, sv, r, s));  // r += -alpha s
    precond(r, sv);
    amg->dot(n, r, sv, sc + 0, s);                         // gamma = <r,s>
    if (prm.two_norm) amg->dot(n, r, r, sc + 5, s);
    read();
    const double flag = hs[6];
    const double gamma = hs[0];
    if (flag != 0.0) {  // zero <s,p> or subnormal alpha: x, r untouched (alpha = 0)
      if (i == 1) i_prod = i_prod_0;
      break;
    }
    i_prod = prm.two_norm ? hs[5] : gamma;
    if (prm.print_level > 1) fprintf(stderr, "% 5d    %e    %e\n", i, std::sqrt(i_prod), std::sqrt(i_prod / bi_prod));
    if (i_prod / bi_prod < eps) break;
    if (!(gamma > 2.2250738585072014e-308)) break;
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
