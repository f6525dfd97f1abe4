// extern "C" entry points of libhypreve.so (declared in include/hypreve.h).
// Each function keeps the reference's name, argument meaning and return
// convention (hypre_error_flag: 0 on success, error bits otherwise).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/hypreve.h"
#include "device/runtime.hpp"
#include "host/hve_host.hpp"
#include "host/layout.hpp"
#include "host/partition.hpp"
#include "host/dsetup.hpp"
#include "host/hostcomm.hpp"

using namespace hve;

// ---------------------------------------------------------------------------
// object layouts
// ---------------------------------------------------------------------------
struct hypre_ParVector_struct {
  HYPRE_Comm comm = nullptr;
  HYPRE_BigInt global_size = 0, first = 0;
  int n = 0;
  double* d = nullptr;
  bool owns = true;
};

struct hypre_ParCSRMatrix_struct {
  HYPRE_Comm comm = nullptr;
  HYPRE_BigInt global_rows = 0, first_row = 0, global_cols = 0, first_col = 0;
  int n = 0;
  CSR diag;         // host: owned rows, GLOBAL column indices, diagonal first
  DevSell dA;       // device copy (SELL-64) used by Matvec (one rank)
  bool dev = false;
  // partitioned path: any communicator with a transport (a 1-rank RCCL
  // communicator included, which runs the partitioned code with one rank)
  bool multi() const { return comm && comm->dc; }
  void ensure_device() {
    if (multi()) throw std::runtime_error("ParCSR matvec across ranks needs a BoomerAMG setup on this matrix");
    if (!dev) { dA.upload(diag); dev = true; }
  }
};

struct hypre_IJMatrix_struct {
  HYPRE_Comm comm = nullptr;
  HYPRE_BigInt ilower = 0, iupper = -1, jlower = 0, jupper = -1;
  std::vector<std::vector<std::pair<int, double>>> rows;
  HYPRE_ParCSRMatrix par = nullptr;
};

struct hypre_IJVector_struct {
  HYPRE_Comm comm = nullptr;
  HYPRE_BigInt jlower = 0, jupper = -1;
  std::vector<double> h;
  HYPRE_ParVector par = nullptr;
};

enum SolverKind { KIND_AMG = 1, KIND_PCG = 2 };

struct hypre_Solver_struct {
  int kind = 0;
  // AMG
  AMGParams prm;
  Hierarchy H;        // global hierarchy (one rank, or rank 0 of a multi-rank setup)
  RankHierarchy RH;   // this rank's part
  HYPRE_Comm comm = nullptr;
  std::unique_ptr<DevAMG> dev;
  int iters = 0;
  double rel_res = 0.0;
  bool use_graph = true;
  // num_blocks 0 (the default): one hybrid-GS row block per kAutoBlockRows
  // local rows, resolved at Setup (hypre's CPU path uses its OpenMP thread
  // count; a single block would run each sweep in one workgroup)
  bool auto_blocks = true;
  // Setup's ext+i, truncation, R = P^T and RAP on the GPU (hypreve_BoomerAMGSetDeviceSetup)
  bool device_setup = true;
  std::vector<int> gs_rank_starts;  // one GPU emulating the GS blocks of an N-rank run
  std::vector<int> rank_emul;       // one process emulating a reference N-rank setup (SetRankEmulation)
  const HYPRE_Int* dof_user = nullptr;  // SetDofFunc: the caller's array, read at Setup (hypre keeps the pointer)
  std::vector<int> coarsen_starts;  // one process coarsening HMIS as N ranks do (SetCoarsenRankStarts)
  // the last Setup's path (hypreve_BoomerAMGGetSetupPath): 0 one process, 1 one
  // process under the rank emulation, 2 distributed (dsetup.cpp), 3 gathered on
  // rank 0 under the rank emulation, 4 gathered one-process (direct interpolation)
  int setup_path = -1;
  // per level: those blocks and their l1 norms (host copies for the introspection calls)
  std::vector<std::vector<int>> gs_blocks_host;
  std::vector<std::vector<double>> gs_l1_host;
  // PCG
  PCGParams pcg;
  HYPRE_Solver precond = nullptr;
  HYPRE_PtrToParSolverFcn precond_solve = nullptr, precond_setup = nullptr;
  std::unique_ptr<DevAMG> ws;
};

// One-process setup, optionally emulating a reference N-rank run (its rows,
// coarsening and GS blocks; no agglomeration, which the reference lacks).
static void setup_one_process(HYPRE_Solver s, HYPRE_ParCSRMatrix A);
// Automatic hybrid Gauss-Seidel block count (num_blocks 0): one block of about
// 4096 rows of the rank's level 0, so a large level's sweep runs on thousands
// of workgroups while every block keeps hypre's exact in-block GS order.  That
// count plays hypre's OMP_NUM_THREADS on every level (AMGParams::blocks_for),
// capped so that a coarse level's blocks keep at least 64 rows.  Measured on
// MI355X (256^3, relax 13/14): blocks of 4096 rows on every level 45.6 ms a
// cycle, 1024 rows 38.5 (the coarse Galerkin levels' long in-block dependency
// chains on few blocks), the level-0 count everywhere (round 2) 11.5.
// The level-0 block size of the automatic hybrid-GS blocks: 4096 rows.
static int auto_block_rows() { return 4096; }
static void resolve_blocks(hypre_Solver_struct* s, int local_rows) {
  s->prm.auto_block_rows = s->auto_blocks ? auto_block_rows() : 0;
  if (s->auto_blocks) s->prm.num_blocks = std::max(1, (local_rows + auto_block_rows() - 1) / auto_block_rows());
}

// ---------------------------------------------------------------------------
// error state (utilities/hypre_error.c semantics)
// ---------------------------------------------------------------------------
static thread_local int g_error = 0;
static thread_local std::string g_msg;
static int g_memloc = HYPRE_MEMORY_HOST;
// per host thread: a virtual rank of the loopback hub runs on its own thread
static thread_local hipStream_t g_stream = nullptr;

static hipStream_t lib_stream() {
  if (!g_stream) HVE_HIP(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
  return g_stream;
}
static int set_err(int code, const std::string& m) {
  g_error |= code;
  g_msg = m;
  return g_error;
}
#define API_BEGIN try {
#define API_END                                              \
  }                                                          \
  catch (const std::exception& e) {                          \
    return set_err(HYPRE_ERROR_GENERIC, e.what());           \
  }                                                          \
  catch (...) {                                              \
    return set_err(HYPRE_ERROR_GENERIC, "unknown exception"); \
  }                                                          \
  return g_error;
#define CHECK_ARG(c, i) \
  if (!(c)) return set_err(HYPRE_ERROR_ARG | ((i) << 3), "invalid argument " #i);

template <typename T>
static std::vector<T> host_copy(const T* p, size_t n) {
  std::vector<T> v(n);
  if (!n) return v;
  if (g_memloc == HYPRE_MEMORY_DEVICE) HVE_HIP(hipMemcpy(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
  else std::memcpy(v.data(), p, n * sizeof(T));
  return v;
}

extern "C" {

// ---------------------------------------------------------------------------
// utilities
// ---------------------------------------------------------------------------
HYPRE_Int HYPRE_Init(void) {
  API_BEGIN
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_err(HYPRE_ERROR_GENERIC, "no HIP device: the hypre-ve_amd solve path runs only on the GPU");
  lib_stream();
  API_END
}
HYPRE_Int HYPRE_Finalize(void) {
  if (g_stream) { hipStreamDestroy(g_stream); g_stream = nullptr; }
  return 0;
}
HYPRE_Int HYPRE_SetMemoryLocation(HYPRE_Int loc) {
  CHECK_ARG(loc == HYPRE_MEMORY_HOST || loc == HYPRE_MEMORY_DEVICE, 1);
  g_memloc = loc;
  return 0;
}
HYPRE_Int HYPRE_GetError(void) { return g_error; }
HYPRE_Int HYPRE_ClearAllErrors(void) { g_error = 0; g_msg.clear(); return 0; }
HYPRE_Int HYPRE_CheckError(HYPRE_Int ierr, HYPRE_Int code) { return ierr & code; }
const char* hypreve_LastErrorMessage(void) { return g_msg.c_str(); }
const char* hypreve_BuildInfo(void) {
  return "hypre-ve_amd: BoomerAMG solve path for gfx950 (SELL-64 lane-per-row operators, f64, "
         "no FMA contraction; host setup PMIS/ext+i/RAP)";
}
HYPRE_Int hypreve_DeviceSynchronize(void) {
  API_BEGIN
  HVE_HIP(hipDeviceSynchronize());
  API_END
}

// ---------------------------------------------------------------------------
// communicators: see comm.hip
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// ParVector
// ---------------------------------------------------------------------------
static HYPRE_ParVector new_vector(HYPRE_Comm comm, HYPRE_BigInt global, HYPRE_BigInt first, int n) {
  auto* v = new hypre_ParVector_struct;
  v->comm = comm;
  v->global_size = global;
  v->first = first;
  v->n = n;
  return v;
}
static void vec_alloc(HYPRE_ParVector v) {
  if (!v->d) {
    HVE_HIP(hipMalloc((void**)&v->d, sizeof(double) * std::max(1, v->n)));
    HVE_HIP(hipMemset(v->d, 0, sizeof(double) * std::max(1, v->n)));
  }
}

HYPRE_Int HYPRE_ParVectorCreate(HYPRE_Comm comm, HYPRE_BigInt global_size, HYPRE_BigInt* partitioning,
                                HYPRE_ParVector* vector) {
  CHECK_ARG(vector, 4);
  HYPRE_BigInt first = 0, last = global_size;
  if (partitioning) { first = partitioning[0]; last = partitioning[1]; }
  *vector = new_vector(comm, global_size, first, (int)(last - first));
  return 0;
}
HYPRE_Int HYPRE_ParVectorInitialize(HYPRE_ParVector v) {
  CHECK_ARG(v, 1);
  API_BEGIN
  vec_alloc(v);
  API_END
}
HYPRE_Int HYPRE_ParVectorDestroy(HYPRE_ParVector v) {
  if (!v) return 0;
  if (v->d && v->owns) hipFree(v->d);
  delete v;
  return 0;
}
HYPRE_Int HYPRE_ParVectorSetConstantValues(HYPRE_ParVector v, HYPRE_Complex value) {
  CHECK_ARG(v, 1);
  API_BEGIN
  vec_alloc(v);
  HVE_HIP(launch_set(v->n, value, v->d, lib_stream()));
  HVE_HIP(hipStreamSynchronize(lib_stream()));
  API_END
}
HYPRE_Int HYPRE_ParVectorCopy(HYPRE_ParVector x, HYPRE_ParVector y) {
  CHECK_ARG(x && y && x->n == y->n, 1);
  API_BEGIN
  vec_alloc(y);
  HVE_HIP(launch_copy(x->n, x->d, y->d, lib_stream()));
  HVE_HIP(hipStreamSynchronize(lib_stream()));
  API_END
}
HYPRE_Int HYPRE_ParVectorScale(HYPRE_Complex value, HYPRE_ParVector x) {
  CHECK_ARG(x, 2);
  API_BEGIN
  HVE_HIP(launch_scale(x->n, nullptr, value, x->d, lib_stream()));
  HVE_HIP(hipStreamSynchronize(lib_stream()));
  API_END
}
HYPRE_Int HYPRE_ParVectorAxpy(HYPRE_Complex alpha, HYPRE_ParVector x, HYPRE_ParVector y) {
  CHECK_ARG(x && y && x->n == y->n, 2);
  API_BEGIN
  HVE_HIP(launch_axpy(x->n, nullptr, alpha, 1.0, x->d, y->d, lib_stream()));
  HVE_HIP(hipStreamSynchronize(lib_stream()));
  API_END
}

static thread_local double* g_dot_part = nullptr;
static thread_local double* g_dot_out = nullptr;
HYPRE_Int HYPRE_ParVectorInnerProd(HYPRE_ParVector x, HYPRE_ParVector y, HYPRE_Real* prod) {
  CHECK_ARG(x && y && x->n == y->n, 1);
  CHECK_ARG(prod, 3);
  API_BEGIN
  if (!g_dot_part) {
    HVE_HIP(hipMalloc((void**)&g_dot_part, 1024 * sizeof(double)));
    HVE_HIP(hipMalloc((void**)&g_dot_out, sizeof(double)));
  }
  HVE_HIP(launch_dot(x->n, x->d, y->d, g_dot_part, g_dot_out, lib_stream()));
  if (x->comm && x->comm->dc) x->comm->dc->allreduce_sum(g_dot_out, 1, lib_stream());
  HVE_HIP(hipMemcpyAsync(prod, g_dot_out, sizeof(double), hipMemcpyDeviceToHost, lib_stream()));
  HVE_HIP(hipStreamSynchronize(lib_stream()));
  API_END
}
HYPRE_Real* hypreve_ParVectorDeviceData(HYPRE_ParVector v) {
  if (!v) return nullptr;
  try { vec_alloc(v); } catch (...) { return nullptr; }
  return v->d;
}
HYPRE_Int hypreve_ParVectorLocalSize(HYPRE_ParVector v) { return v ? v->n : 0; }
HYPRE_Int hypreve_ParVectorCopyToHost(HYPRE_ParVector v, HYPRE_Real* host) {
  CHECK_ARG(v && host, 1);
  API_BEGIN
  HVE_HIP(hipMemcpy(host, v->d, sizeof(double) * v->n, hipMemcpyDeviceToHost));
  API_END
}
HYPRE_Int hypreve_ParVectorCopyFromHost(HYPRE_ParVector v, const HYPRE_Real* host) {
  CHECK_ARG(v && host, 1);
  API_BEGIN
  vec_alloc(v);
  HVE_HIP(hipMemcpy(v->d, host, sizeof(double) * v->n, hipMemcpyHostToDevice));
  API_END
}
// par_vector.c:328 + vector.c:286: SeedRand(seed*(rank+1)); x_i = 2*Rand()-1
HYPRE_Int hypreve_ParVectorSetRandomValues(HYPRE_ParVector v, HYPRE_Int seed) {
  CHECK_ARG(v, 1);
  API_BEGIN
  const int rank = v->comm ? v->comm->rank : 0;
  const int s = seed * (rank + 1);
  std::vector<double> h(v->n);
  for (int i = 0; i < v->n; ++i) h[i] = 2.0 * hypre_rand_at(i, s) - 1.0;
  vec_alloc(v);
  HVE_HIP(hipMemcpy(v->d, h.data(), sizeof(double) * v->n, hipMemcpyHostToDevice));
  API_END
}

// ---------------------------------------------------------------------------
// ParCSR matrix
// ---------------------------------------------------------------------------
static HYPRE_ParCSRMatrix wrap_matrix(HYPRE_Comm comm, CSR&& A, HYPRE_BigInt first, HYPRE_BigInt global) {
  auto* M = new hypre_ParCSRMatrix_struct;
  M->comm = comm;
  M->first_row = M->first_col = first;
  M->global_rows = M->global_cols = global;
  M->n = A.nrows;
  M->diag = std::move(A);
  return M;
}

HYPRE_Int HYPRE_ParCSRMatrixDestroy(HYPRE_ParCSRMatrix M) {
  if (!M) return 0;
  M->dA.release();
  delete M;
  return 0;
}
HYPRE_Int HYPRE_ParCSRMatrixGetLocalRange(HYPRE_ParCSRMatrix M, HYPRE_BigInt* rs, HYPRE_BigInt* re,
                                          HYPRE_BigInt* cs, HYPRE_BigInt* ce) {
  CHECK_ARG(M, 1);
  *rs = M->first_row; *re = M->first_row + M->n - 1;
  *cs = M->first_col; *ce = M->first_col + M->n - 1;
  return 0;
}

static int matvec_general(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A, HYPRE_ParVector x, HYPRE_Complex beta,
                          HYPRE_ParVector b, HYPRE_ParVector y) {
  A->ensure_device();
  vec_alloc(y);
  hipStream_t s = lib_stream();
  if (alpha == 0.0) {
    // y = beta*b
    if (b != y) HVE_HIP(launch_copy(A->n, b->d, y->d, s));
    HVE_HIP(launch_scale(A->n, nullptr, beta, y->d, s));
  } else if (x == y) {
    double* tmp = nullptr;
    HVE_HIP(hipMalloc((void**)&tmp, sizeof(double) * A->n));
    HVE_HIP(launch_copy(A->n, x->d, tmp, s));
    HVE_HIP(launch_sell(K_GENERAL, A->dA.view(), tmp, b->d, nullptr, nullptr, 0, y->d, alpha, beta / alpha, s));
    HVE_HIP(hipStreamSynchronize(s));
    hipFree(tmp);
  } else {
    HVE_HIP(launch_sell(K_GENERAL, A->dA.view(), x->d, b->d, nullptr, nullptr, 0, y->d, alpha, beta / alpha, s));
  }
  HVE_HIP(hipStreamSynchronize(s));
  return 0;
}

HYPRE_Int HYPRE_ParCSRMatrixMatvec(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A, HYPRE_ParVector x, HYPRE_Complex beta,
                                   HYPRE_ParVector y) {
  CHECK_ARG(A, 2);
  CHECK_ARG(x && x->n == A->n, 3);
  CHECK_ARG(y && y->n == A->n, 5);
  API_BEGIN
  matvec_general(alpha, A, x, beta, y, y);
  API_END
}
HYPRE_Int HYPRE_ParCSRMatrixMatvecOutOfPlace(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A, HYPRE_ParVector x,
                                             HYPRE_Complex beta, HYPRE_ParVector b, HYPRE_ParVector y) {
  CHECK_ARG(A, 2);
  CHECK_ARG(x && x->n == A->n, 3);
  CHECK_ARG(b && b->n == A->n, 5);
  CHECK_ARG(y && y->n == A->n, 6);
  API_BEGIN
  matvec_general(alpha, A, x, beta, b, y);
  API_END
}
HYPRE_Int HYPRE_ParCSRMatrixMatvecT(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A, HYPRE_ParVector x,
                                    HYPRE_Complex beta, HYPRE_ParVector y) {
  CHECK_ARG(A, 2);
  API_BEGIN
  // y = alpha*A^T*x + beta*y via an explicit transpose (csr_matvec.c:424 order)
  CSR AT;
  transpose(A->diag, AT);
  DevSell dT;
  dT.upload(AT);
  hipStream_t s = lib_stream();
  double* tmp = nullptr;
  HVE_HIP(hipMalloc((void**)&tmp, sizeof(double) * y->n));
  HVE_HIP(launch_sell(K_RESTRICT, dT.view(), x->d, nullptr, nullptr, nullptr, 0, tmp, 1.0, 0.0, s));
  // y = beta*y + alpha*tmp  (beta/alpha scaling as in the reference)
  if (beta == 0.0) HVE_HIP(launch_set(y->n, 0.0, y->d, s));
  else HVE_HIP(launch_scale(y->n, nullptr, beta, y->d, s));
  HVE_HIP(launch_axpy(y->n, nullptr, alpha, 1.0, tmp, y->d, s));
  HVE_HIP(hipStreamSynchronize(s));
  hipFree(tmp);
  dT.release();
  API_END
}

HYPRE_Int hypreve_ParCSRMatrixCreateFromCSR(HYPRE_Comm comm, HYPRE_BigInt first_row, HYPRE_Int local_rows,
                                            HYPRE_BigInt global_rows, const HYPRE_Int* row_ptr,
                                            const HYPRE_BigInt* cols, const HYPRE_Real* vals, HYPRE_ParCSRMatrix* A) {
  CHECK_ARG(row_ptr && cols && vals && A, 5);
  API_BEGIN
  if (comm && comm->size > 1) throw std::runtime_error("multi-rank matrices: use GenerateLaplacian or IJ per rank");
  CSR M;
  M.resize_rows(local_rows, (int)global_rows);
  for (int r = 0; r <= local_rows; ++r) M.i[r] = row_ptr[r] - row_ptr[0];
  M.j.resize(M.i[local_rows]);
  M.a.resize(M.i[local_rows]);
  for (int r = 0; r < local_rows; ++r) {
    // diagonal first (hypre ParCSR convention), others in given order
    int o = M.i[r];
    const int b = row_ptr[r] - row_ptr[0], e = row_ptr[r + 1] - row_ptr[0];
    int dpos = -1;
    for (int k = b; k < e; ++k)
      if (cols[k] - first_row == r) { dpos = k; break; }
    if (dpos >= 0) { M.j[o] = r; M.a[o++] = vals[dpos]; }
    for (int k = b; k < e; ++k) {
      if (k == dpos) continue;
      M.j[o] = (int)(cols[k] - first_row);
      M.a[o++] = vals[k];
    }
  }
  *A = wrap_matrix(comm, std::move(M), first_row, global_rows);
  API_END
}

// par_laplace.c:15 (P=Q=R=1 in this build; multi-rank grids in comm.hip)
HYPRE_ParCSRMatrix GenerateLaplacian(HYPRE_Comm comm, HYPRE_BigInt nx, HYPRE_BigInt ny, HYPRE_BigInt nz,
                                     HYPRE_Int P, HYPRE_Int Q, HYPRE_Int R, HYPRE_Int p, HYPRE_Int q, HYPRE_Int r,
                                     HYPRE_Real* value) {
  try {
    CSR A;
    if (P * Q * R != 1) {
      if (!comm || comm->size != P * Q * R) throw std::runtime_error("GenerateLaplacian: P*Q*R != communicator size");
      int64_t first = 0;
      generate_laplacian_7pt_block((int)nx, (int)ny, (int)nz, P, Q, R, p, q, r, value, A, first);
      return wrap_matrix(comm, std::move(A), (HYPRE_BigInt)first, (HYPRE_BigInt)nx * ny * nz);
    }
    const double cx = -value[1], cy = -value[2], cz = -value[3];
    generate_laplacian_7pt((int)nx, (int)ny, (int)nz, cx, cy, cz, A);
    // the reference takes value[0] verbatim
    for (int i = 0; i < A.nrows; ++i) A.a[A.i[i]] = value[0];
    return wrap_matrix(comm, std::move(A), 0, (HYPRE_BigInt)nx * ny * nz);
  } catch (const std::exception& e) {
    set_err(HYPRE_ERROR_GENERIC, e.what());
    return nullptr;
  }
}
HYPRE_ParCSRMatrix GenerateLaplacian27pt(HYPRE_Comm comm, HYPRE_BigInt nx, HYPRE_BigInt ny, HYPRE_BigInt nz,
                                         HYPRE_Int P, HYPRE_Int Q, HYPRE_Int R, HYPRE_Int p, HYPRE_Int q,
                                         HYPRE_Int r, HYPRE_Real* value) {
  try {
    CSR A;
    if (P * Q * R != 1) {
      if (!comm || comm->size != P * Q * R) throw std::runtime_error("GenerateLaplacian27pt: P*Q*R != communicator size");
      int64_t first = 0;
      generate_laplacian_27pt_block((int)nx, (int)ny, (int)nz, P, Q, R, p, q, r, value, A, first);
      return wrap_matrix(comm, std::move(A), (HYPRE_BigInt)first, (HYPRE_BigInt)nx * ny * nz);
    }
    generate_laplacian_27pt((int)nx, (int)ny, (int)nz, A);
    for (int i = 0; i < A.nrows; ++i) {
      A.a[A.i[i]] = value[0];
      for (int k = A.i[i] + 1; k < A.i[i + 1]; ++k) A.a[k] = value[1];
    }
    return wrap_matrix(comm, std::move(A), 0, (HYPRE_BigInt)nx * ny * nz);
  } catch (const std::exception& e) {
    set_err(HYPRE_ERROR_GENERIC, e.what());
    return nullptr;
  }
}

// ---------------------------------------------------------------------------
// IJ interface
// ---------------------------------------------------------------------------
HYPRE_Int HYPRE_IJMatrixCreate(HYPRE_Comm comm, HYPRE_BigInt ilower, HYPRE_BigInt iupper, HYPRE_BigInt jlower,
                               HYPRE_BigInt jupper, HYPRE_IJMatrix* matrix) {
  CHECK_ARG(matrix, 6);
  CHECK_ARG(iupper >= ilower - 1, 3);
  auto* M = new hypre_IJMatrix_struct;
  M->comm = comm;
  M->ilower = ilower; M->iupper = iupper; M->jlower = jlower; M->jupper = jupper;
  *matrix = M;
  return 0;
}
HYPRE_Int HYPRE_IJMatrixDestroy(HYPRE_IJMatrix M) {
  if (!M) return 0;
  if (M->par) HYPRE_ParCSRMatrixDestroy(M->par);
  delete M;
  return 0;
}
HYPRE_Int HYPRE_IJMatrixSetObjectType(HYPRE_IJMatrix M, HYPRE_Int type) {
  CHECK_ARG(M, 1);
  CHECK_ARG(type == HYPRE_PARCSR, 2);
  return 0;
}
HYPRE_Int HYPRE_IJMatrixInitialize(HYPRE_IJMatrix M) {
  CHECK_ARG(M, 1);
  M->rows.assign((size_t)(M->iupper - M->ilower + 1), {});
  return 0;
}
static int ij_set(HYPRE_IJMatrix M, HYPRE_Int nrows, HYPRE_Int* ncols, const HYPRE_BigInt* rows,
                  const HYPRE_BigInt* cols, const HYPRE_Complex* values, bool add) {
  if (M->rows.empty() && M->iupper >= M->ilower) HYPRE_IJMatrixInitialize(M);
  auto nc = host_copy(ncols, nrows);
  size_t tot = 0;
  for (int r = 0; r < nrows; ++r) tot += (size_t)nc[r];
  auto rw = host_copy(rows, nrows);
  auto cl = host_copy(cols, tot);
  auto vl = host_copy(values, tot);
  size_t k = 0;
  for (int r = 0; r < nrows; ++r) {
    const HYPRE_BigInt row = rw[r];
    if (row < M->ilower || row > M->iupper) throw std::runtime_error("IJMatrixSetValues: off-process row");
    auto& R = M->rows[row - M->ilower];
    for (int q = 0; q < nc[r]; ++q, ++k) {
      const int c = (int)cl[k];
      auto it = std::find_if(R.begin(), R.end(), [&](const std::pair<int, double>& e) { return e.first == c; });
      if (it == R.end()) R.emplace_back(c, vl[k]);
      else if (add) it->second += vl[k];
      else it->second = vl[k];
    }
  }
  return 0;
}
HYPRE_Int HYPRE_IJMatrixSetValues(HYPRE_IJMatrix M, HYPRE_Int nrows, HYPRE_Int* ncols, const HYPRE_BigInt* rows,
                                  const HYPRE_BigInt* cols, const HYPRE_Complex* values) {
  CHECK_ARG(M, 1);
  API_BEGIN
  ij_set(M, nrows, ncols, rows, cols, values, false);
  API_END
}
HYPRE_Int HYPRE_IJMatrixAddToValues(HYPRE_IJMatrix M, HYPRE_Int nrows, HYPRE_Int* ncols, const HYPRE_BigInt* rows,
                                    const HYPRE_BigInt* cols, const HYPRE_Complex* values) {
  CHECK_ARG(M, 1);
  API_BEGIN
  ij_set(M, nrows, ncols, rows, cols, values, true);
  API_END
}
HYPRE_Int HYPRE_IJMatrixAssemble(HYPRE_IJMatrix M) {
  CHECK_ARG(M, 1);
  API_BEGIN
  if (M->comm && M->comm->size > 1) throw std::runtime_error("IJ assembly across ranks: use per-rank blocks");
  const int n = (int)(M->iupper - M->ilower + 1);
  CSR A;
  A.resize_rows(n, (int)(M->jupper - M->jlower + 1));
  for (int r = 0; r < n; ++r) A.i[r + 1] = A.i[r] + (int)M->rows[r].size();
  A.j.resize(A.i[n]);
  A.a.resize(A.i[n]);
  for (int r = 0; r < n; ++r) {
    int o = A.i[r];
    const auto& R = M->rows[r];
    const int drow = (int)(r + M->ilower - M->jlower);
    for (const auto& e : R)
      if (e.first - (int)M->jlower == drow) { A.j[o] = drow; A.a[o++] = e.second; }
    for (const auto& e : R)
      if (e.first - (int)M->jlower != drow) { A.j[o] = e.first - (int)M->jlower; A.a[o++] = e.second; }
  }
  if (M->par) HYPRE_ParCSRMatrixDestroy(M->par);
  M->par = wrap_matrix(M->comm, std::move(A), M->ilower, M->iupper + 1);
  API_END
}
HYPRE_Int HYPRE_IJMatrixGetObject(HYPRE_IJMatrix M, void** object) {
  CHECK_ARG(M && M->par, 1);
  *object = (void*)M->par;
  return 0;
}

HYPRE_Int HYPRE_IJVectorCreate(HYPRE_Comm comm, HYPRE_BigInt jlower, HYPRE_BigInt jupper, HYPRE_IJVector* vector) {
  CHECK_ARG(vector, 4);
  auto* V = new hypre_IJVector_struct;
  V->comm = comm;
  V->jlower = jlower;
  V->jupper = jupper;
  *vector = V;
  return 0;
}
HYPRE_Int HYPRE_IJVectorDestroy(HYPRE_IJVector V) {
  if (!V) return 0;
  if (V->par) HYPRE_ParVectorDestroy(V->par);
  delete V;
  return 0;
}
HYPRE_Int HYPRE_IJVectorSetObjectType(HYPRE_IJVector V, HYPRE_Int type) {
  CHECK_ARG(V, 1);
  CHECK_ARG(type == HYPRE_PARCSR, 2);
  return 0;
}
HYPRE_Int HYPRE_IJVectorInitialize(HYPRE_IJVector V) {
  CHECK_ARG(V, 1);
  V->h.assign((size_t)(V->jupper - V->jlower + 1), 0.0);
  return 0;
}
HYPRE_Int HYPRE_IJVectorSetValues(HYPRE_IJVector V, HYPRE_Int nvalues, const HYPRE_BigInt* indices,
                                  const HYPRE_Complex* values) {
  CHECK_ARG(V, 1);
  API_BEGIN
  if (V->h.empty()) HYPRE_IJVectorInitialize(V);
  auto vl = host_copy(values, nvalues);
  if (indices) {
    auto ix = host_copy(indices, nvalues);
    for (int k = 0; k < nvalues; ++k) V->h.at(ix[k] - V->jlower) = vl[k];
  } else {
    for (int k = 0; k < nvalues; ++k) V->h.at(k) = vl[k];
  }
  if (V->par) {  // after assembly: write through to the device vector
    HVE_HIP(hipMemcpy(V->par->d, V->h.data(), sizeof(double) * V->h.size(), hipMemcpyHostToDevice));
  }
  API_END
}
HYPRE_Int HYPRE_IJVectorAssemble(HYPRE_IJVector V) {
  CHECK_ARG(V, 1);
  API_BEGIN
  if (V->h.empty()) HYPRE_IJVectorInitialize(V);
  if (!V->par) {
    V->par = new_vector(V->comm, V->jupper + 1, V->jlower, (int)V->h.size());
    vec_alloc(V->par);
  }
  HVE_HIP(hipMemcpy(V->par->d, V->h.data(), sizeof(double) * V->h.size(), hipMemcpyHostToDevice));
  API_END
}
HYPRE_Int HYPRE_IJVectorGetObject(HYPRE_IJVector V, void** object) {
  CHECK_ARG(V && V->par, 1);
  *object = (void*)V->par;
  return 0;
}
HYPRE_Int HYPRE_IJVectorGetValues(HYPRE_IJVector V, HYPRE_Int nvalues, const HYPRE_BigInt* indices,
                                  HYPRE_Complex* values) {
  CHECK_ARG(V && V->par, 1);
  API_BEGIN
  std::vector<double> h(V->par->n);
  HVE_HIP(hipMemcpy(h.data(), V->par->d, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
  std::vector<double> out(nvalues);
  if (indices) {
    auto ix = host_copy(indices, nvalues);
    for (int k = 0; k < nvalues; ++k) out[k] = h.at(ix[k] - V->jlower);
  } else {
    for (int k = 0; k < nvalues; ++k) out[k] = h.at(k);
  }
  if (g_memloc == HYPRE_MEMORY_DEVICE) HVE_HIP(hipMemcpy(values, out.data(), sizeof(double) * nvalues, hipMemcpyHostToDevice));
  else std::memcpy(values, out.data(), sizeof(double) * nvalues);
  API_END
}

// ---------------------------------------------------------------------------
// BoomerAMG
// ---------------------------------------------------------------------------
#define AMG_SET(name, field, type)                          \
  HYPRE_Int HYPRE_BoomerAMGSet##name(HYPRE_Solver s, type v) { \
    CHECK_ARG(s && s->kind == KIND_AMG, 1);                   \
    s->prm.field = v;                                         \
    return 0;                                                 \
  }

HYPRE_Int HYPRE_BoomerAMGCreate(HYPRE_Solver* solver) {
  CHECK_ARG(solver, 1);
  auto* s = new hypre_Solver_struct;
  s->kind = KIND_AMG;
  *solver = s;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGDestroy(HYPRE_Solver s) {
  if (!s) return 0;
  delete s;
  return 0;
}
AMG_SET(ConvergeType, converge_type, HYPRE_Int)
AMG_SET(Tol, tol, HYPRE_Real)
AMG_SET(MaxIter, max_iter, HYPRE_Int)
AMG_SET(MinIter, min_iter, HYPRE_Int)
AMG_SET(MaxCoarseSize, max_coarse_size, HYPRE_Int)
AMG_SET(MinCoarseSize, min_coarse_size, HYPRE_Int)
AMG_SET(MaxLevels, max_levels, HYPRE_Int)
AMG_SET(StrongThreshold, strong_threshold, HYPRE_Real)
AMG_SET(MaxRowSum, max_row_sum, HYPRE_Real)
AMG_SET(CoarsenType, coarsen_type, HYPRE_Int)
AMG_SET(MeasureType, measure_type, HYPRE_Int)
AMG_SET(AggNumLevels, agg_num_levels, HYPRE_Int)
AMG_SET(AggInterpType, agg_interp_type, HYPRE_Int)
AMG_SET(AggTruncFactor, agg_trunc_factor, HYPRE_Real)
AMG_SET(AggP12TruncFactor, agg_P12_trunc_factor, HYPRE_Real)
AMG_SET(AggPMaxElmts, agg_P_max_elmts, HYPRE_Int)
AMG_SET(AggP12MaxElmts, agg_P12_max_elmts, HYPRE_Int)
AMG_SET(NumPaths, num_paths, HYPRE_Int)
AMG_SET(InterpType, interp_type, HYPRE_Int)
AMG_SET(SepWeight, sep_weight, HYPRE_Int)
AMG_SET(SeqThreshold, seq_threshold, HYPRE_Int)
AMG_SET(NumFunctions, num_functions, HYPRE_Int)
// HYPRE_parcsr_ls.h:176: the function of every local row; the array is read at
// Setup (one process, or under the rank emulation: every row)
HYPRE_Int HYPRE_BoomerAMGSetDofFunc(HYPRE_Solver s, HYPRE_Int* dof_func) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  s->dof_user = dof_func;
  return 0;
}
AMG_SET(Redundant, redundant, HYPRE_Int)
AMG_SET(TruncFactor, trunc_factor, HYPRE_Real)
AMG_SET(PMaxElmts, P_max_elmts, HYPRE_Int)
AMG_SET(CycleType, cycle_type, HYPRE_Int)
AMG_SET(RelaxOrder, relax_order, HYPRE_Int)
AMG_SET(PrintLevel, print_level, HYPRE_Int)
AMG_SET(Logging, logging, HYPRE_Int)
AMG_SET(ChebyOrder, cheby_order, HYPRE_Int)
AMG_SET(ChebyFraction, cheby_fraction, HYPRE_Real)
AMG_SET(ChebyScale, cheby_scale, HYPRE_Int)
AMG_SET(ChebyVariant, cheby_variant, HYPRE_Int)
AMG_SET(ChebyEigEst, cheby_eig_est, HYPRE_Int)

// par_amg.c SetRelaxWt / SetOuterWt overwrite every level's weight;
// SetLevelRelaxWt / SetLevelOuterWt (par_amg.c:2368) set one level.  A
// negative weight -k asks for the CG estimate with at most k steps at Setup
// (par_cg_relax_wt.c); a relax weight of 0 asks for 4/3 over the scaled norm
// of the level's matrix at Setup (par_amg_setup.c:3184); an outer weight of 0
// is not restated.
HYPRE_Int HYPRE_BoomerAMGSetRelaxWt(HYPRE_Solver s, HYPRE_Real w) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  s->prm.relax_weight = w;
  s->prm.lev_relax_wt_set = 0;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGSetOuterWt(HYPRE_Solver s, HYPRE_Real w) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  if (!(w != 0.0)) return set_err(HYPRE_ERROR_ARG, "outer weight 0 (scaled-norm weight) is not available");
  s->prm.outer_weight = w;
  s->prm.lev_outer_wt_set = 0;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGSetLevelRelaxWt(HYPRE_Solver s, HYPRE_Real w, HYPRE_Int level) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(level >= 0 && level < AMGParams::kWeightLevels && level < s->prm.max_levels, 3);
  s->prm.lev_relax_wt[level] = w;
  s->prm.lev_relax_wt_set |= (uint64_t)1 << level;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGSetLevelOuterWt(HYPRE_Solver s, HYPRE_Real w, HYPRE_Int level) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(level >= 0 && level < AMGParams::kWeightLevels && level < s->prm.max_levels, 3);
  if (!(w != 0.0)) return set_err(HYPRE_ERROR_ARG, "outer weight 0 (scaled-norm weight) is not available");
  s->prm.lev_outer_wt[level] = w;
  s->prm.lev_outer_wt_set |= (uint64_t)1 << level;
  return 0;
}
// Relaxation weight and outer weight (omega) the cycle uses on `level`.
HYPRE_Int hypreve_BoomerAMGGetLevelWeights(HYPRE_Solver s, HYPRE_Int level, HYPRE_Real* w, HYPRE_Real* omega) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  const AMGParams& p = s->H.lev.empty() ? (s->RH.lev.empty() ? s->prm : s->RH.prm) : s->H.prm;
  if (w) *w = p.wt(level);
  if (omega) *omega = p.omega(level);
  return 0;
}

// par_amg.c:1962 SetNumSweeps: all of [0..2] (coarsest keeps 1), :2084 SetRelaxType
HYPRE_Int HYPRE_BoomerAMGSetNumSweeps(HYPRE_Solver s, HYPRE_Int num_sweeps) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(num_sweeps >= 1, 2);
  for (int i = 0; i < 3; ++i) s->prm.num_sweeps[i] = num_sweeps;
  s->prm.num_sweeps[3] = 1;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGSetCycleNumSweeps(HYPRE_Solver s, HYPRE_Int num_sweeps, HYPRE_Int k) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(num_sweeps >= 0, 2);
  CHECK_ARG(k >= 1 && k <= 3, 3);
  s->prm.num_sweeps[k] = num_sweeps;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGSetRelaxType(HYPRE_Solver s, HYPRE_Int relax_type) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(relax_type >= 0, 2);
  for (int i = 0; i < 3; ++i) s->prm.relax_type[i] = relax_type;
  s->prm.relax_type[3] = 9;
  s->prm.user_relax_type = relax_type;  // par_amg.c:2101-2104
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGSetCycleRelaxType(HYPRE_Solver s, HYPRE_Int relax_type, HYPRE_Int k) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(k >= 1 && k <= 3, 3);
  CHECK_ARG(relax_type >= 0, 2);
  s->prm.relax_type[k] = relax_type;
  return 0;
}
HYPRE_Int hypreve_BoomerAMGSetNumBlocks(HYPRE_Solver s, HYPRE_Int nb) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(nb >= 0, 2);
  s->auto_blocks = nb == 0;
  if (nb >= 1) s->prm.num_blocks = nb;
  return 0;
}
HYPRE_Int hypreve_BoomerAMGSetAggloRows(HYPRE_Solver s, HYPRE_Int rows) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  s->prm.agglo_rows = rows < 0 ? -1 : rows;
  return 0;
}
// Hybrid Gauss-Seidel on one GPU with the row blocks of an N-rank run whose
// level-0 rows start at starts[0..nranks] (num_blocks blocks per rank on
// every level, l1 norms to match): the iterates then equal the N-rank ones.
// nranks <= 1 clears it.  Takes effect at Setup.
HYPRE_Int hypreve_BoomerAMGSetGsRankStarts(HYPRE_Solver s, HYPRE_Int nranks, const HYPRE_Int* starts) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(nranks <= 1 || starts, 3);
  s->gs_rank_starts.clear();
  if (nranks > 1) {
    for (int r = 0; r < nranks; ++r) CHECK_ARG(starts[r] <= starts[r + 1] && starts[0] == 0, 3);
    s->gs_rank_starts.assign(starts, starts + nranks + 1);
  }
  return 0;
}
// HMIS on one process as an N-rank run coarsens it (each rank's Ruge first
// pass, per-rank random streams; dsetup.cpp hmis_dist), everything else the
// one-process setup: a partial rank emulation (SetRankEmulation is the whole).
HYPRE_Int hypreve_BoomerAMGSetCoarsenRankStarts(HYPRE_Solver s, HYPRE_Int nranks, const HYPRE_Int* starts) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(nranks <= 1 || starts, 3);
  s->coarsen_starts.clear();
  if (nranks > 1) {
    for (int r = 0; r < nranks; ++r) CHECK_ARG(starts[r] <= starts[r + 1] && starts[0] == 0, 3);
    s->coarsen_starts.assign(starts, starts + nranks + 1);
  }
  return 0;
}
HYPRE_Int hypreve_BoomerAMGSetRankEmulation(HYPRE_Solver s, HYPRE_Int nranks, const HYPRE_Int* starts) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(nranks <= 1 || starts, 3);
  s->rank_emul.clear();
  s->gs_rank_starts.clear();
  if (nranks > 1) {
    for (int r = 0; r < nranks; ++r) CHECK_ARG(starts[r] <= starts[r + 1] && starts[0] == 0, 3);
    s->rank_emul.assign(starts, starts + nranks + 1);
    s->gs_rank_starts = s->rank_emul;
  }
  return 0;
}
// Tuning: re-key the row-block traversal of the built device hierarchy with
// nbands bands of the grid's y extent (0: natural order; default at Setup:
// 8 bands).  Only the visiting order of row blocks changes.
HYPRE_Int hypreve_BoomerAMGSetBlockBands(HYPRE_Solver s, HYPRE_Int nbands, HYPRE_Int which_mask) {
  CHECK_ARG(s && s->kind == KIND_AMG && s->dev && s->dev->built(), 1);
  CHECK_ARG(nbands >= 0, 2);
  CHECK_ARG(which_mask >= 0 && which_mask <= 7, 3);
  API_BEGIN
  // a one-rank hierarchy lent its matrices for the build only: lend them again
  const bool lent = s->RH.size == 1 && !s->RH.lev.empty() && s->RH.lev[0].A.interior.nrows == 0 &&
                    lend_single_rank(s->H, s->RH, s->gs_rank_starts.empty() ? nullptr : &s->gs_rank_starts);
  try {
    s->dev->set_block_bands(s->RH, nbands, which_mask ? which_mask : 7);
  } catch (...) {
    if (lent) give_back_single_rank(s->H, s->RH);
    throw;
  }
  if (lent) give_back_single_rank(s->H, s->RH);
  HVE_HIP(hipDeviceSynchronize());
  API_END
}
HYPRE_Int hypreve_BoomerAMGSetSellPolicy(HYPRE_Solver s, HYPRE_Int policy) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(policy >= 0 && policy <= 15, 2);
  s->prm.sell_policy = policy;
  return 0;
}
HYPRE_Int hypreve_BoomerAMGSetUseGraph(HYPRE_Solver s, HYPRE_Int g) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  s->use_graph = g != 0;
  if (s->dev) s->dev->set_use_graph(s->use_graph);
  return 0;
}

HYPRE_Int hypreve_BoomerAMGPartitionCheck(HYPRE_Solver s, HYPRE_Int size) {
  CHECK_ARG(s && s->kind == KIND_AMG && !s->H.lev.empty(), 1);
  CHECK_ARG(size >= 1, 2);
  API_BEGIN
  std::string msg;
  const int errs = partition_self_check(s->H, size, msg);
  if (errs) return set_err(HYPRE_ERROR_GENERIC, msg);
  API_END
}

HYPRE_Int hypreve_BoomerAMGDistSetupCheck(HYPRE_Solver s, HYPRE_ParCSRMatrix A, HYPRE_Int size) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(A && !A->multi(), 2);
  CHECK_ARG(size >= 1, 3);
  API_BEGIN
  std::string msg;
  if (!dist_setup_supported(s->prm, &msg)) return set_err(HYPRE_ERROR_ARG, "distributed setup: " + msg);
  const int errs = dist_setup_self_check(A->diag, s->prm, size, msg);
  if (errs) return set_err(HYPRE_ERROR_GENERIC, msg);
  API_END
}

HYPRE_Int hypreve_BoomerAMGSetupHost(HYPRE_Solver s, HYPRE_ParCSRMatrix A) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(A, 2);
  API_BEGIN
  resolve_blocks(s, A->n);
  s->prm.device_setup = 0;  // host only: the reference functions of the device setup
  setup_one_process(s, A);
  API_END
}

HYPRE_Int hypreve_BoomerAMGSetDeviceSetup(HYPRE_Solver s, HYPRE_Int on) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  s->device_setup = on != 0;
  return 0;
}

HYPRE_Int hypreve_BoomerAMGGetSetupPath(HYPRE_Solver s, HYPRE_Int* path) {
  CHECK_ARG(s && s->kind == KIND_AMG && path, 1);
  *path = s->setup_path;
  return 0;
}

HYPRE_Int hypreve_BoomerAMGGetSetupLog(HYPRE_Solver s, char* buf, HYPRE_Int len) {
  CHECK_ARG(s && s->kind == KIND_AMG && buf && len > 0, 1);
  snprintf(buf, (size_t)len, "%s", s->H.log.c_str());
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Multi-rank setup, gathered: for the options the distributed setup
// (dsetup.cpp) does not take, rank 0 gathers the global matrix, runs the
// N-rank emulation of hypre's setup over it (setup.cpp amg_setup with the
// ranks' row starts) and ships every rank its part of each level (RCCL,
// device staging).  An N-GPU solve then reproduces hypre's N-process run,
// and a one-GPU run under hypreve_BoomerAMGSetRankEmulation with the same
// starts bit for bit.
// ---------------------------------------------------------------------------
template <typename T>
static T* dev_copy(const T* h, size_t n) {
  T* d = nullptr;
  HVE_HIP(hipMalloc((void**)&d, std::max<size_t>(1, n) * sizeof(T)));
  if (n) HVE_HIP(hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}
static void setup_multi(hypre_Solver_struct* s, HYPRE_ParCSRMatrix A) {
  HYPRE_Comm c = A->comm;
  DevComm& comm = *c->dc;
  const int rank = c->rank, size = c->size;
  hipStream_t st = lib_stream();
  // 1. sizes
  int64_t mine[3] = {A->n, A->diag.nnz(), A->first_row};
  int64_t* d_all = nullptr;
  HVE_HIP(hipMalloc((void**)&d_all, sizeof(int64_t) * 3 * size));
  int64_t* d_mine = dev_copy(mine, 3);
  comm.allgather(d_mine, d_all, 3 * sizeof(int64_t), st);
  std::vector<int64_t> all(3 * size);
  HVE_HIP(hipMemcpyAsync(all.data(), d_all, sizeof(int64_t) * 3 * size, hipMemcpyDeviceToHost, st));
  HVE_HIP(hipStreamSynchronize(st));
  (void)hipFree(d_all);
  (void)hipFree(d_mine);
  std::vector<int> starts0(size + 1, 0);
  for (int r = 0; r < size; ++r) {
    if (all[3 * r + 2] != starts0[r]) throw std::runtime_error("ParCSR row blocks must be contiguous in rank order");
    starts0[r + 1] = starts0[r] + (int)all[3 * r];
  }
  // 2. gather the rows on rank 0
  int* d_i = dev_copy(A->diag.i.data(), A->diag.i.size());
  int* d_j = dev_copy(A->diag.j.data(), A->diag.j.size());
  double* d_a = dev_copy(A->diag.a.data(), A->diag.a.size());
  std::vector<int*> ri(size, nullptr), rj(size, nullptr);
  std::vector<double*> ra(size, nullptr);
  {
    std::vector<P2PMsg> sends, recvs;
    if (rank == 0) {
      for (int r = 1; r < size; ++r) {
        HVE_HIP(hipMalloc((void**)&ri[r], sizeof(int) * (all[3 * r] + 1)));
        HVE_HIP(hipMalloc((void**)&rj[r], sizeof(int) * std::max<int64_t>(1, all[3 * r + 1])));
        HVE_HIP(hipMalloc((void**)&ra[r], sizeof(double) * std::max<int64_t>(1, all[3 * r + 1])));
        recvs.push_back({r, ri[r], sizeof(int) * (size_t)(all[3 * r] + 1)});
        recvs.push_back({r, rj[r], sizeof(int) * (size_t)all[3 * r + 1]});
        recvs.push_back({r, ra[r], sizeof(double) * (size_t)all[3 * r + 1]});
      }
    } else {
      sends.push_back({0, d_i, sizeof(int) * (size_t)(A->n + 1)});
      sends.push_back({0, d_j, sizeof(int) * (size_t)A->diag.nnz()});
      sends.push_back({0, d_a, sizeof(double) * (size_t)A->diag.nnz()});
    }
    comm.exchange(sends, recvs, st);
  }
  HVE_HIP(hipStreamSynchronize(st));
  std::vector<std::vector<char>> bufs;
  if (rank == 0) {
    CSR G;
    G.resize_rows(starts0[size], starts0[size]);
    std::vector<int64_t> nnzoff(size + 1, 0);
    for (int r = 0; r < size; ++r) nnzoff[r + 1] = nnzoff[r] + all[3 * r + 1];
    if (nnzoff[size] > 0x7fffffffLL) throw std::runtime_error("global matrix exceeds 2^31 nonzeros");
    G.j.resize(nnzoff[size]);
    G.a.resize(nnzoff[size]);
    for (int r = 0; r < size; ++r) {
      std::vector<int> li(all[3 * r] + 1);
      if (r == 0) {
        li = A->diag.i;
        std::copy(A->diag.j.begin(), A->diag.j.end(), G.j.begin());
        std::copy(A->diag.a.begin(), A->diag.a.end(), G.a.begin());
      } else {
        HVE_HIP(hipMemcpy(li.data(), ri[r], sizeof(int) * li.size(), hipMemcpyDeviceToHost));
        HVE_HIP(hipMemcpy(G.j.data() + nnzoff[r], rj[r], sizeof(int) * all[3 * r + 1], hipMemcpyDeviceToHost));
        HVE_HIP(hipMemcpy(G.a.data() + nnzoff[r], ra[r], sizeof(double) * all[3 * r + 1], hipMemcpyDeviceToHost));
        (void)hipFree(ri[r]); (void)hipFree(rj[r]); (void)hipFree(ra[r]);
      }
      for (int q = 0; q < (int)all[3 * r]; ++q) G.i[starts0[r] + q + 1] = (int)(nnzoff[r] + li[q + 1]);
    }
    if (s->dof_user && s->prm.num_functions > 1)
      throw std::runtime_error("HYPRE_BoomerAMGSetDofFunc with more than one rank is not available");
    // One contract for every N-rank setup: hypre's own setup on `size`
    // processes, as the rank emulation restates it (pinned to the reference's
    // np > 1 runs; dsetup.cpp follows the same rules distributed).  The
    // direct interpolation (3), which the emulation does not restate, keeps
    // the one-process hierarchy with HMIS coarsened per rank.
    const int it = s->prm.interp_type;
    const bool emulated = size > 1 && (it == 6 || it == 7 || it == 8 || it == 9 || it == 14 || (it >= 16 && it <= 18));
    if (emulated) amg_setup(G, s->prm, s->H, &starts0, nullptr);
    else amg_setup(G, s->prm, s->H, nullptr, &starts0);
    s->setup_path = emulated ? 3 : 4;
    { CSR().swap(G); }  // the gathered matrix is level 0 of H now
    bufs.resize(size);
    std::vector<RankHierarchy> parts;
    partition_hierarchy_all(s->H, starts0, size, parts);
    for (int r = 0; r < size; ++r) {
      serialize(parts[r], bufs[r]);
      parts[r] = RankHierarchy();  // release as we go
    }
  }
  (void)hipFree(d_i); (void)hipFree(d_j); (void)hipFree(d_a);
  // 3. scatter the serialized parts
  std::vector<int64_t> lens(size, 0);
  if (rank == 0) for (int r = 0; r < size; ++r) lens[r] = (int64_t)bufs[r].size();
  int64_t* d_lens = dev_copy(lens.data(), size);
  comm.bcast(d_lens, sizeof(int64_t) * size, 0, st);
  HVE_HIP(hipMemcpyAsync(lens.data(), d_lens, sizeof(int64_t) * size, hipMemcpyDeviceToHost, st));
  HVE_HIP(hipStreamSynchronize(st));
  (void)hipFree(d_lens);
  std::vector<char> mybuf;
  if (rank == 0) {
    std::vector<char*> dsend(size, nullptr);
    std::vector<P2PMsg> sends;
    for (int r = 1; r < size; ++r) {
      dsend[r] = dev_copy(bufs[r].data(), bufs[r].size());
      sends.push_back({r, dsend[r], (size_t)lens[r]});
    }
    comm.exchange(sends, {}, st);
    HVE_HIP(hipStreamSynchronize(st));
    for (int r = 1; r < size; ++r) (void)hipFree(dsend[r]);
    mybuf.swap(bufs[0]);
  } else {
    char* drecv = nullptr;
    HVE_HIP(hipMalloc((void**)&drecv, std::max<int64_t>(1, lens[rank])));
    comm.exchange({}, {{0, drecv, (size_t)lens[rank]}}, st);
    HVE_HIP(hipStreamSynchronize(st));
    mybuf.resize(lens[rank]);
    HVE_HIP(hipMemcpy(mybuf.data(), drecv, lens[rank], hipMemcpyDeviceToHost));
    (void)hipFree(drecv);
  }
  deserialize(mybuf, s->RH);
}

// HostComm over the device communicator (RCCL, or the loopback hub): host
// buffers staged through device memory.  The byte counts of every pair go
// round first (an all-gather of each rank's send sizes), then one grouped
// exchange moves all non-empty messages; a rank's message to itself is a
// host copy.
class DevHostComm final : public HostComm {
 public:
  explicit DevHostComm(DevComm& dc) : HostComm(dc.rank(), dc.size()), dc_(dc) {
    HVE_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
  }
  ~DevHostComm() override { (void)hipStreamDestroy(st_); }

  void alltoallv(const std::vector<std::vector<char>>& send, std::vector<std::vector<char>>& recv) override {
    const int n = size_, r = rank_;
    std::vector<int64_t> mine(n), all((size_t)n * n);
    for (int p = 0; p < n; ++p) mine[p] = (int64_t)send[p].size();
    {
      int64_t *dm = nullptr, *da = nullptr;
      HVE_HIP(hipMalloc((void**)&dm, sizeof(int64_t) * n));
      HVE_HIP(hipMalloc((void**)&da, sizeof(int64_t) * n * n));
      HVE_HIP(hipMemcpyAsync(dm, mine.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, st_));
      dc_.allgather(dm, da, sizeof(int64_t) * n, st_);
      HVE_HIP(hipMemcpyAsync(all.data(), da, sizeof(int64_t) * n * n, hipMemcpyDeviceToHost, st_));
      HVE_HIP(hipStreamSynchronize(st_));
      (void)hipFree(dm);
      (void)hipFree(da);
    }
    // all[p * n + q] = bytes p sends to q
    std::vector<size_t> soff(n + 1, 0), roff(n + 1, 0);
    for (int p = 0; p < n; ++p) {
      soff[p + 1] = soff[p] + (p == r ? 0 : (size_t)all[(size_t)r * n + p]);
      roff[p + 1] = roff[p] + (p == r ? 0 : (size_t)all[(size_t)p * n + r]);
    }
    char *ds = nullptr, *dr = nullptr;
    HVE_HIP(hipMalloc((void**)&ds, std::max<size_t>(1, soff[n])));
    HVE_HIP(hipMalloc((void**)&dr, std::max<size_t>(1, roff[n])));
    std::vector<P2PMsg> sends, recvs;
    for (int p = 0; p < n; ++p) {
      if (p == r) continue;
      const size_t sb = soff[p + 1] - soff[p], rb = roff[p + 1] - roff[p];
      if (sb) {
        HVE_HIP(hipMemcpyAsync(ds + soff[p], send[p].data(), sb, hipMemcpyHostToDevice, st_));
        sends.push_back({p, ds + soff[p], sb});
      }
      if (rb) recvs.push_back({p, dr + roff[p], rb});
    }
    dc_.exchange(sends, recvs, st_);
    recv.assign(n, {});
    for (int p = 0; p < n; ++p) {
      if (p == r) {
        recv[p] = send[p];
        continue;
      }
      recv[p].resize(roff[p + 1] - roff[p]);
      if (!recv[p].empty())
        HVE_HIP(hipMemcpyAsync(recv[p].data(), dr + roff[p], recv[p].size(), hipMemcpyDeviceToHost, st_));
    }
    HVE_HIP(hipStreamSynchronize(st_));
    (void)hipFree(ds);
    (void)hipFree(dr);
  }

  std::vector<int64_t> allgather(int64_t v) override {
    const int n = size_;
    std::vector<int64_t> out(n);
    int64_t *dm = nullptr, *da = nullptr;
    HVE_HIP(hipMalloc((void**)&dm, sizeof(int64_t)));
    HVE_HIP(hipMalloc((void**)&da, sizeof(int64_t) * n));
    HVE_HIP(hipMemcpyAsync(dm, &v, sizeof(int64_t), hipMemcpyHostToDevice, st_));
    dc_.allgather(dm, da, sizeof(int64_t), st_);
    HVE_HIP(hipMemcpyAsync(out.data(), da, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st_));
    HVE_HIP(hipStreamSynchronize(st_));
    (void)hipFree(dm);
    (void)hipFree(da);
    return out;
  }

 private:
  DevComm& dc_;
  hipStream_t st_ = nullptr;
};

// Multi-rank setup path: every rank sets up its own rows (dsetup.cpp) where
// the parameters allow it, the rank-0 gather (setup_multi) otherwise.
// HVE_SETUP=gather forces the gather path.
static bool use_dist_setup(const AMGParams& prm) {
  const char* e = getenv("HVE_SETUP");
  if (e && std::string(e) == "gather") return false;
  return dist_setup_supported(prm);
}

static void setup_dist(hypre_Solver_struct* s, HYPRE_ParCSRMatrix A) {
  DevHostComm hc(*A->comm->dc);
  s->H = Hierarchy();
  std::string log;
  if (amg_setup_dist(A->diag, A->first_row, s->prm, hc, s->RH, &log) != 0)
    throw std::runtime_error("distributed setup refused its parameters");
  if (s->prm.print_level > 0) fputs(log.c_str(), stderr);
  s->H.log = log;
  s->setup_path = 2;
}

static void setup_one_process(HYPRE_Solver s, HYPRE_ParCSRMatrix A) {
  s->setup_path = s->rank_emul.empty() ? 0 : 1;
  if (s->rank_emul.empty()) {
    std::vector<int> dof;
    if (s->dof_user && s->prm.num_functions > 1) dof.assign(s->dof_user, s->dof_user + A->diag.nrows);
    amg_setup(A->diag, s->prm, s->H, nullptr, s->coarsen_starts.empty() ? nullptr : &s->coarsen_starts,
              dof.empty() ? nullptr : &dof);
  } else {
    AMGParams prm = s->prm;
    prm.agglo_rows = 0;
    std::vector<int> dof;
    if (s->dof_user && s->prm.num_functions > 1) dof.assign(s->dof_user, s->dof_user + A->diag.nrows);
    amg_setup(A->diag, prm, s->H, &s->rank_emul, nullptr, dof.empty() ? nullptr : &dof);
  }
  gs_rank_blocks_host(s->H, s->gs_rank_starts, s->gs_blocks_host, s->gs_l1_host);
  if (s->gs_blocks_host.empty() && s->prm.auto_block_rows > 0) {
    // per-level automatic blocks: exported for the introspection calls (the
    // l1 norms of L.l1 already follow them)
    for (const Level& L : s->H.lev) s->gs_blocks_host.push_back(hypre_block_starts(L.A.nrows, s->prm.blocks_for(L.A.nrows)));
  }
}

extern "C" {

HYPRE_Int HYPRE_BoomerAMGSetup(HYPRE_Solver s, HYPRE_ParCSRMatrix A, HYPRE_ParVector b, HYPRE_ParVector x) {
  CHECK_ARG(s && s->kind == KIND_AMG, 1);
  CHECK_ARG(A, 2);
  API_BEGIN
  s->comm = A->comm;
  resolve_blocks(s, A->n);
  s->prm.device_setup = s->device_setup ? 1 : 0;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = now();
  if (A->multi()) {
    if (use_dist_setup(s->prm)) setup_dist(s, A);
    else setup_multi(s, A);
  } else {
    setup_one_process(s, A);
  }
  const double t1 = now();
  // one rank: the device build reads the hierarchy's own matrices (lent, no
  // copy: 11 s and ~45 GB of host memory at 512^3) and they go back to H after
  bool lent = false;
  const std::vector<int>* gsr = s->gs_rank_starts.empty() ? nullptr : &s->gs_rank_starts;
  if (!A->multi()) {
    lent = lend_single_rank(s->H, s->RH, gsr);
    if (!lent) single_rank_hierarchy(s->H, s->RH, gsr);
  }
  const double t2 = now();
  if (!s->dev) s->dev.reset(new DevAMG);
  try {
    s->dev->build(s->RH, A->multi() ? A->comm->dc.get() : nullptr);
  } catch (...) {
    if (lent) give_back_single_rank(s->H, s->RH);
    throw;
  }
  if (lent) give_back_single_rank(s->H, s->RH);
  s->dev->set_use_graph(s->use_graph);
  const double t3 = now();
  char tb[224];
  double rss_c, rss_p;
  host_rss_gb(&rss_c, &rss_p);
  snprintf(tb, sizeof tb,
           "setup: hierarchy %.3fs, rank partition %.3fs, device layouts and upload %.3fs (host RSS %.1f GB, peak "
           "%.1f GB)\n",
           t1 - t0, t2 - t1, t3 - t2, rss_c, rss_p);
  s->H.log += tb;
  if (s->prm.print_level > 0) fputs(tb, stderr);
  API_END
}

HYPRE_Int HYPRE_BoomerAMGSolve(HYPRE_Solver s, HYPRE_ParCSRMatrix A, HYPRE_ParVector b, HYPRE_ParVector x) {
  CHECK_ARG(s && s->kind == KIND_AMG && s->dev && s->dev->built(), 1);
  CHECK_ARG(A, 2);
  CHECK_ARG(b && b->n == s->dev->n0(), 3);
  CHECK_ARG(x && x->n == s->dev->n0(), 4);
  API_BEGIN
  vec_alloc(x);
  s->dev->prm.tol = s->prm.tol;
  s->dev->prm.max_iter = s->prm.max_iter;
  s->dev->prm.min_iter = s->prm.min_iter;
  s->dev->prm.converge_type = s->prm.converge_type;
  s->dev->prm.print_level = s->prm.print_level;
  const int rc = s->dev->solve(b->d, x->d, s->dev->stream(), &s->iters, &s->rel_res);
  HVE_HIP(hipStreamSynchronize(s->dev->stream()));
  if (rc) g_error |= rc;
  API_END
}
HYPRE_Int hypreve_BoomerAMGCycle(HYPRE_Solver s, HYPRE_ParVector f, HYPRE_ParVector u) {
  CHECK_ARG(s && s->kind == KIND_AMG && s->dev && s->dev->built(), 1);
  CHECK_ARG(f && u && f->n == s->dev->n0() && u->n == s->dev->n0(), 2);
  API_BEGIN
  s->dev->cycle(f->d, u->d, s->dev->stream());
  HVE_HIP(hipStreamSynchronize(s->dev->stream()));
  API_END
}
HYPRE_Int HYPRE_BoomerAMGGetNumIterations(HYPRE_Solver s, HYPRE_Int* it) {
  CHECK_ARG(s && it, 1);
  *it = s->iters;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGGetFinalRelativeResidualNorm(HYPRE_Solver s, HYPRE_Real* r) {
  CHECK_ARG(s && r, 1);
  *r = s->rel_res;
  return 0;
}
HYPRE_Int HYPRE_BoomerAMGGetNumLevels(HYPRE_Solver s, HYPRE_Int* nl) {
  CHECK_ARG(s && nl, 1);
  *nl = s->H.lev.empty() ? (int)s->RH.lev.size() : (int)s->H.lev.size();
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetComplexities(HYPRE_Solver s, HYPRE_Real* grid, HYPRE_Real* oper, HYPRE_Real* cycle) {
  CHECK_ARG(s, 1);
  if (grid) *grid = s->H.lev.empty() ? s->RH.grid_complexity : s->H.grid_complexity;
  if (oper) *oper = s->H.lev.empty() ? s->RH.operator_complexity : s->H.operator_complexity;
  if (cycle) {
    // par_cycle.c op count: one smoothing sweep costs nnz(A_l)
    double ops = 0;
    const bool dist = s->H.lev.empty();
    const int nl = dist ? (int)s->RH.nnz_A.size() : (int)s->H.lev.size();
    const AMGParams& p = dist ? s->RH.prm : s->H.prm;
    auto nnz = [&](int l) { return dist ? (double)s->RH.nnz_A[l] : (double)s->H.lev[l].A.nnz(); };
    for (int l = 0; l < nl; ++l) {
      const double nz = nnz(l);
      if (nl == 1) ops += nz;
      else if (l < nl - 1) ops += nz * (p.num_sweeps[1] + p.num_sweeps[2]);
      else ops += nz * p.num_sweeps[3];
    }
    *cycle = nl ? ops / nnz(0) : 0.0;
  }
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetLevelInfo(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int* rows, int64_t* nnz_A,
                                        int64_t* nnz_P) {
  CHECK_ARG(s, 1);
  if (s->H.lev.empty()) {  // distributed setup: global rows / nnz of A only
    CHECK_ARG(level >= 0 && level < (int)s->RH.rows.size(), 2);
    if (rows) *rows = (int)s->RH.rows[level];
    if (nnz_A) *nnz_A = s->RH.nnz_A[level];
    if (nnz_P) *nnz_P = -1;
    return 0;
  }
  CHECK_ARG(level >= 0 && level < (int)s->H.lev.size(), 2);
  const Level& L = s->H.lev[level];
  if (rows) *rows = L.A.nrows;
  if (nnz_A) *nnz_A = L.A.nnz();
  if (nnz_P) *nnz_P = L.P.nnz();
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetLevelMatrix(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int which, HYPRE_Int* nrows,
                                          HYPRE_Int* ncols, int64_t* nnz, HYPRE_Int* row_ptr, HYPRE_Int* cols,
                                          HYPRE_Real* vals) {
  CHECK_ARG(s && level >= 0 && level < (int)s->H.lev.size(), 2);
  const Level& L = s->H.lev[level];
  const CSR& M = which == 0 ? L.A : which == 1 ? L.P : L.R;
  if (nrows) *nrows = M.nrows;
  if (ncols) *ncols = M.ncols;
  if (nnz) *nnz = M.nnz();
  if (row_ptr && !M.i.empty()) std::memcpy(row_ptr, M.i.data(), sizeof(int) * M.i.size());
  if (cols && M.nnz()) std::memcpy(cols, M.j.data(), sizeof(int) * M.nnz());
  if (vals && M.nnz()) std::memcpy(vals, M.a.data(), sizeof(double) * M.nnz());
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetLevelVector(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int which, HYPRE_Int* n,
                                          void* data) {
  CHECK_ARG(s && level >= 0 && level < (int)s->H.lev.size(), 2);
  const Level& L = s->H.lev[level];
  if (which == 0) {
    if (n) *n = (int)L.cf.size();
    if (data && !L.cf.empty()) std::memcpy(data, L.cf.data(), sizeof(int) * L.cf.size());
  } else if (which == 1) {
    // with the N-rank GS emulation: the norms of its blocks (what the device sweeps with)
    const std::vector<double>& l1 = level < (int)s->gs_l1_host.size() ? s->gs_l1_host[level] : L.l1;
    if (n) *n = (int)l1.size();
    if (data && !l1.empty()) std::memcpy(data, l1.data(), sizeof(double) * l1.size());
  } else if (which == 3) {
    // hybrid-GS block starts of the N-rank emulation (empty: hypre's num_blocks partition)
    static const std::vector<int> none;
    const std::vector<int>& b = level < (int)s->gs_blocks_host.size() ? s->gs_blocks_host[level] : none;
    if (n) *n = (int)b.size();
    if (data && !b.empty()) std::memcpy(data, b.data(), sizeof(int) * b.size());
  } else {
    if (n) *n = (int)L.cheby_ds.size();
    if (data && !L.cheby_ds.empty()) std::memcpy(data, L.cheby_ds.data(), sizeof(double) * L.cheby_ds.size());
  }
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetChebyInfo(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int* ncoefs, HYPRE_Real* coefs,
                                        HYPRE_Real* eig, HYPRE_Int* params) {
  CHECK_ARG(s && level >= 0 && level < (int)s->H.lev.size(), 2);
  const Level& L = s->H.lev[level];
  if (params) { params[0] = s->H.prm.cheby_order; params[1] = s->H.prm.cheby_scale; params[2] = s->H.prm.cheby_variant; }
  if (ncoefs) *ncoefs = (int)L.cheby_coefs.size();
  if (coefs && !L.cheby_coefs.empty()) std::memcpy(coefs, L.cheby_coefs.data(), sizeof(double) * L.cheby_coefs.size());
  if (eig) { eig[0] = L.max_eig; eig[1] = L.min_eig; }
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetCoarseMatrix(HYPRE_Solver s, HYPRE_Int* n, HYPRE_Real* dense) {
  CHECK_ARG(s, 1);
  if (n) *n = s->H.coarse_n;
  if (dense && !s->H.coarse_dense.empty())
    std::memcpy(dense, s->H.coarse_dense.data(), sizeof(double) * s->H.coarse_dense.size());
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetRelaxInfo(HYPRE_Solver s, HYPRE_Int* rt, HYPRE_Int* ns, HYPRE_Real* w, HYPRE_Int* misc) {
  CHECK_ARG(s, 1);
  const AMGParams& p = s->H.lev.empty() ? (s->RH.lev.empty() ? s->prm : s->RH.prm) : s->H.prm;
  for (int i = 0; i < 4; ++i) { if (rt) rt[i] = p.relax_type[i]; if (ns) ns[i] = p.num_sweeps[i]; }
  if (w) { w[0] = p.relax_weight; w[1] = p.outer_weight; }
  if (misc) { misc[0] = p.relax_order; misc[1] = p.cycle_type; misc[2] = p.num_blocks; misc[3] = p.user_relax_type; }
  return 0;
}
HYPRE_Int hypreve_BoomerAMGGetKernelStats(HYPRE_Solver s, HYPRE_Real* stats, HYPRE_Int n) {
  CHECK_ARG(s && stats, 1);
  for (int i = 0; i < n; ++i) stats[i] = 0.0;
  if (n > 0 && s->dev) stats[0] = s->dev->cycle_op_count();
  return 0;
}

// Finest-level residual SpMV timed with HIP events on the solver's stream.
// Algorithmic bytes per launch: nnz*(8 val + 4 col) + n*(8 x + 8 b + 8 y)
// + slice pointers (4 per 64 rows).
HYPRE_Int hypreve_BenchFineSpMV(HYPRE_Solver s, HYPRE_Int reps, HYPRE_Real* avg_ms, HYPRE_Real* bytes) {
  CHECK_ARG(s && s->dev && s->dev->built(), 1);
  API_BEGIN
  DevAMG& D = *s->dev;
  const DevSell& A = D.level(0).A.in;
  hipStream_t st = D.stream();
  double* x = D.scratch(0);
  double* b = D.scratch(1);
  double* y = D.scratch(2);
  HVE_HIP(launch_set(A.nrows, 1.0, x, st));
  HVE_HIP(launch_set(A.nrows, 0.5, b, st));
  for (int w = 0; w < 3; ++w)
    HVE_HIP(launch_sell(K_RESID, A.view(), x, b, nullptr, nullptr, 0, y, -1.0, 0.0, st));
  hipEvent_t e0, e1;
  HVE_HIP(hipEventCreate(&e0));
  HVE_HIP(hipEventCreate(&e1));
  HVE_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r)
    HVE_HIP(launch_sell(K_RESID, A.view(), x, b, nullptr, nullptr, 0, y, -1.0, 0.0, st));
  HVE_HIP(hipEventRecord(e1, st));
  HVE_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  HVE_HIP(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (avg_ms) *avg_ms = ms / reps;
  if (bytes) *bytes = (double)A.nnz * 12.0 + (double)A.nrows * 24.0 + (double)(A.nslices + 1) * 4.0;
  API_END
}

// Bytes the finest residual SpMV streams in its stored layout (padding, 16-bit
// column deltas and their slot bases included) plus the three vectors: what
// the layout moves, beside BenchFineSpMV's algorithmic (CSR) bytes.
HYPRE_Int hypreve_BenchFineSpMVStoredBytes(HYPRE_Solver s, HYPRE_Real* bytes) {
  CHECK_ARG(s && s->dev && s->dev->built() && bytes, 1);
  API_BEGIN
  const DevSell& A = s->dev->level(0).A.in;
  *bytes = (double)A.bytes() + (double)A.nrows * 24.0;
  API_END
}

// Device layout of a level operator's interior rows (which: 0 A, 1 P, 2 R):
// 0 padded SELL-64, 1 jagged, 2 workgroup-per-slice, 3 jagged wave-product,
// 4 dictionary (LDS x-tile), 5 16-bit column deltas, 6 deltas + 8-bit value
// table, 7 deltas + 16-bit value table, 8 padded + 16-bit value table,
// 9 jagged + 16-bit value table, 10 range dictionary, 11 slot-uniform stencil
// (no per-entry data), 12 offset-coded, 13 packed codes, 14 the stencil's grid
// form, 15 dictionary with lane-packed streams (k_sell_dictw).
HYPRE_Int hypreve_BoomerAMGGetLevelLayout(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int which, HYPRE_Int* kind) {
  CHECK_ARG(s && s->dev && s->dev->built() && kind, 1);
  CHECK_ARG(level >= 0 && level < s->dev->num_levels(), 2);
  CHECK_ARG(which >= 0 && which <= 2 && (which == 0 || level < s->dev->num_levels() - 1), 3);
  API_BEGIN
  const DevLevel& L = s->dev->level(level);
  const DevSell& M = which == 0 ? L.A.in : which == 1 ? L.P.in : L.R.in;
  *kind = M.code32 ? 13 : M.code16 ? (M.rowlen ? 16 : 12) : M.slot_mask ? (grid_stencil_on(M.view()) ? 14 : 11)
         : M.dcol ? (M.vidx16 ? 7 : M.vidx ? 6 : 5)
                 : M.vidx16 ? (M.rowlen ? 9 : 8) : M.col16 ? (M.dict_ranges ? 10 : M.wptr ? 15 : 4) : M.pw ? 3 : M.rowlen ? 1
                 : M.wide ? 2 : 0;
  API_END
}

// Host check of every hybrid Gauss-Seidel level schedule of the hierarchy
// (both directions, diagonal and l1 scaling) against the sequential sweep.
HYPRE_Int hypreve_BoomerAMGGsScheduleCheck(HYPRE_Solver s, HYPRE_Int num_blocks) {
  CHECK_ARG(s && s->kind == KIND_AMG && !s->H.lev.empty(), 1);
  CHECK_ARG(num_blocks >= 1, 2);
  API_BEGIN
  for (size_t l = 0; l < s->H.lev.size(); ++l) {
    const CSR& A = s->H.lev[l].A;
    std::vector<double> l1 = s->H.lev[l].l1;
    if (l1.empty()) {
      l1.resize(A.nrows);
      for (int i = 0; i < A.nrows; ++i) {
        double t = 0;
        for (int k = A.i[i]; k < A.i[i + 1]; ++k) t += std::fabs(A.a[k]);
        l1[i] = t;
      }
    }
    // teams of about 64 rows a step (the default) and of a few rows (many
    // steps per team level: ring reach and fences exercised)
    for (int team_rows : {64, 3})
      for (int fwd = 0; fwd < 2; ++fwd)
        for (int use_l1 = 0; use_l1 < 2; ++use_l1)
          for (int wgt = 0; wgt < 2; ++wgt) {
            std::string msg;
            if (gs_schedule_self_check(A, num_blocks, fwd != 0, use_l1 != 0, l1, msg, team_rows, wgt != 0))
              throw std::runtime_error("level " + std::to_string(l) + (fwd ? " forward" : " backward") +
                                       (use_l1 ? " l1" : "") + (wgt ? " weighted" : "") + " team_rows " +
                                       std::to_string(team_rows) + ": " + msg);
          }
  }
  API_END
}

// This rank's communication in one V-cycle (the last cycle the solver emitted):
// out = {halo exchanges, bytes they send, all-gathers, all-gather bytes sent,
// all-reduces} on level `level`; zeros on one rank.
HYPRE_Int hypreve_BoomerAMGGetCycleCommStats(HYPRE_Solver s, HYPRE_Int level, int64_t* out) {
  CHECK_ARG(s && s->kind == KIND_AMG && s->dev, 1);
  CHECK_ARG(out, 3);
  API_BEGIN
  const auto& cc = s->dev->cycle_comm();
  for (int k = 0; k < 5; ++k) out[k] = 0;
  if (level >= 0 && level < (HYPRE_Int)cc.size()) {
    out[0] = cc[level].exchanges;
    out[1] = cc[level].bytes;
    out[2] = cc[level].allgathers;
    out[3] = cc[level].allgather_bytes;
    out[4] = cc[level].allreduces;
  }
  API_END
}

// Size of the packed hybrid Gauss-Seidel schedule of a level's A for a block
// count (host only): out = {nnz, stored entries, steps, teams, longest team
// (steps), blocks}.
HYPRE_Int hypreve_BoomerAMGGsScheduleStats(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int forward, HYPRE_Int num_blocks,
                                           int64_t* out) {
  CHECK_ARG(s && s->kind == KIND_AMG && !s->H.lev.empty(), 1);
  CHECK_ARG(level >= 0 && level < (HYPRE_Int)s->H.lev.size(), 2);
  CHECK_ARG(num_blocks >= 1, 4);
  CHECK_ARG(out, 5);
  API_BEGIN
  const CSR& A = s->H.lev[level].A;
  GsSchedule S;
  build_gs_schedule(A, hypre_block_starts(A.nrows, num_blocks), forward != 0, S);
  out[0] = S.nnz;
  out[1] = (int64_t)S.code.size();
  out[2] = S.team_step.back();
  out[3] = S.nteams;
  out[4] = S.max_steps;
  out[5] = num_blocks;
  API_END
}

// Host check of the slot-uniform stencil layout of a level's A: every row's
// (column, value) sequence rebuilt from its slice's pattern equals the CSR row
// entry for entry (bit patterns of the values included).  *width = 0 when the
// operator is not a constant-coefficient stencil (the layout does not build).
HYPRE_Int hypreve_GridStencilAddressable(HYPRE_BigInt nx, HYPRE_BigInt ny, HYPRE_BigInt nz) {
  return grid_stencil_addressable(nx, ny, nz) ? 1 : 0;
}
HYPRE_Int hypreve_BoomerAMGStencilLayoutCheck(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int* width,
                                              HYPRE_Int* npatterns) {
  CHECK_ARG(s && s->kind == KIND_AMG && !s->H.lev.empty(), 1);
  CHECK_ARG(level >= 0 && level < (HYPRE_Int)s->H.lev.size(), 2);
  API_BEGIN
  const CSR& A = s->H.lev[level].A;
  std::vector<int> pat, off, vi;
  std::vector<uint64_t> mask;
  std::vector<double> tab;
  int W = 0;
  if (width) *width = 0;
  if (npatterns) *npatterns = 0;
  // not a constant-coefficient stencil: success with width 0 (not the sticky error flag)
  if (!build_sell_stencil_host(A, 64, W, pat, off, vi, mask, tab)) return 0;
  for (int r = 0; r < A.nrows; ++r) {
    const size_t p0 = (size_t)pat[r >> 6] * W;
    int e = A.i[r];
    for (int k = 0; k < W; ++k) {
      if (!((mask[p0 + k] >> (r & 63)) & 1)) continue;
      if (e >= A.i[r + 1] || (int64_t)A.j[e] - r != off[p0 + k] ||
          std::memcmp(&tab[vi[p0 + k]], &A.a[e], 8) != 0)
        throw std::runtime_error("stencil layout: row " + std::to_string(r) + " differs at its entry " +
                                 std::to_string(e - A.i[r]));
      ++e;
    }
    if (e != A.i[r + 1]) throw std::runtime_error("stencil layout: row " + std::to_string(r) + " loses entries");
    if (A.i[r + 1] > A.i[r] && !(mask[p0] >> (r & 63) & 1))
      throw std::runtime_error("stencil layout: row " + std::to_string(r) + " does not start in slot 0");
  }
  if (width) *width = W;
  if (npatterns) *npatterns = (HYPRE_Int)((off.size() - 16) / std::max(W, 1));
  API_END
}

// Host check of the offset-coded layout of level's P (which 1) or R (which 2):
// every row decoded from its 16-bit codes (offset and value tables, anchors,
// fine -> coarse map) equals the CSR row entry for entry, values bitwise.
HYPRE_Int hypreve_BoomerAMGCodedLayoutCheck(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int which, HYPRE_Int* noffsets,
                                            HYPRE_Int* nvalues) {
  CHECK_ARG(s && s->kind == KIND_AMG && !s->H.lev.empty(), 1);
  CHECK_ARG(level >= 0 && level + 1 < (HYPRE_Int)s->H.lev.size(), 2);
  CHECK_ARG(which == 1 || which == 2, 3);
  API_BEGIN
  const auto& L = s->H.lev[level];
  const CSR& M = which == 1 ? L.P : L.R;
  if (noffsets) *noffsets = 0;
  if (nvalues) *nvalues = 0;
  std::vector<int> fc, cidx(L.A.nrows, -1);
  for (int i = 0; i < (int)L.cf.size() && i < L.A.nrows; ++i)
    if (L.cf[i] == 1) {
      cidx[i] = (int)fc.size();
      fc.push_back(i);
    }
  static const std::vector<int> none;
  std::vector<int> sp, ot;
  hvec<unsigned short> code;
  std::vector<double> tab;
  int vb = 0;
  // not coded (too many offsets or values): success with zero counts
  if (!build_sell_coded_host(M, none, which == 2 ? fc : none, which == 1 ? fc : none, which == 1 ? cidx : none, sp,
                             code, ot, tab, vb))
    return 0;
  for (int r = 0; r < M.nrows; ++r) {
    const int s0 = r >> 6, w = (sp[s0 + 1] - sp[s0]) >> 6;
    const int64_t a = which == 2 ? fc[r] : r;
    int e = M.i[r];
    for (int k = 0; k < w; ++k) {
      const unsigned c = code[(size_t)sp[s0] + (size_t)k * 64 + (r & 63)];
      if (c == 0xFFFF) break;
      const int64_t pos = a + ot[c >> vb];
      const int64_t col = which == 1 ? cidx[pos] : pos;
      if (e >= M.i[r + 1] || col != M.j[e] || std::memcmp(&tab[c & ((1u << vb) - 1)], &M.a[e], 8) != 0)
        throw std::runtime_error("coded layout: row " + std::to_string(r) + " differs at its entry " +
                                 std::to_string(e - M.i[r]));
      ++e;
    }
    if (e != M.i[r + 1]) throw std::runtime_error("coded layout: row " + std::to_string(r) + " loses entries");
  }
  if (noffsets) *noffsets = (HYPRE_Int)ot.size();
  if (nvalues) *nvalues = (HYPRE_Int)tab.size();
  API_END
}

// Average time of one application of a level operator (which: 0 = A_l as the
// residual r = f - A u, 1 = P_l as prolongation u_l += P u_{l+1}, 2 = R_l as
// restriction f_{l+1} = R r_l) with its algorithmic bytes: every stored
// nonzero once (8 B value + 4 B column), each input vector entry once, each
// output entry read and/or written once.  Interior rows only on multi-rank.
HYPRE_Int hypreve_BenchOperator(HYPRE_ParCSRMatrix A, HYPRE_Int op, HYPRE_Int policy, HYPRE_Int nbands,
                                HYPRE_Int reps, HYPRE_Real* avg_ms, HYPRE_Real* stored_bytes, char* layout, HYPRE_Int len) {
  CHECK_ARG(A && !A->multi(), 1);
  CHECK_ARG(op == K_RESID || op == K_MATVEC || op == K_L1JAC || op == K_RESID_L1JAC, 2);
  CHECK_ARG(reps > 0, 5);
  API_BEGIN
  const double ms = bench_operator(A->diag, op, policy, nbands, reps, stored_bytes, layout, len);
  if (avg_ms) *avg_ms = ms;
  API_END
}
HYPRE_Int hypreve_BenchLevelOp(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int which, HYPRE_Int reps,
                               HYPRE_Real* avg_ms, HYPRE_Real* bytes, HYPRE_Real* padded_nnz) {
  CHECK_ARG(s && s->dev && s->dev->built(), 1);
  CHECK_ARG(level >= 0 && level < s->dev->num_levels(), 2);
  CHECK_ARG(which >= 0 && which <= 3 && (which == 0 || which == 3 || level < s->dev->num_levels() - 1), 3);
  CHECK_ARG(reps > 0, 4);
  API_BEGIN
  DevAMG& D = *s->dev;
  const DevLevel& L = D.level(level);
  const DevSell& M = (which == 0 || which == 3) ? L.A.in : which == 1 ? L.P.in : L.R.in;
  const int op = which == 0 ? K_RESID : which == 1 ? K_PROLONG : which == 2 ? K_RESTRICT : K_L1JAC;
  hipStream_t st = D.stream();
  double* x = D.scratch(0);
  double* b = D.scratch(1);
  double* y = D.scratch(2);
  HVE_HIP(launch_set(D.ws_n(), 1.0, x, st));
  HVE_HIP(launch_set(D.ws_n(), 0.5, b, st));
  HVE_HIP(launch_set(D.ws_n(), 0.0, y, st));
  // which 3: A as the l1-Jacobi sweep, with b standing in for the l1 norms
  const double* l1 = which == 3 ? b : nullptr;
  auto launch = [&] { HVE_HIP(launch_sell(op, M.view(), x, b, l1, nullptr, 0, y, -1.0, 0.0, st)); };
  for (int w = 0; w < 3; ++w) launch();
  hipEvent_t e0, e1;
  HVE_HIP(hipEventCreate(&e0));
  HVE_HIP(hipEventCreate(&e1));
  HVE_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) launch();
  HVE_HIP(hipEventRecord(e1, st));
  HVE_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  HVE_HIP(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (avg_ms) *avg_ms = ms / reps;
  const double out_rw = which == 0 ? 16.0 : which == 1 ? 16.0 : 8.0;  // b read + y write / y rw / y write
  if (bytes)
    *bytes = (double)M.nnz * 12.0 + (double)M.nrows * out_rw + (double)M.ncols * 8.0 + (double)(M.nslices + 1) * 4.0 +
             (M.rowmap ? (double)M.nrows * 4.0 : 0.0) + (M.rowlen ? (double)M.nrows * 4.0 : 0.0);
  if (padded_nnz) *padded_nnz = (double)M.nnz_pad;
  API_END
}

// Tuning knobs read by the launch code (kernels.h set_knob): variants compared
// in one process on one hierarchy.
HYPRE_Int hypreve_SetKnob(HYPRE_Int id, HYPRE_Int value) {
  CHECK_ARG(id >= 0 && id < 32, 1);
  set_knob(id, value);
  return 0;
}

// Bytes one hypreve_BenchLevelOp launch streams in the operator's stored layout
// (DevSell::bytes: compressed columns / values, padding, bases, dictionaries,
// row maps) plus its vectors counted as BenchLevelOp counts them.
HYPRE_Int hypreve_BenchLevelOpStoredBytes(HYPRE_Solver s, HYPRE_Int level, HYPRE_Int which, HYPRE_Real* bytes) {
  CHECK_ARG(s && s->dev && s->dev->built() && bytes, 1);
  CHECK_ARG(level >= 0 && level < s->dev->num_levels(), 2);
  CHECK_ARG(which >= 0 && which <= 3 && (which == 0 || which == 3 || level < s->dev->num_levels() - 1), 3);
  API_BEGIN
  const DevLevel& L = s->dev->level(level);
  const DevSell& M = (which == 0 || which == 3) ? L.A.in : which == 1 ? L.P.in : L.R.in;
  // b read + y write / y rw / y write / f, u_g, l1 read + u' write
  const double out_rw = which == 0 ? 16.0 : which == 1 ? 16.0 : which == 2 ? 8.0 : 32.0;
  *bytes = (double)M.bytes() + (double)M.nrows * out_rw + (double)M.ncols * 8.0;
  API_END
}

// Read-only streaming kernel over n elements of elem_bytes (4, 8 or 16) each: the
// calibration pass for rocprofv3 FETCH_SIZE at this access width and the
// achievable-bandwidth reference for the roofline.
HYPRE_Int hypreve_BenchStream(HYPRE_Int elem_bytes, int64_t n, HYPRE_Int reps, HYPRE_Real* avg_ms) {
  CHECK_ARG(elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8 || elem_bytes == 16 || elem_bytes == -1 ||
                elem_bytes == -2 || elem_bytes == -5 || elem_bytes == -8 || elem_bytes == -9,
            1);
  CHECK_ARG(n > 0, 2);
  CHECK_ARG(reps > 0, 3);
  API_BEGIN
  if (elem_bytes == -8 || elem_bytes == -9) {  // n doubles in per-wave segments (-9: interleaved)
    double *buf = nullptr, *out = nullptr;
    hipStream_t st = lib_stream();
    HVE_HIP(hipMalloc((void**)&buf, (size_t)n * sizeof(double)));
    HVE_HIP(hipMalloc((void**)&out, sizeof(double)));
    HVE_HIP(hipMemsetAsync(buf, 0, (size_t)n * sizeof(double), st));
    for (int w = 0; w < 2; ++w) HVE_HIP(launch_stream_seg(n, elem_bytes == -9, buf, out, st));
    hipEvent_t e0, e1;
    HVE_HIP(hipEventCreate(&e0));
    HVE_HIP(hipEventCreate(&e1));
    HVE_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) HVE_HIP(launch_stream_seg(n, elem_bytes == -9, buf, out, st));
    HVE_HIP(hipEventRecord(e1, st));
    HVE_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    HVE_HIP(hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    (void)hipFree(buf);
    (void)hipFree(out);
    if (avg_ms) *avg_ms = ms / reps;
    return 0;
  }
  if (elem_bytes < 0) {  // read/write mix: -R = R double reads + 1 double write per element
    const int R = -elem_bytes;
    double *src = nullptr, *y = nullptr;
    hipStream_t st = lib_stream();
    HVE_HIP(hipMalloc((void**)&src, (size_t)n * R * sizeof(double)));
    HVE_HIP(hipMalloc((void**)&y, (size_t)n * sizeof(double)));
    HVE_HIP(hipMemsetAsync(src, 0, (size_t)n * R * sizeof(double), st));
    for (int w = 0; w < 2; ++w) HVE_HIP(launch_stream_mix(n, R, src, y, st));
    hipEvent_t e0, e1;
    HVE_HIP(hipEventCreate(&e0));
    HVE_HIP(hipEventCreate(&e1));
    HVE_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) HVE_HIP(launch_stream_mix(n, R, src, y, st));
    HVE_HIP(hipEventRecord(e1, st));
    HVE_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    HVE_HIP(hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    (void)hipFree(src);
    (void)hipFree(y);
    if (avg_ms) *avg_ms = ms / reps;
    return 0;
  }
  void* buf = nullptr;
  double* out = nullptr;
  hipStream_t st = lib_stream();
  HVE_HIP(hipMalloc(&buf, (size_t)n * elem_bytes));
  HVE_HIP(hipMalloc((void**)&out, sizeof(double)));
  HVE_HIP(hipMemsetAsync(buf, 0, (size_t)n * elem_bytes, st));
  for (int w = 0; w < 2; ++w) HVE_HIP(launch_stream_read((int64_t)n * elem_bytes, elem_bytes, buf, out, st));
  hipEvent_t e0, e1;
  HVE_HIP(hipEventCreate(&e0));
  HVE_HIP(hipEventCreate(&e1));
  HVE_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) HVE_HIP(launch_stream_read((int64_t)n * elem_bytes, elem_bytes, buf, out, st));
  HVE_HIP(hipEventRecord(e1, st));
  HVE_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  HVE_HIP(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  (void)hipFree(buf);
  (void)hipFree(out);
  if (avg_ms) *avg_ms = ms / reps;
  API_END
}

// ---------------------------------------------------------------------------
// PCG
// ---------------------------------------------------------------------------
HYPRE_Int HYPRE_ParCSRPCGCreate(HYPRE_Comm comm, HYPRE_Solver* solver) {
  CHECK_ARG(solver, 2);
  auto* s = new hypre_Solver_struct;
  s->kind = KIND_PCG;
  *solver = s;
  return 0;
}
HYPRE_Int HYPRE_ParCSRPCGDestroy(HYPRE_Solver s) {
  if (!s) return 0;
  delete s;
  return 0;
}
HYPRE_Int HYPRE_ParCSRPCGSetTol(HYPRE_Solver s, HYPRE_Real tol) { CHECK_ARG(s, 1); s->pcg.tol = tol; return 0; }
HYPRE_Int HYPRE_ParCSRPCGSetMaxIter(HYPRE_Solver s, HYPRE_Int m) { CHECK_ARG(s, 1); s->pcg.max_iter = m; return 0; }
HYPRE_Int HYPRE_ParCSRPCGSetTwoNorm(HYPRE_Solver s, HYPRE_Int t) { CHECK_ARG(s, 1); s->pcg.two_norm = t; return 0; }
HYPRE_Int HYPRE_ParCSRPCGSetPrintLevel(HYPRE_Solver s, HYPRE_Int l) { CHECK_ARG(s, 1); s->pcg.print_level = l; return 0; }
HYPRE_Int HYPRE_ParCSRPCGSetPrecond(HYPRE_Solver s, HYPRE_PtrToParSolverFcn precond,
                                    HYPRE_PtrToParSolverFcn precond_setup, HYPRE_Solver precond_solver) {
  CHECK_ARG(s && s->kind == KIND_PCG, 1);
  s->precond_solve = precond;
  s->precond_setup = precond_setup;
  s->precond = precond_solver;
  return 0;
}
HYPRE_Int HYPRE_ParCSRPCGSetup(HYPRE_Solver s, HYPRE_ParCSRMatrix A, HYPRE_ParVector b, HYPRE_ParVector x) {
  CHECK_ARG(s && s->kind == KIND_PCG, 1);
  CHECK_ARG(A, 2);
  API_BEGIN
  if (s->precond_setup && s->precond) {
    int rc = s->precond_setup(s->precond, A, b, x);
    if (rc) return rc;
  }
  if (!(s->precond && s->precond->kind == KIND_AMG && s->precond->dev)) {
    A->ensure_device();
    s->ws.reset(new DevAMG);
    s->ws->init_workspace(A->n, nullptr);
  }
  API_END
}
HYPRE_Int HYPRE_ParCSRPCGSolve(HYPRE_Solver s, HYPRE_ParCSRMatrix A, HYPRE_ParVector b, HYPRE_ParVector x) {
  CHECK_ARG(s && s->kind == KIND_PCG, 1);
  CHECK_ARG(A, 2);
  CHECK_ARG(b && b->n == A->n, 3);
  CHECK_ARG(x && x->n == A->n, 4);
  API_BEGIN
  vec_alloc(x);
  DevAMG* amg = (s->precond && s->precond->kind == KIND_AMG && s->precond->dev) ? s->precond->dev.get() : nullptr;
  DevAMG* ws = amg ? amg : s->ws.get();
  if (!ws) throw std::runtime_error("PCGSolve called before PCGSetup");
  hipStream_t st = ws->stream();
  Precond pre;
  if (amg && s->precond_solve == (HYPRE_PtrToParSolverFcn)HYPRE_BoomerAMGSolve) {
    // HYPRE_BoomerAMGSolve(precond, A, r, z) on device buffers, honoring the
    // preconditioner's tol / max_iter (tol 0, max_iter 1 = one cycle)
    hypre_Solver_struct* P = s->precond;
    pre = [amg, P, st](const double* r, double* z, bool z_zero) {
      amg->prm.tol = P->prm.tol;
      amg->prm.max_iter = P->prm.max_iter;
      amg->prm.min_iter = P->prm.min_iter;
      amg->prm.converge_type = P->prm.converge_type;
      amg->prm.print_level = 0;
      if (P->prm.tol == 0.0 && P->prm.max_iter == 1) {
        amg->cycle(r, z, st, nullptr, z_zero);  // one cycle from the cleared z: zero-guess first sweep
      } else {
        if (z_zero) HVE_HIP(launch_set(amg->n0(), 0.0, z, st));
        amg->solve(r, z, st, &P->iters, &P->rel_res);
      }
    };
  } else if (s->precond_solve && s->precond) {
    const int n = A->n;
    hypre_Solver_struct* P = s->precond;
    auto fn = s->precond_solve;
    pre = [fn, P, A, n, st](const double* r, double* z, bool z_zero) {
      if (z_zero) HVE_HIP(launch_set(n, 0.0, z, st));
      HVE_HIP(hipStreamSynchronize(st));
      hypre_ParVector_struct rv, zv;
      rv.n = zv.n = n; rv.d = const_cast<double*>(r); zv.d = z; rv.owns = zv.owns = false;
      fn(P, A, &rv, &zv);
    };
  } else {
    const int n = A->n;
    pre = [n, st](const double* r, double* z, bool) { HVE_HIP(launch_copy(n, r, z, st)); };
  }
  MatvecFn Aop;
  if (amg) {
    Aop = [amg, st](int op, const double* xx, const double* bb, double* yy, double* dot) {
      if (op == K_MATVEC && dot) amg->fine_matvec_dot(xx, yy, dot, st);
      else amg->fine_apply(op, xx, bb, yy, op == K_RESID ? -1.0 : 1.0, 0.0, st);
    };
  } else {
    A->ensure_device();
    DevSell* dA = &A->dA;
    Aop = [dA, ws, n = A->n, st](int op, const double* xx, const double* bb, double* yy, double* dot) {
      HVE_HIP(launch_sell(op, dA->view(), xx, bb, nullptr, nullptr, 0, yy, op == K_RESID ? -1.0 : 1.0, 0.0, st));
      if (dot) ws->dot(n, yy, xx, dot, st);
    };
  }
  const int rc = pcg_solve(ws, A->n, Aop, s->pcg, pre, b->d, x->d, st, &s->iters, &s->rel_res);
  if (rc) g_error |= rc;
  API_END
}
HYPRE_Int HYPRE_ParCSRPCGGetNumIterations(HYPRE_Solver s, HYPRE_Int* it) {
  CHECK_ARG(s && it, 1);
  *it = s->iters;
  return 0;
}
HYPRE_Int HYPRE_ParCSRPCGGetFinalRelativeResidualNorm(HYPRE_Solver s, HYPRE_Real* r) {
  CHECK_ARG(s && r, 1);
  *r = s->rel_res;
  return 0;
}

}  // extern "C"
