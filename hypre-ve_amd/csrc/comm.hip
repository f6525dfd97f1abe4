// Communicator handles of the C ABI (the reference passes an MPI_Comm; here a
// HYPRE_Comm wraps a DevComm: RCCL over xGMI, one process per GPU, or the
// in-process loopback hub used by the parity tests).
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/hypreve.h"
#include "device/comm.hpp"

using namespace hve;

extern "C" {

HYPRE_Int hypreve_CommGetUniqueId(void* nccl_id_128) {
  if (!nccl_id_128) return HYPRE_ERROR_ARG;
  try {
    rccl_unique_id(nccl_id_128);
  } catch (...) {
    return HYPRE_ERROR_GENERIC;
  }
  return 0;
}

HYPRE_Int hypreve_CommCreate(HYPRE_Int rank, HYPRE_Int size, const void* nccl_id_128, HYPRE_Comm* comm) {
  if (!comm || size < 1 || rank < 0 || rank >= size || (size > 1 && !nccl_id_128)) return HYPRE_ERROR_ARG;
  auto* c = new hypreve_comm_struct;
  c->rank = rank;
  c->size = size;
  // size 1 with an id: a 1-rank RCCL communicator (the partitioned path with
  // one rank; used to exercise RCCL on a single-GPU box)
  if (size > 1 || nccl_id_128) {
    try {
      c->dc = make_rccl_comm(rank, size, nccl_id_128);
    } catch (...) {
      delete c;
      return HYPRE_ERROR_GENERIC;
    }
  }
  *comm = c;
  return 0;
}

HYPRE_Int hypreve_CommCreateShm(HYPRE_Int rank, HYPRE_Int size, const char* shm_name, HYPRE_Comm* comm) {
  if (!comm || !shm_name || size < 1 || rank < 0 || rank >= size) return HYPRE_ERROR_ARG;
  auto* c = new hypreve_comm_struct;
  c->rank = rank;
  c->size = size;
  if (size > 1) {
    try {
      c->dc = make_shm_comm(rank, size, shm_name);
    } catch (...) {
      delete c;
      return HYPRE_ERROR_GENERIC;
    }
  }
  *comm = c;
  return 0;
}

HYPRE_Int hypreve_CommCreateLoopback(HYPRE_Int size, HYPRE_Comm* comms) {
  if (!comms || size < 1) return HYPRE_ERROR_ARG;
  try {
    auto v = make_loopback_comms(size);
    for (int r = 0; r < size; ++r) {
      auto* c = new hypreve_comm_struct;
      c->rank = r;
      c->size = size;
      if (size > 1) c->dc = std::move(v[r]);
      comms[r] = c;
    }
  } catch (...) {
    return HYPRE_ERROR_GENERIC;
  }
  return 0;
}

// Transport self-test: a grouped exchange with every rank (self included: a
// send to one's own rank), an all-reduce, an all-gather and a broadcast on
// device buffers, each checked on the host.  Collective over the communicator.
HYPRE_Int hypreve_CommSelfTest(HYPRE_Comm comm) {
  if (!comm) return HYPRE_ERROR_ARG;
  if (!comm->dc) return 0;  // single rank without a transport: nothing to test
  try {
    DevComm& dc = *comm->dc;
    const int r = dc.rank(), n = dc.size();
    const int m = 1000;  // doubles per message
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return HYPRE_ERROR_GENERIC;
    std::vector<double> h((size_t)n * m);
    double *dsend = nullptr, *drecv = nullptr, *dsum = nullptr, *dall = nullptr, *dmine = nullptr;
    auto ok = [](hipError_t e) { if (e != hipSuccess) throw std::runtime_error(hipGetErrorString(e)); };
    ok(hipMalloc((void**)&dsend, sizeof(double) * n * m));
    ok(hipMalloc((void**)&drecv, sizeof(double) * n * m));
    ok(hipMalloc((void**)&dsum, sizeof(double) * 4));
    ok(hipMalloc((void**)&dall, sizeof(double) * n));
    ok(hipMalloc((void**)&dmine, sizeof(double)));
    for (int p = 0; p < n; ++p)
      for (int i = 0; i < m; ++i) h[(size_t)p * m + i] = 1e6 * r + 1e3 * p + i;  // from r to p
    ok(hipMemcpy(dsend, h.data(), sizeof(double) * n * m, hipMemcpyHostToDevice));
    std::vector<P2PMsg> sends, recvs;
    for (int p = 0; p < n; ++p) {
      sends.push_back({p, dsend + (size_t)p * m, sizeof(double) * m});
      recvs.push_back({p, drecv + (size_t)p * m, sizeof(double) * m});
    }
    dc.exchange(sends, recvs, st);
    const double v4[4] = {1.0 + r, 2.0 * r, 0.5, (double)(r == 0)};
    ok(hipMemcpyAsync(dsum, v4, sizeof(v4), hipMemcpyHostToDevice, st));
    dc.allreduce_sum(dsum, 4, st);
    const double mine = 10.0 + r;
    ok(hipMemcpyAsync(dmine, &mine, sizeof(double), hipMemcpyHostToDevice, st));
    dc.allgather(dmine, dall, sizeof(double), st);
    double root_val = r == 0 ? 42.0 : -1.0;
    ok(hipMemcpyAsync(dmine, &root_val, sizeof(double), hipMemcpyHostToDevice, st));
    dc.bcast(dmine, sizeof(double), 0, st);
    std::vector<double> got((size_t)n * m), all(n);
    double sum[4], bc = 0;
    ok(hipMemcpyAsync(got.data(), drecv, sizeof(double) * n * m, hipMemcpyDeviceToHost, st));
    ok(hipMemcpyAsync(sum, dsum, sizeof(sum), hipMemcpyDeviceToHost, st));
    ok(hipMemcpyAsync(all.data(), dall, sizeof(double) * n, hipMemcpyDeviceToHost, st));
    ok(hipMemcpyAsync(&bc, dmine, sizeof(double), hipMemcpyDeviceToHost, st));
    ok(hipStreamSynchronize(st));
    int bad = 0;
    for (int p = 0; p < n; ++p)
      for (int i = 0; i < m; ++i) bad += got[(size_t)p * m + i] != 1e6 * p + 1e3 * r + i;
    bad += sum[0] != n * (n + 1) / 2.0;
    bad += sum[1] != (double)n * (n - 1);
    bad += sum[2] != 0.5 * n;
    bad += sum[3] != 1.0;
    for (int p = 0; p < n; ++p) bad += all[p] != 10.0 + p;
    bad += bc != 42.0;
    for (void* q : {(void*)dsend, (void*)drecv, (void*)dsum, (void*)dall, (void*)dmine}) (void)hipFree(q);
    (void)hipStreamDestroy(st);
    return bad ? HYPRE_ERROR_GENERIC : 0;
  } catch (...) {
    return HYPRE_ERROR_GENERIC;
  }
}

HYPRE_Int hypreve_CommDestroy(HYPRE_Comm comm) {
  delete comm;
  return 0;
}

}  // extern "C"
