// Communicator handles of the C ABI (the reference passes an MPI_Comm; here a
// HYPRE_Comm wraps a DevComm: RCCL over xGMI, one process per GPU, or the
// in-process loopback hub used by the parity tests).
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>

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
  if (size > 1) {
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

HYPRE_Int hypreve_CommDestroy(HYPRE_Comm comm) {
  delete comm;
  return 0;
}

}  // extern "C"
