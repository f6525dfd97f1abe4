// RCCL communicator plumbing (one process per GPU; the reference uses MPI_Comm).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/hypreve.h"

struct hypreve_comm_struct {
  int rank = 0, size = 1;
  void* nccl = nullptr;
};

static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(r) + " in " + what);
}

extern "C" {

HYPRE_Int hypreve_CommGetUniqueId(void* nccl_id_128) {
  if (!nccl_id_128) return HYPRE_ERROR_ARG;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  try {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::memcpy(nccl_id_128, &id, sizeof(id));
  } catch (...) {
    return HYPRE_ERROR_GENERIC;
  }
  return 0;
}

HYPRE_Int hypreve_CommCreate(HYPRE_Int rank, HYPRE_Int size, const void* nccl_id_128, HYPRE_Comm* comm) {
  if (!comm || size < 1 || rank < 0 || rank >= size) return HYPRE_ERROR_ARG;
  auto* c = new hypreve_comm_struct;
  c->rank = rank;
  c->size = size;
  if (size > 1) {
    try {
      ncclUniqueId id;
      std::memcpy(&id, nccl_id_128, sizeof(id));
      ncclComm_t nc;
      nccl_check(ncclCommInitRank(&nc, size, id, rank), "ncclCommInitRank");
      c->nccl = (void*)nc;
    } catch (...) {
      delete c;
      return HYPRE_ERROR_GENERIC;
    }
  }
  *comm = c;
  return 0;
}

}  // extern "C"
