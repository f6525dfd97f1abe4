// Device communicator of the multi-GPU solve path (one rank per GPU).
//
// The solve needs exactly two data-path operations: a grouped point-to-point
// exchange (the ParCSR halo, par_csr_communication.c
// hypre_ParCSRCommHandleCreate) and an in-place sum over ranks (inner products,
// the gathered coarse right-hand side).  Two back ends implement them:
//   * RCCL over xGMI (ncclGroupStart / ncclSend / ncclRecv / ncclAllReduce),
//     one process per GPU -- the production path;
//   * an in-process loopback hub: `size` virtual ranks, one host thread each,
//     sharing one GPU, exchanging through device-to-device copies ordered by
//     HIP events.  RCCL refuses two ranks on one device, so this is how the
//     partitioned data path is checked against the 1-rank iterates on a
//     single-GPU box.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <vector>

namespace hve {

struct P2PMsg {
  int peer;
  void* buf;
  size_t bytes;
};

class DevComm {
 public:
  DevComm(int rank, int size) : rank_(rank), size_(size) {}
  virtual ~DevComm() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual const char* kind() const = 0;
  // Whether exchange / allreduce_sum may be recorded into a hipGraph (stream
  // capture): RCCL's grouped send/recv and all-reduce can; the loopback hub and
  // the shared-memory transport block on the host and cannot.
  virtual bool capturable() const { return false; }
  // Grouped exchange on stream s with ncclGroupStart/Send/Recv/GroupEnd
  // semantics: the k-th message this rank sends to p matches p's k-th receive
  // from this rank.  All transfers, sends included, complete in stream order,
  // so the send buffers may be rewritten by work enqueued after the call.
  virtual void exchange(const std::vector<P2PMsg>& sends, const std::vector<P2PMsg>& recvs, hipStream_t s) = 0;
  // In-place element-wise sum over all ranks of n device doubles (collective).
  virtual void allreduce_sum(double* buf, size_t n, hipStream_t s) = 0;

  // Collectives built on exchange (device buffers, collective over all ranks).
  void allgather(const void* mine, void* all, size_t bytes_each, hipStream_t s);
  void bcast(void* buf, size_t bytes, int root, hipStream_t s);

 protected:
  int rank_, size_;
};

// 128-byte ncclUniqueId generated on the rank that creates the clique.
void rccl_unique_id(void* id128);
std::unique_ptr<DevComm> make_rccl_comm(int rank, int size, const void* id128);
// `size` communicators sharing one in-process hub; rank r must only be used
// from one host thread at a time, and every rank from its own thread.
std::vector<std::unique_ptr<DevComm>> make_loopback_comms(int size);
// Host-staged transport over the POSIX shared-memory segment `name` (rank 0
// creates it): `size` processes on one host, e.g. several ranks on one GPU,
// where RCCL refuses.  Exchanges and all-reduces synchronise the stream.
std::unique_ptr<DevComm> make_shm_comm(int rank, int size, const char* name);

}  // namespace hve

// Object behind the C ABI's HYPRE_Comm handle.
struct hypreve_comm_struct {
  int rank = 0, size = 1;
  std::unique_ptr<hve::DevComm> dc;  // null for a single rank
};
