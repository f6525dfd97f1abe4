// Host-side communicator of the distributed setup (one rank per GPU).
//
// The setup exchanges host data: ghost rows, coarse-point flags, request
// lists.  Everything goes through one personalised all-to-all of byte
// buffers plus small all-gathers, the operations hypre's setup performs with
// MPI (hypre_ParCSRCommHandle, MPI_Allgather).  Two implementations:
//   * over the device communicator (RCCL between processes; staging through
//     device buffers) -- runtime.hip, make_host_comm_over_device();
//   * an in-process hub of host threads -- the CPU test suite runs the
//     distributed setup on N threads and checks it against the
//     single-process setup without a GPU.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

namespace hve {

class HostComm {
 public:
  HostComm(int rank, int size) : rank_(rank), size_(size) {}
  virtual ~HostComm() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  // send[p] goes to rank p (send[rank] to itself); recv[p] receives what p
  // sent here.  Collective.
  virtual void alltoallv(const std::vector<std::vector<char>>& send, std::vector<std::vector<char>>& recv) = 0;
  // every rank's value, in rank order.  Collective.
  virtual std::vector<int64_t> allgather(int64_t v) = 0;

  int64_t allreduce_sum(int64_t v) {
    int64_t s = 0;
    for (int64_t x : allgather(v)) s += x;
    return s;
  }
  int64_t allreduce_max(int64_t v) {
    int64_t s = INT64_MIN;
    for (int64_t x : allgather(v)) s = x > s ? x : s;
    return s;
  }
  // typed all-to-all of plain-old-data vectors
  template <typename T>
  void exchange(const std::vector<std::vector<T>>& send, std::vector<std::vector<T>>& recv) {
    std::vector<std::vector<char>> sb(size_), rb;
    for (int p = 0; p < size_; ++p) {
      sb[p].resize(send[p].size() * sizeof(T));
      if (!send[p].empty()) std::memcpy(sb[p].data(), send[p].data(), sb[p].size());
    }
    alltoallv(sb, rb);
    recv.assign(size_, {});
    for (int p = 0; p < size_; ++p) {
      recv[p].resize(rb[p].size() / sizeof(T));
      if (!recv[p].empty()) std::memcpy(recv[p].data(), rb[p].data(), rb[p].size());
    }
  }
  // every rank's vector, concatenated in rank order
  template <typename T, typename Al>
  std::vector<T> allgatherv(const std::vector<T, Al>& mine) {
    std::vector<std::vector<T>> send(size_, std::vector<T>(mine.begin(), mine.end())), recv;
    exchange(send, recv);
    std::vector<T> out;
    for (auto& v : recv) out.insert(out.end(), v.begin(), v.end());
    return out;
  }

 protected:
  int rank_, size_;
};

// `size` communicators over one in-process hub; rank r used from its own thread.
std::vector<std::unique_ptr<HostComm>> make_thread_host_comms(int size);

}  // namespace hve
