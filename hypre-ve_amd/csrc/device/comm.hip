// DevComm back ends: RCCL (production, one process per GPU) and the in-process
// loopback hub (virtual ranks on one GPU, for the parity tests).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>

#include "kernels.h"
#include "runtime.hpp"

namespace hve {

void DevComm::allgather(const void* mine, void* all, size_t bytes_each, hipStream_t s) {
  std::vector<P2PMsg> sends, recvs;
  for (int p = 0; p < size_; ++p) {
    if (p == rank_) continue;
    sends.push_back({p, const_cast<void*>(mine), bytes_each});
    recvs.push_back({p, (char*)all + (size_t)p * bytes_each, bytes_each});
  }
  HVE_HIP(hipMemcpyAsync((char*)all + (size_t)rank_ * bytes_each, mine, bytes_each, hipMemcpyDeviceToDevice, s));
  exchange(sends, recvs, s);
}

void DevComm::bcast(void* buf, size_t bytes, int root, hipStream_t s) {
  std::vector<P2PMsg> sends, recvs;
  if (rank_ == root) {
    for (int p = 0; p < size_; ++p)
      if (p != root) sends.push_back({p, buf, bytes});
  } else {
    recvs.push_back({root, buf, bytes});
  }
  exchange(sends, recvs, s);
}

// ---------------------------------------------------------------------------
// RCCL
// ---------------------------------------------------------------------------
static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error '") + ncclGetErrorString(r) + "' in " + what);
}

void rccl_unique_id(void* id128) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(id128, &id, sizeof(id));
}

class RcclComm final : public DevComm {
 public:
  RcclComm(int rank, int size, const void* id128) : DevComm(rank, size) {
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    nccl_check(ncclCommInitRank(&comm_, size, id, rank), "ncclCommInitRank");
  }
  ~RcclComm() override {
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  const char* kind() const override { return "rccl"; }
  void exchange(const std::vector<P2PMsg>& sends, const std::vector<P2PMsg>& recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return;
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (const auto& m : sends)
      if (m.bytes) nccl_check(ncclSend(m.buf, m.bytes, ncclUint8, m.peer, comm_, s), "ncclSend");
    for (const auto& m : recvs)
      if (m.bytes) nccl_check(ncclRecv(m.buf, m.bytes, ncclUint8, m.peer, comm_, s), "ncclRecv");
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }
  void allreduce_sum(double* buf, size_t n, hipStream_t s) override {
    nccl_check(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm_, s), "ncclAllReduce");
  }

 private:
  ncclComm_t comm_ = nullptr;
};

std::unique_ptr<DevComm> make_rccl_comm(int rank, int size, const void* id128) {
  return std::unique_ptr<DevComm>(new RcclComm(rank, size, id128));
}

// ---------------------------------------------------------------------------
// Loopback hub.  Point-to-point: per (src, dst) FIFO mailboxes.  A send posts
// {buffer, bytes, ready event}; the receiver waits for the post, orders its
// stream after the ready event, copies, and answers with a done event that the
// sender's stream then waits on (a send completes when it has been received,
// as with RCCL).  Host threads block only on posts, never on GPU work.
// All-reduce: a true collective with a barrier; sums in rank order.
// ---------------------------------------------------------------------------
struct LoopHub {
  explicit LoopHub(int n) : size(n), mail((size_t)n * n), ack((size_t)n * n), slot(n, nullptr), slot_n(n, 0),
                            ready(n, nullptr), done(n, nullptr) {}
  ~LoopHub() {
    for (double* p : slot)
      if (p) (void)hipFree(p);
  }
  struct Post {
    void* buf;
    size_t bytes;
    hipEvent_t ev;
  };
  int size;
  std::mutex m;
  std::condition_variable cv;
  std::vector<std::deque<Post>> mail;        // [src * size + dst]
  std::vector<std::deque<hipEvent_t>> ack;   // [src * size + dst]: done events for src's sends
  // all-reduce state
  int arrived = 0;
  unsigned long gen = 0;
  std::vector<double*> slot;
  std::vector<size_t> slot_n;
  std::vector<hipEvent_t> ready, done;

  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const unsigned long g = gen;
    if (++arrived == size) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

static hipEvent_t new_event() {
  hipEvent_t e;
  HVE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}

class LoopComm final : public DevComm {
 public:
  LoopComm(int rank, std::shared_ptr<LoopHub> hub) : DevComm(rank, hub->size), hub_(std::move(hub)) {}
  const char* kind() const override { return "loopback"; }

  void exchange(const std::vector<P2PMsg>& sends, const std::vector<P2PMsg>& recvs, hipStream_t s) override {
    LoopHub& H = *hub_;
    const int n = size_;
    // 1. post the sends (one ready event covers all of them)
    if (!sends.empty()) {
      hipEvent_t ev = new_event();
      HVE_HIP(hipEventRecord(ev, s));
      std::lock_guard<std::mutex> lk(H.m);
      for (const auto& m : sends) {
        if (m.peer < 0 || m.peer >= n) throw std::runtime_error("loopback: bad send peer");
        hipEvent_t e = ev;
        if (&m != &sends.front()) e = dup_event(s);
        H.mail[(size_t)rank_ * n + m.peer].push_back({m.buf, m.bytes, e});
      }
      H.cv.notify_all();
    }
    // 2. receive: wait for the matching post, copy after its ready event
    for (const auto& m : recvs) {
      if (m.peer < 0 || m.peer >= n) throw std::runtime_error("loopback: bad recv peer");
      LoopHub::Post p;
      {
        std::unique_lock<std::mutex> lk(H.m);
        auto& q = H.mail[(size_t)m.peer * n + rank_];
        H.cv.wait(lk, [&] { return !q.empty(); });
        p = q.front();
        q.pop_front();
      }
      if (p.bytes != m.bytes) throw std::runtime_error("loopback: message size mismatch");
      HVE_HIP(hipStreamWaitEvent(s, p.ev, 0));
      HVE_HIP(hipEventDestroy(p.ev));  // released once complete
      if (m.bytes) HVE_HIP(hipMemcpyAsync(m.buf, p.buf, m.bytes, hipMemcpyDeviceToDevice, s));
      hipEvent_t d = new_event();
      HVE_HIP(hipEventRecord(d, s));
      {
        std::lock_guard<std::mutex> lk(H.m);
        H.ack[(size_t)m.peer * n + rank_].push_back(d);
      }
      H.cv.notify_all();
    }
    // 3. sends complete when received
    for (const auto& m : sends) {
      hipEvent_t d;
      {
        std::unique_lock<std::mutex> lk(H.m);
        auto& q = H.ack[(size_t)rank_ * n + m.peer];
        H.cv.wait(lk, [&] { return !q.empty(); });
        d = q.front();
        q.pop_front();
      }
      HVE_HIP(hipStreamWaitEvent(s, d, 0));
      HVE_HIP(hipEventDestroy(d));
    }
  }

  void allreduce_sum(double* buf, size_t n, hipStream_t s) override {
    LoopHub& H = *hub_;
    if (H.slot_n[rank_] < n) {
      if (H.slot[rank_]) HVE_HIP(hipFree(H.slot[rank_]));
      HVE_HIP(hipMalloc((void**)&H.slot[rank_], n * sizeof(double)));
      H.slot_n[rank_] = n;
    }
    HVE_HIP(hipMemcpyAsync(H.slot[rank_], buf, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    hipEvent_t r = new_event();
    HVE_HIP(hipEventRecord(r, s));
    H.ready[rank_] = r;
    H.barrier();
    for (int q = 0; q < size_; ++q) HVE_HIP(hipStreamWaitEvent(s, H.ready[q], 0));
    HVE_HIP(hipMemcpyAsync(buf, H.slot[0], n * sizeof(double), hipMemcpyDeviceToDevice, s));
    for (int q = 1; q < size_; ++q) HVE_HIP(launch_axpy((int)n, nullptr, 1.0, 1.0, H.slot[q], buf, s));
    hipEvent_t d = new_event();
    HVE_HIP(hipEventRecord(d, s));
    H.done[rank_] = d;
    H.barrier();
    for (int q = 0; q < size_; ++q) HVE_HIP(hipStreamWaitEvent(s, H.done[q], 0));
    H.barrier();
    HVE_HIP(hipEventDestroy(r));
    HVE_HIP(hipEventDestroy(d));
  }

 private:
  static hipEvent_t dup_event(hipStream_t s) {
    hipEvent_t e = new_event();
    HVE_HIP(hipEventRecord(e, s));
    return e;
  }
  std::shared_ptr<LoopHub> hub_;
};

std::vector<std::unique_ptr<DevComm>> make_loopback_comms(int size) {
  auto hub = std::make_shared<LoopHub>(size);
  std::vector<std::unique_ptr<DevComm>> v;
  for (int r = 0; r < size; ++r) v.emplace_back(new LoopComm(r, hub));
  return v;
}

}  // namespace hve
