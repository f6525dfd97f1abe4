// DevComm back ends: RCCL (production, one process per GPU) and the in-process
// loopback hub (virtual ranks on one GPU, for the parity tests).
#include "comm.hpp"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
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
  bool capturable() const override { return true; }
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

// ---------------------------------------------------------------------------
// Host-staged transport over POSIX shared memory: `size` processes on one host
// (one GPU each, or several sharing one GPU, where RCCL refuses).  Every
// ordered pair (src, dst) owns a one-slot mailbox of kShmChunk bytes; a message
// moves chunk by chunk (post: write data, publish the length, bump `posted`;
// take: copy out, bump `taken`).  An exchange first drains the stream, stages
// the send buffers to the host, then runs one progress loop over all of its
// sends and receives (so two ranks streaming large messages at each other
// cannot deadlock), and finally copies the received bytes to the device.
// Messages between a pair keep their order.  The all-reduce gathers every
// rank's vector and sums it in rank order on the host: the loopback hub's
// arithmetic (buf = v_0, buf += v_q, q = 1..n-1), so the two transports give
// the same bits.
// ---------------------------------------------------------------------------
namespace {
constexpr size_t kShmChunk = (size_t)1 << 20;
constexpr uint64_t kShmMagic = 0x68766573686d3031ULL;  // "hveshm01"
struct alignas(64) ShmSlot {
  std::atomic<uint64_t> posted;
  std::atomic<uint64_t> taken;
  std::atomic<uint64_t> len;
};
struct ShmHeader {
  std::atomic<uint64_t> magic;
  std::atomic<int> size;
  std::atomic<int> attached;
  std::atomic<int> detached;
};
size_t shm_bytes(int n) {
  return 4096 + (size_t)n * n * (sizeof(ShmSlot) + kShmChunk);
}
}  // namespace

class ShmComm final : public DevComm {
 public:
  ShmComm(int rank, int size, const std::string& name) : DevComm(rank, size), name_(name) {
    const size_t bytes = shm_bytes(size);
    int fd = -1;
    if (rank == 0) {
      ::shm_unlink(name.c_str());
      fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm comm: shm_open(create) failed for " + name);
      if (::ftruncate(fd, (off_t)bytes) != 0) {
        ::close(fd);
        throw std::runtime_error("shm comm: ftruncate failed");
      }
    } else {
      for (int tries = 0; tries < 60000 && fd < 0; ++tries) {  // up to ~60 s for rank 0
        fd = ::shm_open(name.c_str(), O_RDWR, 0600);
        if (fd < 0) ::usleep(1000);
      }
      if (fd < 0) throw std::runtime_error("shm comm: rank " + std::to_string(rank) + " cannot open " + name);
      struct stat st;
      for (int tries = 0; tries < 60000; ++tries) {
        if (::fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
        ::usleep(1000);
      }
    }
    void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("shm comm: mmap failed");
    base_ = (char*)p;
    bytes_ = bytes;
    hdr_ = reinterpret_cast<ShmHeader*>(base_);
    if (rank == 0) {
      for (int i = 0; i < size * size; ++i) {
        ShmSlot* sl = slot_at(i);
        new (sl) ShmSlot;
        sl->posted.store(0);
        sl->taken.store(0);
        sl->len.store(0);
      }
      hdr_->size.store(size);
      hdr_->attached.store(0);
      hdr_->detached.store(0);
      hdr_->magic.store(kShmMagic, std::memory_order_release);
    } else {
      for (int tries = 0; tries < 60000 && hdr_->magic.load(std::memory_order_acquire) != kShmMagic; ++tries)
        ::usleep(1000);
      if (hdr_->magic.load(std::memory_order_acquire) != kShmMagic || hdr_->size.load() != size) {
        unmap();
        throw std::runtime_error("shm comm: segment not initialised by rank 0");
      }
    }
    hdr_->attached.fetch_add(1);
    // every rank is mapped; a peer that died during startup ends the wait
    const auto t0 = std::chrono::steady_clock::now();
    while (hdr_->attached.load() < size) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(kShmAttachSeconds)) {
        const int seen = hdr_->attached.load();
        unmap();
        if (rank == 0) ::shm_unlink(name_.c_str());
        throw std::runtime_error("shm comm: only " + std::to_string(seen) + " of " + std::to_string(size) +
                                 " ranks attached within " + std::to_string(kShmAttachSeconds) + " s");
      }
      ::usleep(100);
    }
  }
  ~ShmComm() override {
    if (!base_) return;
    hdr_->detached.fetch_add(1);
    if (rank_ == 0) {
      for (int tries = 0; tries < 10000 && hdr_->detached.load() < size_; ++tries) ::usleep(1000);
      ::shm_unlink(name_.c_str());
    }
    unmap();
  }
  const char* kind() const override { return "shm"; }

  void exchange(const std::vector<P2PMsg>& sends, const std::vector<P2PMsg>& recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return;
    HVE_HIP(hipStreamSynchronize(s));
    std::vector<std::vector<char>> sh(sends.size()), rh(recvs.size());
    for (size_t k = 0; k < sends.size(); ++k) {
      if (sends[k].peer < 0 || sends[k].peer >= size_) throw std::runtime_error("shm comm: bad send peer");
      sh[k].resize(sends[k].bytes);
      if (sends[k].bytes) HVE_HIP(hipMemcpy(sh[k].data(), sends[k].buf, sends[k].bytes, hipMemcpyDeviceToHost));
    }
    for (size_t k = 0; k < recvs.size(); ++k) {
      if (recvs[k].peer < 0 || recvs[k].peer >= size_) throw std::runtime_error("shm comm: bad recv peer");
      rh[k].resize(recvs[k].bytes);
    }
    host_exchange(sends, sh, recvs, rh);
    for (size_t k = 0; k < recvs.size(); ++k)
      if (recvs[k].bytes) HVE_HIP(hipMemcpy(recvs[k].buf, rh[k].data(), recvs[k].bytes, hipMemcpyHostToDevice));
  }

  void allreduce_sum(double* buf, size_t n, hipStream_t s) override {
    HVE_HIP(hipStreamSynchronize(s));
    std::vector<char> mine(n * sizeof(double));
    if (n) HVE_HIP(hipMemcpy(mine.data(), buf, n * sizeof(double), hipMemcpyDeviceToHost));
    std::vector<P2PMsg> sends, recvs;
    std::vector<std::vector<char>> sh, rh;
    for (int p = 0; p < size_; ++p) {
      if (p == rank_) continue;
      sends.push_back({p, nullptr, n * sizeof(double)});
      sh.push_back(mine);
      recvs.push_back({p, nullptr, n * sizeof(double)});
      rh.emplace_back(n * sizeof(double));
    }
    host_exchange(sends, sh, recvs, rh);
    std::vector<const double*> v(size_);
    for (int p = 0, k = 0; p < size_; ++p) v[p] = p == rank_ ? (const double*)mine.data() : (const double*)rh[k++].data();
    std::vector<double> out(n);
    for (size_t i = 0; i < n; ++i) {
      double t = v[0][i];
      for (int q = 1; q < size_; ++q) t = t + 1.0 * v[q][i];  // k_axpy: y += 1.0 * x
      out[i] = t;
    }
    if (n) HVE_HIP(hipMemcpy(buf, out.data(), n * sizeof(double), hipMemcpyHostToDevice));
  }

 private:
  // startup and per-exchange deadlines: a peer that is gone ends the wait with an error
  static constexpr int kShmAttachSeconds = 60;
  static constexpr int kShmIdleSeconds = 300;
  void unmap() {
    if (base_) ::munmap(base_, bytes_);
    base_ = nullptr;
    hdr_ = nullptr;
  }
  ShmSlot* slot_at(int i) const { return reinterpret_cast<ShmSlot*>(base_ + 4096 + (size_t)i * sizeof(ShmSlot)); }
  ShmSlot* slot(int src, int dst) const { return slot_at(src * size_ + dst); }
  char* data(int src, int dst) const {
    return base_ + 4096 + (size_t)size_ * size_ * sizeof(ShmSlot) + (size_t)(src * size_ + dst) * kShmChunk;
  }

  // Progress loop over host-staged messages (per pair in order, chunked).
  void host_exchange(const std::vector<P2PMsg>& sends, std::vector<std::vector<char>>& sh,
                     const std::vector<P2PMsg>& recvs, std::vector<std::vector<char>>& rh) {
    std::vector<size_t> soff(sends.size(), 0), roff(recvs.size(), 0);
    std::vector<int> sdone(sends.size(), 0), rdone(recvs.size(), 0);
    // messages to / from each peer in order: the head is the first unfinished one
    auto head = [](const std::vector<P2PMsg>& v, const std::vector<int>& done, int peer) -> int {
      for (size_t k = 0; k < v.size(); ++k)
        if (v[k].peer == peer && !done[k]) return (int)k;
      return -1;
    };
    for (size_t k = 0; k < sends.size(); ++k) sdone[k] = sends[k].bytes == 0;
    for (size_t k = 0; k < recvs.size(); ++k) rdone[k] = recvs[k].bytes == 0;
    size_t left = 0;
    for (int d : sdone) left += !d;
    for (int d : rdone) left += !d;
    long idle = 0;
    auto last = std::chrono::steady_clock::now();
    while (left) {
      bool progress = false;
      for (int p = 0; p < size_; ++p) {
        const int ks = head(sends, sdone, p);
        if (ks >= 0) {
          ShmSlot* sl = slot(rank_, p);
          if (sl->posted.load(std::memory_order_acquire) == sl->taken.load(std::memory_order_acquire)) {
            const size_t c = std::min(kShmChunk, sends[ks].bytes - soff[ks]);
            std::memcpy(data(rank_, p), sh[ks].data() + soff[ks], c);
            sl->len.store(c, std::memory_order_relaxed);
            sl->posted.fetch_add(1, std::memory_order_release);
            soff[ks] += c;
            if (soff[ks] == sends[ks].bytes) { sdone[ks] = 1; --left; }
            progress = true;
          }
        }
        const int kr = head(recvs, rdone, p);
        if (kr >= 0) {
          ShmSlot* sl = slot(p, rank_);
          if (sl->posted.load(std::memory_order_acquire) > sl->taken.load(std::memory_order_acquire)) {
            const size_t c = sl->len.load(std::memory_order_relaxed);
            if (roff[kr] + c > recvs[kr].bytes) throw std::runtime_error("shm comm: message size mismatch");
            std::memcpy(rh[kr].data() + roff[kr], data(p, rank_), c);
            sl->taken.fetch_add(1, std::memory_order_release);
            roff[kr] += c;
            if (roff[kr] == recvs[kr].bytes) { rdone[kr] = 1; --left; }
            progress = true;
          }
        }
      }
      if (progress) {
        idle = 0;
      } else if (++idle > 64) {
        ::usleep(idle > 100000 ? 1000 : 20);
        if ((idle & 1023) == 0) {
          if (std::chrono::steady_clock::now() - last > std::chrono::seconds(kShmIdleSeconds))
            throw std::runtime_error("shm comm: exchange made no progress for " + std::to_string(kShmIdleSeconds) +
                                     " s (peer gone?)");
        }
      }
      if (progress) last = std::chrono::steady_clock::now();
    }
  }

  std::string name_;
  char* base_ = nullptr;
  size_t bytes_ = 0;
  ShmHeader* hdr_ = nullptr;
};

std::unique_ptr<DevComm> make_shm_comm(int rank, int size, const char* name) {
  return std::unique_ptr<DevComm>(new ShmComm(rank, size, name));
}

}  // namespace hve
