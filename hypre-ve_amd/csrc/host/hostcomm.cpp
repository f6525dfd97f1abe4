// In-process host-thread hub behind HostComm (see hostcomm.hpp).
#include "hostcomm.hpp"

#include <condition_variable>
#include <mutex>

namespace hve {

namespace {

struct Hub {
  explicit Hub(int n) : size(n), box((size_t)n * n), vals(n) {}
  int size;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long gen = 0;
  std::vector<std::vector<char>> box;  // [src * size + dst]
  std::vector<int64_t> vals;

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

class ThreadHostComm final : public HostComm {
 public:
  ThreadHostComm(int rank, std::shared_ptr<Hub> hub) : HostComm(rank, hub->size), hub_(std::move(hub)) {}

  void alltoallv(const std::vector<std::vector<char>>& send, std::vector<std::vector<char>>& recv) override {
    Hub& H = *hub_;
    for (int p = 0; p < size_; ++p) H.box[(size_t)rank_ * size_ + p] = send[p];
    H.barrier();  // every rank has posted
    recv.assign(size_, {});
    for (int p = 0; p < size_; ++p) recv[p] = H.box[(size_t)p * size_ + rank_];
    H.barrier();  // every rank has read before the boxes are reused
  }

  std::vector<int64_t> allgather(int64_t v) override {
    Hub& H = *hub_;
    H.vals[rank_] = v;
    H.barrier();
    std::vector<int64_t> out = H.vals;
    H.barrier();
    return out;
  }

 private:
  std::shared_ptr<Hub> hub_;
};

}  // namespace

std::vector<std::unique_ptr<HostComm>> make_thread_host_comms(int size) {
  auto hub = std::make_shared<Hub>(size);
  std::vector<std::unique_ptr<HostComm>> v;
  for (int r = 0; r < size; ++r) v.emplace_back(new ThreadHostComm(r, hub));
  return v;
}

}  // namespace hve
