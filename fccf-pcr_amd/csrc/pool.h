// pool.h — small persistent host thread pool for the independent per-candidate
// host stages (quick_verify + LM).  parallel_for writes results into per-index
// slots, so the outcome does not depend on scheduling.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace fccf {

class Pool {
 public:
  explicit Pool(int n = 0) {
    if (n <= 0) {
      const char* e = std::getenv("FCCF_HOST_THREADS");
      n = e ? std::atoi(e) : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    }
    for (int i = 1; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size() + 1; }
  // Runs f(i) for i in [0, n); the caller participates.
  void parallel_for(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (workers_.empty() || n == 1) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &f;
      n_ = n;
      next_.store(0);
      active_ = (int)workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    run();
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [this] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void run() {
    for (int i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
      }
      run();
      std::lock_guard<std::mutex> g(m_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> next_{0};
  int n_ = 0, active_ = 0;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

}  // namespace fccf
