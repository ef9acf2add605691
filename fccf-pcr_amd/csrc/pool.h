// pool.h — small persistent host thread pool for the independent per-candidate
// host stages (quick_verify + LM, clustering neighbour lists).  parallel_for
// writes results into per-index slots, so the outcome does not depend on
// scheduling.
//
// Latency matters more than throughput here: a registration makes a few
// parallel_for calls of ~10-100 items, each item 1-50 us.  So
//  * idle workers spin on the job word for a while before sleeping on a condition
//    variable (a futex wake-up costs tens of microseconds per thread);
//  * items are claimed with a CAS on one 64-bit word holding (job id, next index),
//    so a worker that wakes late can never claim an item of a finished job;
//  * the caller returns as soon as every item is done, without waiting for
//    workers that never woke up.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
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
    const char* s = std::getenv("FCCF_POOL_SPIN_US");
    spin_us_ = s ? std::atoi(s) : 500;
    for (int i = 1; i < n; ++i) workers_.emplace_back([this, i] { loop(i - 1); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      quit_.store(true);
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size() + 1; }
  // Wakes sleeping workers and keeps the first `nw` workers (all by default) spinning
  // for `us` microseconds, so a parallel_for issued within that window starts on those
  // threads at once (call it before a wait whose end is followed by parallel work).
  // Spinning threads take CPU time from the caller's other threads: keep nw to what the
  // next parallel_for needs.
  void warm(int us, int nw = 1 << 30) {
    if (workers_.empty()) return;
    warm_n_.store(nw, std::memory_order_relaxed);
    warm_until_.store(now_us() + us, std::memory_order_relaxed);
    warm_gen_.fetch_add(1, std::memory_order_release);
    {
      std::lock_guard<std::mutex> g(m_);
    }
    cv_.notify_all();
  }
  // Runs f(i) for i in [0, n); the caller participates.  Not reentrant.
  void parallel_for(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (workers_.empty() || n == 1) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    const uint64_t job = (job_ + 1) & 0xffffffffu;
    job_ = job;
    fn_ = &f;
    n_.store(n, std::memory_order_relaxed);
    done_.store(0, std::memory_order_relaxed);
    word_.store(job << 32, std::memory_order_release);  // publishes fn_, n_, done_
    {
      std::lock_guard<std::mutex> g(m_);  // pairs with the sleepers' predicate check
    }
    cv_.notify_all();
    run(job);
    while (done_.load(std::memory_order_acquire) != n) relax();
  }

 private:
  static int64_t now_us() {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  static void relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  // Claims and runs items of job `job` until none is left.
  void run(uint64_t job) {
    uint64_t w = word_.load(std::memory_order_acquire);
    while ((w >> 32) == job) {
      const int i = (int)(w & 0xffffffffu);
      if (i >= n_.load(std::memory_order_relaxed)) return;
      if (!word_.compare_exchange_weak(w, w + 1, std::memory_order_acq_rel, std::memory_order_acquire)) continue;
      (*fn_)(i);
      done_.fetch_add(1, std::memory_order_acq_rel);
      w = word_.load(std::memory_order_acquire);
    }
  }
  void loop(int id) {
    uint64_t seen = 0;
    while (true) {
      int64_t until = now_us() + spin_us_;
      uint64_t w;
      int k = 0;
      while (((w = word_.load(std::memory_order_acquire)) >> 32) == seen && !quit_.load()) {
        relax();
        if ((++k & 255) == 0 &&
            now_us() > std::max(until, id < warm_n_.load(std::memory_order_relaxed)
                                           ? warm_until_.load(std::memory_order_relaxed)
                                           : int64_t(0))) {
          std::unique_lock<std::mutex> g(m_);
          const uint64_t wg = warm_gen_.load();
          cv_.wait(g, [&] {  // (a warm() wakes only the workers it keeps spinning)
            return quit_.load() || (word_.load() >> 32) != seen ||
                   (warm_gen_.load() != wg && id < warm_n_.load(std::memory_order_relaxed));
          });
          until = now_us() + spin_us_;
        }
      }
      if (quit_.load()) return;
      seen = w >> 32;
      run(seen);
    }
  }
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<uint64_t> word_{0};  // (job id << 32) | next item
  std::atomic<int> done_{0};
  std::atomic<bool> quit_{false};
  std::atomic<int64_t> warm_until_{0};
  std::atomic<uint64_t> warm_gen_{0};
  std::atomic<int> warm_n_{1 << 30};
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> n_{0};
  uint64_t job_ = 0;
  int spin_us_ = 500;
};

// One background thread running one task at a time (the batch driver enqueues the
// next pair's cloud stage there while the caller runs this pair's host stages).
// wait() joins the current task and rethrows its exception, if any.
class AsyncTask {
 public:
  AsyncTask() : th_([this] { loop(); }) {}
  ~AsyncTask() {
    {
      std::lock_guard<std::mutex> g(m_);
      quit_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void submit(std::function<void()> f) {
    wait();
    {
      std::lock_guard<std::mutex> g(m_);
      task_ = std::move(f);
      busy_ = true;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [this] { return !busy_; });
    if (err_) {
      std::exception_ptr e = err_;
      err_ = nullptr;
      std::rethrow_exception(e);
    }
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    while (true) {
      cv_.wait(g, [this] { return quit_ || busy_; });
      if (quit_) return;
      std::function<void()> f = std::move(task_);
      g.unlock();
      std::exception_ptr e;
      try {
        f();
      } catch (...) {
        e = std::current_exception();
      }
      g.lock();
      err_ = e;
      busy_ = false;
      done_cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::function<void()> task_;
  std::exception_ptr err_;
  bool busy_ = false, quit_ = false;
  std::thread th_;
};

}  // namespace fccf
