// Persistent host-thread pool of the graphed multi-replica step's group launches
// (runtime/graph_launch.cpp): run(n, f) calls f(0) .. f(n - 1) on n worker threads and returns
// once every call returned.  Header-only and HIP-free, so csrc/tests/launch_pool_test.cpp drives
// it natively under ThreadSanitizer (scripts/sanitize_host.sh).
#pragma once
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace pddl {

// Persistent worker threads (joined by the destructor; the process-wide pool is never destroyed).
// Worker i runs task i of each generation; a worker spins ~200 us for the next generation
// before it sleeps, so the back-to-back phases of one step see no futex wake-up latency.
class LaunchPool {
 public:
  LaunchPool() = default;
  LaunchPool(const LaunchPool&) = delete;
  LaunchPool& operator=(const LaunchPool&) = delete;
  ~LaunchPool() {   // (graph_launch.cpp's pool is never destroyed; tests' pools are)
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true, std::memory_order_release);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }

  void run(size_t n, const std::function<void(size_t)>& f) {
    std::lock_guard<std::mutex> one(run_mu_);   // (one group launch at a time)
    while (workers_ < n) {   // (a new worker waits for the NEXT generation, never a finished one's fn_)
      const size_t i = workers_++;
      const uint64_t g0 = gen_.load(std::memory_order_acquire);
      threads_.emplace_back([this, i, g0] { loop(i, g0); });
    }
    fn_ = &f;
    n_ = n;
    pending_.store((int)workers_, std::memory_order_relaxed);   // every worker checks in
    {
      std::lock_guard<std::mutex> lk(mu_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    if (!spin([&] { return pending_.load(std::memory_order_acquire) == 0; })) {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [&] { return pending_.load(std::memory_order_acquire) == 0; });
    }
  }

 private:
  template <class P>
  static bool spin(P&& ready) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!ready()) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) return false;
      _mm_pause();
    }
    return true;
  }

  void loop(size_t i, uint64_t seen) {
    for (;;) {
      if (!spin([&] { return gen_.load(std::memory_order_acquire) != seen; })) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
      }
      seen = gen_.load(std::memory_order_acquire);
      if (stop_.load(std::memory_order_acquire)) return;
      if (i < n_) (*fn_)(i);
      if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_one();
      }
    }
  }

  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> stop_{false};
  std::vector<std::thread> threads_;
  size_t workers_ = 0;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
};

}  // namespace pddl
