// Native ThreadSanitizer / ASan driver of the collective stall watchdog (runtime/comm_watch.h)
// used by the native RCCL communicator: a caller thread registering collectives whose
// completion flags are set by a fake "device" thread after random delays, then one collective
// that never completes -> the verdict, the abort action (once), check() raising.
//   clang++ -std=c++17 -O1 -g -fsanitize=thread -I csrc csrc/tests/comm_watch_test.cpp -lpthread
#include <cassert>
#include <cstdio>
#include <memory>
#include <random>
#include <vector>

#include "runtime/comm_watch.h"

using namespace pddl;

struct Device {   // completes "events" after a delay (or never, for the hung one)
  std::mutex mu;
  std::deque<std::pair<double, std::shared_ptr<std::atomic<bool>>>> q;
  std::atomic<bool> stop{false};
  std::thread th;
  Device() {
    th = std::thread([this] {
      while (!stop.load()) {
        std::shared_ptr<std::atomic<bool>> f;
        {
          std::lock_guard<std::mutex> lk(mu);
          if (!q.empty() && q.front().first <= cw_now_s()) {
            f = q.front().second;
            q.pop_front();
          }
        }
        if (f) f->store(true, std::memory_order_release);
        else std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    });
  }
  ~Device() {
    stop.store(true);
    th.join();
  }
  void submit(std::shared_ptr<std::atomic<bool>> f, double delay_s) {
    std::lock_guard<std::mutex> lk(mu);
    q.emplace_back(cw_now_s() + delay_s, std::move(f));
  }
};

int main() {
  // 1. many collectives, all complete: every one retired, no verdict, releases run once each
  {
    Device dev;
    std::atomic<int> aborts{0}, released{0};
    CommWatch w(2.0, 0.0, 0, [&](const std::string&) { aborts++; });
    std::mt19937 rng(3);
    const int N = 2000;
    for (int i = 0; i < N; ++i) {
      auto f = std::make_shared<std::atomic<bool>>(false);
      dev.submit(f, 1e-4 * (rng() % 20));
      w.add("bucket " + std::to_string(i % 5) + " all_reduce", [f] { return f->load(std::memory_order_acquire); },
            [&released] { released++; });
      w.check();
    }
    const double t0 = cw_now_s();
    while (w.retired() < N && cw_now_s() - t0 < 10) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    assert(w.retired() == N && w.outstanding() == 0 && !w.stalled() && aborts.load() == 0);
    assert(released.load() == N && w.issued() == N);
    std::printf("comm watch: %d collectives retired in order, no false stall\n", N);
  }
  // 2. one collective never completes: verdict names it, abort runs exactly once, check() raises
  {
    Device dev;
    std::atomic<int> aborts{0}, released{0};
    std::string seen;
    std::mutex seen_mu;
    CommWatch w(0.3, 0.0, 5, [&](const std::string& m) {
      std::lock_guard<std::mutex> lk(seen_mu);
      seen = m;
      aborts++;
    });
    auto ok = std::make_shared<std::atomic<bool>>(false);
    dev.submit(ok, 0.01);
    w.add("bucket 0 all_reduce", [ok] { return ok->load(); }, [&released] { released++; });
    auto never = std::make_shared<std::atomic<bool>>(false);
    w.add("bucket 1 all_reduce", [never] { return never->load(); }, [&released] { released++; });
    const double t0 = cw_now_s();
    bool threw = false;
    while (!threw && cw_now_s() - t0 < 5) {
      try {
        w.check();
      } catch (const std::runtime_error& e) {
        threw = std::string(e.what()).find("bucket 1 all_reduce") != std::string::npos;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    assert(threw && cw_now_s() - t0 < 3.0);
    std::this_thread::sleep_for(std::chrono::milliseconds(200));   // no second verdict / abort
    assert(aborts.load() == 1 && w.stalled());
    {
      std::lock_guard<std::mutex> lk(seen_mu);
      assert(seen.find("rank 5") != std::string::npos);
    }
    w.stop();
    assert(released.load() == 2);   // the retired one and the one left at stop()
    std::printf("comm watch: hung collective -> one verdict + one abort, check() raises\n");
  }
  std::printf("comm_watch_test: ok\n");
  return 0;
}
