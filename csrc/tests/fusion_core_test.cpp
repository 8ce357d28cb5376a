// Native ThreadSanitizer / ASan driver of the fusion engine's scheduling core
// (runtime/fusion_core.h): the caller thread, the core's worker and watchdog threads, and a
// fake "network" thread that completes collectives after random delays.
//   g++ -std=c++17 -O1 -g -fsanitize=thread -I csrc csrc/tests/fusion_core_test.cpp -lpthread
#include <cassert>
#include <cstdio>
#include <cstring>
#include <random>

#include "runtime/fusion_core.h"

using namespace pddl;

struct FakeWork : FusionWork {
  std::atomic<bool> done{false};
  int bucket = -1;
  bool completed() override { return done.load(std::memory_order_acquire); }
};

// Completes works after a random delay (or never, when told to hang bucket `hang`).
struct Network {
  std::mutex mu;
  std::deque<std::pair<double, std::shared_ptr<FakeWork>>> q;
  std::atomic<bool> stop{false};
  std::atomic<int> hang{-1};
  std::thread th;
  Network() {
    th = std::thread([this] {
      while (!stop.load()) {
        std::shared_ptr<FakeWork> w;
        {
          std::lock_guard<std::mutex> lk(mu);
          if (!q.empty() && q.front().first <= fc_now_us()) {
            w = q.front().second;
            q.pop_front();
          }
        }
        if (w) {
          if (w->bucket != hang.load()) w->done.store(true, std::memory_order_release);
        } else {
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
      }
    });
  }
  ~Network() {
    stop.store(true);
    th.join();
  }
  void submit(std::shared_ptr<FakeWork> w, double delay_us) {
    std::lock_guard<std::mutex> lk(mu);
    q.emplace_back(fc_now_us() + delay_us, std::move(w));
  }
};

struct Payload {
  std::vector<int> order;   // (plain data written by the issuer, read by the caller after drain)
};

int main() {
  const int NB = 6, STEPS = 200;
  // 1. many steps, in-order issue, every bucket completes
  {
    Network net;
    std::mt19937 rng(1);
    std::vector<int> issue_order;   // written only by the worker thread, read after drain
    FusionCore<Payload> core(NB, 5.0, 0, [&](FusionCore<Payload>::Item& it) {
      auto w = std::make_shared<FakeWork>();
      w->bucket = it.bucket;
      it.t_issue = fc_now_us();
      it.payload.order.push_back(it.bucket);
      issue_order.push_back(it.bucket);
      net.submit(w, 20 + (it.bucket * 37 % 200));
      it.work = w;
    });
    core.start();
    for (int s = 0; s < STEPS; ++s) {
      core.begin_step();
      for (int b = 0; b < NB; ++b) {
        FusionCore<Payload>::Item it;
        it.bucket = b;
        it.t_ready = fc_now_us();
        core.ready(std::move(it));
        if (rng() % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 100));
      }
      auto done = core.drain();
      assert((int)done.size() == NB);
      for (int b = 0; b < NB; ++b) {
        assert(done[b].bucket == b && done[b].payload.order.size() == 1 && done[b].payload.order[0] == b);
        core.wait_polling(done[b]);
      }
    }
    assert(core.issued() == (int64_t)NB * STEPS);
    for (int i = 0; i < NB * STEPS; ++i) assert(issue_order[i] == i % NB);
    // out-of-order readiness is rejected
    core.begin_step();
    FusionCore<Payload>::Item bad;
    bad.bucket = 1;
    bool threw = false;
    try {
      core.ready(std::move(bad));
    } catch (const std::runtime_error&) {
      threw = true;
    }
    assert(threw);
    core.shutdown();
    std::printf("fusion core: %d steps x %d buckets issued in order, out-of-order rejected\n", STEPS, NB);
  }
  // 2. a collective that never completes: the watchdog flags it, the waits end with an error
  {
    Network net;
    net.hang.store(2);
    FusionCore<Payload> core(NB, 0.3, 7, [&](FusionCore<Payload>::Item& it) {
      auto w = std::make_shared<FakeWork>();
      w->bucket = it.bucket;
      it.t_issue = fc_now_us();
      net.submit(w, 10);
      it.work = w;
    });
    core.start();
    core.begin_step();
    for (int b = 0; b < NB; ++b) {
      FusionCore<Payload>::Item it;
      it.bucket = b;
      it.t_ready = fc_now_us();
      core.ready(std::move(it));
    }
    auto done = core.drain();
    std::string msg;
    const double t0 = fc_now_us();
    try {
      for (auto& it : done) core.wait_polling(it);
    } catch (const std::runtime_error& e) {
      msg = e.what();
    }
    assert(msg.find("stall detected") != std::string::npos && msg.find("bucket 2") != std::string::npos);
    assert((fc_now_us() - t0) * 1e-6 < 3.0);
    bool threw = false;
    try {
      core.begin_step();
    } catch (const std::runtime_error&) {
      threw = true;
    }
    assert(threw);
    core.shutdown();
    std::printf("fusion core: hung collective reported by the stall inspector\n");
  }
  std::printf("fusion_core_test: ok\n");
  return 0;
}
