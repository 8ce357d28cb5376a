// Native ThreadSanitizer / ASan driver of the collective stall watchdog (runtime/comm_watch.h)
// used by the native RCCL communicator: a caller thread registering collectives whose
// completion flags are set by a fake "device" thread after random delays, then one collective
// that never completes -> the verdict, the abort action (once), check() raising.
//   clang++ -std=c++17 -O1 -g -fsanitize=thread -I csrc csrc/tests/comm_watch_test.cpp -lpthread
#include <sys/wait.h>
#include <unistd.h>

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
  // 3. the abort action itself blocks (a lock held by a thread stuck in the collective, or a hung
  //    ncclCommAbort): the verdict still reaches check(), the loop keeps running beside the action,
  //    and the shutdown deadline still ends the process with 124 (in a forked child)
  {
    std::mutex held;
    held.lock();   // never released while the action waits on it (until the end of the case)
    std::atomic<int> started{0};
    CommWatch w(0.2, 0.0, 1, [&](const std::string&) {
      started++;
      std::lock_guard<std::mutex> lk(held);
    });
    auto never = std::make_shared<std::atomic<bool>>(false);
    w.add("bucket 2 all_reduce", [never] { return never->load(); }, nullptr);
    const double t0 = cw_now_s();
    while (!w.stalled() && cw_now_s() - t0 < 3) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    while (started.load() == 0 && cw_now_s() - t0 < 3) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    assert(w.stalled() && started.load() == 1 && !w.action_done());
    bool threw = false;
    try {
      w.check();
    } catch (const std::runtime_error&) {
      threw = true;
    }
    assert(threw);
    held.unlock();   // let the action finish so stop() can join it
    w.stop();
    assert(w.action_done());
    fflush(stdout);
    const pid_t pid = fork();
    if (pid == 0) {
      std::mutex forever;
      forever.lock();
      CommWatch wc(0.2, 0.3, 2, [&](const std::string&) { std::lock_guard<std::mutex> lk(forever); });
      auto nv = std::make_shared<std::atomic<bool>>(false);
      wc.add("bucket 0 all_reduce", [nv] { return nv->load(); }, nullptr);
      std::this_thread::sleep_for(std::chrono::seconds(20));
      std::_Exit(3);   // not reached when the watchdog enforces its deadline
    }
    int st = 0;
    const double tf = cw_now_s();
    waitpid(pid, &st, 0);
    assert(WIFEXITED(st) && WEXITSTATUS(st) == 124 && cw_now_s() - tf < 5.0);
    std::printf("comm watch: blocked abort action -> loop still exits 124 at the deadline\n");
  }
  // 4. report-only mode: a slow collective is reported once, nothing aborts, check() never
  //    raises, and it retires when it completes late
  {
    Device dev;
    std::atomic<int> aborts{0};
    CommWatch w(0.1, 0.0, 0, [&](const std::string&) { aborts++; }, /*fatal=*/false);
    auto slow = std::make_shared<std::atomic<bool>>(false);
    dev.submit(slow, 0.5);
    w.add("bucket 3 all_reduce", [slow] { return slow->load(); }, nullptr);
    const double t0 = cw_now_s();
    while (w.retired() < 1 && cw_now_s() - t0 < 5) {
      w.check();   // never raises in report-only mode
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    assert(w.retired() == 1 && w.warnings() == 1 && aborts.load() == 0 && !w.stalled());
    std::printf("comm watch: report-only mode -> one warning, no abort, late completion retires\n");
  }
  std::printf("comm_watch_test: ok\n");
  return 0;
}
