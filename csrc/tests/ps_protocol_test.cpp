// Native ThreadSanitizer / ASan driver of the parameter-server control protocol
// (runtime/ps_protocol.h): the service loop and W worker threads exchange through one control
// segment, with plain mailbox / receive-buffer traffic ordered only by the protocol's
// release / acquire sequence numbers (as across processes in ps_service.cpp).
//   g++ -std=c++17 -O1 -g -fsanitize=thread -I csrc csrc/tests/ps_protocol_test.cpp -lpthread
#include <cassert>
#include <cstdio>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "runtime/ps_protocol.h"

using namespace pddl::ps;

int main() {
  const int W = 4, N = 1024, ITERS = 400;
  std::unique_ptr<unsigned char[]> mem(new unsigned char[sizeof(PSCtrl) + 128]);
  void* aligned = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(mem.get()) + 127) & ~uintptr_t(127));
  PSCtrl* ctrl = new (aligned) PSCtrl();
  ctrl->magic = kMagic;
  ctrl->n = N;
  ctrl->workers = W;
  std::vector<float> params(N, 0.f);
  std::vector<std::vector<float>> mailbox(W, std::vector<float>(N)), rx(W, std::vector<float>(N));
  std::atomic<bool> stop{false};
  std::vector<int> dead;
  int idles = 0;
  // A fake in-order "PS stream": apply / snapshot only enqueue jobs, a device thread runs them
  // later and bumps the worker's completion count (the GPU path's event), so done_seq must be
  // published on completion, not on enqueue, for the workers' reads below to be race-free.
  std::mutex qmu;
  std::deque<std::function<void()>> q;
  std::vector<std::atomic<int>> enq(W), fin(W);
  for (int w = 0; w < W; ++w) enq[w] = fin[w] = 0;
  std::atomic<bool> dev_stop{false};
  std::thread device([&] {
    while (!dev_stop.load()) {
      std::function<void()> job;
      {
        std::lock_guard<std::mutex> lk(qmu);
        if (!q.empty()) {
          job = std::move(q.front());
          q.pop_front();
        }
      }
      if (job) job();
      else std::this_thread::sleep_for(std::chrono::microseconds(30));
    }
  });
  std::thread server([&] {
    serve(
        ctrl, W, stop,
        [&](int w, float lr) {   // "SGD" with lr = 1: params += grad (deterministic sum of all pushes)
          std::lock_guard<std::mutex> lk(qmu);
          q.push_back([&, w, lr] {
            for (int i = 0; i < N; ++i) params[i] += lr * mailbox[w][i];
          });
        },
        [&](int w) {
          enq[w]++;
          std::lock_guard<std::mutex> lk(qmu);
          q.push_back([&, w] {
            rx[w] = params;
            fin[w].fetch_add(1, std::memory_order_release);
          });
        },
        [&](int w) { return fin[w].load(std::memory_order_acquire) == enq[w].load(); }, [&] { ++idles; },
        [](int) { return true; }, &dead);
  });
  ctrl->ready.store(1, std::memory_order_release);
  std::vector<std::thread> workers;
  for (int w = 0; w < W; ++w) {
    workers.emplace_back([&, w] {
      while (ctrl->ready.load(std::memory_order_acquire) != 1) std::this_thread::yield();
      WorkerSlot& s = ctrl->slot[w];
      s.pid.store(1000 + w);
      uint64_t seq = s.done_seq.load();
      float last = -1.f;
      for (int it = 0; it < ITERS; ++it) {
        const bool push = it % 4 != 3;
        if (push)
          for (int i = 0; i < N; ++i) mailbox[w][i] = 1.f;   // plain writes before the release
        post(s, ++seq, push ? OP_PUSH : OP_PULL, 1.f);
        wait_done(s, seq, 30.0, 0);
        const float v = rx[w][0];                             // plain read after the acquire
        for (int i = 1; i < N; i += 97) assert(rx[w][i] == v);   // a consistent snapshot
        assert(v >= last);                                    // updates are never lost or reordered
        last = v;
      }
      post(s, ++seq, OP_STOP, 0.f);
      wait_done(s, seq, 30.0, 0);
    });
  }
  for (auto& t : workers) t.join();
  server.join();
  dev_stop.store(true);
  device.join();
  const float expect = (float)(W * (ITERS - ITERS / 4));
  for (int i = 0; i < N; ++i) assert(params[i] == expect);
  assert(ctrl->updates.load() == (uint64_t)(W * (ITERS - ITERS / 4)) && dead.empty());
  std::printf("ps_protocol_test: ok (%d workers x %d exchanges, %llu updates, %d idle polls)\n", W, ITERS,
              (unsigned long long)ctrl->updates.load(), idles);
  ctrl->~PSCtrl();
  return 0;
}
