// Control-plane protocol of the parameter-server data plane (ps_service.cpp),
// free of torch and HIP so ThreadSanitizer can drive it natively (csrc/tests/ps_protocol_test.cpp
// runs the service loop and several clients as threads over one segment).
//
// One control segment per PS (POSIX shared memory across processes) with a slot per worker.
// A request is: the worker writes its gradient into its mailbox and the learning rate into the
// slot (plain stores), then publishes `req_seq` with RELEASE; the service loop ACQUIREs
// `req_seq`, applies the update, writes the fresh shard into the worker's receive buffer
// (plain stores) and publishes `done_seq` with RELEASE; the worker ACQUIREs `done_seq` before
// reading the receive buffer.  Those two release/acquire pairs are the only ordering the
// plain mailbox / receive-buffer traffic relies on.  (GPU roles: the mailbox and receive
// buffers are HIP-IPC device memory written by kernels and peer copies; the worker's pack
// kernel is fenced by an event synchronize on the worker's poster thread before its release
// store, the PS's Adam + snapshot copy by an event query before the PS's release store.)
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace pddl {
namespace ps {

constexpr uint64_t kMagic = 0x5044444c50535631ull;   // "PDDLPSV1"
constexpr int kMaxWorkers = 64;
constexpr int kIpcHandleBytes = 64;                  // hipIpcMemHandle_t
enum { OP_PUSH = 0, OP_PULL = 1, OP_STOP = 2 };

struct alignas(128) WorkerSlot {
  std::atomic<uint64_t> req_seq;
  std::atomic<uint64_t> done_seq;
  std::atomic<int32_t> op;
  std::atomic<int32_t> rx_ready;
  std::atomic<int32_t> pid;
  float lr;                                    // plain: published by req_seq
  unsigned char rx_handle[kIpcHandleBytes];    // worker receive buffer (GPU roles); published by rx_ready
};

struct PSCtrl {
  uint64_t magic;
  int64_t n;            // shard elements (padded to a multiple of 4)
  int32_t workers;
  int32_t gpu;          // 1: data in GPU memory (IPC), 0: shared memory
  int32_t wire;         // element type of mailboxes / snapshots: 0 fp32, 1 bf16 (GPU roles only)
  std::atomic<int32_t> ready;
  std::atomic<uint64_t> updates;
  unsigned char mailbox_handle[kIpcHandleBytes];
  WorkerSlot slot[kMaxWorkers];
};

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Service loop of one PS: serve every worker's requests in arrival order until each has sent
// OP_STOP or vanished.  apply(w, lr): ENQUEUE the update of worker w's mailbox; snapshot(w):
// ENQUEUE the copy of the fresh shard into w's receive buffer; complete(w): true once both have
// finished (GPU roles: an event recorded after the copy on the PS stream -- the loop never
// blocks on the device, so requests of other workers are enqueued behind it while the copy
// runs; host roles: always true).  `done_seq` is published only on completion.  idle(): called
// when nothing happened in a sweep (housekeeping); alive(pid): false once a worker process is
// gone (polled every 0.5 s while idle).
template <class Apply, class Snapshot, class Complete, class Idle, class Alive>
void serve(PSCtrl* ctrl, int W, const std::atomic<bool>& stop, Apply apply, Snapshot snapshot, Complete complete,
           Idle idle, Alive alive, std::vector<int>* dead) {
  std::vector<uint64_t> seen(W, 0), pending(W, 0);
  std::vector<char> finished(W, 0), busy(W, 0), pushed(W, 0);
  int n_done = 0, n_busy = 0;
  double last_check = now_s();
  auto retire = [&](int w) {   // the enqueued work of w's request finished: publish it
    if (pushed[w]) ctrl->updates.fetch_add(1);
    ctrl->slot[w].done_seq.store(pending[w], std::memory_order_release);
    busy[w] = 0;
    --n_busy;
  };
  while ((n_done < W || n_busy > 0) && !stop.load()) {
    bool any = false;
    for (int w = 0; w < W; ++w) {
      if (busy[w]) {
        if (complete(w)) {
          retire(w);
          any = true;
        }
        continue;
      }
      if (finished[w]) continue;
      WorkerSlot& s = ctrl->slot[w];
      const uint64_t r = s.req_seq.load(std::memory_order_acquire);
      if (r == seen[w]) continue;
      any = true;
      seen[w] = r;
      const int op = s.op.load(std::memory_order_relaxed);
      if (op == OP_STOP) {
        finished[w] = 1;
        ++n_done;
        s.done_seq.store(r, std::memory_order_release);
      } else {
        pushed[w] = op == OP_PUSH;
        if (pushed[w]) apply(w, s.lr);
        snapshot(w);
        pending[w] = r;
        busy[w] = 1;
        ++n_busy;
        if (complete(w)) retire(w);
      }
    }
    if (!any) {
      idle();
      const double t = now_s();
      if (t - last_check > 0.5) {   // a worker process that vanished counts as finished
        last_check = t;
        for (int w = 0; w < W; ++w) {
          const int pid = ctrl->slot[w].pid.load();
          if (!finished[w] && pid > 0 && !alive(pid)) {
            finished[w] = 1;
            ++n_done;
            if (dead) dead->push_back(w);
          }
        }
      }
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

// Client side: publish request `seq` (after the mailbox / lr writes) ...
inline void post(WorkerSlot& s, uint64_t seq, int op, float lr) {
  s.lr = lr;
  s.op.store(op, std::memory_order_relaxed);
  s.req_seq.store(seq, std::memory_order_release);
}

// ... and wait for its completion (then the receive buffer holds the fresh shard).
// `failed` (optional): a local failure flag (e.g. the worker's poster thread could not post the
// request) checked in the spin, so a failure that means no answer will ever come surfaces at
// once instead of after the whole timeout as a misleading "did not answer".
inline void wait_done(WorkerSlot& s, uint64_t seq, double timeout_s, int p,
                      const std::atomic<bool>* failed = nullptr) {
  const double t0 = now_s();
  int spins = 0;
  while (s.done_seq.load(std::memory_order_acquire) != seq) {
    if (failed && failed->load(std::memory_order_acquire))
      throw std::runtime_error("pddl ps client: request to parameter server " + std::to_string(p) +
                               " was never posted (local failure)");
    if (++spins > 64) {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
      if (now_s() - t0 >= timeout_s)
        throw std::runtime_error("pddl ps client: parameter server " + std::to_string(p) + " did not answer within " +
                                 std::to_string(timeout_s) + " s (PS failure aborts the job)");
    }
  }
}

}  // namespace ps
}  // namespace pddl
