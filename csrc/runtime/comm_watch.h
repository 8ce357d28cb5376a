// Stall watchdog for stream-ordered collectives, free of torch and HIP so
// ThreadSanitizer can drive it natively (csrc/tests/comm_watch_test.cpp).
//
// The native RCCL communicator (rccl_comm.cpp: Mirrored's ncclCommInitAll, MWMS's multi-rank
// ncclCommInitRank) enqueues collectives on HIP streams and returns at once, so a peer that
// never joins shows up only as a device synchronize that never returns.  Every collective is
// registered here with a completion probe (a HIP event query on each local stream) and a tag
// (e.g. "bucket 3 all_reduce"); a watchdog thread retires completed entries in issue order and,
// when the oldest outstanding one exceeds the timeout, records the verdict, runs the `on_stall`
// action (ncclCommAbort of every local communicator, which makes the blocked kernels exit) and
// -- when `shutdown_s` > 0 -- terminates the process with exit status 124 once that grace has
// also passed (Horovod's HOROVOD_STALL_SHUTDOWN_TIME_SECONDS; the reference's fail-fast intent,
// imagenet-resnet50-ps.py:67-69).  `check()` rethrows the verdict on the caller thread.
// The action runs on a thread of its own: an abort that blocks (on a lock held by a thread stuck
// inside the collective, or inside ncclCommAbort itself) never delays the shutdown deadline,
// which the watchdog loop keeps checking independently.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>

namespace pddl {

inline double cw_now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class CommWatch {
 public:
  using Probe = std::function<bool()>;   // true once the collective completed (non-blocking)
  using Release = std::function<void()>; // frees the probe's resources (called by the watchdog)

  // fatal = false: report only (Horovod's default stall check) -- each collective older than the
  // timeout is reported once, nothing is aborted, check() never raises, and a late completion
  // simply retires it; fatal = true: the verdict + action + shutdown deadline described above.
  CommWatch(double timeout_s, double shutdown_s, int rank, std::function<void(const std::string&)> on_stall,
            bool fatal = true)
      : timeout_s_(timeout_s), shutdown_s_(shutdown_s), rank_(rank), on_stall_(std::move(on_stall)), fatal_(fatal) {
    th_ = std::thread([this] { loop(); });
  }
  ~CommWatch() { stop(); }
  CommWatch(const CommWatch&) = delete;
  CommWatch& operator=(const CommWatch&) = delete;

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    if (act_th_.joinable()) act_th_.join();
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& e : q_)
      if (e.release) e.release();
    q_.clear();
  }

  void add(std::string tag, Probe probe, Release release) {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back({std::move(tag), std::move(probe), std::move(release), cw_now_s(), false});
    ++issued_;
  }

  // Raise the watchdog's verdict (if any) on the caller's thread.
  void check() const {
    std::lock_guard<std::mutex> lk(mu_);
    if (stalled_) throw std::runtime_error("pddl comm watchdog: " + msg_);
  }
  bool stalled() const {
    std::lock_guard<std::mutex> lk(mu_);
    return stalled_;
  }
  bool action_done() const { return act_done_.load(); }
  std::string message() const {
    std::lock_guard<std::mutex> lk(mu_);
    return msg_;
  }
  size_t outstanding() const {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }
  int64_t issued() const {
    std::lock_guard<std::mutex> lk(mu_);
    return issued_;
  }
  int64_t retired() const { return retired_.load(); }
  int64_t warnings() const { return warnings_.load(); }

 private:
  struct Entry {
    std::string tag;
    Probe probe;
    Release release;
    double t_issue;
    bool warned;
  };

  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      cv_.wait_for(lk, std::chrono::milliseconds(20), [this] { return stop_; });
      if (stop_) break;
      // retire completed collectives in issue order (probes are cheap, non-blocking queries)
      while (!q_.empty() && q_.front().probe()) {
        if (q_.front().release) q_.front().release();
        q_.pop_front();
        retired_++;
      }
      const double now = cw_now_s();
      if (!fatal_ && timeout_s_ > 0 && !q_.empty() && !q_.front().warned && now - q_.front().t_issue > timeout_s_) {
        q_.front().warned = true;
        warnings_++;
        std::fprintf(stderr, "[pddl comm watchdog] rank %d: %s issued %.1f s ago has not completed (%zu outstanding)"
                     " - reporting only (set PDDL_STALL_SHUTDOWN > 0 or PDDL_STALL_ABORT=1 to abort)\n", rank_,
                     q_.front().tag.c_str(), now - q_.front().t_issue, q_.size());
        std::fflush(stderr);
      }
      if (fatal_ && !stalled_ && timeout_s_ > 0 && !q_.empty() && now - q_.front().t_issue > timeout_s_) {
        std::ostringstream os;
        os << "rank " << rank_ << ": " << q_.front().tag << " issued " << (now - q_.front().t_issue)
           << " s ago has not completed (" << q_.size() << " collective(s) outstanding) - a peer rank is"
           << " likely stuck, dead or diverged";
        msg_ = os.str();
        stalled_ = true;
        t_stall_ = now;
        std::fprintf(stderr, "[pddl comm watchdog] %s\n", msg_.c_str());
        std::fflush(stderr);
        auto act = on_stall_;
        const std::string m = msg_;
        // the action (communicator abort) may block; it runs beside this loop, which keeps
        // enforcing the shutdown deadline below
        act_th_ = std::thread([this, act, m] {
          if (act) act(m);
          act_done_ = true;
        });
      }
      if (stalled_ && shutdown_s_ > 0 && now - t_stall_ > shutdown_s_) {
        std::fprintf(stderr, "[pddl comm watchdog] rank %d: still stalled %.1f s after the verdict; "
                     "terminating the process (exit 124)\n", rank_, now - t_stall_);
        std::fflush(stderr);
        std::_Exit(124);
      }
    }
  }

  const double timeout_s_, shutdown_s_;
  const int rank_;
  std::function<void(const std::string&)> on_stall_;
  const bool fatal_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Entry> q_;
  bool stop_ = false, stalled_ = false;
  double t_stall_ = 0;
  std::string msg_;
  int64_t issued_ = 0;
  std::atomic<int64_t> retired_{0};
  std::atomic<bool> act_done_{false};
  std::atomic<int64_t> warnings_{0};
  std::thread th_, act_th_;
};

}  // namespace pddl
