// Scheduling core of the gradient fusion engine (fusion_engine.cpp), free of
// torch and HIP so ThreadSanitizer can drive it natively (csrc/tests/fusion_core_test.cpp;
// a libtorch Python process cannot run under TSan here).
//
// Threads: the caller (main / training thread: begin_step, ready, drain, wait_polling), the
// worker (issues each ready bucket's collective in bucket order through `issue`) and the
// watchdog (stall inspector: a bucket queued but not issued, or issued but not completed,
// for longer than the timeout).  Every shared field is guarded by mu_; `issued_` is atomic.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace pddl {

inline double fc_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A collective in flight, as the transport sees it (c10d::Work on the engine, a fake in tests).
struct FusionWork {
  virtual ~FusionWork() = default;
  virtual bool completed() = 0;   // non-blocking
};

template <class Payload>
struct FusionItem {
  int bucket = 0;
  double t_ready = 0, t_issue = 0, t_done = 0;
  Payload payload;                  // the transport's per-bucket state (events, timeline stamps)
  std::shared_ptr<FusionWork> work; // set by `issue`
};

template <class Payload>
class FusionCore {
 public:
  using Item = FusionItem<Payload>;
  using IssueFn = std::function<void(Item&)>;   // enqueue item.bucket's collective, set work / t_issue

  FusionCore(int nbuckets, double stall_s, int rank, IssueFn issue)
      : nb_(nbuckets), stall_s_(stall_s), rank_(rank), issue_(std::move(issue)) {}
  ~FusionCore() { shutdown(); }
  FusionCore(const FusionCore&) = delete;
  FusionCore& operator=(const FusionCore&) = delete;

  void start() {
    worker_ = std::thread([this] { run(); });
    watchdog_ = std::thread([this] { watch(); });
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
    if (watchdog_.joinable()) watchdog_.join();
  }

  void begin_step() {
    std::lock_guard<std::mutex> lk(mu_);
    if (stalled_) throw std::runtime_error("pddl fusion: stall detected: " + stall_msg_);
    if (!pending_.empty() || !inflight_.empty())
      throw std::runtime_error("pddl fusion: begin_step with outstanding buckets");
    next_expected_ = 0;
    ++step_;
  }

  // Hand bucket it.bucket to the worker (buckets must become ready in id order: the static
  // negotiation every rank agreed on).
  void ready(Item&& it) {
    if (it.bucket < 0 || it.bucket >= nb_) throw std::runtime_error("pddl fusion: bad bucket id");
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (it.bucket != next_expected_) {
        std::ostringstream os;
        os << "pddl fusion: buckets must become ready in order (got " << it.bucket << ", expected " << next_expected_
           << ")";
        throw std::runtime_error(os.str());
      }
      ++next_expected_;
      pending_.push_back(std::move(it));
    }
    cv_.notify_all();
  }

  // Wait until every queued bucket has been issued; return the in-flight items (the caller
  // completes them: stream-ordered waits on the GPU, wait_polling on a host backend).
  std::vector<Item> drain() {
    std::vector<Item> done;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return (pending_.empty() && !busy_) || stalled_ || stop_ || !error_.empty(); });
    if (!error_.empty()) throw std::runtime_error("pddl fusion: collective failed: " + error_);
    if (stalled_) throw std::runtime_error("pddl fusion: stall detected: " + stall_msg_);
    done.swap(inflight_);
    return done;
  }

  // Host-blocking completion with the watchdog's verdict able to end the wait.
  void wait_polling(Item& it) {
    while (!it.work->completed()) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (stalled_) throw std::runtime_error("pddl fusion: stall detected: " + stall_msg_);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }

  int step() const {
    std::lock_guard<std::mutex> lk(mu_);
    return step_;
  }
  // Horovod's HOROVOD_STALL_SHUTDOWN_TIME_SECONDS: once a stall has been reported and `s` more
  // seconds pass without the caller ending the job, terminate the process (exit 124) -- on the
  // GPU the caller may sit in a device synchronize behind the stuck collective and never see
  // the verdict.  0 = report only.
  void set_shutdown(double s) {
    std::lock_guard<std::mutex> lk(mu_);
    shutdown_s_ = s;
  }
  int64_t issued() const { return issued_.load(); }

 private:
  struct Watch {
    std::shared_ptr<FusionWork> work;
    double t_issue;
    int bucket;
  };

  void report_stall(const std::string& msg) {   // (mu_ held)
    stall_msg_ = msg;
    stalled_ = true;
    t_stall_ = fc_now_us();
    std::fprintf(stderr, "[pddl stall inspector] %s\n", stall_msg_.c_str());
  }

  void run() {
    while (true) {
      Item it;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !pending_.empty(); });
        if (stop_) return;
        it = std::move(pending_.front());
        pending_.pop_front();
        busy_ = true;
      }
      try {
        issue_(it);
        issued_++;
        std::lock_guard<std::mutex> lk(mu_);
        watch_.push_back({it.work, it.t_issue, it.bucket});
        inflight_.push_back(std::move(it));
        busy_ = false;
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu_);
        error_ = e.what();
        busy_ = false;
      }
      cv_.notify_all();
    }
  }

  void watch() {
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (cv_.wait_for(lk, std::chrono::milliseconds(50), [this] { return stop_; })) return;
        if (stall_s_ > 0 && !pending_.empty() && !stalled_) {
          const double age = (fc_now_us() - pending_.front().t_ready) * 1e-6;
          if (age > stall_s_) {
            std::ostringstream os;
            os << "rank " << rank_ << ": bucket " << pending_.front().bucket << " queued for " << age
               << " s without being issued (" << pending_.size() << " pending, " << inflight_.size()
               << " in flight) - a peer rank is likely stuck or diverged";
            report_stall(os.str());
          }
        }
        // issued collectives that never complete: a peer never joined (stream-ordered waits on
        // the GPU do not block the host, so this is where a stuck peer becomes visible)
        while (!watch_.empty() && watch_.front().work->completed()) watch_.pop_front();
        if (stall_s_ > 0 && !watch_.empty() && !stalled_) {
          const double age = (fc_now_us() - watch_.front().t_issue) * 1e-6;
          if (age > stall_s_) {
            std::ostringstream os;
            os << "rank " << rank_ << ": all-reduce of bucket " << watch_.front().bucket << " issued " << age
               << " s ago has not completed (" << watch_.size() << " outstanding) - a peer rank is likely stuck"
               << " or diverged";
            report_stall(os.str());
          }
        }
        if (stalled_ && shutdown_s_ > 0 && (fc_now_us() - t_stall_) * 1e-6 > shutdown_s_) {
          std::fprintf(stderr, "[pddl stall inspector] rank %d: still stalled %.1f s after the report; terminating"
                       " the process (exit 124)\n", rank_, (fc_now_us() - t_stall_) * 1e-6);
          std::fflush(stderr);
          std::_Exit(124);
        }
      }
      cv_.notify_all();
    }
  }

  const int nb_;
  const double stall_s_;
  const int rank_;
  IssueFn issue_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> pending_;
  std::vector<Item> inflight_;
  std::deque<Watch> watch_;
  bool stop_ = false, busy_ = false, stalled_ = false;
  double shutdown_s_ = 0, t_stall_ = 0;
  std::string error_, stall_msg_;
  int next_expected_ = 0, step_ = 0;
  std::atomic<int64_t> issued_{0};
  std::thread worker_, watchdog_;
};

}  // namespace pddl
