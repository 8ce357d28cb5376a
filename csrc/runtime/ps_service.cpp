// Asynchronous parameter-server data plane (the gRPC servers + RecvTensor /
// remote ApplyAdam of the reference's ParameterServerStrategy, imagenet-resnet50-ps.py:31-84).
//
// MI355X-native design (one node, one GPU per role, e.g. 2 PS + 6 workers):
//   * PS p owns its shard of the flat fp32 parameters plus the Adam slots m, v, and a
//     per-worker gradient MAILBOX [W][n] in its own HBM.
//   * Control plane: one POSIX shared-memory segment per PS with a slot per worker
//     (request / done sequence numbers, op, learning rate, pid, IPC handles).  Lock-free
//     process-shared atomics with release / acquire ordering; no RPC layer at all.
//   * Data plane over xGMI with HIP IPC (dmabuf): a worker's pack kernel gathers its gradient
//     ranges and writes them STRAIGHT into its mailbox slot on the PS GPU (peer writes), then
//     bumps its request sequence number.  The PS service thread sees the request, ENQUEUES the
//     fused Adam kernel (optim.hip, TF epsilon-hat form) on the mailbox, which also writes the
//     requester's own snapshot buffer of the fresh shard, on the PS stream; the copy of that
//     snapshot into the worker's receive buffer on the worker GPU (peer copy over the worker's
//     xGMI link) runs on the worker's own copy stream, so the PS stream serialises only the
//     updates while the copies to different workers proceed in parallel over their links.  It
//     records the worker's completion event and moves on to the next request; `done`
//     is published when that event has completed (the service thread never blocks on the
//     device, so the Adam / copy work of several workers' requests queues back to back on the
//     PS GPU).  Updates are applied one at a time in arrival order on the PS stream, so every
//     pull is a consistent snapshot of the shard; workers never wait for each other
//     (unbounded staleness, as the reference's asynchronous coordinator).
//   * Worker side, `begin()` returns right after enqueueing the pack kernel: a poster thread
//     waits for the pack's event and only then publishes the request, so the training thread
//     goes on launching the next step instead of synchronizing with the end of backward.
//   * CPU roles (tests, `--device cpu`): the same protocol with the mailboxes and receive
//     buffers in shared memory and a host Adam loop.
//   * The request / completion protocol and the service loop are in runtime/ps_protocol.h
//     (torch-free; ThreadSanitizer drives it natively: csrc/tests/ps_protocol_test.cpp).
//   * Wire precision (`wire` = 1, --ps-wire bf16): the worker's pack kernel rounds its gradient
//     ranges to bf16 into a bf16 mailbox, the PS's fused Adam reads them and also writes a bf16
//     snapshot of the updated shard, and the pull copies that snapshot: half the xGMI bytes in
//     both directions; the PS keeps fp32 master weights and Adam slots.
//   * Failure handling: a worker that dies never bumps its sequence number again (its
//     half-written mailbox is never applied); the service loop treats a vanished worker pid
//     as finished, and the coordinator re-queues its closure (parameter_server.py).  A worker
//     waiting on a dead PS times out with an error (reference: a PS failure aborts the job).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels/kernels.h"
#include "runtime/ps_protocol.h"

namespace py = pybind11;
using torch::Tensor;

namespace {

using pddl::ps::kMagic;
using pddl::ps::kMaxWorkers;
using pddl::ps::PSCtrl;
using pddl::ps::WorkerSlot;
using pddl::ps::OP_PUSH;
using pddl::ps::OP_PULL;
using pddl::ps::OP_STOP;
using pddl::ps::now_s;
static_assert(sizeof(hipIpcMemHandle_t) == pddl::ps::kIpcHandleBytes, "IPC handle size");

void hck(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, "pddl ps ", what, ": ", hipGetErrorString(e)); }
void kck(const char* err, const char* what) { TORCH_CHECK(err == nullptr, "pddl ps ", what, ": ", err ? err : ""); }

std::string seg_name(const std::string& job, int p, const char* what) {
  return "/pddl_" + job + "_ps" + std::to_string(p) + what;
}

// POSIX shared-memory mapping (created by the PS, attached by workers).
struct Shm {
  std::string name;
  void* ptr = nullptr;
  size_t bytes = 0;
  bool owner = false;
  void create(const std::string& n, size_t b) {
    name = n; bytes = b; owner = true;
    shm_unlink(n.c_str());
    int fd = shm_open(n.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    TORCH_CHECK(fd >= 0, "pddl ps: shm_open(create) ", n, ": ", strerror(errno));
    TORCH_CHECK(ftruncate(fd, (off_t)b) == 0, "pddl ps: ftruncate ", n);
    ptr = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    TORCH_CHECK(ptr != MAP_FAILED, "pddl ps: mmap ", n);
  }
  bool attach(const std::string& n, size_t b) {
    int fd = shm_open(n.c_str(), O_RDWR, 0600);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < b) { close(fd); return false; }
    name = n; bytes = b;
    ptr = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    return ptr != MAP_FAILED;
  }
  void unlink() {   // the mapping stays valid; the name disappears from /dev/shm
    if (owner) shm_unlink(name.c_str());
    owner = false;
  }
  ~Shm() {
    if (ptr && ptr != MAP_FAILED) munmap(ptr, bytes);
    unlink();
  }
};

// ------------------------------------------------------------------------------ server
class PSServer {
 public:
  PSServer(const std::string& job, int p, Tensor init, int workers, int device, double b1, double b2, double eps,
           int wire)
      : p_(p), W_(workers), dev_(device), wire_(wire), b1_(b1), b2_(b2), eps_(eps) {
    TORCH_CHECK(workers >= 1 && workers <= kMaxWorkers, "pddl ps: 1..64 workers");
    TORCH_CHECK(wire == 0 || (wire == 1 && device >= 0), "pddl ps: the bf16 wire needs GPU roles");
    TORCH_CHECK(init.scalar_type() == torch::kFloat32 && init.dim() == 1, "pddl ps: init must be a flat fp32 shard");
    n_real_ = init.numel();
    n_ = (n_real_ + 3) / 4 * 4;
    ctrl_shm_.create(seg_name(job, p, ""), sizeof(PSCtrl));
    ctrl_ = new (ctrl_shm_.ptr) PSCtrl();
    ctrl_->magic = kMagic;
    ctrl_->n = n_;
    ctrl_->workers = W_;
    ctrl_->gpu = dev_ >= 0;
    ctrl_->wire = wire_;
    const size_t esz = wire_ ? 2 : 4;
    Tensor host = init.to(torch::kCPU).contiguous();
    if (dev_ >= 0) {
      hck(hipSetDevice(dev_), "set device");
      hck(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "stream");
      hck(hipMalloc(&params_, 3 * n_ * sizeof(float)), "malloc params");
      m_ = params_ + n_;
      v_ = params_ + 2 * n_;
      hck(hipMemset(params_, 0, 3 * n_ * sizeof(float)), "memset");
      hck(hipMemcpy(params_, host.data_ptr<float>(), n_real_ * sizeof(float), hipMemcpyHostToDevice), "init copy");
      hck(hipMalloc(&mailbox_, (size_t)W_ * n_ * esz), "malloc mailbox");
      hck(hipMemset(mailbox_, 0, (size_t)W_ * n_ * esz), "memset mailbox");
      // per-worker snapshot buffers: request r of worker w writes ITS snapshot into snap_[w]
      // on the PS stream, then the copy to w's receive buffer runs on w's own copy stream over
      // w's xGMI link while the PS stream goes on with the next request (w's next request --
      // the only writer of snap_[w] -- comes after w saw this one done)
      hck(hipMalloc(&snap_, (size_t)W_ * n_ * esz), "malloc snapshots");
      cstream_.assign(W_, nullptr);
      for (auto& cs : cstream_) hck(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "copy stream");
      hipIpcMemHandle_t mh;
      hck(hipIpcGetMemHandle(&mh, mailbox_), "ipc handle");
      std::memcpy(ctrl_->mailbox_handle, &mh, sizeof(mh));
      hck(hipDeviceSynchronize(), "init sync");
      rx_ptr_.assign(W_, nullptr);
      done_ev_.assign(W_, nullptr);
      start_ev_.assign(W_, nullptr);
      snap_ev_.assign(W_, nullptr);
      for (auto& e : done_ev_) hck(hipEventCreate(&e), "event");   // (timed: per-request service time)
      for (auto& e : start_ev_) hck(hipEventCreate(&e), "event");
      for (auto& e : snap_ev_) hck(hipEventCreate(&e), "event");
    } else {
      host_.assign(3 * n_, 0.f);
      std::memcpy(host_.data(), host.data_ptr<float>(), n_real_ * sizeof(float));
      params_ = host_.data(); m_ = params_ + n_; v_ = params_ + 2 * n_;
      mb_shm_.create(seg_name(job, p, "_mb"), (size_t)W_ * n_ * sizeof(float));
      rx_shm_.create(seg_name(job, p, "_rx"), (size_t)W_ * n_ * sizeof(float));
      mailbox_ = mb_shm_.ptr;
    }
    ctrl_->ready.store(1, std::memory_order_release);
  }
  ~PSServer() {
    stop_.store(true);
    if (thr_.joinable()) thr_.join();
    if (dev_ >= 0) {
      hipSetDevice(dev_);
      for (void* r : rx_ptr_) if (r) hipIpcCloseMemHandle(r);
      for (auto e : done_ev_) if (e) hipEventDestroy(e);
      for (auto e : start_ev_) if (e) hipEventDestroy(e);
      for (auto e : snap_ev_) if (e) hipEventDestroy(e);
      for (auto cs : cstream_) if (cs) hipStreamDestroy(cs);
      if (mailbox_) hipFree(mailbox_);
      if (snap_) hipFree(snap_);
      if (params_) hipFree(params_);
      if (stream_) hipStreamDestroy(stream_);
    }
  }

  void start() { thr_ = std::thread([this] { serve(); }); }
  int64_t join() {
    if (thr_.joinable()) thr_.join();
    TORCH_CHECK(err_.empty(), "pddl ps server: ", err_);
    return (int64_t)ctrl_->updates.load();
  }
  int64_t updates() const { return (int64_t)ctrl_->updates.load(); }
  // Per-request GPU service time (start of Adam -> end of the snapshot copy), after join().
  py::dict service_stats() const {
    py::dict d;
    d["requests"] = svc_n_;
    d["mean_ms"] = svc_n_ ? svc_sum_ms_ / svc_n_ : 0.0;          // start of Adam -> copy landed
    d["max_ms"] = svc_max_ms_;
    d["total_ms"] = svc_sum_ms_;
    d["busy_mean_ms"] = svc_n_ ? busy_sum_ms_ / svc_n_ : 0.0;     // the PS stream's share (serialised)
    d["busy_total_ms"] = busy_sum_ms_;
    d["shard_elems"] = n_real_;
    return d;
  }
  std::vector<int> dead() const { return dead_; }
  Tensor params() const {
    Tensor out = torch::empty({n_real_}, torch::kFloat32);
    if (dev_ >= 0) {
      hipSetDevice(dev_);
      hck(hipStreamSynchronize(stream_), "sync");
      hck(hipMemcpy(out.data_ptr<float>(), params_, n_real_ * sizeof(float), hipMemcpyDeviceToHost), "params d2h");
    } else {
      std::memcpy(out.data_ptr<float>(), params_, n_real_ * sizeof(float));
    }
    return out;
  }

 private:
  void apply_adam(int w, float lr) {
    ++t_;
    const double lr_t = lr * std::sqrt(1.0 - std::pow(b2_, t_)) / (1.0 - std::pow(b1_, t_));
    const float* g = static_cast<const float*>(mailbox_) + (size_t)w * n_;
    if (dev_ >= 0) {
      hck(hipEventRecord(start_ev_[w], stream_), "record start");
      started_[w] = true;
      if (wire_)
        kck(pddl::adam_bf16_wire_launch(params_, static_cast<const uint16_t*>(mailbox_) + (size_t)w * n_, m_, v_,
                                        static_cast<uint16_t*>(snap_) + (size_t)w * n_, n_, (float)lr_t, (float)b1_,
                                        (float)b2_, (float)eps_, stream_),
            "adam (bf16 wire)");
      else
        kck(pddl::adam_launch(params_, g, m_, v_, n_, (float)lr_t, (float)b1_, (float)b2_, (float)eps_, 1.f, nullptr,
                              stream_),
            "adam");
    } else {
      const float b1 = (float)b1_, b2 = (float)b2_, eps = (float)eps_, lt = (float)lr_t;
      for (int64_t i = 0; i < n_; ++i) {
        m_[i] = b1 * m_[i] + (1.f - b1) * g[i];
        v_[i] = b2 * v_[i] + (1.f - b2) * g[i] * g[i];
        params_[i] -= lt * m_[i] / (std::sqrt(v_[i]) + eps);
      }
    }
  }
  void send_snapshot(int w) {
    WorkerSlot& s = ctrl_->slot[w];
    if (dev_ >= 0) {
      if (!rx_ptr_[w]) {
        TORCH_CHECK(s.rx_ready.load(std::memory_order_acquire) == 1, "worker ", w, " has no receive buffer");
        void* ptr = nullptr;
        hipIpcMemHandle_t h;
        std::memcpy(&h, s.rx_handle, sizeof(h));
        hck(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess), "open rx handle");
        rx_ptr_[w] = ptr;
      }
      const bool pushed = started_[w];
      if (!started_[w]) hck(hipEventRecord(start_ev_[w], stream_), "record start");   // (pull: snapshot only)
      started_[w] = false;
      // w's snapshot of the shard as of this point of the PS stream (bf16 push: written by the
      // fused Adam already), then the cross-link copy on w's copy stream
      if (wire_) {
        uint16_t* sw = static_cast<uint16_t*>(snap_) + (size_t)w * n_;
        if (!pushed) kck(pddl::cast_bf16_launch(params_, sw, n_, stream_), "snapshot cast");
        hck(hipEventRecord(snap_ev_[w], stream_), "record snapshot");
        hck(hipStreamWaitEvent(cstream_[w], snap_ev_[w], 0), "copy stream wait");
        hck(hipMemcpyAsync(rx_ptr_[w], sw, n_ * sizeof(uint16_t), hipMemcpyDeviceToDevice, cstream_[w]), "snapshot");
      } else {
        float* sw = static_cast<float*>(snap_) + (size_t)w * n_;
        hck(hipMemcpyAsync(sw, params_, n_ * sizeof(float), hipMemcpyDeviceToDevice, stream_), "snapshot");
        hck(hipEventRecord(snap_ev_[w], stream_), "record snapshot");
        hck(hipStreamWaitEvent(cstream_[w], snap_ev_[w], 0), "copy stream wait");
        hck(hipMemcpyAsync(rx_ptr_[w], sw, n_ * sizeof(float), hipMemcpyDeviceToDevice, cstream_[w]), "snapshot");
      }
      hck(hipEventRecord(done_ev_[w], cstream_[w]), "record done");
    } else {
      std::memcpy(static_cast<float*>(rx_shm_.ptr) + (size_t)w * n_, params_, n_ * sizeof(float));
    }
  }
  void serve() {
    try {
      if (dev_ >= 0) hck(hipSetDevice(dev_), "set device");
      pddl::ps::serve(
          ctrl_, W_, stop_, [this](int w, float lr) { apply_adam(w, lr); }, [this](int w) { send_snapshot(w); },
          [this](int w) {
            if (dev_ < 0) return true;
            const hipError_t q = hipEventQuery(done_ev_[w]);
            if (q == hipErrorNotReady) return false;
            hck(q, "completion event");
            float ms = 0.f, busy = 0.f;   // request: Adam start -> copy landed; busy: the PS stream's part
            if (hipEventElapsedTime(&ms, start_ev_[w], done_ev_[w]) == hipSuccess &&
                hipEventElapsedTime(&busy, start_ev_[w], snap_ev_[w]) == hipSuccess) {
              svc_n_++;
              svc_sum_ms_ += ms;
              busy_sum_ms_ += busy;
              svc_max_ms_ = std::max(svc_max_ms_, (double)ms);
            }
            return true;
          },
          [this] {
            if (!unlinked_) {   // every worker attached: drop the names (no /dev/shm leak on a crash)
              bool all = true;
              for (int w = 0; w < W_; ++w) all = all && ctrl_->slot[w].pid.load() > 0;
              if (all) {
                ctrl_shm_.unlink(); mb_shm_.unlink(); rx_shm_.unlink();
                unlinked_ = true;
              }
            }
          },
          [](int pid) { return !(kill(pid, 0) != 0 && errno == ESRCH); }, &dead_);
      if (dev_ >= 0) {
        hipStreamSynchronize(stream_);
        for (auto cs : cstream_) hipStreamSynchronize(cs);
      }
    } catch (const std::exception& e) {
      err_ = e.what();
    }
  }

  int p_, W_, dev_, wire_;
  double b1_, b2_, eps_;
  int64_t n_real_ = 0, n_ = 0, t_ = 0;
  Shm ctrl_shm_, mb_shm_, rx_shm_;
  PSCtrl* ctrl_ = nullptr;
  float* params_ = nullptr;
  float* m_ = nullptr;
  float* v_ = nullptr;
  void* mailbox_ = nullptr;            // [W][n] fp32 or (bf16 wire) bf16
  void* snap_ = nullptr;               // [W][n] per-worker snapshots (bf16 or fp32 wire)
  std::vector<hipStream_t> cstream_;   // per worker: its snapshot's copy over its link
  std::vector<float> host_;
  std::vector<void*> rx_ptr_;
  std::vector<hipEvent_t> done_ev_;   // per worker: its request's Adam + snapshot copy finished
  std::vector<hipEvent_t> start_ev_;  // per worker: its request's work started (timing)
  std::vector<hipEvent_t> snap_ev_;   // per worker: its snapshot is written (end of the PS stream's part)
  std::vector<char> started_ = std::vector<char>(pddl::ps::kMaxWorkers, 0);
  int64_t svc_n_ = 0;
  double svc_sum_ms_ = 0, svc_max_ms_ = 0, busy_sum_ms_ = 0;
  hipStream_t stream_ = nullptr;
  std::thread thr_;
  std::atomic<bool> stop_{false};
  std::vector<int> dead_;
  bool unlinked_ = false;
  std::string err_;
};

// ------------------------------------------------------------------------------ client
struct Remote {
  Shm ctrl_shm, mb_shm, rx_shm;
  PSCtrl* ctrl = nullptr;
  int64_t n = 0;
  int wire = 0;               // 1: bf16 mailbox / receive buffer
  void* mailbox = nullptr;    // this worker's slot (peer GPU memory or shared memory)
  void* mb_base = nullptr;    // IPC mapping base (GPU)
  void* rx = nullptr;         // this worker's receive buffer
  Tensor rows;                // device RangeRow table (GPU) / host (CPU)
  std::vector<pddl::RangeRow> host_rows;
  uint64_t seq = 0;
};

class PSClient {
 public:
  PSClient(const std::string& job, std::vector<std::vector<std::pair<int64_t, int64_t>>> ranges, int worker,
           int device, double timeout_s)
      : w_(worker), dev_(device), timeout_(timeout_s) {
    const int P = (int)ranges.size();
    rem_.resize(P);
    if (dev_ >= 0) hck(hipSetDevice(dev_), "set device");
    for (int p = 0; p < P; ++p) {
      Remote& r = rem_[p];
      const double t0 = now_s();
      while (!r.ctrl_shm.attach(seg_name(job, p, ""), sizeof(PSCtrl))) {
        TORCH_CHECK(now_s() - t0 < timeout_, "pddl ps client: PS ", p, " never came up");
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
      r.ctrl = static_cast<PSCtrl*>(r.ctrl_shm.ptr);
      while (r.ctrl->ready.load(std::memory_order_acquire) != 1) {
        TORCH_CHECK(now_s() - t0 < timeout_, "pddl ps client: PS ", p, " not ready");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      TORCH_CHECK(r.ctrl->magic == kMagic && w_ < r.ctrl->workers, "pddl ps client: bad control segment");
      TORCH_CHECK((r.ctrl->gpu != 0) == (dev_ >= 0), "pddl ps client: PS and worker must both be GPU or both CPU");
      r.n = r.ctrl->n;
      r.wire = r.ctrl->wire;
      const size_t esz = r.wire ? 2 : 4;
      int64_t packed = 0;
      for (auto& fr : ranges[p]) {
        TORCH_CHECK(fr.first >= 0 && fr.second >= 0, "pddl ps client: negative range");
        r.host_rows.push_back({(long)fr.first, (long)packed, (long)fr.second});
        packed += fr.second;
        flat_end_ = std::max<int64_t>(flat_end_, fr.first + fr.second);
      }
      TORCH_CHECK(packed <= r.n && (packed + 3) / 4 * 4 == r.n, "pddl ps client: ranges do not match shard ", p);
      WorkerSlot& s = r.ctrl->slot[w_];
      r.seq = s.done_seq.load();
      if (dev_ >= 0) {
        hipIpcMemHandle_t mh;
        std::memcpy(&mh, r.ctrl->mailbox_handle, sizeof(mh));
        hck(hipIpcOpenMemHandle(&r.mb_base, mh, hipIpcMemLazyEnablePeerAccess), "open mailbox");
        r.mailbox = static_cast<char*>(r.mb_base) + (size_t)w_ * r.n * esz;
        void* rx = nullptr;
        hck(hipMalloc(&rx, r.n * esz), "malloc rx");
        hck(hipMemset(rx, 0, r.n * esz), "memset rx");
        hck(hipDeviceSynchronize(), "rx sync");
        r.rx = rx;
        hipIpcMemHandle_t rh;
        hck(hipIpcGetMemHandle(&rh, r.rx), "rx handle");
        std::memcpy(s.rx_handle, &rh, sizeof(rh));
        s.rx_ready.store(1, std::memory_order_release);
        auto opts = torch::TensorOptions().dtype(torch::kUInt8);
        Tensor hrows = torch::empty({(int64_t)(r.host_rows.size() * sizeof(pddl::RangeRow))}, opts);
        std::memcpy(hrows.data_ptr(), r.host_rows.data(), hrows.numel());
        r.rows = hrows.to(torch::Device(torch::kCUDA, dev_));
      } else {
        TORCH_CHECK(r.mb_shm.attach(seg_name(job, p, "_mb"), (size_t)r.ctrl->workers * r.n * sizeof(float)) &&
                        r.rx_shm.attach(seg_name(job, p, "_rx"), (size_t)r.ctrl->workers * r.n * sizeof(float)),
                    "pddl ps client: cannot attach shard buffers of PS ", p);
        r.mailbox = static_cast<float*>(r.mb_shm.ptr) + (size_t)w_ * r.n;
        r.rx = static_cast<float*>(r.rx_shm.ptr) + (size_t)w_ * r.n;
      }
      s.pid.store((int32_t)getpid());
    }
    if (dev_ >= 0) {
      hck(hipEventCreateWithFlags(&pack_ev_, hipEventDisableTiming), "pack event");
      poster_ = std::thread([this] { post_loop(); });
    }
  }
  ~PSClient() {
    {
      std::lock_guard<std::mutex> lk(post_mu_);
      post_stop_ = true;
    }
    post_stopping_.store(true);
    post_cv_.notify_all();
    // bounded: the poster polls its event and leaves once stopping, even if the pack never ends
    if (poster_.joinable()) poster_.join();
    if (dev_ >= 0) {
      hipSetDevice(dev_);
      if (pack_ev_) hipEventDestroy(pack_ev_);
      for (Remote& r : rem_) {
        if (r.mb_base) hipIpcCloseMemHandle(r.mb_base);
        if (r.rx) hipFree(r.rx);
      }
    }
  }

  // push (op 0): send this worker's gradients, receive the updated shards; pull (op 1):
  // receive only.  Writes the received shards into `params` (flat).
  void exchange(Tensor grads, Tensor params, double lr, bool push) {
    begin(grads, params, lr, push);
    end(params);
  }

  // Split form, so a worker can overlap the round trip with its next step (the PS applies the
  // update and snapshots the shard while the worker computes): begin() packs the gradients into
  // the PS mailboxes and publishes the requests; end() waits for every PS and unpacks the fresh
  // shards into `params`.  The mailbox is not touched again before end() returned.
  void begin(Tensor grads, Tensor params, double lr, bool push) {
    TORCH_CHECK(!in_flight_, "pddl ps: begin() while an exchange is in flight");
    TORCH_CHECK(params.is_contiguous() && params.scalar_type() == torch::kFloat32, "pddl ps: flat fp32 params");
    TORCH_CHECK((dev_ >= 0) == params.is_cuda(), "pddl ps: params on the worker's device");
    TORCH_CHECK(params.numel() >= flat_end_ && (!push || grads.numel() >= flat_end_),
                "pddl ps: flat buffers shorter than the shard ranges");
    hipStream_t st = nullptr;
    if (dev_ >= 0) st = at::hip::getCurrentHIPStream(dev_).stream();
    for (Remote& r : rem_) {
      WorkerSlot& s = r.ctrl->slot[w_];
      if (push) {
        TORCH_CHECK(grads.is_contiguous() && grads.scalar_type() == torch::kFloat32, "pddl ps: flat fp32 grads");
        if (dev_ >= 0 && r.wire) {
          kck(pddl::range_copy_cvt_launch(grads.data_ptr<float>(), r.mailbox,
                                          reinterpret_cast<const pddl::RangeRow*>(r.rows.data_ptr()),
                                          (int)r.host_rows.size(), 0, st),
              "pack (bf16)");
        } else if (dev_ >= 0) {
          kck(pddl::range_copy_launch(grads.data_ptr<float>(), static_cast<float*>(r.mailbox),
                                      reinterpret_cast<const pddl::RangeRow*>(r.rows.data_ptr()),
                                      (int)r.host_rows.size(), 0, st),
              "pack");
        } else {
          const float* g = grads.data_ptr<float>();
          float* mb = static_cast<float*>(r.mailbox);
          for (auto& row : r.host_rows) std::memcpy(mb + row.packed, g + row.flat, row.len * sizeof(float));
        }
      }
    }
    const int op = push ? OP_PUSH : OP_PULL;
    for (Remote& r : rem_) ++r.seq;
    in_flight_ = true;
    if (dev_ >= 0 && push) {
      // The peer writes must be complete and visible before the release store of the request:
      // hand the event wait + post to the poster thread instead of blocking this thread.
      hck(hipEventRecord(pack_ev_, st), "record pack");
      std::lock_guard<std::mutex> lk(post_mu_);
      post_job_ = {true, op, (float)lr};
      post_cv_.notify_all();
      return;
    }
    for (Remote& r : rem_) pddl::ps::post(r.ctrl->slot[w_], r.seq, op, (float)lr);
  }

  void end(Tensor params) {
    TORCH_CHECK(in_flight_, "pddl ps: end() without begin()");
    TORCH_CHECK(params.is_contiguous() && params.scalar_type() == torch::kFloat32 && params.numel() >= flat_end_,
                "pddl ps: flat fp32 params");
    hipStream_t st = nullptr;
    if (dev_ >= 0) st = at::hip::getCurrentHIPStream(dev_).stream();
    in_flight_ = false;
    for (size_t p = 0; p < rem_.size(); ++p) {
      Remote& r = rem_[p];
      wait_done(r, (int)p);
      if (dev_ >= 0 && r.wire) {
        kck(pddl::range_copy_cvt_launch(r.rx, params.data_ptr<float>(),
                                        reinterpret_cast<const pddl::RangeRow*>(r.rows.data_ptr()),
                                        (int)r.host_rows.size(), 1, st),
            "unpack (bf16)");
      } else if (dev_ >= 0) {
        kck(pddl::range_copy_launch(static_cast<const float*>(r.rx), params.data_ptr<float>(),
                                    reinterpret_cast<const pddl::RangeRow*>(r.rows.data_ptr()),
                                    (int)r.host_rows.size(), 1, st),
            "unpack");
      } else {
        float* pp = params.data_ptr<float>();
        const float* rx = static_cast<const float*>(r.rx);
        for (auto& row : r.host_rows) std::memcpy(pp + row.flat, rx + row.packed, row.len * sizeof(float));
      }
    }
  }
  bool in_flight() const { return in_flight_; }

  void stop() {
    TORCH_CHECK(!in_flight_, "pddl ps: stop() while an exchange is in flight");
    for (Remote& r : rem_) pddl::ps::post(r.ctrl->slot[w_], ++r.seq, OP_STOP, 0.f);
    for (size_t p = 0; p < rem_.size(); ++p) wait_done(rem_[p], (int)p);
  }

 private:
  void wait_done(Remote& r, int p) {
    try {
      pddl::ps::wait_done(r.ctrl->slot[w_], r.seq, timeout_, p, &post_failed_);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(post_mu_);
      TORCH_CHECK(post_err_.empty(), "pddl ps client: ", post_err_);
      throw;
    }
    std::lock_guard<std::mutex> lk(post_mu_);
    TORCH_CHECK(post_err_.empty(), "pddl ps client: ", post_err_);
  }

  // Poster thread (GPU workers): wait for the pack kernel's event, then publish the requests.
  void post_loop() {
    hipSetDevice(dev_);
    while (true) {
      PostJob job;
      {
        std::unique_lock<std::mutex> lk(post_mu_);
        post_cv_.wait(lk, [this] { return post_stop_ || post_job_.valid; });
        if (post_stop_ && !post_job_.valid) return;
        job = post_job_;
        post_job_.valid = false;
      }
      // poll (not hipEventSynchronize) so that a destructor can always stop this thread
      hipError_t e;
      int spins = 0;
      while ((e = hipEventQuery(pack_ev_)) == hipErrorNotReady) {
        if (post_stopping_.load()) return;
        if (++spins > 256) std::this_thread::sleep_for(std::chrono::microseconds(10));
      }
      if (e != hipSuccess) {
        {
          std::lock_guard<std::mutex> lk(post_mu_);
          post_err_ = std::string("pack event: ") + hipGetErrorString(e);
        }
        post_failed_.store(true, std::memory_order_release);   // end()'s wait fails at once
        continue;   // (the requests are never posted)
      }
      for (Remote& r : rem_) pddl::ps::post(r.ctrl->slot[w_], r.seq, job.op, job.lr);
    }
  }

  struct PostJob {
    bool valid = false;
    int op = OP_PUSH;
    float lr = 0.f;
  };
  int w_, dev_;
  double timeout_;
  bool in_flight_ = false;
  hipEvent_t pack_ev_ = nullptr;
  std::thread poster_;
  std::mutex post_mu_;
  std::condition_variable post_cv_;
  PostJob post_job_;
  bool post_stop_ = false;
  std::atomic<bool> post_stopping_{false}, post_failed_{false};
  std::string post_err_;
  int64_t flat_end_ = 0;
  std::vector<Remote> rem_;
};

}  // namespace

void register_ps(py::module& m) {
  py::class_<PSServer, std::shared_ptr<PSServer>>(m, "PSServer")
      .def(py::init<const std::string&, int, Tensor, int, int, double, double, double, int>(), py::arg("job"),
           py::arg("ps_index"), py::arg("init_shard"), py::arg("workers"), py::arg("device"), py::arg("beta1"),
           py::arg("beta2"), py::arg("eps"), py::arg("wire") = 0)
      .def("start", &PSServer::start)
      .def("join", &PSServer::join, py::call_guard<py::gil_scoped_release>())
      .def("params", &PSServer::params)
      .def_property_readonly("updates", &PSServer::updates)
      .def("service_stats", &PSServer::service_stats)
      .def_property_readonly("dead", &PSServer::dead);
  py::class_<PSClient, std::shared_ptr<PSClient>>(m, "PSClient")
      .def(py::init<const std::string&, std::vector<std::vector<std::pair<int64_t, int64_t>>>, int, int, double>(),
           py::arg("job"), py::arg("ranges"), py::arg("worker"), py::arg("device"), py::arg("timeout_s") = 120.0,
           py::call_guard<py::gil_scoped_release>())
      .def("exchange", &PSClient::exchange, py::call_guard<py::gil_scoped_release>())
      .def("begin", &PSClient::begin, py::call_guard<py::gil_scoped_release>())
      .def("end", &PSClient::end, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("in_flight", &PSClient::in_flight)
      .def("stop", &PSClient::stop, py::call_guard<py::gil_scoped_release>());
}
