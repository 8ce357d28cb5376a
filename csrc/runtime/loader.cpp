// Native input-pipeline gatherer (the tf.data C++ runtime's parallel map /
// batch role).  A memory-mapped uint8 record file is gathered row by row into a (pinned)
// host batch buffer by a pool of worker threads, so the Python process only issues one call
// per batch and the H2D copy of the previous batch overlaps the gather of the next.
#include <torch/extension.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace py = pybind11;
using torch::Tensor;

namespace {

class Loader {
 public:
  Loader(const std::string& path, int64_t row_bytes, int threads) : row_(row_bytes) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    TORCH_CHECK(fd_ >= 0, "pddl loader: cannot open ", path);
    struct stat st;
    TORCH_CHECK(fstat(fd_, &st) == 0, "pddl loader: stat failed");
    size_ = st.st_size;
    TORCH_CHECK(row_ > 0 && size_ % row_ == 0, "pddl loader: file size is not a multiple of the row size");
    base_ = static_cast<const uint8_t*>(mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0));
    TORCH_CHECK(base_ != MAP_FAILED, "pddl loader: mmap failed");
    madvise(const_cast<uint8_t*>(base_), size_, MADV_RANDOM);
    nthreads_ = threads > 0 ? threads : 1;
    for (int i = 0; i < nthreads_; ++i) pool_.emplace_back([this, i] { work(i); });
  }
  ~Loader() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : pool_) t.join();
    if (base_ && base_ != MAP_FAILED) munmap(const_cast<uint8_t*>(base_), size_);
    if (fd_ >= 0) ::close(fd_);
  }

  int64_t rows() const { return size_ / row_; }

  // out[i, :] = record[idx[i], :]   (idx int64 CPU, out uint8 CPU [n, row_bytes])
  void gather(Tensor idx, Tensor out) {
    TORCH_CHECK(idx.scalar_type() == torch::kInt64 && !idx.is_cuda() && idx.is_contiguous(), "idx int64 CPU");
    TORCH_CHECK(out.scalar_type() == torch::kUInt8 && !out.is_cuda() && out.is_contiguous(), "out uint8 CPU");
    TORCH_CHECK(out.numel() >= idx.numel() * row_, "out too small");
    const int64_t* ip = idx.data_ptr<int64_t>();
    const int64_t n = idx.numel();
    for (int64_t i = 0; i < n; ++i) TORCH_CHECK(ip[i] >= 0 && ip[i] < rows(), "pddl loader: index out of range");
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_idx_ = ip;
      job_n_ = n;
      job_out_ = out.data_ptr<uint8_t>();
      next_.store(0);
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return done_ == nthreads_; });
  }

 private:
  void work(int) {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      while (true) {
        const int64_t i = next_.fetch_add(1);
        if (i >= job_n_) break;
        memcpy(job_out_ + i * row_, base_ + job_idx_[i] * row_, row_);
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++done_;
      }
      done_cv_.notify_all();
    }
  }

  int fd_ = -1;
  int64_t row_, size_ = 0;
  const uint8_t* base_ = nullptr;
  int nthreads_ = 1;
  std::vector<std::thread> pool_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  uint64_t gen_ = 0;
  int done_ = 0;
  const int64_t* job_idx_ = nullptr;
  int64_t job_n_ = 0;
  uint8_t* job_out_ = nullptr;
  std::atomic<int64_t> next_{0};
};

}  // namespace

void register_loader(py::module& m) {
  py::class_<Loader, std::shared_ptr<Loader>>(m, "Loader")
      .def(py::init<const std::string&, int64_t, int>(), py::arg("path"), py::arg("row_bytes"), py::arg("threads") = 8)
      .def("gather", &Loader::gather, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rows", &Loader::rows);
}
