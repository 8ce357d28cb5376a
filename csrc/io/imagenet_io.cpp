// Native ImageNet reader (tfds ImageNet2012 -> decode -> resize_with_crop
// -> batch, the tf.data C++ runtime's role behind imagenet-resnet50.py:28-49).
//
//   * TFRecord shards as written by tfds (`imagenet2012-train.tfrecord-00000-of-01024`): every
//     record framed as  len:u64 | crc(len):u32 | data | crc(data):u32  (masked CRC32C, checked),
//     data a serialized tf.Example with features "image" (JPEG bytes) and "label" (int64).
//     Records are indexed once; batches are random access with pread, so shuffling, sharding
//     (Horovod batch-shard, MWMS element-shard) and repeat() stay in the Python sampler.
//   * Plain JPEG files (the untarred ILSVRC class folders): label supplied by the caller.
//   * Decode with libjpeg (RGB; grayscale expanded, CMYK / inverted-CMYK converted) and
//     tf.image.resize_with_crop_or_pad to S x S (central crop of larger dims, centred zero
//     pad of smaller ones) straight into the caller's (pinned) uint8 [n, S, S, 3] batch buffer.
//   * A persistent thread pool decodes one image per task; Python releases the GIL.
// Separate module (`_pddl_io`) so the GPU kernels never depend on libjpeg being loadable.
#include <torch/extension.h>

#include "io/io_core.h"

namespace py = pybind11;
using torch::Tensor;

namespace {

using namespace pddl_io;

// ----------------------------------------------------------------------------- readers
class TFRecordImageNet {
 public:
  TFRecordImageNet(std::vector<std::string> files, int size, int threads, bool verify_crc, std::string image_key,
                   std::string label_key)
      : files_(std::move(files)), S_(size), verify_(verify_crc), image_key_(std::move(image_key)),
        label_key_(std::move(label_key)), pool_(threads) {
    for (size_t f = 0; f < files_.size(); ++f) {
      const int fd = ::open(files_[f].c_str(), O_RDONLY);
      TORCH_CHECK(fd >= 0, "pddl io: cannot open ", files_[f]);
      fds_.push_back(fd);
      const off_t fsize = lseek(fd, 0, SEEK_END);
      off_t off = 0;
      uint8_t hdr[12];
      while (pread_all(fd, hdr, 12, off)) {
        uint64_t len;
        uint32_t lcrc;
        std::memcpy(&len, hdr, 8);
        std::memcpy(&lcrc, hdr + 8, 4);
        TORCH_CHECK(!verify_ || lcrc == masked_crc(hdr, 8), "pddl io: corrupt TFRecord length in ", files_[f],
                    " at ", (long long)off);
        TORCH_CHECK(len <= (uint64_t)fsize && off + 12 + (off_t)len + 4 <= fsize, "pddl io: truncated TFRecord ",
                    files_[f], " at ", (long long)off);
        recs_.push_back({(int)f, off + 12, (int64_t)len});
        off += 12 + (off_t)len + 4;
      }
    }
  }
  ~TFRecordImageNet() {
    for (int fd : fds_) ::close(fd);
  }
  int64_t size() const { return (int64_t)recs_.size(); }

  // images uint8 [n, S, S, 3] (pinned or plain host), labels int64 [n]
  void fetch(Tensor idx, Tensor images, Tensor labels) {
    check_out(idx, images, labels);
    const int64_t* ip = idx.data_ptr<int64_t>();
    for (int64_t i = 0; i < idx.numel(); ++i) TORCH_CHECK(ip[i] >= 0 && ip[i] < size(), "pddl io: index out of range");
    uint8_t* out = images.data_ptr<uint8_t>();
    int64_t* lab = labels.data_ptr<int64_t>();
    const size_t per = (size_t)S_ * S_ * 3;
    pool_.run(idx.numel(), [&](int64_t i) {
      const Rec& r = recs_[ip[i]];
      std::vector<uint8_t> buf((size_t)r.len + 4);
      if (!pread_all(fds_[r.file], buf.data(), buf.size(), r.off)) throw std::runtime_error("pddl io: short read");
      if (verify_) {
        uint32_t dcrc;
        std::memcpy(&dcrc, buf.data() + r.len, 4);
        if (dcrc != masked_crc(buf.data(), (size_t)r.len)) throw std::runtime_error("pddl io: corrupt TFRecord data");
      }
      const uint8_t* img = nullptr;
      size_t img_n = 0;
      int64_t label = -1;
      if (!parse_example(buf.data(), (size_t)r.len, &img, &img_n, &label, image_key_, label_key_))
        throw std::runtime_error("pddl io: record without image/label features");
      decode_crop_pad(img, img_n, S_, out + (size_t)i * per);
      lab[i] = label;
    });
  }
  // labels of every record (one pass, no decode): for class-balanced checks / metadata
  Tensor all_labels() {
    Tensor out = torch::empty({size()}, torch::kInt64);
    int64_t* lab = out.data_ptr<int64_t>();
    pool_.run(size(), [&](int64_t i) {
      const Rec& r = recs_[i];
      std::vector<uint8_t> buf((size_t)r.len);
      if (!pread_all(fds_[r.file], buf.data(), buf.size(), r.off)) throw std::runtime_error("pddl io: short read");
      const uint8_t* img = nullptr;
      size_t img_n = 0;
      int64_t label = -1;
      parse_example(buf.data(), buf.size(), &img, &img_n, &label, image_key_, label_key_);
      lab[i] = label;
    });
    return out;
  }

 private:
  void check_out(const Tensor& idx, const Tensor& images, const Tensor& labels) {
    TORCH_CHECK(idx.scalar_type() == torch::kInt64 && !idx.is_cuda() && idx.is_contiguous(), "idx int64 CPU");
    TORCH_CHECK(images.scalar_type() == torch::kUInt8 && !images.is_cuda() && images.is_contiguous() &&
                    images.numel() >= idx.numel() * S_ * S_ * 3,
                "images uint8 CPU [n, S, S, 3]");
    TORCH_CHECK(labels.scalar_type() == torch::kInt64 && !labels.is_cuda() && labels.numel() >= idx.numel(),
                "labels int64 CPU [n]");
  }
  struct Rec { int file; off_t off; int64_t len; };
  std::vector<std::string> files_;
  std::vector<int> fds_;
  std::vector<Rec> recs_;
  int S_;
  bool verify_;
  std::string image_key_, label_key_;
  Pool pool_;
};

class JpegFiles {
 public:
  JpegFiles(int size, int threads) : S_(size), pool_(threads) {}
  // decode files[i] -> images[i]
  void fetch(std::vector<std::string> files, Tensor images) {
    TORCH_CHECK(images.scalar_type() == torch::kUInt8 && !images.is_cuda() && images.is_contiguous() &&
                    images.numel() >= (int64_t)files.size() * S_ * S_ * 3,
                "images uint8 CPU [n, S, S, 3]");
    uint8_t* out = images.data_ptr<uint8_t>();
    const size_t per = (size_t)S_ * S_ * 3;
    pool_.run((int64_t)files.size(), [&](int64_t i) {
      const int fd = ::open(files[i].c_str(), O_RDONLY);
      if (fd < 0) throw std::runtime_error("pddl io: cannot open " + files[i]);
      const off_t n = lseek(fd, 0, SEEK_END);
      std::vector<uint8_t> buf((size_t)n);
      const bool ok = pread_all(fd, buf.data(), buf.size(), 0);
      ::close(fd);
      if (!ok) throw std::runtime_error("pddl io: short read " + files[i]);
      decode_crop_pad(buf.data(), buf.size(), S_, out + (size_t)i * per);
    });
  }

 private:
  int S_;
  Pool pool_;
};

}  // namespace

PYBIND11_MODULE(_pddl_io, m) {
  m.doc() = "pddl native ImageNet reader: TFRecord (tfds) / JPEG decode + resize_with_crop_or_pad";
  py::class_<TFRecordImageNet, std::shared_ptr<TFRecordImageNet>>(m, "TFRecordImageNet")
      .def(py::init<std::vector<std::string>, int, int, bool, std::string, std::string>(), py::arg("files"),
           py::arg("size") = 224, py::arg("threads") = 8, py::arg("verify_crc") = true,
           py::arg("image_key") = "image", py::arg("label_key") = "label",
           py::call_guard<py::gil_scoped_release>())
      .def("__len__", &TFRecordImageNet::size)
      .def("fetch", &TFRecordImageNet::fetch, py::call_guard<py::gil_scoped_release>())
      .def("all_labels", &TFRecordImageNet::all_labels, py::call_guard<py::gil_scoped_release>());
  py::class_<JpegFiles, std::shared_ptr<JpegFiles>>(m, "JpegFiles")
      .def(py::init<int, int>(), py::arg("size") = 224, py::arg("threads") = 8)
      .def("fetch", &JpegFiles::fetch, py::call_guard<py::gil_scoped_release>());
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return masked_crc(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
}
