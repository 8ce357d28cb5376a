// Native RCCL communicator: in-process multi-GPU collectives over xGMI.
//
// Reference parity: MirroredStrategy's NcclAllReduce across the local GPUs of one process
// (imagenet-resnet50-mirror.py:21) and MultiWorkerMirroredStrategy with several replicas per
// worker process over CommunicationImplementation.NCCL (imagenet-resnet50-multiworkers.py:20-25).
// torch.distributed supports one rank per process, so the multi-device-per-process layouts
// use this communicator directly:
//   * init_all(devices)                      -> ncclCommInitAll (one process, all local GPUs)
//   * RcclComm(nranks, uid, ranks, devices)  -> ncclCommInitRank for each local rank inside
//                                               one ncclGroupStart/End (P processes x R GPUs)
// Every collective is issued for all local ranks inside one group, each on the CURRENT HIP
// stream of its tensor's device, so it is ordered after the kernels that produced the data.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <rccl/rccl.h>

#include <memory>
#include <string>
#include <vector>

namespace py = pybind11;
using torch::Tensor;

namespace {

void nck(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "pddl rccl ", what, ": ", ncclGetErrorString(r));
}

ncclDataType_t dtype_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return ncclFloat32;
    case torch::kBFloat16: return ncclBfloat16;
    case torch::kFloat16: return ncclFloat16;
    case torch::kInt64: return ncclInt64;
    case torch::kInt32: return ncclInt32;
    case torch::kUInt8: return ncclUint8;
    default: TORCH_CHECK(false, "pddl rccl: unsupported dtype");
  }
  return ncclFloat32;
}

ncclRedOp_t op_of(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "avg") return ncclAvg;
  TORCH_CHECK(false, "pddl rccl: unknown op ", op);
  return ncclSum;
}

hipStream_t stream_of(const Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "pddl rccl: GPU tensor expected");
  return at::hip::getCurrentHIPStream(t.device().index()).stream();
}

class RcclComm {
 public:
  RcclComm(int nranks, const std::string& uid, std::vector<int> ranks, std::vector<int> devices)
      : nranks_(nranks), ranks_(std::move(ranks)), devs_(std::move(devices)) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "pddl rccl: bad unique id size");
    TORCH_CHECK(ranks_.size() == devs_.size() && !ranks_.empty(), "pddl rccl: ranks/devices mismatch");
    ncclUniqueId id;
    memcpy(&id, uid.data(), sizeof(id));
    comms_.resize(devs_.size());
    nck(ncclGroupStart(), "group start");
    for (size_t i = 0; i < devs_.size(); ++i) {
      c10::hip::HIPGuardMasqueradingAsCUDA g(devs_[i]);
      nck(ncclCommInitRank(&comms_[i], nranks_, id, ranks_[i]), "comm init rank");
    }
    nck(ncclGroupEnd(), "group end (init)");
  }
  explicit RcclComm(std::vector<int> devices) : devs_(std::move(devices)) {
    nranks_ = (int)devs_.size();
    comms_.resize(devs_.size());
    for (int i = 0; i < nranks_; ++i) ranks_.push_back(i);
    nck(ncclCommInitAll(comms_.data(), nranks_, devs_.data()), "comm init all");
  }
  ~RcclComm() {
    for (auto c : comms_)
      if (c) ncclCommDestroy(c);
  }

  static py::bytes unique_id() {
    ncclUniqueId id;
    nck(ncclGetUniqueId(&id), "get unique id");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  }

  void all_reduce(std::vector<Tensor> ts, const std::string& op) {
    check_local(ts);
    nck(ncclGroupStart(), "group start");
    for (size_t i = 0; i < ts.size(); ++i) {
      c10::hip::HIPGuardMasqueradingAsCUDA g(devs_[i]);
      nck(ncclAllReduce(ts[i].data_ptr(), ts[i].data_ptr(), ts[i].numel(), dtype_of(ts[i]), op_of(op), comms_[i],
                        stream_of(ts[i])),
          "all_reduce");
    }
    nck(ncclGroupEnd(), "group end (all_reduce)");
  }

  // Same, on explicit streams (one per local rank, e.g. the comm streams of a replica driver
  // that overlaps bucket all-reduces with the next graph segment's compute).
  void all_reduce_on(std::vector<Tensor> ts, const std::string& op, std::vector<int64_t> streams) {
    check_local(ts);
    TORCH_CHECK(streams.size() == ts.size(), "pddl rccl: one stream per local rank");
    nck(ncclGroupStart(), "group start");
    for (size_t i = 0; i < ts.size(); ++i) {
      c10::hip::HIPGuardMasqueradingAsCUDA g(devs_[i]);
      nck(ncclAllReduce(ts[i].data_ptr(), ts[i].data_ptr(), ts[i].numel(), dtype_of(ts[i]), op_of(op), comms_[i],
                        reinterpret_cast<hipStream_t>(streams[i])),
          "all_reduce");
    }
    nck(ncclGroupEnd(), "group end (all_reduce)");
  }

  void broadcast(std::vector<Tensor> ts, int root) {
    check_local(ts);
    nck(ncclGroupStart(), "group start");
    for (size_t i = 0; i < ts.size(); ++i) {
      c10::hip::HIPGuardMasqueradingAsCUDA g(devs_[i]);
      nck(ncclBroadcast(ts[i].data_ptr(), ts[i].data_ptr(), ts[i].numel(), dtype_of(ts[i]), root, comms_[i],
                        stream_of(ts[i])),
          "broadcast");
    }
    nck(ncclGroupEnd(), "group end (broadcast)");
  }

  // Point-to-point from local rank `li` (PS push/pull over xGMI).
  void send(Tensor t, int peer, int li) {
    c10::hip::HIPGuardMasqueradingAsCUDA g(devs_.at(li));
    nck(ncclSend(t.data_ptr(), t.numel(), dtype_of(t), peer, comms_.at(li), stream_of(t)), "send");
  }
  void recv(Tensor t, int peer, int li) {
    c10::hip::HIPGuardMasqueradingAsCUDA g(devs_.at(li));
    nck(ncclRecv(t.data_ptr(), t.numel(), dtype_of(t), peer, comms_.at(li), stream_of(t)), "recv");
  }

  // Failure path (stall watchdog / PS failure): abort every local communicator.
  void abort() {
    for (auto& c : comms_)
      if (c) {
        ncclCommAbort(c);
        c = nullptr;
      }
  }
  std::string async_error() {
    for (auto c : comms_) {
      if (!c) continue;
      ncclResult_t e;
      if (ncclCommGetAsyncError(c, &e) == ncclSuccess && e != ncclSuccess) return ncclGetErrorString(e);
    }
    return "";
  }

  int nranks() const { return nranks_; }
  std::vector<int> ranks() const { return ranks_; }
  std::vector<int> devices() const { return devs_; }

 private:
  void check_local(const std::vector<Tensor>& ts) {
    TORCH_CHECK(ts.size() == comms_.size(), "pddl rccl: need one tensor per local rank");
    for (size_t i = 0; i < ts.size(); ++i) {
      TORCH_CHECK(ts[i].is_cuda() && ts[i].device().index() == devs_[i], "pddl rccl: tensor ", i,
                  " must live on device ", devs_[i]);
      TORCH_CHECK(ts[i].is_contiguous(), "pddl rccl: contiguous tensors only");
      TORCH_CHECK(ts[i].numel() == ts[0].numel(), "pddl rccl: equal sizes across local ranks");
      TORCH_CHECK(comms_[i] != nullptr, "pddl rccl: communicator aborted");
    }
  }
  int nranks_;
  std::vector<int> ranks_, devs_;
  std::vector<ncclComm_t> comms_;
};

}  // namespace

void register_rccl(py::module& m) {
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<int, const std::string&, std::vector<int>, std::vector<int>>(), py::arg("nranks"),
           py::arg("uid"), py::arg("ranks"), py::arg("devices"))
      .def_static("init_all", [](std::vector<int> devs) { return std::make_shared<RcclComm>(devs); })
      .def_static("unique_id", &RcclComm::unique_id)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("tensors"), py::arg("op") = "sum",
           py::call_guard<py::gil_scoped_release>())
      .def("all_reduce_on", &RcclComm::all_reduce_on, py::arg("tensors"), py::arg("op"), py::arg("streams"),
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::arg("tensors"), py::arg("root") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("send", &RcclComm::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &RcclComm::recv, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort)
      .def("async_error", &RcclComm::async_error)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("ranks", &RcclComm::ranks)
      .def_property_readonly("devices", &RcclComm::devices);
}
