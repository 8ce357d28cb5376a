// Host side of the graphed multi-replica step (parallel/strategies.py _LocalReplicas): HIP graph
// executables launched straight from their raw handles, one native call per step phase of R
// devices, optionally fanned out over a pool of host threads (one per device slot).
//
// Why: the runtime submits a graph from the host.  A single-stream graph goes out as pre-built
// packets (~0.5 us per kernel node: ~19 us for a b32 step segment), a multi-branch one node by
// node (~3.5 us per node); and torch's per-launch device / stream contexts and event objects
// cost more Python time than the launches themselves.  At R = 8 and b32 one thread issuing
// every replica's 6 graphs, 5 event forks and 1 join per step took 5.7 ms (two-stream graphs)
// or 2.0 ms (one stream) against a 4.4 ms GPU step (profiles/r6_mirror_host_loop.txt).  With
// the pool, a phase costs the slowest device's launch, not the sum over devices.
//
// The pool runs only single-stream graphs in parallel: concurrent hipGraphLaunch of
// multi-branch graphs (the two-stream backward) on one device segfaulted inside the runtime
// (3 replicas on one GPU, round 6); those phases run in the calling thread.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "launch_pool.h"

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;

namespace {

pddl::LaunchPool& pool() {
  static pddl::LaunchPool* p = new pddl::LaunchPool();   // (leaked: its threads outlive static destruction)
  return *p;
}

std::string hip_err(hipError_t e, const char* what, size_t i) {
  return std::string(what) + " [" + std::to_string(i) + "]: " + hipGetErrorString(e);
}

}  // namespace

void register_graph_launch(py::module& m) {
  // Replay an instantiated graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()) on a stream, GIL
  // released (train/graph.py _replay).
  m.def("graph_launch", [](int64_t exec, int64_t stream) {
    hipError_t e;
    {
      py::gil_scoped_release nogil;
      e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), reinterpret_cast<hipStream_t>(stream));
    }
    if (e != hipSuccess) throw std::runtime_error(hip_err(e, "hipGraphLaunch", 0));
  });
  // One step phase of R replicas, GIL released: per i, on device devices[i] --
  //   pre[i]   != 0: record pre[i] on pre_src[i] and make streams[i] wait on it (joins a comm stream);
  //   execs[i] != 0: hipGraphLaunch(execs[i], streams[i]);
  //   post[i]  != 0: record post[i] on streams[i] and make post_dst[i] wait on it (forks to a comm stream).
  // parallel: the R items run on the launch pool (single-stream graphs only, see the header).
  m.def(
      "graph_launch_group",
      [](std::vector<int64_t> devices, std::vector<int64_t> execs, std::vector<int64_t> streams,
         std::vector<int64_t> pre, std::vector<int64_t> pre_src, std::vector<int64_t> post,
         std::vector<int64_t> post_dst, bool parallel) {
        const size_t n = execs.size();
        if (devices.size() != n || streams.size() != n)
          throw std::invalid_argument("graph_launch_group: one device / stream per exec");
        if (!(pre.empty() || (pre.size() == n && pre_src.size() == n)) ||
            !(post.empty() || (post.size() == n && post_dst.size() == n)))
          throw std::invalid_argument("graph_launch_group: event lists must be empty or one per exec");
        std::vector<std::string> err(n);
        {
          py::gil_scoped_release nogil;
          auto item = [&](size_t i) {
            auto ck = [&](hipError_t e, const char* what) {
              if (e != hipSuccess && err[i].empty()) err[i] = hip_err(e, what, i);
            };
            ck(hipSetDevice((int)devices[i]), "hipSetDevice");
            auto st = reinterpret_cast<hipStream_t>(streams[i]);
            if (!pre.empty() && pre[i]) {
              ck(hipEventRecord(reinterpret_cast<hipEvent_t>(pre[i]), reinterpret_cast<hipStream_t>(pre_src[i])),
                 "hipEventRecord");
              ck(hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(pre[i]), 0), "hipStreamWaitEvent");
            }
            if (execs[i]) ck(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(execs[i]), st), "hipGraphLaunch");
            if (!post.empty() && post[i]) {
              ck(hipEventRecord(reinterpret_cast<hipEvent_t>(post[i]), st), "hipEventRecord");
              ck(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(post_dst[i]), reinterpret_cast<hipEvent_t>(post[i]), 0),
                 "hipStreamWaitEvent");
            }
          };
          if (parallel && n > 1) {
            pool().run(n, item);
          } else {
            int dev0 = 0;
            hipGetDevice(&dev0);
            for (size_t i = 0; i < n; ++i) item(i);
            hipSetDevice(dev0);
          }
        }
        for (const auto& e : err)
          if (!e.empty()) throw std::runtime_error("graph_launch_group: " + e);
      },
      py::arg("devices"), py::arg("execs"), py::arg("streams"), py::arg("pre"), py::arg("pre_src"), py::arg("post"),
      py::arg("post_dst"), py::arg("parallel") = false);
}
