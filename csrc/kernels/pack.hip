// Range gather / scatter between the flat parameter (or gradient) buffer and a packed
// parameter-server shard (the fusion-buffer pack of Horovod and the
// RecvTensor / remote-assign traffic of the reference's PS, imagenet-resnet50-ps.py:75-84).
//
// A shard is a list of (flat offset, length) ranges -- MinSizePartitioner splits of the 214
// trainable variables (parallel/parameter_server.py) -- laid end to end in the packed buffer.
// One launch moves every range: blockIdx.y picks the range, blocks stride over its elements.
// `dst` may be a peer GPU's memory opened through HIP IPC: the gather then writes the packed
// gradient straight into the parameter server's mailbox over xGMI (no staging copy).
#include "common.h"
#include "kernels.h"

namespace pddl {

__global__ void range_copy_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                  const RangeRow* __restrict__ rows, int scatter) {
  const RangeRow r = rows[blockIdx.y];
  const long so = scatter ? r.packed : r.flat;
  const long d0 = scatter ? r.flat : r.packed;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < r.len; i += (long)gridDim.x * blockDim.x)
    dst[d0 + i] = src[so + i];
}

const char* range_copy_launch(const float* src, float* dst, const RangeRow* rows_dev, int nrows, int scatter,
                              hipStream_t s) {
  if (nrows <= 0) return nullptr;
  if (nrows > 65535) return "range_copy: too many ranges";
  hipLaunchKernelGGL(range_copy_kernel, dim3(32, nrows), dim3(256), 0, s, src, dst, rows_dev, scatter);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
