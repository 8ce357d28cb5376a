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


// bf16 wire of the parameter server (--ps-wire bf16): the same range gather / scatter with the
// precision change fused in -- gather: flat fp32 -> packed bf16 (round to nearest even, the
// worker's gradient push into a bf16 mailbox); scatter: packed bf16 -> flat fp32 (the pulled
// bf16 shard snapshot into the worker's fp32 parameters).
__global__ void range_copy_cvt_kernel(const void* __restrict__ src, void* __restrict__ dst,
                                      const RangeRow* __restrict__ rows, int scatter) {
  const RangeRow r = rows[blockIdx.y];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < r.len; i += (long)gridDim.x * blockDim.x) {
    if (scatter)
      static_cast<float*>(dst)[r.flat + i] = bf2f(static_cast<const uint16_t*>(src)[r.packed + i]);
    else
      static_cast<uint16_t*>(dst)[r.packed + i] = f2bf(static_cast<const float*>(src)[r.flat + i]);
  }
}

const char* range_copy_cvt_launch(const void* src, void* dst, const RangeRow* rows_dev, int nrows, int scatter,
                                  hipStream_t s) {
  if (nrows <= 0) return nullptr;
  if (nrows > 65535) return "range_copy_cvt: too many ranges";
  hipLaunchKernelGGL(range_copy_cvt_kernel, dim3(32, nrows), dim3(256), 0, s, src, dst, rows_dev, scatter);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ------------------------------------------------------------------------------ comm proxy
// Stand-in for one RCCL ring all-reduce's footprint on THIS GPU (bench.py --comm-proxy): a 1-GPU
// model of what a multi-GPU backward shares its CUs with.  `nch` workgroups (RCCL's channel
// count) each stream their slice of the gradient bucket -- read the gradient, write a scratch
// copy -- `passes` times (a ring all-reduce moves ~2 (N-1)/N bucket sizes through each GPU),
// paced by the constant-rate realtime counter (100 MHz) so the launch holds its CUs for the
// collective's modelled duration `ticks` (bytes x 2 (N-1)/N / bus bandwidth), then exits: the
// wait is bounded by `ticks`, which the launcher caps.  The gradient is only read.
__global__ void __launch_bounds__(256) comm_proxy_kernel(const float4* __restrict__ src, float4* __restrict__ scratch,
                                                         long n4, int passes, long ticks) {
  const long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long lo = blockIdx.x * per, hi = lmin(n4, lo + per);
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  constexpr long CH = 4 * 256;   // float4s per workgroup iteration
  const long nck = lmax(1, passes * ((hi - lo + CH - 1) / CH));
  long k = 0;
  for (int p = 0; p < passes; ++p)
    for (long i = lo; i < hi; i += CH, ++k) {
      const long due = t0 + (ticks * k) / nck;
      while ((long)__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long e = i + j * 256 + threadIdx.x;
        if (e < hi) scratch[e] = src[e];
      }
    }
  while ((long)__builtin_amdgcn_s_memrealtime() < t0 + ticks) __builtin_amdgcn_s_sleep(8);
}

const char* comm_proxy_launch(const float* src, float* scratch, long n, int passes, long ticks, int nch,
                              hipStream_t s) {
  if (n % 4) return "comm_proxy: element count must be a multiple of 4";
  if (ticks < 0 || ticks > 100L * 1000 * 1000) return "comm_proxy: duration must be within 0..1 s";
  if (nch < 1 || nch > 1024 || passes < 1 || passes > 16) return "comm_proxy: bad channel / pass count";
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(nch), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                     reinterpret_cast<float4*>(scratch), n / 4, passes, ticks);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
