// Range gather / scatter between the flat parameter (or gradient) buffer and a packed
// parameter-server shard (the fusion-buffer pack of Horovod and the
// RecvTensor / remote-assign traffic of the reference's PS, imagenet-resnet50-ps.py:75-84).
//
// A shard is a list of (flat offset, length) ranges -- MinSizePartitioner splits of the 214
// trainable variables (parallel/parameter_server.py) -- laid end to end in the packed buffer
// (callers check that order).  One launch moves every range.
// `dst` may be a peer GPU's memory opened through HIP IPC: the gather then writes the packed
// gradient straight into the parameter server's mailbox over xGMI (no staging copy).
#include "common.h"
#include "kernels.h"

namespace pddl {

// One flat walk over the packed shard for every range: block chunks of 2048 consecutive packed
// elements (8 per thread, coalesced: element k * 256 + tid of the chunk), the chunk's first range
// found by a binary search over the rows (laid end to end in packed order: igemm-style wide
// grids never see a 64-element BN range hold a whole workgroup) and each thread advancing its
// row as its elements cross range ends; all 8 addresses are resolved before the loads issue.
// (The former one-range-per-grid-row form -- 32 workgroups per range, 214 ranges -- moved a
// ResNet-50 shard at 290 us per b32 worker step, pack + unpack, profiles/r6_ps_worker.txt.)
// T_SRC / T_DST: float or uint16_t (bf16 wire: round to nearest even on the gather, widen on
// the scatter).
template <class T_SRC, class T_DST>
__global__ void __launch_bounds__(256) range_move_kernel(const T_SRC* __restrict__ src, T_DST* __restrict__ dst,
                                                         const RangeRow* __restrict__ rows, int nrows, int scatter) {
  constexpr int PER = 8;
  constexpr long CHUNK = 256L * PER;
  const long p0 = rows[0].packed;
  const long total = rows[nrows - 1].packed + rows[nrows - 1].len - p0;
  for (long c = (long)blockIdx.x * CHUNK; c < total; c += (long)gridDim.x * CHUNK) {
    const long q = p0 + c;
    int lo = 0, hi = nrows - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (rows[mid].packed <= q) lo = mid;
      else hi = mid - 1;
    }
    int row = lo;
    RangeRow r = rows[row];
    long si[PER], di[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const long pk = q + k * 256 + threadIdx.x;
      si[k] = -1;
      if (pk - p0 < total) {
        while (pk >= r.packed + r.len) r = rows[++row];
        const long fl = r.flat + (pk - r.packed);
        si[k] = scatter ? pk : fl;
        di[k] = scatter ? fl : pk;
      }
    }
    T_SRC v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (si[k] >= 0) v[k] = src[si[k]];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (si[k] < 0) continue;
      if constexpr (sizeof(T_SRC) == sizeof(T_DST)) dst[di[k]] = v[k];
      else if constexpr (sizeof(T_DST) == 2) dst[di[k]] = f2bf(v[k]);
      else dst[di[k]] = bf2f(v[k]);
    }
  }
}

static int range_move_grid() { return 4 * num_cus(); }   // (grid-stride: a 25.6M-element shard is ~12.5k chunks)

const char* range_copy_launch(const float* src, float* dst, const RangeRow* rows_dev, int nrows, int scatter,
                              hipStream_t s) {
  if (nrows <= 0) return nullptr;
  hipLaunchKernelGGL((range_move_kernel<float, float>), dim3(range_move_grid()), dim3(256), 0, s, src,
                     dst, rows_dev, nrows, scatter);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// bf16 wire of the parameter server (--ps-wire bf16): the same range gather / scatter with the
// precision change fused in -- gather: flat fp32 -> packed bf16 (round to nearest even, the
// worker's gradient push into a bf16 mailbox); scatter: packed bf16 -> flat fp32 (the pulled
// bf16 shard snapshot into the worker's fp32 parameters).
const char* range_copy_cvt_launch(const void* src, void* dst, const RangeRow* rows_dev, int nrows, int scatter,
                                  hipStream_t s) {
  if (nrows <= 0) return nullptr;
  const int g = range_move_grid();
  if (scatter)
    hipLaunchKernelGGL((range_move_kernel<uint16_t, float>), dim3(g), dim3(256), 0, s,
                       static_cast<const uint16_t*>(src), static_cast<float*>(dst), rows_dev, nrows, 1);
  else
    hipLaunchKernelGGL((range_move_kernel<float, uint16_t>), dim3(g), dim3(256), 0, s,
                       static_cast<const float*>(src), static_cast<uint16_t*>(dst), rows_dev, nrows, 0);
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
