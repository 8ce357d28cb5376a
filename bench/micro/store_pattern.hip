// Store-pattern microbenchmark: HBM write bandwidth of the epilogue shapes the 1x1 conv
// kernels use, on a [M][256] bf16 tensor (M = 1024*56*56, the conv2-stage activation).
//   linear : each wave instruction stores 1 KiB contiguous (grid-stride)
//   tile   : 128x128 block tiles, 4 waves as 2x2 of 64x64; one instruction = 8 rows x 128 B
//            (the igemm epilogue's shape)
//   rows   : 64-row x 256-col block tiles; one instruction = 2 rows x 512 B (full rows)
//   tile_rd: the tile pattern plus a same-shaped read of a second tensor (residual add)
//   rows_rd: the rows pattern plus the same read
//   read   : pure streaming read (1 KiB per wave instruction), copy: streaming read + write
// hipcc --offload-arch=gfx950 -O3 bench/micro/store_pattern.hip -o /tmp/store_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) k_linear(uint4* out, long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = make_uint4(i, 1, 2, 3);
}

// out: [M][256] bf16 = [M][32] uint4.  Block tile 128 rows x 128 cols (16 uint4), wave 64x64
template <bool RD>
__global__ void __launch_bounds__(256) k_tile(uint4* out, const uint4* in, int M) {
  const int nt = 2, tile = blockIdx.x, tn = tile % nt, tm = tile / nt;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wm = wave >> 1, wn = wave & 1;
  const int c8 = lane & 7, rr = lane >> 3;
  const int col = tn * 16 + wn * 8 + c8;
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const long row = (long)tm * 128 + wm * 64 + it * 8 + rr;
    if (row < M) {
      uint4 v = make_uint4(row, col, 0, 0);
      if (RD) { uint4 a = in[row * 32 + col]; v.z = a.x + acc.x; v.w = a.y; }
      out[row * 32 + col] = v;
    }
  }
}

// Block tile 64 rows x 256 cols; a wave instruction = 2 rows x 32 uint4 (2 x 512 B)
template <bool RD>
__global__ void __launch_bounds__(256) k_rows(uint4* out, const uint4* in, int M) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = lane & 31, rr = lane >> 5;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const long row = (long)blockIdx.x * 64 + wave * 16 + it * 2 + rr;
    if (row < M) {
      uint4 v = make_uint4(row, c, 0, 0);
      if (RD) { uint4 a = in[row * 32 + c]; v.z = a.x; v.w = a.y; }
      out[row * 32 + c] = v;
    }
  }
}

// pure read: every wave instruction loads 1 KiB contiguous; the per-thread sum is stored once
__global__ void __launch_bounds__(256) k_read(const uint4* in, uint4* out, long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = in[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  out[(long)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
// streaming copy (read 1 KiB + write 1 KiB per wave instruction pair)
__global__ void __launch_bounds__(256) k_copy(const uint4* in, uint4* out, long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

int main() {
  const int M = 1024 * 56 * 56;
  const long n16 = (long)M * 32;
  uint4 *out, *in;
  CK(hipMalloc(&out, n16 * 16));
  CK(hipMalloc(&in, n16 * 16));
  CK(hipMemset(in, 1, n16 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = (double)n16 * 16;
  for (int pat = 0; pat < 7; ++pat) {
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipEventRecord(e0));
      if (pat == 0) hipLaunchKernelGGL(k_linear, dim3(256 * 32), dim3(256), 0, 0, out, n16);
      if (pat == 1) hipLaunchKernelGGL(k_tile<false>, dim3((M / 128) * 2), dim3(256), 0, 0, out, in, M);
      if (pat == 2) hipLaunchKernelGGL(k_rows<false>, dim3(M / 64), dim3(256), 0, 0, out, in, M);
      if (pat == 3) hipLaunchKernelGGL(k_tile<true>, dim3((M / 128) * 2), dim3(256), 0, 0, out, in, M);
      if (pat == 4) hipLaunchKernelGGL(k_rows<true>, dim3(M / 64), dim3(256), 0, 0, out, in, M);
      if (pat == 5) hipLaunchKernelGGL(k_read, dim3(256 * 32), dim3(256), 0, 0, in, out, n16);
      if (pat == 6) hipLaunchKernelGGL(k_copy, dim3(256 * 32), dim3(256), 0, 0, in, out, n16);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
    }
    const char* nm[] = {"linear", "tile", "rows", "tile_rd", "rows_rd", "read", "copy"};
    const double b = bytes * ((pat == 3 || pat == 4 || pat == 6) ? 2 : 1);
    printf("{\"pattern\": \"%s\", \"us\": %.1f, \"TBps\": %.2f}\n", nm[pat], best * 1e3, b / (best * 1e-3) / 1e12);
  }
  return 0;
}
