// Cross-layer fusion at a 64-channel bottleneck boundary (gfx950): conv3 of block b (1x1, 64 -> 256,
// folded BN, + residual, ReLU) and conv1 of block b + 1 (1x1, 256 -> 64, folded BN, ReLU) in one
// launch.  Block b's 256-channel output is still written (it is block b + 1's residual and the
// backward's input), but block b + 1's conv1 reads it from LDS instead of HBM: at b2560 that is one
// 4.1 GB read fewer per boundary (stage 2: conv2_block1 -> 2 and 2 -> 3; conv2_block3 feeds the
// stride-2 projection block and keeps the separate launches).
//
// A workgroup owns 64 rows (pixels), 4 waves:
//   phase 1  out[64][256] = y2[64][64] . W3^T  -- wave w: output channels [64 w, 64 w + 64)
//   epilogue relu(acc * scale3 + shift3 (+ res)) -> bf16 into an LDS tile [64][256], then row stores
//            of that tile (+ the ReLU bits of the block output)
//   phase 2  y1[64][64] = out[64][256] . W1^T -- wave w: channels [16 w, 16 w + 16), K = 256 from LDS
//   epilogue relu(acc * scale1 + shift1) -> bf16 -> row stores (+ ReLU bits)
// Both MFMA phases run with the weights as the A operand (fragments loaded once per workgroup from
// L2 into registers), so a lane's accumulator holds 4 consecutive channels of one pixel and the
// epilogues write 8-byte chunks; the residual tile is DMA'd into the output tile's LDS at the start
// and each lane reads its 8 bytes of it where it then writes its 8 bytes of output.  LDS: 8 KiB A
// tile + 32 KiB output tile.  Same arithmetic as the unfused igemm epilogues (fp32 scale / shift / residual, one
// bf16 rounding), so the outputs match the two-launch form bitwise up to MFMA operand order.
// Reference: the conv*_block*_3_conv -> add -> relu -> conv*_block*_1_conv chain of the Keras
// ResNet50 (imagenet-resnet50.py:56).  (A dual-source form for the projection
// boundary conv2_block1 -> 2, K = 128 with the shortcut conv, measured no gain -- 2.77 ms fused vs
// 1.87 + 0.90 ms separate at b2560, profiles/r4_c3c1.txt -- and was removed.)
#include "common.h"
#include "kernels.h"

namespace pddl {

namespace {
constexpr int CC_BM = 64;
// LDS swizzles: [rows][128 B] A tiles -- chunk ^ ((row >> 1) & 7) (igemm / conv3x3c64 images);
// [rows][512 B] output tile -- chunk ^ (row & 15): 16 consecutive rows at one chunk hit 16 distinct
// 16-byte slots of the 256-byte bank row (a 512-byte row pitch is a whole number of bank rows)
__device__ __forceinline__ int cc_sw(int row) { return (row >> 1) & 7; }
}  // namespace

__global__ void __launch_bounds__(256, 2) c3c1_kernel(C3C1Params p) {
  constexpr int K1 = 64;
  constexpr int A_BYTES = CC_BM * 128;                 // the 64-channel source tile
  __shared__ __attribute__((aligned(16))) char smem[A_BYTES + CC_BM * 512];
  char* at = smem;                                     // A1 tile; later the y1 staging tile
  char* ot = smem + A_BYTES;                           // block-b output tile [64][512 B]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int m0 = blockIdx.x * CC_BM;

  // ---- A tile by LDS-DMA: 8 pieces of 8 rows, 2 per wave
  {
    const __amdgpu_buffer_rsrc_t ra = make_rsrc_at(p.a, (long)m0 * 64, (long)p.M * 64);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pc = wave * 2 + q, row = pc * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ cc_sw(row);
      buf_lds16(ra, LDS_PTR(at + pc * 1024), m0 + row < p.M ? (uint32_t)((row * 64 + ch * 8) * 2) : OOB_OFF, 0);
    }
  }
  // ---- residual tile by LDS-DMA straight into the output tile (same swizzled image): the epilogue
  //      reads each lane's 8 bytes of residual where it then writes its 8 bytes of output.
  //      32 pieces of 2 rows x 512 B, 8 per wave.
  const bool has_res = p.res != nullptr;
  if (has_res) {
    const __amdgpu_buffer_rsrc_t rr = make_rsrc_at(p.res, (long)m0 * 256, (long)p.M * 256);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int pc = wave * 8 + q, row = 2 * pc + (lane >> 5);
      const int ch = (lane & 31) ^ (row & 15);
      buf_lds16(rr, LDS_PTR(ot + pc * 1024), m0 + row < p.M ? (uint32_t)((row * 256 + ch * 8) * 2) : OOB_OFF, 0);
    }
  }
  // ---- weight fragments (A operand): W3 rows 64 wave + 16 jb + r16, k = 32 ks + 8 kq .. + 7
  v8bf w3[4][K1 / 32];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int ks = 0; ks < K1 / 32; ++ks)
      w3[jb][ks] = *reinterpret_cast<const v8bf*>(p.w3 + (64 * wave + 16 * jb + r16) * K1 + 32 * ks + 8 * kq);

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- phase 1
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[i][jb] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < K1 / 32; ++ks) {
    const char* src = at + (ks >> 1) * A_BYTES;
    const int ch = (ks & 1) * 4 + kq;
    v8bf bx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + r16;
      bx[i] = *reinterpret_cast<const v8bf*>(src + row * 128 + ((ch ^ cc_sw(row)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3[jb][ks], bx[i], acc[i][jb], 0, 0, 0);
  }
  // phase-2 weights (loaded while phase 1 drains): W1 rows 16 wave + r16, k = 32 kk + 8 kq .. + 7
  v8bf w1[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) w1[kk] = *reinterpret_cast<const v8bf*>(p.w1 + (16 * wave + r16) * 256 + 32 * kk + 8 * kq);

  // ---- epilogue 1 -> output tile (bf16, 8-byte chunks)
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int n = 64 * wave + 16 * jb + 4 * kq;
    const float4 s4 = *reinterpret_cast<const float4*>(p.scale3 + n);
    const float4 h4 = *reinterpret_cast<const float4*>(p.shift3 + n);
    const float sc[4] = {s4.x, s4.y, s4.z, s4.w}, sh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + r16;
      const int chunk = n >> 3;                         // 16-byte chunk of the 512-byte row
      uint2* slot = reinterpret_cast<uint2*>(ot + row * 512 + ((chunk ^ (row & 15)) << 4) + 8 * (kq & 1));
      const uint2 rv = has_res ? *slot : make_uint2(0u, 0u);
      const float r4[4] = {__uint_as_float(rv.x << 16), __uint_as_float(rv.x & 0xffff0000u),
                           __uint_as_float(rv.y << 16), __uint_as_float(rv.y & 0xffff0000u)};
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][jb][e] * sc[e] + sh[e] + r4[e];
      *slot = make_uint2(relu_pk2(pack2(v[0], v[1])), relu_pk2(pack2(v[2], v[3])));
    }
  }
  __syncthreads();

  // ---- block-b output: row stores from the tile (32 threads per 512-byte row), + its ReLU bits
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 256 + tid, row = idx >> 5, c = idx & 31;
    const uint4 pk = *reinterpret_cast<const uint4*>(ot + row * 512 + ((c ^ (row & 15)) << 4));
    if (m0 + row < p.M) {
      *reinterpret_cast<uint4*>(p.out + (long)(m0 + row) * 256 + c * 8) = pk;
      if (p.bits3) p.bits3[(long)(m0 + row) * 32 + c] = (uint8_t)pos_bits8(pk);
    }
  }

  // ---- phase 2: y1[64][16 wave .. +16) over K = 256 from the output tile
  v4f acc2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc2[i] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    v8bf bx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + r16, ch = kk * 4 + kq;
      bx[i] = *reinterpret_cast<const v8bf*>(ot + row * 512 + ((ch ^ (row & 15)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[kk], bx[i], acc2[i], 0, 0, 0);
  }
  // ---- epilogue 2 -> y1 staging tile (the A tile's LDS: every wave finished phase 1 before the
  //      barrier above) -> row stores (+ ReLU bits)
  {
    const int n = 16 * wave + 4 * kq;
    const float4 s4 = *reinterpret_cast<const float4*>(p.scale1 + n);
    const float4 h4 = *reinterpret_cast<const float4*>(p.shift1 + n);
    const float sc[4] = {s4.x, s4.y, s4.z, s4.w}, sh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + r16;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc2[i][e] * sc[e] + sh[e];
      const int chunk = n >> 3;
      *reinterpret_cast<uint2*>(at + row * 128 + ((chunk ^ cc_sw(row)) << 4) + 8 * (kq & 1)) =
          make_uint2(relu_pk2(pack2(v[0], v[1])), relu_pk2(pack2(v[2], v[3])));
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = it * 256 + tid, row = idx >> 3, c = idx & 7;
    const uint4 pk = *reinterpret_cast<const uint4*>(at + row * 128 + ((c ^ cc_sw(row)) << 4));
    if (m0 + row < p.M) {
      *reinterpret_cast<uint4*>(p.y1 + (long)(m0 + row) * 64 + c * 8) = pk;
      if (p.bits1) p.bits1[(long)(m0 + row) * 8 + c] = (uint8_t)pos_bits8(pk);
    }
  }
}

const char* c3c1_launch(const C3C1Params& p, hipStream_t s) {
  if (p.M <= 0) return "c3c1: empty";
  if (!p.a || !p.w3 || !p.scale3 || !p.shift3 || !p.out || !p.w1 || !p.scale1 || !p.shift1 || !p.y1)
    return "c3c1: missing operand";
  const dim3 grid((unsigned)((p.M + CC_BM - 1) / CC_BM));
  hipLaunchKernelGGL(c3c1_kernel, grid, dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
