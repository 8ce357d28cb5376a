// Fused backward of a stride-1 1x1 convolution: data gradient AND weight gradient from ONE
// read of the output gradient (gfx950).
//
//   out[m, ci]  = bit(m, ci) * sum_co g[m, co] * Wd[ci, co]        (dgrad, ReLU bits of x fused)
//   dW[co, ci] += sum_m g[m, co] * x[m, ci]                        (wgrad)
//   colsum[row, ci] = per-wave partial column sums of out          (BN beta / gamma gradients)
//
// Reference parity: the backward of the third (expansion) conv of every stage-2 bottleneck of
// keras.applications.ResNet50 (imagenet-resnet50.py:56, SURVEY.md §2.5: conv2_block{1,2} conv3,
// 1x1 64 -> 256).  The separate launches (wgrad_kernel, then the igemm dgrad) each stream the
// 256-channel gradient g from HBM -- the largest operand of both (M x 256 x 2 bytes, 1.6 GB at
// b1024), so the layer pair is bound by reading it twice.  Here every 64-row tile of g is staged
// into LDS once (16-byte LDS-DMA, double-buffered) and serves both GEMMs:
//   * dgrad: g rows as MFMA B operand, the 64 x 256 data-gradient weights held in registers for
//     the whole launch (each wave owns 16 ci columns: 8 k-steps of 8 bf16 per lane) as MFMA A,
//     so a lane ends with 4 consecutive ci of one row; staged through LDS (fp32) and stored as
//     128-byte row segments with the ReLU bits applied and the column sums accumulated;
//   * wgrad: g and x read back transposed with ds_read_b64_tr_b16 (the wgrad_kernel images:
//     [64 m][128 co] halves with tr_swz rows, [64 m][64 ci] with tr_swz128), the 256 x 64 dW
//     tile accumulated in registers across ALL of the workgroup's tiles (persistent grid of
//     2 x #CUs workgroups, tiles b, b + G, ...) and added once at the end with row-contiguous
//     fp32 atomics.
// Every LDS access inside the tile loop is inline asm: the compiler cannot tell those addresses
// from the LDS-DMA targets in flight and would drain the prefetch (vmcnt(0)) before each one.
#include "common.h"
#include "kernels.h"

namespace pddl {

namespace {

constexpr int B1_CO = 256, B1_CI = 64, B1_MT = 64;

// the wgrad_kernel swizzles (wgrad.hip): [m][128 bf16] rows and [m][64 bf16] rows
__device__ __forceinline__ int b1_swz256(int row) { return ((row & 3) | ((row >> 1) & 4)) << 1; }
__device__ __forceinline__ int b1_swz128(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }

__device__ __forceinline__ v4bf b1_tr_read(const char* p) {
  v4bf r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}
typedef unsigned int b1_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ b1_v4u b1_read16(const char* p) {
  b1_v4u r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}

__global__ void __launch_bounds__(256, 2) bwd1x1_kernel(Bwd1x1Params p) {
  constexpr int CO = B1_CO, CI = B1_CI, MT = B1_MT;
  constexpr int GH_BYTES = MT * 128 * 2;                 // one 128-co half image: 16 KiB
  constexpr int G_BYTES = 2 * GH_BYTES, X_BYTES = MT * CI * 2;
  constexpr int STAGE = G_BYTES + X_BYTES;               // 40 KiB: two stages, two workgroups per CU
  constexpr int LDF = CI + 4;                            // fp32 staging row of the dgrad tile
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = (p.M + MT - 1) / MT;
  const int G = gridDim.x, b = blockIdx.x;
  const int nit = b < T ? (T - b + G - 1) / G : 0;

  // LDS-DMA lane offsets relative to the tile's first row: g half h, piece i covers rows
  // (wave*4 + i)*4 + lane/16 (16 chunks of 16 B); x piece i covers rows (wave*2 + i)*8 + lane/8
  const int lrow = lane >> 4, lpos = lane & 15;
  uint32_t g_off[8], x_off[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (wave * 4 + i) * 4 + lrow;
      g_off[h * 4 + i] = (uint32_t)((row * CO + h * 128 + (lpos ^ b1_swz256(row)) * 8) * 2);
    }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3);
    x_off[i] = (uint32_t)((row * CI + ((lane & 7) ^ b1_swz128(row)) * 8) * 2);
  }
  auto load_tile = [&](int tile, int buf) {
    const long m0 = (long)tile * MT;
    const __amdgpu_buffer_rsrc_t rg = make_rsrc_at(p.g, m0 * CO, (long)p.M * CO);   // rows >= M read zeros
    const __amdgpu_buffer_rsrc_t rx = make_rsrc_at(p.x, m0 * CI, (long)p.M * CI);
    char* gb = smem + buf * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) buf_lds16(rg, LDS_PTR(gb + h * GH_BYTES + (wave * 4 + i) * 1024), g_off[h * 4 + i], 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) buf_lds16(rx, LDS_PTR(gb + G_BYTES + (wave * 2 + i) * 1024), x_off[i], 0);
  };

  // dgrad weights of this wave's 16 ci columns (MFMA A operand: row ci, 8 co per lane per k-step)
  v8bf wa[8];
  {
    const uint16_t* wr = p.wd + (long)(16 * wave + (lane & 15)) * p.ld_wd + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) wa[ks] = *reinterpret_cast<const v8bf*>(wr + 32 * ks);
  }

  v4f accw[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int er = tid >> 3, ec = tid & 7;          // epilogue: rows er, er + 32; ci 8ec .. 8ec + 7
  const int wm = wave & 1;                        // wgrad: co rows 64*wave .. +63 (half wave >> 1)
  const int Gq = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;

  uint32_t bt_next[2];
  auto load_bits = [&](int tile) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {   // row clamped, value zeroed: no branch around the load
      const long r = (long)tile * MT + er + 32 * q;
      const uint32_t v = p.bits[(r < p.M ? r : p.M - 1) * (CI / 8) + ec];
      bt_next[q] = r < p.M ? v : 0u;
    }
  };
  if (nit > 0) {
    load_tile(b, 0);
    load_bits(b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int it = 0; it < nit; ++it) {
    const int cur = it & 1, tile = b + it * G;
    const long m0 = (long)tile * MT;
    // next tile (unconditional: past the last tile the descriptor is empty and the DMA writes
    // zeros into the idle buffer), then the next tile's ReLU bits into registers: both land by
    // the vmcnt(0) that ends this iteration, so no wait the compiler places for the bytes can
    // hold back a DMA (waiting for them here, before the GEMMs, drained the prefetch)
    load_tile(tile + G, cur ^ 1);
    const uint32_t bt[2] = {bt_next[0], bt_next[1]};
    load_bits(tile + G);
    const char* gb = smem + cur * STAGE;
    const char* xb = gb + G_BYTES;

    // ---- data gradient: D[ci][m] = sum_co Wd[ci][co] g[m][co]; lane (grp, r): ci 4grp..4grp+3
    // (of the wave's 16), m = 16i + r.  Reads of k-step ks + 1 are issued before the MFMAs of ks.
    v4f accd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) accd[i] = v4f{0.f, 0.f, 0.f, 0.f};
    b1_v4u ga[2][4];
    auto read_ks = [&](int ks, b1_v4u (&dst)[4]) {
      const int c = 4 * ks + (lane >> 4);         // logical 16-byte chunk (8 co) of the k-step
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + (lane & 15);
        dst[i] = b1_read16(gb + (c >> 4) * GH_BYTES + row * 256 + (((c & 15) ^ b1_swz256(row)) << 4));
      }
    };
    read_ks(0, ga[0]);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + 1 < 8) {
        read_ks(ks + 1, ga[(ks + 1) & 1]);
        asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        accd[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks], __builtin_bit_cast(v8bf, ga[ks & 1][i]), accd[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- weight gradient: dW[co][ci] += sum_m g[m][co] x[m][ci] (transposed fragment reads)
    const char* gh = gb + (wave >> 1) * GH_BYTES;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      int goff[2], gsw[2], xoff[2], xsw[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int row = kh * 32 + 8 * Gq + 4 * h2 + q4;
        goff[h2] = row * 256 + (pp & 1) * 8; gsw[h2] = b1_swz256(row);
        xoff[h2] = row * 128 + (pp & 1) * 8; xsw[h2] = b1_swz128(row);
      }
      v8bf af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ch = wm * 8 + i * 2 + (pp >> 1);
        const v4bf lo = b1_tr_read(gh + goff[0] + ((ch ^ gsw[0]) << 4));
        const v4bf hi = b1_tr_read(gh + goff[1] + ((ch ^ gsw[1]) << 4));
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = j * 2 + (pp >> 1);
        const v4bf lo = b1_tr_read(xb + xoff[0] + ((ch ^ xsw[0]) << 4));
        const v4bf hi = b1_tr_read(xb + xoff[1] + ((ch ^ xsw[1]) << 4));
        bfr[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) accw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], accw[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- dgrad epilogue: fp32 tile staged over this buffer's g image (every wave is done with it)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    char* st = smem + cur * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + (lane & 15), col = 16 * wave + 4 * (lane >> 4);
      const uint32_t a = (uint32_t)(uintptr_t)LDS_PTR(st + (row * LDF + col) * 4);
      asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(accd[i]) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float w[2][8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int row = er + 32 * q;
      const uint32_t a = (uint32_t)(uintptr_t)LDS_PTR(st + (row * LDF + ec * 8) * 4);
      float4 v0, v1;
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(v0), "=&v"(v1) : "v"(a) : "memory");
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        w[q][e] = ((bt[q] >> e) & 1u) ? v[e] : 0.f;
        csum[e] += w[q][e];
      }
    }
    // (both rows' bits consumed before the first store: a store under a branch in between would
    // make the compiler's wait for the second byte a vmcnt(0))
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const long gm = m0 + er + 32 * q;
      if (gm < p.M) *reinterpret_cast<uint4*>(p.out + gm * CI + ec * 8) = pack8(w[q]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next tile landed
    __syncthreads();                                    // ... and every wave is done with this buffer
  }

  // per-wave partial column sums (one row per wave; the launch reports 4 x grid rows)
#pragma unroll
  for (int o = 8; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] += __shfl_xor(csum[e], o, 64);
  if (lane < 8) {
    float4* dst = reinterpret_cast<float4*>(p.colsum + (long)(b * 4 + wave) * CI + ec * 8);
    dst[0] = make_float4(csum[0], csum[1], csum[2], csum[3]);
    dst[1] = make_float4(csum[4], csum[5], csum[6], csum[7]);
  }
  if (nit == 0) return;

  // dW: per-wave 32-row fp32 staging, then one 256-byte row-contiguous atomic per row
  __syncthreads();
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * LDF);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          stage[(i2 * 16 + (lane >> 4) * 4 + jj) * LDF + j * 16 + (lane & 15)] = accw[pass * 2 + i2][j][jj];
    __syncthreads();
    for (int r = 0; r < 32; ++r) {
      const int co = 64 * wave + pass * 32 + r;
      unsafeAtomicAdd(p.dw + (long)co * p.ld_dw + lane, stage[r * LDF + lane]);
    }
    __syncthreads();
  }
}

}  // namespace

int bwd1x1_grid(int M) {
  const long T = (M + B1_MT - 1) / B1_MT, G = 2L * num_cus();
  return (int)(T < G ? T : G);
}
int bwd1x1_partial_rows(int M) { return 4 * bwd1x1_grid(M); }

const char* bwd1x1_launch(const Bwd1x1Params& p, hipStream_t stream) {
  if (p.M <= 0) return "bwd1x1: empty problem";
  if ((long)p.M * B1_CO >= (1L << 31)) return "bwd1x1: gradient has more than 2^31 elements";
  if (p.ld_wd < B1_CO || p.ld_wd % 8 || p.ld_dw < B1_CI) return "bwd1x1: weight / gradient row strides";
  hipLaunchKernelGGL(bwd1x1_kernel, dim3(bwd1x1_grid(p.M)), dim3(256), 0, stream, p);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
