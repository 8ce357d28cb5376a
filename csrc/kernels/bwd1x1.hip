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

constexpr int B1_MT = 64;

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

// CO: gradient channels (256 stage 2, 512 stage 3); NW: waves (4: two 80 KiB workgroups per CU;
// 8: one 144 KiB workgroup).  A workgroup owns input-channel columns [64 half, 64 half + 64) of
// CI = 64 NH: with NH = 2 (stage 3: CI = 128 would need 272 registers per lane for the dW tile and
// the weight fragments) the two halves of a tile run as a PAIR of workgroups b, b + 8 -- the same
// XCD under the round-robin dispatch -- in lockstep, so the second read of each g tile hits L2.
__device__ __forceinline__ uint2 b1_read8(const char* p) {
  uint2 r;
  asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}
__device__ __forceinline__ void b1_write8(char* p, uint2 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"((uint32_t)(uintptr_t)LDS_PTR(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t b1_read_u8(const char* p) {
  uint32_t r;
  asm volatile("ds_read_u8 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}

// PRE (stage 2 only): the g tile is computed in LDS from the next block's conv1 gradient instead
// of read -- the next block's conv1 data gradient fused in front (one 4.1 GB read of g fewer per
// stage-2 block boundary at b2560): the shortcut gradient is DMA'd into the g images, the next
// block's conv1 gradient g1 and this block's output ReLU bits into two small images, and
//   g = bit * (g1 . w1d^T + shortcut gradient)
// overwrites the images in place (each lane reads its 8 bytes of the shortcut gradient where it
// writes its 8 bytes of g), is stored to HBM and summed per channel, then both GEMMs below run
// on it unchanged.  One 100 KiB workgroup per CU.
template <int CO, int NW, bool S2, bool PRE = false>
__global__ void __launch_bounds__(NW * 64, (NW == 8 || PRE) ? 1 : 2) bwd1x1_kernel(Bwd1x1Params p) {
  constexpr int CB = 64, MT = B1_MT;
  constexpr int NIMG = CO / 128;                         // 128-co half images
  constexpr int GH_BYTES = MT * 256;                     // one image: 16 KiB
  constexpr int G_BYTES = NIMG * GH_BYTES, X_BYTES = MT * CB * 2;
  constexpr int G1_BYTES = PRE ? MT * 128 : 0, GM_BYTES = PRE ? MT * CO / 8 : 0;
  constexpr int STAGE = G_BYTES + X_BYTES + G1_BYTES + GM_BYTES;   // 40 KiB (256; PRE 50) / 72 KiB (512)
  static_assert(!PRE || (CO == 256 && NW == 4 && !S2), "the pre form is the stage-2 stride-1 kernel");
  constexpr int GP = NIMG * 16 / NW, XP = 8 / NW;        // LDS-DMA pieces per wave per tile
  constexpr int KSPLIT = NW / 4;                         // waves per 16-column dgrad block (co split)
  constexpr int KS = CO / 32 / KSPLIT;                   // dgrad k-steps per wave
  constexpr int RPT = 512 / (NW * 64);                   // epilogue rows per thread (8 columns each)
  constexpr int LDF = CB + 4;                            // fp32 staging row of the dgrad tile
  constexpr int PART = MT * LDF * 4;                     // one staged partial dgrad tile
  static_assert(CO == 64 * NW && KS == 8 && GP * NW == NIMG * 16 && XP * NW == 8, "bwd1x1 shape");
  static_assert(KSPLIT * PART <= G_BYTES, "dgrad staging must fit over the g images");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int CI = p.CI, nh = CI / CB;
  int pid = blockIdx.x, half = 0, np = gridDim.x;
  if (nh == 2) {   // workgroups b and b + 8 of every 16 share an XCD: one is each half of a pair
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    half = k & 1; pid = (k >> 1) * 8 + x; np = gridDim.x / 2;
  }
  const int T = (p.M + MT - 1) / MT;
  const int nit = pid < T ? (T - pid + np - 1) / np : 0;

  // LDS-DMA lane offsets relative to the tile's first row: g piece pi = wave * GP + i fills image
  // pi / 16, rows (pi % 16) * 4 + lane / 16 (16 chunks of 16 B); x piece xi rows xi * 8 + lane / 8
  const int lrow = lane >> 4, lpos = lane & 15;
  uint32_t g_off[GP], x_off[XP];
#pragma unroll
  for (int i = 0; i < GP; ++i) {
    const int pi = wave * GP + i, row = (pi & 15) * 4 + lrow;
    g_off[i] = (uint32_t)((row * CO + (pi >> 4) * 128 + (lpos ^ b1_swz256(row)) * 8) * 2);
  }
#pragma unroll
  for (int i = 0; i < XP; ++i) {
    const int row = (wave * XP + i) * 8 + (lane >> 3);
    x_off[i] = (uint32_t)((row * CI + half * CB + ((lane & 7) ^ b1_swz128(row)) * 8) * 2);
  }
  // S2 (the block feeds a stride-2 block): the gradient g and the compact copy out2 are on the
  // stride-2 grid (M = N * Hc * Wc rows), x, out and the bits at full resolution Hf x Wf: compact
  // row m is full-resolution pixel (n, 2i, 2j)
  const int HWc = p.Hc * p.Wc;
  auto full_row = [&](long m) -> long {
    const int n = fdiv((int)m, p.mg_hwc), rem = (int)m - n * HWc, i = fdiv(rem, p.mg_wc), j = rem - i * p.Wc;
    return ((long)n * p.Hf + 2 * i) * p.Wf + 2 * j;
  };
  auto load_tile = [&](int tile, int buf) {
    const long m0 = (long)tile * MT;
    const __amdgpu_buffer_rsrc_t rg = make_rsrc_at(p.g, m0 * CO, (long)p.M * CO);   // rows >= M read zeros
    char* gb = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < GP; ++i) {
      const int pi = wave * GP + i;
      buf_lds16(rg, LDS_PTR(gb + (pi >> 4) * GH_BYTES + (pi & 15) * 1024), g_off[i], 0);
    }
    if constexpr (S2) {   // x rows gathered at the grid pixels, descriptor rebased at the tile's first image
      const int n_first = fdiv((int)(m0 < p.M ? m0 : 0), p.mg_hwc);
      const long HWf = (long)p.Hf * p.Wf;
      const __amdgpu_buffer_rsrc_t rx =
          make_rsrc_at(p.x, m0 < p.M ? n_first * HWf * CI : 0, m0 < p.M ? (long)p.N * HWf * CI : 0);
#pragma unroll
      for (int i = 0; i < XP; ++i) {
        const int row = (wave * XP + i) * 8 + (lane >> 3);
        const long m = m0 + row;
        const long pf = full_row(m < p.M ? m : 0) - n_first * HWf;
        const uint32_t off = m < p.M ? (uint32_t)((pf * CI + half * CB + ((lane & 7) ^ b1_swz128(row)) * 8) * 2) : OOB_OFF;
        buf_lds16(rx, LDS_PTR(gb + G_BYTES + (wave * XP + i) * 1024), off, 0);
      }
    } else {
      const __amdgpu_buffer_rsrc_t rx = make_rsrc_at(p.x, m0 * CI, (long)p.M * CI);
#pragma unroll
      for (int i = 0; i < XP; ++i) buf_lds16(rx, LDS_PTR(gb + G_BYTES + (wave * XP + i) * 1024), x_off[i], 0);
    }
    if constexpr (PRE) {
      // g1 tile [64 m][64 ch] (chunk ^ ((row >> 1) & 7)): 8 pieces, 2 per wave; the output's ReLU
      // bits [64 m][32 B] lane-linear: 2 pieces (waves 0, 1)
      const __amdgpu_buffer_rsrc_t r1 = make_rsrc_at(p.g1, m0 * 64, (long)p.M * 64);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pc = wave * 2 + i, row = pc * 8 + (lane >> 3);
        buf_lds16(r1, LDS_PTR(gb + G_BYTES + X_BYTES + pc * 1024),
                  (uint32_t)((row * 64 + ((lane & 7) ^ ((row >> 1) & 7)) * 8) * 2), 0);
      }
      if (wave < 2) {
        const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(p.gmask) + m0 * (CO / 8), (short)0,
            (int)(m0 < p.M ? lmin(((long)p.M - m0) * (CO / 8), 0x7fffffffL) : 0), 0x00020000);
        buf_lds16(rm, LDS_PTR(gb + G_BYTES + X_BYTES + G1_BYTES + wave * 1024), (uint32_t)((wave * 64 + lane) * 16), 0);
      }
    }
  };

  // dgrad roles: 16-column block cb of this half, co range kp * CO / KSPLIT ..; the weights of
  // that block and range stay in registers (MFMA A operand: row ci, 8 co per lane per k-step)
  const int cb = wave & 3, kp = wave >> 2;
  v8bf wa[KS];
  {
    const uint16_t* wr = p.wd + (long)(half * CB + 16 * cb + (lane & 15)) * p.ld_wd + kp * (CO / KSPLIT) + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wa[ks] = *reinterpret_cast<const v8bf*>(wr + 32 * ks);
  }

  // PRE: the next block's conv1 data-gradient weights as MFMA A fragments: rows co = 64 wave +
  // 16 jb + (lane & 15), k = 32 kh + 8 (lane >> 4) .. + 7 (the g tile's 64 co columns of this wave)
  v8bf w1f[PRE ? 4 : 1][2];
  float csx[PRE ? 16 : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
        w1f[jb][kh] = *reinterpret_cast<const v8bf*>(p.w1d + (64 * wave + 16 * jb + (lane & 15)) * 64 + 32 * kh + 8 * (lane >> 4));
#pragma unroll
    for (int e = 0; e < 16; ++e) csx[e] = 0.f;
  }

  v4f accw[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int er = tid >> 3, ec = tid & 7;          // epilogue: rows er + NW * 8 * q; ci 8ec .. 8ec + 7
  const int wm = wave & 1;                        // wgrad: co rows 64*wave .. +63 (image wave >> 1)
  const int Gq = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;

  uint32_t bt_next[RPT];
  auto load_bits = [&](int tile) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {   // row clamped, value zeroed: no branch around the load
      const long r = (long)tile * MT + er + NW * 8 * q;
      const long rc = r < p.M ? r : p.M - 1;
      const uint32_t v = p.bits[(S2 ? full_row(rc) : rc) * (CI / 8) + half * 8 + ec];
      bt_next[q] = r < p.M ? v : 0u;
    }
  };
  if (nit > 0) {
    load_tile(pid, 0);
    load_bits(pid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int it = 0; it < nit; ++it) {
    const int cur = it & 1, tile = pid + it * np;
    const long m0 = (long)tile * MT;
    // next tile (unconditional: past the last tile the descriptor is empty and the DMA writes
    // zeros into the idle buffer), then the next tile's ReLU bits into registers: both land by
    // the vmcnt(0) that ends this iteration, so no wait the compiler places for the bytes can
    // hold back a DMA (waiting for them here, before the GEMMs, drained the prefetch)
    load_tile(tile + np, cur ^ 1);
    uint32_t bt[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) bt[q] = bt_next[q];
    load_bits(tile + np);
    const char* gb = smem + cur * STAGE;
    const char* xb = gb + G_BYTES;

    if constexpr (PRE) {
      // ---- g = bit * (g1 . w1d^T + shortcut gradient), in place in the g images
      const char* g1b = gb + G_BYTES + X_BYTES;
      const char* gmb = g1b + G1_BYTES;
      v4f acc1[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc1[i][jb] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        b1_v4u bx[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * i + (lane & 15), ch = kh * 4 + (lane >> 4);
          bx[i] = b1_read16(g1b + row * 128 + ((ch ^ ((row >> 1) & 7)) << 4));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jb = 0; jb < 4; ++jb)
            acc1[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[jb][kh], __builtin_bit_cast(v8bf, bx[i]), acc1[i][jb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // lane: co = 64 wave + 16 jb + 4 kq + e (image wave >> 1), row 16 i + (lane & 15)
      const int kq = lane >> 4;
      char* gw = const_cast<char*>(gb) + (wave >> 1) * GH_BYTES;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + (lane & 15);
        uint2 ad[4];
        uint32_t mb[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          const int cc = 64 * (wave & 1) + 16 * jb + 4 * kq;   // column within the 128-co image
          ad[jb] = b1_read8(gw + row * 256 + (((cc >> 3) ^ b1_swz256(row)) << 4) + 8 * (kq & 1));
          mb[jb] = b1_read_u8(gmb + row * (CO / 8) + ((64 * wave + 16 * jb + 4 * kq) >> 3));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);   // (the asm reads' results: nothing may move above the wait)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          const int cc = 64 * (wave & 1) + 16 * jb + 4 * kq;
          const float a4[4] = {__uint_as_float(ad[jb].x << 16), __uint_as_float(ad[jb].x & 0xffff0000u),
                               __uint_as_float(ad[jb].y << 16), __uint_as_float(ad[jb].y & 0xffff0000u)};
          const int sh = (kq & 1) * 4;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = ((mb[jb] >> (sh + e)) & 1u) ? acc1[i][jb][e] + a4[e] : 0.f;
            if (m0 + row < p.M) csx[4 * jb + e] += v[e];
          }
          b1_write8(gw + row * 256 + (((cc >> 3) ^ b1_swz256(row)) << 4) + 8 * (kq & 1),
                    make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3])));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // g tile -> HBM (256 threads x 8 x 16 B, 512-byte rows)
      b1_v4u gv[8];
#pragma unroll
      for (int it2 = 0; it2 < 8; ++it2) {
        const int idx = it2 * 256 + tid, row = idx >> 5, c32 = idx & 31;
        gv[it2] = b1_read16(gb + (c32 >> 4) * GH_BYTES + row * 256 + (((c32 & 15) ^ b1_swz256(row)) << 4));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int it2 = 0; it2 < 8; ++it2) {
        const int idx = it2 * 256 + tid, row = idx >> 5, c32 = idx & 31;
        if (m0 + row < p.M) *reinterpret_cast<b1_v4u*>(p.gx + (m0 + row) * CO + c32 * 8) = gv[it2];
      }
    }

    // ---- data gradient: D[ci][m] = sum_co Wd[ci][co] g[m][co]; lane (grp, r): ci 4grp..4grp+3
    // of block cb, m = 16i + r.  Reads of k-step ks + 1 are issued before the MFMAs of ks.
    v4f accd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) accd[i] = v4f{0.f, 0.f, 0.f, 0.f};
    b1_v4u ga[2][4];
    auto read_ks = [&](int ks, b1_v4u (&dst)[4]) {
      const int c = 4 * (kp * KS + ks) + (lane >> 4);   // logical 16-byte chunk (8 co) of the k-step
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + (lane & 15);
        dst[i] = b1_read16(gb + (c >> 4) * GH_BYTES + row * 256 + (((c & 15) ^ b1_swz256(row)) << 4));
      }
    };
    read_ks(0, ga[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
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

    // ---- dgrad epilogue: the KSPLIT partial fp32 tiles staged over this buffer's g images
    // (every wave is done with them), summed on the read-back
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    char* st = smem + cur * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + (lane & 15), col = 16 * cb + 4 * (lane >> 4);
      const uint32_t a = (uint32_t)(uintptr_t)LDS_PTR(st + kp * PART + (row * LDF + col) * 4);
      asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(accd[i]) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float w[RPT][8];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int row = er + NW * 8 * q;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KSPLIT; ++k) {
        const uint32_t a = (uint32_t)(uintptr_t)LDS_PTR(st + k * PART + (row * LDF + ec * 8) * 4);
        float4 v0, v1;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(v0), "=&v"(v1) : "v"(a) : "memory");
        v[0] += v0.x; v[1] += v0.y; v[2] += v0.z; v[3] += v0.w; v[4] += v1.x; v[5] += v1.y; v[6] += v1.z; v[7] += v1.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        w[q][e] = ((bt[q] >> e) & 1u) ? v[e] : 0.f;
        csum[e] += w[q][e];
      }
    }
    // (every row's bits consumed before the first store: a store under a branch in between would
    // make the compiler's wait for the next byte a vmcnt(0))
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const long gm = m0 + er + NW * 8 * q;
      if (gm < p.M) {
        const uint4 pk = pack8(w[q]);
        *reinterpret_cast<uint4*>(p.out + (S2 ? full_row(gm) : gm) * CI + half * CB + ec * 8) = pk;
        if (S2) *reinterpret_cast<uint4*>(p.out2 + gm * CI + half * CB + ec * 8) = pk;   // compact copy
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next tile landed
    __syncthreads();                                    // ... and every wave is done with this buffer
  }

  // per-wave partial column sums: row pid * NW + wave, this half's 64 columns (the launch
  // reports np * NW rows of CI columns)
#pragma unroll
  for (int o = 8; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] += __shfl_xor(csum[e], o, 64);
  if (lane < 8) {
    float4* dst = reinterpret_cast<float4*>(p.colsum + (long)(pid * NW + wave) * CI + half * CB + ec * 8);
    dst[0] = make_float4(csum[0], csum[1], csum[2], csum[3]);
    dst[1] = make_float4(csum[4], csum[5], csum[6], csum[7]);
  }
  if constexpr (PRE) {   // g's per-channel partial sums: row pid * NW + wave, this wave's 64 columns
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int e = 0; e < 16; ++e) csx[e] += __shfl_xor(csx[e], o, 64);
    if ((lane & 15) == 0) {
      float* row = p.colsum_gx + (long)(pid * NW + wave) * CO + 64 * wave + 4 * (lane >> 4);
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        *reinterpret_cast<float4*>(row + 16 * jb) = make_float4(csx[4 * jb], csx[4 * jb + 1], csx[4 * jb + 2], csx[4 * jb + 3]);
    }
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
      unsafeAtomicAdd(p.dw + (long)co * p.ld_dw + half * CB + lane, stage[r * LDF + lane]);
    }
    __syncthreads();
  }
}

}  // namespace

// Launch geometry: (workgroups, pairs).  NW = 4 (CO 256): two per CU, one per tile column
// block; NW = 8 (CO 512, CI 128): one per CU, as pairs (a multiple of 8 pairs: the XCD pairing).
static void bwd1x1_geom(int M, int CO, int CI, int* grid, int* np) {
  const long T = (M + B1_MT - 1) / B1_MT;
  if (CO == 256) {
    const long G = 2L * num_cus();
    *np = *grid = (int)(T < G ? T : G);
    return;
  }
  long P = (num_cus() / 2) / 8 * 8;
  if (P < 8) P = 8;
  *np = (int)P;
  *grid = (int)(P * (CI / 64));
}
int bwd1x1_partial_rows(int M, int CO, int CI) {
  int grid, np;
  bwd1x1_geom(M, CO, CI, &grid, &np);
  return np * (CO == 256 ? 4 : 8);
}

const char* bwd1x1_launch(const Bwd1x1Params& p, hipStream_t stream) {
  if (p.M <= 0) return "bwd1x1: empty problem";
  if (!((p.CO == 256 && p.CI == 64) || (p.CO == 512 && p.CI == 128))) return "bwd1x1: (CO, CI) must be (256, 64) or (512, 128)";
  if ((long)p.M * p.CO >= (1L << 31)) return "bwd1x1: gradient has more than 2^31 elements";
  if (p.ld_wd < p.CO || p.ld_wd % 8 || p.ld_dw < p.CI) return "bwd1x1: weight / gradient row strides";
  int grid, np;
  bwd1x1_geom(p.M, p.CO, p.CI, &grid, &np);
  if (p.s2 && (!p.out2 || p.Hc != (p.Hf + 1) / 2 || p.Wc != (p.Wf + 1) / 2 || (long)p.N * p.Hc * p.Wc != p.M))
    return "bwd1x1: stride-2 grid geometry";
  Bwd1x1Params q = p;
  if (q.s2) { q.mg_hwc = fdiv_magic(q.Hc * q.Wc); q.mg_wc = fdiv_magic(q.Wc); }
  if (q.g1) {
    if (q.CO != 256 || q.s2 || !q.w1d || !q.gmask || !q.gx || !q.colsum_gx) return "bwd1x1: pre form operands";
    // (partial rows of other waves' columns stay zero: every row is written by exactly one wave's
    // 64 columns)
    (void)hipMemsetAsync(q.colsum_gx, 0, (size_t)np * 4 * 256 * sizeof(float), stream);
    hipLaunchKernelGGL((bwd1x1_kernel<256, 4, false, true>), dim3(grid), dim3(256), 0, stream, q);
  } else if (q.CO == 256) {
    if (q.s2) hipLaunchKernelGGL((bwd1x1_kernel<256, 4, true>), dim3(grid), dim3(256), 0, stream, q);
    else hipLaunchKernelGGL((bwd1x1_kernel<256, 4, false>), dim3(grid), dim3(256), 0, stream, q);
  } else {
    if (q.s2) hipLaunchKernelGGL((bwd1x1_kernel<512, 8, true>), dim3(grid), dim3(512), 0, stream, q);
    else hipLaunchKernelGGL((bwd1x1_kernel<512, 8, false>), dim3(grid), dim3(512), 0, stream, q);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
