// Weight-gradient of the implicit-GEMM convolution on MFMA (gfx950).
//
//   dW[co, k] += sum_m g[m, co] * im2col(x)[m, k]        (k = (r, s, c), c fastest)
//
// Reference parity: the backward-filter half of every Keras Conv2D / Dense weight update
// (ResourceApplyAdam consumes these, imagenet-resnet50.py:62); SURVEY.md §2.4 N3.
//
// Both operands are row-major along the reduction axis m in NHWC memory (g is [M][Cout],
// x rows are [M][K]), which is the "TN" GEMM case.  Instead of transposing in memory, the
// tiles are staged lane-linearly into LDS as [m][col] by 16-byte LDS-DMA and read with the
// gfx950 transposing LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10): one
// read gives a lane 4 consecutive m for one column, two reads give the 8-deep k fragment of
// a 16x16x32 bf16 MFMA operand.
//
// The reduction over M = N*Ho*Wo (up to 800k rows) is split across workgroups; partial
// tiles go through LDS and are added with row-contiguous (256 B per wave instruction)
// no-return fp32 atomics into the flat fp32 gradient buffer (MI355X_MICROARCH.md "Global
// float atomics": ~1.3 TB/s chip-wide, so splits are sized to keep atomic bytes small).
#include <array>
#include <map>
#include <mutex>

#include "common.h"
#include "kernels.h"

namespace pddl {

// Bank-conflict swizzle for the [m][128 x bf16] (256-byte row) images: the 8 rows a
// 32-lane half of ds_read_b64_tr_b16 touches get distinct even chunk XORs, so the 16
// 16-byte chunks they read cover all 64 banks exactly once.
__device__ __forceinline__ int tr_swz(int row) { return ((row & 3) | ((row >> 1) & 4)) << 1; }
// Same property for [m][64 x bf16] (128-byte row) images: two rows share a 256-byte bank
// row, so the even/odd rows of a half take chunk XORs {0,2,4,6} within their 8 chunks.
__device__ __forceinline__ int tr_swz128(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }

// BM = 128: 2x2 waves, wave tile 64 (co) x 64 (k).  BM = 64 (Cout = 64 layers: the stem and
// stage 2): 1x4 waves, wave tile 64 x 32, gradient tile with 128-byte rows.
// ds_read_b64_tr_b16 as inline asm: the builtin form makes the compiler drain every LDS-DMA
// load in flight (vmcnt(0)) before each transposed read, which serialises the staging pipeline;
// the asm form is invisible to its wait insertion, so the kernel waits itself (lgkmcnt(0) before
// the MFMAs that consume the fragments).
__device__ __forceinline__ v4bf tr_read(const char* p) {
  v4bf r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}

// NSTAGE: LDS buffers.  2: the next m-tile's LDS-DMA overlaps this tile's MFMAs; 1: load ->
// compute -> load in one buffer at half the LDS, so more blocks share a CU and overlap each
// other's phases instead (measured faster on the short / narrow layers, knob wgrad1).
template <bool FAST, int BM, int NSTAGE>
__global__ void __launch_bounds__(256, 2) wgrad_kernel(WgradParams p, int m_per_split, const int2* __restrict__ rowinfo) {
  constexpr int G_BYTES = 64 * BM * 2;        // 64 m-rows x BM bf16
  constexpr int X_BYTES = 64 * 256;           // 64 m-rows x 128 bf16
  constexpr int STAGE = G_BYTES + X_BYTES;
  constexpr int WAVES_N = BM == 128 ? 2 : 4;
  constexpr int WTN = 128 / WAVES_N;          // k columns per wave
  constexpr int TN = WTN / 16;
  constexpr int EPI_LD = WTN + 4;
  constexpr int GI = G_BYTES / 4096;          // 1 KiB G pieces per wave
  constexpr int EPI_BYTES = 4 * 32 * EPI_LD * 4;
  constexpr int SMEM = NSTAGE * STAGE > EPI_BYTES ? NSTAGE * STAGE : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tco = (p.Cout + BM - 1) / BM, tk = (p.K + 127) / 128, ntiles = tco * tk;
  const int splits = (p.M + m_per_split - 1) / m_per_split;
  const int wg = xcd_remap(blockIdx.x, ntiles * splits);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int co0 = (tile % tco) * BM, k0 = (tile / tco) * 128;
  const int mbeg = split * m_per_split;
  const int mend = min(p.M, mbeg + m_per_split);

  // buffer descriptors: 32-bit lane offsets, the m-step in the scalar soffset, and
  // out-of-range offsets (padding taps, tile overhang) load zeros.  They are rebased at the
  // split's first row (gradient, 1x1 input) or first image (gathered input), so the offsets
  // span one split whatever the batch (the launcher bounds the split span).
  const int pix0 = FAST ? 0 : (mbeg / (p.Ho * p.Wo)) * p.H * p.W;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_at(p.g, (long)mbeg * p.ldg, (long)p.M * p.ldg);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_at(p.x, FAST ? (long)mbeg * p.ldx : (long)pix0 * p.C,
                                                 FAST ? (long)p.M * p.ldx : (long)p.N * p.H * p.W * p.C);

  // (r, s, c0) of the two 64-column halves of this k tile (generic path only).
  int hr[2], hs[2], hc[2]; bool hv[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kk = k0 + h * 64;
    hv[h] = kk < p.K;
    const int rs = kk / p.C; hc[h] = kk - rs * p.C; hr[h] = rs / p.S; hs[h] = rs - hr[h] * p.S;
  }

  // Loader lane geometry: piece i of wave w covers rows (w*4+i)*4 .. +3, 16 chunks per row.
  const int lrow = lane >> 4, lpos = lane & 15;
  // loop-invariant lane offsets of the gradient pieces (relative to row mb) and their source
  uint32_t g_off[GI]; int g_row[GI];
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    int row, chunk;
    if (BM == 128) { row = (wave * GI + i) * 4 + lrow; chunk = lpos ^ tr_swz(row); }
    else { row = (wave * GI + i) * 8 + (lane >> 3); chunk = (lane & 7) ^ tr_swz128(row); }
    const int co = co0 + chunk * 8;
    g_row[i] = row;
    g_off[i] = co >= p.Cout ? OOB_OFF : (uint32_t)((row * p.ldg + co) * 2);
  }
  uint32_t x_off[4];   // FAST: loop-invariant input offsets
  int x_delta[4], x_tap[4];   // generic: per-piece element shift of the lane's (r, s, c) and tap bit
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 4 + lrow;
    const int chunk = lpos ^ tr_swz(row);
    const int kc = k0 + chunk * 8;
    x_off[i] = (FAST && kc < p.K) ? (uint32_t)((row * p.ldx + kc) * 2) : OOB_OFF;
    const int h = chunk >> 3;
    const int r = h ? hr[1] : hr[0], s = h ? hs[1] : hs[0], c = h ? hc[1] : hc[0];
    x_delta[i] = (r * p.W + s) * p.C + c + (chunk & 7) * 8;
    x_tap[i] = (h ? hv[1] : hv[0]) ? r * p.S + s : 31 + 1;   // bit 32: never set -> zero
  }
  // Generic path: the im2col row geometry comes from a per-layer table rowinfo[m] =
  // {pixel index of tap (0, 0), bitmask of in-bounds taps}, prefetched one tile ahead into
  // registers (4 rows per lane), so the gather costs a mask test and one multiply-add.
  int2 ri[4];
  auto fetch_rows = [&](int mb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(mb + (wave * 4 + i) * 4 + lrow, p.M - 1);
      ri[i] = rowinfo[m];
    }
  };

  auto load_tile = [&](int mb, int buf) {
    char* gb = smem + buf * STAGE;
    char* xb = gb + G_BYTES;
    const bool full = mb + 64 <= mend;   // scalar: only the split's last tile has dead rows
#pragma unroll
    for (int i = 0; i < GI; ++i) {  // gradient operand
      const uint32_t off = (full || mb + g_row[i] < mend) ? g_off[i] : OOB_OFF;
      buf_lds16(rg, LDS_PTR(gb + (wave * GI + i) * 1024), off, (mb - mbeg) * p.ldg * 2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // input operand
      const int row = (wave * 4 + i) * 4 + lrow;
      const bool mok = full || mb + row < mend;
      if (FAST) {
        buf_lds16(rx, LDS_PTR(xb + (wave * 4 + i) * 1024), mok ? x_off[i] : OOB_OFF, (mb - mbeg) * p.ldx * 2);
      } else {
        const bool ok = mok && x_tap[i] < 32 && ((ri[i].y >> x_tap[i]) & 1);
        const uint32_t off = ok ? (uint32_t)(((ri[i].x - pix0) * p.C + x_delta[i]) * 2) : OOB_OFF;
        buf_lds16(rx, LDS_PTR(xb + (wave * 4 + i) * 1024), off, 0);
      }
    }
    if (!FAST) fetch_rows(mb + 64);   // next tile's rows (landed by the loop's vmcnt(0))
  };

  v4f acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // Fragment-read lane geometry (T10): group G = lane>>4 reads rows 8G + 4h + q, q = (lane&15)>>2,
  // columns 4p..4p+3, p = lane&3.
  const int G = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int nit = (mend - mbeg + 63) / 64;
  if (nit > 0) {
    if (!FAST) fetch_rows(mbeg);
    load_tile(mbeg, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int it = 0; it < nit; ++it) {
    const int cur = NSTAGE == 2 ? (it & 1) : 0;
    if (NSTAGE == 2 && it + 1 < nit) load_tile(mbeg + (it + 1) * 64, cur ^ 1);
    const char* gb = smem + cur * STAGE;
    const char* xb = gb + G_BYTES;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      int roff[2], rsw[2], goff[2], gsw[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int row = kh * 32 + 8 * G + 4 * h2 + q;
        roff[h2] = row * 256 + (pp & 1) * 8;
        rsw[h2] = tr_swz(row);
        goff[h2] = row * (BM * 2) + (pp & 1) * 8;
        gsw[h2] = BM == 128 ? rsw[h2] : tr_swz128(row);
      }
      v8bf af[4], bfr[TN];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ch = wm * 8 + i * 2 + (pp >> 1);
        v4bf lo = tr_read(gb + goff[0] + ((ch ^ gsw[0]) << 4));
        v4bf hi = tr_read(gb + goff[1] + ((ch ^ gsw[1]) << 4));
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int ch = wn * (WTN / 8) + j * 2 + (pp >> 1);
        v4bf lo = tr_read(xb + roff[0] + ((ch ^ rsw[0]) << 4));
        v4bf hi = tr_read(xb + roff[1] + ((ch ^ rsw[1]) << 4));
        bfr[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (the asm fragment reads)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (NSTAGE == 1 && it + 1 < nit) {
      __syncthreads();            // every wave is done reading the single buffer
      load_tile(mbeg + (it + 1) * 64, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nit == 0) return;

  // Epilogue: per-wave 32 x WTN fp32 staging, then row-contiguous atomics (256 B per wave
  // instruction: one 64-float row, or two 32-float rows for WTN = 32).
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * EPI_LD);
  constexpr int RPA = 64 / WTN;  // rows per atomic instruction
  const int kcol = k0 + wn * WTN + (lane % WTN);
  const int rsub = lane / WTN;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          stage[(i2 * 16 + (lane >> 4) * 4 + jj) * EPI_LD + j * 16 + (lane & 15)] = acc[pass * 2 + i2][j][jj];
    __syncthreads();
    if (kcol < p.K) {
      for (int r = 0; r < 32; r += RPA) {
        const int co = co0 + wm * 64 + pass * 32 + r + rsub;
        if (co < p.Cout)
          unsafeAtomicAdd(p.dw + (long)co * p.ld_dw + kcol, stage[(r + rsub) * EPI_LD + (lane % WTN)]);
      }
    }
    __syncthreads();
  }
}


// ---------------------------------------------------------------------------------------
// 8-phase 256 (co) x 256 (k) weight gradient: the igemm8_kernel schedule (igemm.hip) on the
// transposed-operand GEMM.  8 waves, one 128 KiB block per CU; per 64-row m-tile four 16 KiB
// half-tiles {G cols 0-127, X cols 0-127, X cols 128-255, G cols 128-255} ([64 m][128] bf16,
// tr_swz-swizzled rows) staged LEAD = 5 halves ahead with counted vmcnt and raw barriers; each
// m-tile is reduced in 4 phases over the 128x128 output quadrants in snake order (every wave
// owns a 64 (co) x 32 (k) sub-tile of each quadrant: 16 MFMAs per phase), fragments read with
// ds_read_b64_tr_b16 as in wgrad_kernel.  The m reduction is split over workgroups sized to one
// block per CU and the fp32 partial tiles are added with row-contiguous atomics.  The generic
// (padded / strided) gather decodes each row's im2col geometry arithmetically (magic-number
// division) when its m-tile is staged: an ordinary global load of a row table would make the
// compiler drain the LDS-DMA queue (vmcnt(0)) at its first use.
// Host-computed im2col stepping of wgrad8_kernel's generic gather (64 rows per m-tile).
struct Wg8Geom {
  uint64_t mg_howo, mg_wo;   // magic divisors for the starting row of a split
  int dho, dwo, dpix;        // 64 rows as (output rows, output cols) and the tap-(0,0) pixel delta
  int carry_w, carry_h;      // pixel delta of a column -> row carry and of a row -> image carry
  uint32_t row_unit;         // bit r*S for every kernel row r
};

template <bool FAST, bool STAGGER>
__global__ void __launch_bounds__(512, 1) wgrad8_kernel(WgradParams p, int m_per_split, Wg8Geom geo, int probe) {
  constexpr int HALF = 16384, BUF = 4 * HALF, LEAD = 5;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tco = (p.Cout + 255) / 256, tk = (p.K + 255) / 256, ntiles = tco * tk;
  const int splits = (p.M + m_per_split - 1) / m_per_split;
  const int wg = xcd_remap(blockIdx.x, ntiles * splits);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int co0 = (tile % tco) * 256, k0 = (tile / tco) * 256;
  const int mbeg = split * m_per_split;
  const int mend = min(p.M, mbeg + m_per_split);
  const int nit = (mend - mbeg + 63) / 64;
  if (nit <= 0) return;   // (block-uniform, before any barrier)
  // descriptors rebased at the split's first row / first image (as in wgrad_kernel)
  const int n_first = FAST ? 0 : fdiv(mbeg, geo.mg_howo);
  const long pix0 = (long)n_first * p.H * p.W;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_at(p.g, (long)mbeg * p.ldg, (long)p.M * p.ldg);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_at(p.x, FAST ? (long)mbeg * p.ldx : pix0 * p.C,
                                                 FAST ? (long)p.M * p.ldx : (long)p.N * p.H * p.W * p.C);

  // staging lanes: piece i of a half covers m-rows (2*wave + i)*4 .. +3, 16 chunks per row
  const int lrow = lane >> 4, lpos = lane & 15;
  int prow[2], pch[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    prow[i] = (2 * wave + i) * 4 + lrow;
    pch[i] = lpos ^ tr_swz(prow[i]);
  }
  uint32_t g_off[2][2], x_off[2][2], x_bit[2][2];
  int x_delta2[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = co0 + 128 * h + pch[i] * 8;
      g_off[h][i] = co >= p.Cout ? OOB_OFF : (uint32_t)((prow[i] * p.ldg + co) * 2);
      const int kc = k0 + 128 * h + pch[i] * 8;
      x_off[h][i] = (FAST && kc < p.K) ? (uint32_t)((prow[i] * p.ldx + kc) * 2) : OOB_OFF;
      const int kk = k0 + 128 * h + (pch[i] >> 3) * 64;   // the lane's 64-column sub-half
      const int rs = kk / p.C, c0 = kk - rs * p.C, r = rs / p.S, s = rs - r * p.S;
      x_delta2[h][i] = ((r * p.W + s) * p.C + c0 + (pch[i] & 7) * 8) * 2;
      x_bit[h][i] = kk < p.K ? 1u << (r * p.S + s) : 0u;   // the lane's tap in a row's valid-tap mask
    }
  // generic gather: each lane stages 2 rows of every m-tile (m = mb + prow[i]).  Their im2col
  // geometry -- output position (ho, wo) and the input pixel of tap (0, 0) -- advances by 64
  // rows per m-tile with mixed-radix carries (host-computed steps, no divisions or full-rate
  // multiplies in the loop); the valid-tap mask follows from the window's clipped row / column
  // ranges: (column bits) x (row-start bits of the valid rows).
  int gho[2] = {0, 0}, gwo[2] = {0, 0}, gpix[2] = {0, 0};
  int rpix2[2] = {0, 0};
  uint32_t rmask[2] = {0u, 0u};
  if (!FAST) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = mbeg + prow[i];
      const int n = fdiv(m, geo.mg_howo), rem = m - n * p.Ho * p.Wo;
      gho[i] = fdiv(rem, geo.mg_wo);
      gwo[i] = rem - gho[i] * p.Wo;
      gpix[i] = ((n - n_first) * p.H + gho[i] * p.stride - p.pad) * p.W + gwo[i] * p.stride - p.pad;
    }
  }
  auto row_geometry = [&](int mb) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int hi = __mul24(gho[i], p.stride) - p.pad, wi = __mul24(gwo[i], p.stride) - p.pad;
      const int rmin = max(0, -hi), rmax = min(p.R, p.H - hi);
      const int cmin = max(0, -wi), cmax = min(p.S, p.W - wi);
      const uint32_t cols = (cmax > cmin) ? (~0u >> (32 - cmax)) & ~((1u << cmin) - 1u) : 0u;
      const uint32_t rows = (rmax > rmin) ? geo.row_unit & (~0u >> (32 - rmax * p.S)) & ~((1u << (rmin * p.S)) - 1u) : 0u;
      rmask[i] = mb + prow[i] < mend ? cols * rows : 0u;
      rpix2[i] = __mul24(gpix[i], 2 * p.C);
      // advance to the next m-tile (64 rows)
      gwo[i] += geo.dwo;
      gho[i] += geo.dho;
      gpix[i] += geo.dpix;
      if (gwo[i] >= p.Wo) { gwo[i] -= p.Wo; gho[i] += 1; gpix[i] += geo.carry_w; }
      if (gho[i] >= p.Ho) { gho[i] -= p.Ho; gpix[i] += geo.carry_h; }
    }
  };
  const int NH = 4 * nit;
  // half-tile j = 4 t + part of m-tile t: part 0 G cols 0-127, 1 X cols 0-127, 2 X cols 128-255,
  // 3 G cols 128-255 (first read in phases 0, 0, 1, 2 of the tile, as in igemm8_kernel)
  auto stage_half = [&](int j, int part) {
    const int mb = mbeg + (j >> 2) * 64;
    char* base = smem + ((j >> 2) & 1) * BUF;
    const bool full = mb + 64 <= mend;
    if (part == 0 || part == 3) {
      const int h = part == 0 ? 0 : 1;
      char* hb = base + (part == 0 ? 0 : 3) * HALF;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t off = (full || mb + prow[i] < mend) ? g_off[h][i] : OOB_OFF;
        buf_lds16(rg, LDS_PTR(hb + (2 * wave + i) * 1024), off, (mb - mbeg) * p.ldg * 2);
      }
    } else {
      const int h = part == 1 ? 0 : 1;
      char* hb = base + part * HALF;
      if (!FAST && part == 1) row_geometry(mb);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (FAST) {
          const bool mok = full || mb + prow[i] < mend;
          buf_lds16(rx, LDS_PTR(hb + (2 * wave + i) * 1024), mok ? x_off[h][i] : OOB_OFF, (mb - mbeg) * p.ldx * 2);
        } else {
          const uint32_t off = (rmask[i] & x_bit[h][i]) ? (uint32_t)(rpix2[i] + x_delta2[h][i]) : OOB_OFF;
          buf_lds16(rx, LDS_PTR(hb + (2 * wave + i) * 1024), off, 0);
        }
      }
    }
  };
#define WG8_WAIT_BARRIER(need, last)                                                              \
  {                                                                                               \
    const int after_ = (last) - (need);                                                           \
    if (after_ >= 3) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");                \
    else if (after_ == 2) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");           \
    else if (after_ == 1) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");           \
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");                            \
  }

  v4f acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = v4f{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int j = 0; j < LEAD; ++j)
    if (j < NH) stage_half(j, j & 3);
  {
    const int last = (LEAD < NH ? LEAD : NH) - 1;
    WG8_WAIT_BARRIER(1, last)
  }
  if (STAGGER && wm == 1) asm volatile("s_barrier" ::: "memory");

  // fragment-read geometry (T10): group G = lane>>4 reads m-rows 8G + 4h + q, q = (lane&15)>>2,
  // columns 4p..4p+3 of its 8-column chunk, p = lane&3
  const int Gq = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  int roff[2][2], rsw[2][2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int row = kh * 32 + 8 * Gq + 4 * h2 + qq;
      roff[kh][h2] = row * 256 + (pp & 1) * 8;
      rsw[kh][h2] = tr_swz(row);
    }
  v8bf af[2][4], bfr[2][2];
  for (int t = 0; t < nit; ++t) {
    const char* buf = smem + (t & 1) * BUF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qm = (q == 0 || q == 1) ? 0 : 1;
      const int qn = (q == 0 || q == 3) ? 0 : 1;
      const bool loadA = (q == 0 || q == 2), loadB = (q != 2);
      if (loadB) {
        const char* Xs = buf + (qn == 0 ? 1 : 2) * HALF;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int ch = wn * 4 + j * 2 + (pp >> 1);
            v4bf lo = tr_read(Xs + roff[kh][0] + ((ch ^ rsw[kh][0]) << 4));
            v4bf hi = tr_read(Xs + roff[kh][1] + ((ch ^ rsw[kh][1]) << 4));
            bfr[kh][j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (loadA) {
        const char* Gs = buf + (qm == 0 ? 0 : 3) * HALF;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int ch = wm * 8 + i * 2 + (pp >> 1);
            v4bf lo = tr_read(Gs + roff[kh][0] + ((ch ^ rsw[kh][0]) << 4));
            v4bf hi = tr_read(Gs + roff[kh][1] + ((ch ^ rsw[kh][1]) << 4));
            af[kh][i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
      }
      const int js = 4 * t + q + LEAD;
      if (js < NH) stage_half(js, (q + LEAD) & 3);
      const int last = (js < NH ? js : NH - 1);
      if (q == 0) WG8_WAIT_BARRIER(4 * t + 2, last)
      else if (q == 1) WG8_WAIT_BARRIER(4 * t + 3, last)
      else if (q == 3 && t + 1 < nit) WG8_WAIT_BARRIER(4 * t + 5, last)
      else asm volatile("s_barrier" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (the asm fragment reads)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qm][qn][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kh][i], bfr[kh][j], acc[qm][qn][i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
    }
  }
#undef WG8_WAIT_BARRIER
  if (STAGGER && wm == 0) asm volatile("s_barrier" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (probe & 1) {   // (timing probe only: main loop without the atomic epilogue)
    if (acc[0][0][0][0][0] == 12345.f && acc[1][1][3][1][3] == 54321.f) p.dw[tid] = 0.f;
    return;
  }

  // epilogue: per quadrant, the wave's 64 x 32 partial tile through LDS (2 passes of 32 rows),
  // then row-contiguous atomics: 2 rows of 32 floats (2 x 128 B) per wave instruction
  constexpr int EPI_LD = 36;
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * EPI_LD);
  const int rsub = lane >> 5, cl = lane & 31;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn) {
      const int kcol = k0 + qn * 128 + wn * 32 + cl;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              stage[(i2 * 16 + (lane >> 4) * 4 + jj) * EPI_LD + j * 16 + (lane & 15)] = acc[qm][qn][pass * 2 + i2][j][jj];
        __syncthreads();
        if (kcol < p.K) {
          for (int r = 0; r < 32; r += 2) {
            const int co = co0 + qm * 128 + wm * 64 + pass * 32 + r + rsub;
            if (co < p.Cout) unsafeAtomicAdd(p.dw + (long)co * p.ld_dw + kcol, stage[(r + rsub) * EPI_LD + cl]);
          }
        }
        __syncthreads();
      }
    }
}

// rowinfo[m] = {(n*H + ho*stride - pad)*W + wo*stride - pad, bit (r*S + s) set iff tap (r, s)
// of output row m reads inside the image}.
__global__ void rowinfo_kernel(int2* __restrict__ out, int M, int Ho, int Wo, int H, int W, int stride, int pad,
                               int R, int S) {
  for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < M; m += gridDim.x * blockDim.x) {
    const int n = m / (Ho * Wo), rem = m - n * Ho * Wo, ho = rem / Wo, wo = rem - ho * Wo;
    const int hi = ho * stride - pad, wi = wo * stride - pad;
    uint32_t mk = 0;
    for (int r = 0; r < R; ++r)
      for (int s = 0; s < S; ++s)
        if ((unsigned)(hi + r) < (unsigned)H && (unsigned)(wi + s) < (unsigned)W) mk |= 1u << (r * S + s);
    out[m] = make_int2((n * H + hi) * W + wi, (int)mk);
  }
}

// One table per (device, geometry), built on first use on the caller's stream and kept for
// the process lifetime (a handful of geometries per network; first use must not be inside a
// graph capture -- the engines always run one eager step first).
static const int2* rowinfo_for(const WgradParams& p, hipStream_t stream, const char** why) {
  static std::mutex mu;
  static std::map<std::array<int, 10>, int2*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  const std::array<int, 10> key{dev, p.M, p.Ho, p.Wo, p.H, p.W, p.stride, p.pad, p.R, p.S};
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int2* buf = nullptr;
  if (hipMalloc(&buf, sizeof(int2) * (size_t)p.M) != hipSuccess) { *why = "wgrad: rowinfo allocation failed"; return nullptr; }
  hipLaunchKernelGGL(rowinfo_kernel, dim3((p.M + 255) / 256 < 8192 ? (p.M + 255) / 256 : 8192), dim3(256), 0, stream,
                     buf, p.M, p.Ho, p.Wo, p.H, p.W, p.stride, p.pad, p.R, p.S);
  // The table is shared by every stream of the device (engines of several replicas, side
  // streams), so it must be complete before any other caller gets the pointer: finish the
  // build here, under the lock.  (Without this a second engine on another stream read a table
  // still being written -- a 1-GPU Mirrored rehearsal with two replicas in threads.)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
    if (hipStreamSynchronize(stream) != hipSuccess) { *why = "wgrad: rowinfo build failed"; return nullptr; }
  }
  cache[key] = buf;
  return buf;
}

int g_wgrad1 = 1;          // LDS stages of the 128/64-wide wgrad kernel: 1 = single stage except the
                           // long-reduction direct layers and grids of at most one block per CU (1x1 / stem window, M >= 2M rows: stage-2
                           // 1x1s -4..-12 %, stem -8 %, 3x3 and stage 3+ +8..+13 % with 2 stages;
                           // per-layer A/B at b1024), 0 = 2 stages everywhere, 2 = single everywhere
int g_wgrad8 = 1;          // 8-phase 256x256 wgrad8_kernel for Cout >= 256, K >= 256: 0 off, 1 on where its grid
                           // each block's reduction amortises its atomic burst (wgrad_launch_one), 2 with the wave-row stagger (slower here);
                           // +8 (probe): skip the atomic epilogue; +16: whatever the grid

int g_wgrad8_min_rows = 512;    // wgrad8 m-reduction split: at least this many rows per split (knob;
                                // b32: 1024 -> 512 rows 5.32 -> 5.06 ms/step, 256: 5.26)

static const char* wgrad_launch_one(const WgradParams& pin, hipStream_t stream);

// A second gradient source (rows >= co_split of dW: projection blocks, where conv1 and the
// shortcut conv share the input) runs as its own launch over the same input, so every
// tile reads one descriptor-addressed gradient.
const char* wgrad_launch(const WgradParams& pin, hipStream_t stream) {
  if (!pin.g2) return wgrad_launch_one(pin, stream);
  if (pin.co_split <= 0 || pin.co_split >= pin.Cout) return "wgrad: co_split out of range";
  WgradParams a = pin, b = pin;
  a.g2 = nullptr; a.Cout = pin.co_split;
  b.g2 = nullptr; b.g = pin.g2; b.ldg = pin.ldg2; b.Cout = pin.Cout - pin.co_split;
  b.dw = pin.dw + (long)pin.co_split * pin.ld_dw;
  const char* e = wgrad_launch_one(a, stream);
  return e ? e : wgrad_launch_one(b, stream);
}

static const char* wgrad_launch_one(const WgradParams& pin, hipStream_t stream) {
  WgradParams p = pin;
  const bool fast = (p.R == 1 && p.S == 1 && p.stride == 1 && p.pad == 0);
  // window form (space-to-depth stem): S taps x C channels = 64 contiguous elements
  const bool window = (p.C * p.S == 64) && p.stride == 1 && p.pad == 0;
  if (!fast && p.C % 64 && !window) return "wgrad: C must be a multiple of 64 for the gather path";
  if (p.Cout % 8 || p.ldg % 8 || (fast && p.ldx % 8)) return "wgrad: Cout / ldg / ldx must be multiples of 8";
  if (p.M <= 0 || p.Cout <= 0 || p.K <= 0) return "wgrad: empty problem";
  if (!fast && p.R * p.S > 32) return "wgrad: at most 32 taps";
  // element indices are ints; buffer byte offsets are 31-bit (0x80000000 marks out-of-range
  // lanes) relative to each split's first row / image (the kernels rebase their descriptors
  // there), so only one split's span has to fit
  if ((long)p.N * p.H * p.W * p.C >= (1L << 31) || (long)p.M * p.ldg >= (1L << 31) ||
      (fast && (long)p.M * p.ldx >= (1L << 31)))
    return "wgrad: tensor has more than 2^31 elements";
  const long HoWo = (long)p.Ho * p.Wo;
  auto span_pix = [&](int mps) { return ((mps + 64) / HoWo + 2) * p.H * p.W; };
  auto span_ok = [&](int mps) {
    const long rows = mps + 64;
    const long xs = fast ? rows * p.ldx : span_pix(mps) * p.C;
    return xs * 2 < (1L << 31) - (1L << 24) && rows * p.ldg * 2 < (1L << 31) - (1L << 24);
  };
  // 128-wide tiles (4 waves, 2 blocks per CU): the m-split plan.
  const int BM = p.Cout <= 64 ? 64 : 128;
  const int ntiles = ((p.Cout + BM - 1) / BM) * ((p.K + 127) / 128);
  int splits = p.splits;
  if (splits <= 0) {
    // Every split adds one 64 KiB fp32 atomic tile (~1.3 TB/s chip-wide), so a workgroup
    // should own >= ~48 m-iterations (3072 rows); but keep >= 256 workgroups when the
    // tile count alone cannot fill the 256 CUs.
    const int fill = (1536 + ntiles - 1) / ntiles;
    const int work = (p.M + 3071) / 3072;
    splits = fill < work ? fill : work;
    if ((long)ntiles * splits < 256) {
      const int f2 = (256 + ntiles - 1) / ntiles, w2 = (p.M + 511) / 512;
      splits = f2 < w2 ? f2 : w2;
    }
    if (splits < 1) splits = 1;
  }
  int mps = (p.M + splits - 1) / splits;
  mps = (mps + 63) / 64 * 64;
  while (!span_ok(mps) && mps > 64) mps = (mps / 2 + 63) / 64 * 64;   // (batches beyond ~1.5k)
  const bool plan1_ok = span_ok(mps);
  splits = (p.M + mps - 1) / mps;
  const int nwg = ntiles * splits;

  // 8-phase 256x256 tiles (one block per CU): split the m reduction so tiles x splits ~ one
  // round of CUs, each split at least g_wgrad8_min_rows rows.
  const int nt8 = ((p.Cout + 255) / 256) * ((p.K + 255) / 256);
  int sp = (num_cus() + nt8 / 2) / nt8;
  const int cap = (p.M + g_wgrad8_min_rows - 1) / g_wgrad8_min_rows;
  if (sp > cap) sp = cap;
  if (sp < 1) sp = 1;
  const int mps8 = ((p.M + sp - 1) / sp + 63) / 64 * 64;
  sp = (p.M + mps8 - 1) / mps8;
  // (the generic gather steps pixel indices through 24-bit multiplies: < 2^22 pixels per split)
  const bool elig8 = g_wgrad8 && p.Cout >= 256 && p.K >= 256 && !window && p.splits <= 0 && span_ok(mps8) &&
                     (fast || (span_pix(mps8) < (1L << 22) && 2L * p.C < (1L << 23)));
  // Which tiling.  Every 8-phase block ends with a burst of fp32 atomics of its 256 KiB partial
  // tile, and one round of blocks (one per CU) is ~64 MiB of atomics at the chip's ~1.3 TB/s
  // atomic rate (MI355X_MICROARCH.md "Global float atomics"): ~50 us that no block's MFMA work
  // overlaps, since the blocks finish together (wgrad8=9 probe: 48-51 us of a 84-124 us layer at
  // b256, 17-26 us of 340-740 at b2560; scripts/wgrad_probe.sh).  The 8-phase tiles pay off when
  // each block's reduction is long enough to amortise that burst -- >= 0.4 GFLOP per block
  // (~47 us of MFMA work) -- and the grid covers at least half the CUs; otherwise the 128-wide
  // tiles (64 KiB partials, 2 blocks per CU) win: b256 whole step 11.72 -> 11.03 ms, b32 3.95 ->
  // 3.85 ms, b1024 / b2560 unchanged (profiles/r5_b32_wgrad_ab.txt, profiles/r5_b256_wgrad_ab.txt).
  bool use8 = false;
  if (elig8) {
    const double F = 2.0 * p.M * (double)p.Cout * p.K, w8 = (double)nt8 * sp;
    use8 = (g_wgrad8 & 16) || !plan1_ok || (F >= 4e8 * w8 && 2 * w8 >= num_cus());
  }
  if (use8) {
    const int mps = mps8;
    Wg8Geom geo{};
    geo.mg_howo = fdiv_magic(p.Ho * p.Wo);
    geo.mg_wo = fdiv_magic(p.Wo);
    {
      const int HoWo = p.Ho * p.Wo, dn = 64 / HoWo, rem = 64 % HoWo;
      geo.dho = rem / p.Wo;
      geo.dwo = rem % p.Wo;
      geo.dpix = dn * p.H * p.W + geo.dho * p.stride * p.W + geo.dwo * p.stride;
      geo.carry_w = p.stride * p.W - p.Wo * p.stride;
      geo.carry_h = p.H * p.W - p.Ho * p.stride * p.W;
      for (int r = 0; r < p.R; ++r) geo.row_unit |= 1u << (r * p.S);
    }
    if ((g_wgrad8 & 7) == 2) {
      if (fast) hipLaunchKernelGGL((wgrad8_kernel<true, true>), dim3(nt8 * sp), dim3(512), 0, stream, p, mps, geo, g_wgrad8 >> 3);
      else hipLaunchKernelGGL((wgrad8_kernel<false, true>), dim3(nt8 * sp), dim3(512), 0, stream, p, mps, geo, g_wgrad8 >> 3);
    } else {
      if (fast) hipLaunchKernelGGL((wgrad8_kernel<true, false>), dim3(nt8 * sp), dim3(512), 0, stream, p, mps, geo, g_wgrad8 >> 3);
      else hipLaunchKernelGGL((wgrad8_kernel<false, false>), dim3(nt8 * sp), dim3(512), 0, stream, p, mps, geo, g_wgrad8 >> 3);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? nullptr : hipGetErrorString(e);
  }
  if (!plan1_ok) return "wgrad: one 64-row tile spans more than 2 GiB";
  // 2 LDS stages + 2 blocks/CU (a 3-stage ring at 1 block/CU measured slower and was removed)
  const int2* ri = nullptr;
  if (!fast) {
    const char* why = nullptr;
    ri = rowinfo_for(p, stream, &why);
    if (!ri) return why;
  }
#define WG_LAUNCH(F_, BM_, NS_) hipLaunchKernelGGL((wgrad_kernel<F_, BM_, NS_>), dim3(nwg), dim3(256), 0, stream, p, mps, ri);
  // (a grid of at most one block per CU has no co-resident block to overlap a single stage's
  // load and MFMA phases: small batches take the 2-stage pipeline)
  const bool one_stage = g_wgrad1 == 2 || (g_wgrad1 == 1 && nwg > num_cus() && !((fast || window) && p.M >= (1 << 21)));
  if (one_stage) {
    if (BM == 64) {
      if (fast) WG_LAUNCH(true, 64, 1) else WG_LAUNCH(false, 64, 1)
    } else {
      if (fast) WG_LAUNCH(true, 128, 1) else WG_LAUNCH(false, 128, 1)
    }
  } else {
    if (BM == 64) {
      if (fast) WG_LAUNCH(true, 64, 2) else WG_LAUNCH(false, 64, 2)
    } else {
      if (fast) WG_LAUNCH(true, 128, 2) else WG_LAUNCH(false, 128, 2)
    }
  }
#undef WG_LAUNCH
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
