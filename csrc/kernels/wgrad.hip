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
template <bool FAST, int BM, int NSTAGE>  // NSTAGE: LDS buffers (the loop is written for 2)
__global__ void __launch_bounds__(256, 2) wgrad_kernel(WgradParams p, int m_per_split, const int2* __restrict__ rowinfo) {
  constexpr int G_BYTES = 64 * BM * 2;        // 64 m-rows x BM bf16
  constexpr int X_BYTES = 64 * 256;           // 64 m-rows x 128 bf16
  constexpr int STAGE = G_BYTES + X_BYTES;
  constexpr int WAVES_N = BM == 128 ? 2 : 4;
  constexpr int WTN = 128 / WAVES_N;          // k columns per wave
  constexpr int TN = WTN / 16;
  constexpr int EPI_LD = WTN + 4;
  constexpr int GI = G_BYTES / 4096;          // 1 KiB G pieces per wave
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];

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
  // out-of-range offsets (padding taps, tile overhang) load zeros
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.g, p.M * p.ldg * 2);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, FAST ? p.M * p.ldx * 2 : p.N * p.H * p.W * p.C * 2);

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
      buf_lds16(rg, LDS_PTR(gb + (wave * GI + i) * 1024), off, mb * p.ldg * 2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // input operand
      const int row = (wave * 4 + i) * 4 + lrow;
      const bool mok = full || mb + row < mend;
      if (FAST) {
        buf_lds16(rx, LDS_PTR(xb + (wave * 4 + i) * 1024), mok ? x_off[i] : OOB_OFF, mb * p.ldx * 2);
      } else {
        const bool ok = mok && x_tap[i] < 32 && ((ri[i].y >> x_tap[i]) & 1);
        const uint32_t off = ok ? (uint32_t)((ri[i].x * p.C + x_delta[i]) * 2) : OOB_OFF;
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
    const int cur = it & 1;
    if (it + 1 < nit) load_tile(mbeg + (it + 1) * 64, cur ^ 1);
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
        v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) v4bf*)(gb + goff[0] + ((ch ^ gsw[0]) << 4)));
        v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) v4bf*)(gb + goff[1] + ((ch ^ gsw[1]) << 4)));
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int ch = wn * (WTN / 8) + j * 2 + (pp >> 1);
        v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) v4bf*)(xb + roff[0] + ((ch ^ rsw[0]) << 4)));
        v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) v4bf*)(xb + roff[1] + ((ch ^ rsw[1]) << 4)));
        bfr[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
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
  cache[key] = buf;
  return buf;
}

int g_wgrad_variant = 0;   // A/B knob (unused: one pipeline depth remains)

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
  // 31-bit buffer byte offsets (0x80000000 marks out-of-range lanes)
  if ((fast ? (long)p.M * p.ldx : (long)p.N * p.H * p.W * p.C) * 2 >= (1L << 31) ||
      (long)p.M * p.ldg * 2 >= (1L << 31))
    return "wgrad: operand too large for 31-bit buffer offsets";
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
  splits = (p.M + mps - 1) / mps;
  const int nwg = ntiles * splits;
  // 2 LDS stages + 2 blocks/CU (a 3-stage ring at 1 block/CU measured slower and was removed)
  const int2* ri = nullptr;
  if (!fast) {
    const char* why = nullptr;
    ri = rowinfo_for(p, stream, &why);
    if (!ri) return why;
  }
#define WG_LAUNCH(F_, BM_) hipLaunchKernelGGL((wgrad_kernel<F_, BM_, 2>), dim3(nwg), dim3(256), 0, stream, p, mps, ri);
  if (BM == 64) {
    if (fast) WG_LAUNCH(true, 64) else WG_LAUNCH(false, 64)
  } else {
    if (fast) WG_LAUNCH(true, 128) else WG_LAUNCH(false, 128)
  }
#undef WG_LAUNCH
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
