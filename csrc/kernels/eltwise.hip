// Memory-bound kernels around the implicit-GEMM convs (gfx950):
//   * stem_s2d     : Rescaling(1/255) -> RandomCrop/resize -> RandomFlip -> ZeroPadding2D(3)
//                    -> 2x2 space-to-depth (16 ch), in one pass (reference imagenet-resnet50.py:53-55
//                    and the Keras ResNet50 stem)
//   * maxpool      : ZeroPadding2D(1) + MaxPooling2D(3, 2) forward (argmax byte) and backward
//                    (gather form, fused with the ReLU mask of conv1's output)  (N6)
//   * gap          : GlobalAveragePooling2D forward / backward (+ ReLU mask)   (N7)
//   * colsum       : per-channel sum of a gradient (BN beta / conv-bias grads)
//   * softmax_xent : softmax + sparse categorical cross-entropy + accuracy, fwd+bwd fused (N9)
//   * prep / wgrad_finalize / bn_grad : frozen-BN folding and per-channel parameter grads (N4)
// Every kernel moves 16 bytes per lane (8 x bf16) where the layout allows (Guideline 13).
#include "common.h"
#include "kernels.h"

namespace pddl {

// ------------------------------------------------------------------------------ stem
__device__ __forceinline__ float stem_pix(const StemParams& p, int b, int y, int x, int c) {
  if (p.flip && p.flip[b]) x = p.Wc - 1 - x;
  auto fetch = [&](int yy, int xx) -> float {
    const long idx = (((long)b * p.Hin + yy) * p.Win + xx) * 3 + c;
    return p.in_u8 ? (float)reinterpret_cast<const uint8_t*>(p.in)[idx]
                   : reinterpret_cast<const float*>(p.in)[idx];
  };
  float v;
  if (p.mode == 0) {
    v = fetch(y, x);
  } else if (p.mode == 2) {
    v = fetch(y + p.oy, x + p.ox);
  } else {  // bilinear, half-pixel centers (tf.image.resize / keras smart_resize)
    const float sy = (y + 0.5f) * ((float)p.Hin / p.Hc) - 0.5f;
    const float sx = (x + 0.5f) * ((float)p.Win / p.Wc) - 0.5f;
    const float fy = floorf(sy), fx = floorf(sx);
    const int y0 = max((int)fy, 0), x0 = max((int)fx, 0);
    const int y1 = min((int)ceilf(sy), p.Hin - 1), x1 = min((int)ceilf(sx), p.Win - 1);
    const float ly = sy - fy, lx = sx - fx;
    const float top = fetch(y0, x0) + (fetch(y0, x1) - fetch(y0, x0)) * lx;
    const float bot = fetch(y1, x0) + (fetch(y1, x1) - fetch(y1, x0)) * lx;
    v = top + (bot - top) * ly;
  }
  return v * p.scale;
}

// Space-to-depth stem input: one thread per s2d pixel, two 16-byte stores.
__global__ void stem_s2d_kernel(StemParams p, int npix, uint64_t mg_ws, uint64_t mg_hs) {
  if (p.crop_dev) { p.oy = p.crop_dev[0]; p.ox = p.crop_dev[1]; }   // graph-replayable crop offset
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < npix; q += gridDim.x * blockDim.x) {
    const int t = fdiv(q, mg_ws);
    const int j = q - t * p.Ws;
    const int b = fdiv(t, mg_hs);
    const int i = t - b * p.Hs;
    float v[16];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int y = 2 * i + (d >> 1) - 3, x = 2 * j + (d & 1) - 3;
      const bool in = y >= 0 && y < p.Hc && x >= 0 && x < p.Wc;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[d * 4 + c] = in ? stem_pix(p, b, y, x, c) : 0.f;
      v[d * 4 + 3] = 0.f;
    }
    uint4* o = reinterpret_cast<uint4*>(p.out + (long)q * 16);
    o[0] = pack8(v);
    o[1] = pack8(v + 8);
  }
}

// fp32 form (the reference-precision engine): same values, 16 fp32 channels per s2d pixel.
__global__ void stem_s2d_f32_kernel(StemParams p, float* __restrict__ out, int npix, uint64_t mg_ws, uint64_t mg_hs) {
  if (p.crop_dev) { p.oy = p.crop_dev[0]; p.ox = p.crop_dev[1]; }
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < npix; q += gridDim.x * blockDim.x) {
    const int t = fdiv(q, mg_ws);
    const int j = q - t * p.Ws;
    const int b = fdiv(t, mg_hs);
    const int i = t - b * p.Hs;
    float4* o = reinterpret_cast<float4*>(out + (long)q * 16);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int y = 2 * i + (d >> 1) - 3, x = 2 * j + (d & 1) - 3;
      const bool in = y >= 0 && y < p.Hc && x >= 0 && x < p.Wc;
      o[d] = make_float4(in ? stem_pix(p, b, y, x, 0) : 0.f, in ? stem_pix(p, b, y, x, 1) : 0.f,
                         in ? stem_pix(p, b, y, x, 2) : 0.f, 0.f);
    }
  }
}
const char* stem_s2d_f32_launch(const StemParams& p, float* out, hipStream_t s) {
  if ((p.Hc + 6) != 2 * p.Hs || (p.Wc + 6) != 2 * p.Ws) return "stem_s2d_f32: Hs must be (Hc + 6) / 2 (even crop)";
  const long npix = (long)p.B * p.Hs * p.Ws;
  if (npix >= (1L << 31) - (1L << 24)) return "stem_s2d_f32: too many pixels for 32-bit indexing";
  const int grid = (int)lmin((npix + 255) / 256, 16384);
  hipLaunchKernelGGL(stem_s2d_f32_kernel, dim3(grid), dim3(256), 0, s, p, out, (int)npix, fdiv_magic(p.Ws),
                     fdiv_magic(p.Hs));
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// Row form for uint8 identity / crop input (modes 0 and 2, the training path): one block per
// s2d row (b, i) stages the two preprocessed source rows 2i-3, 2i-2 through LDS with
// coalesced 4-byte loads (the per-pixel form issues 12 scattered byte loads per thread and
// ran at 1.8 TB/s), then thread j assembles s2d pixel j (flip applied on the LDS read).
// Bitwise equal to the per-pixel form (same (float)u8 * scale -> bf16).
constexpr int STEM_ROW_MAXW = 1024;   // preprocessed width the LDS row buffer holds
__global__ void __launch_bounds__(128) stem_s2d_rows_kernel(StemParams p) {
  __shared__ uint32_t rowbuf[2][(STEM_ROW_MAXW * 3) / 4 + 2];
  if (p.crop_dev) { p.oy = p.crop_dev[0]; p.ox = p.crop_dev[1]; }
  const int i = blockIdx.x % p.Hs, b = blockIdx.x / p.Hs;
  const int oy = p.mode == 2 ? p.oy : 0, ox = p.mode == 2 ? p.ox : 0;
  const uint8_t* in = reinterpret_cast<const uint8_t*>(p.in);
  int shift[2];
  bool rok[2];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    const int y = 2 * i + dy - 3;
    rok[dy] = y >= 0 && y < p.Hc;
    shift[dy] = 0;
    if (!rok[dy]) continue;
    const uint8_t* src = in + (((long)b * p.Hin + y + oy) * p.Win + ox) * 3;
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(src) & ~uintptr_t(3);
    shift[dy] = (int)(reinterpret_cast<uintptr_t>(src) - a0);
    const int nw = (shift[dy] + p.Wc * 3 + 3) / 4;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a0);
    for (int k = threadIdx.x; k < nw; k += blockDim.x) rowbuf[dy][k] = w[k];
  }
  __syncthreads();
  const bool fl = p.flip && p.flip[b];
  const uint8_t* rb = reinterpret_cast<const uint8_t*>(&rowbuf[0][0]);
  constexpr int ROWB = ((STEM_ROW_MAXW * 3) / 4 + 2) * 4;
  for (int j = threadIdx.x; j < p.Ws; j += blockDim.x) {
    float v[16];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dy = d >> 1;
      int x = 2 * j + (d & 1) - 3;
      const bool in_ = rok[dy] && x >= 0 && x < p.Wc;
      if (fl) x = p.Wc - 1 - x;
      const int o = dy * ROWB + shift[dy] + x * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[d * 4 + c] = in_ ? (float)rb[o + c] * p.scale : 0.f;
      v[d * 4 + 3] = 0.f;
    }
    uint4* o = reinterpret_cast<uint4*>(p.out + (((long)b * p.Hs + i) * p.Ws + j) * 16);
    o[0] = pack8(v);
    o[1] = pack8(v + 8);
  }
}
int g_stem_variant = 1;   // 1: row form for uint8 modes 0 / 2 (default), 0: per-pixel form everywhere

const char* stem_s2d_launch(const StemParams& p, hipStream_t s) {
  if ((p.Hc + 6) != 2 * p.Hs || (p.Wc + 6) != 2 * p.Ws) return "stem_s2d: Hs must be (Hc + 6) / 2 (even crop)";
  const long npix = (long)p.B * p.Hs * p.Ws;
  if (npix >= (1L << 31) - (1L << 24)) return "stem_s2d: too many pixels for 32-bit indexing";
  if (g_stem_variant == 1 && p.in_u8 && p.mode != 1 && p.Wc <= STEM_ROW_MAXW) {
    hipLaunchKernelGGL(stem_s2d_rows_kernel, dim3(p.B * p.Hs), dim3(128), 0, s, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? nullptr : hipGetErrorString(e);
  }
  const int grid = (int)lmin((npix + 255) / 256, 16384);
  hipLaunchKernelGGL(stem_s2d_kernel, dim3(grid), dim3(256), 0, s, p, (int)npix, fdiv_magic(p.Ws), fdiv_magic(p.Hs));
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

__device__ __forceinline__ int s2d_col(int r, int s, int c) {
  return ((r >> 1) * 4 + (s >> 1)) * 16 + ((r & 1) * 2 + (s & 1)) * 4 + c;
}

__global__ void stem_wgrad_fold_kernel(const float* __restrict__ g2, float* __restrict__ dw, int cout) {
  const int n = cout * 147;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int co = e / 147, k = e - co * 147;
    const int r = k / 21, rm = k - r * 21, s = rm / 3, c = rm - s * 3;
    dw[e] += g2[co * 256 + s2d_col(r, s, c)];
  }
}
const char* stem_wgrad_fold_launch(const float* g2, float* dw, int cout, hipStream_t s) {
  hipLaunchKernelGGL(stem_wgrad_fold_kernel, dim3((cout * 147 + 255) / 256), dim3(256), 0, s, g2, dw, cout);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

int g_pool_blocks = 8192;   // grid cap of the pool / GAP kernels: 4096 -> 8192 -> 16384 blocks
                            // measured 772 -> 742 -> 733 us (fwd); 16384 not adopted (1%, twice the
                            // backward colsum partial rows; profiles/r1_pool_grid_sweep.log)
static int grid_for(long n) { return (int)lmin((n + 255) / 256, g_pool_blocks); }

// --------------------------------------------------------------------------- maxpool
// Window of output (ho, wo) covers input rows 2ho-1 .. 2ho+1 (ZeroPadding2D(1) then 3x3/s2
// valid).  Padded taps are real zeros (as in Keras); the first maximum in scan order wins.
// Index math is 32-bit with magic-number division (the launchers check the element counts
// fit): 64-bit div / mod per element made these kernels ALU-bound.
struct PoolDiv { uint64_t cg, w, h; };
__global__ void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                   uint8_t* __restrict__ bits, int B, int H, int W, int C, int Ho, int Wo, PoolDiv dv) {
  const int cg = C / 8;
  const int total = B * Ho * Wo * cg;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int pix = fdiv(t, dv.cg);
    const int g = t - pix * cg;
    const int t2 = fdiv(pix, dv.w);
    const int wo = pix - t2 * Wo;
    const int b = fdiv(t2, dv.h);
    const int ho = t2 - b * Ho;
    float best[8]; uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int hi = 2 * ho - 1 + r, wi = 2 * wo - 1 + s;
        float v[8];
        if (hi >= 0 && hi < H && wi >= 0 && wi < W) {
          unpack8(*reinterpret_cast<const uint4*>(x + (((long)b * H + hi) * W + wi) * C + g * 8), v);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = (uint8_t)(r * 3 + s); }
      }
    const long o = (long)pix * C + g * 8;
    const uint4 yv = pack8(best);
    *reinterpret_cast<uint4*>(y + o) = yv;
    if (bits) bits[o >> 3] = (uint8_t)pos_bits8(yv);
    uint2 pk;
    pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = pk;
  }
}

// Column sums of the output are accumulated per thread: with a grid stride that is a
// multiple of C/8 every thread keeps one channel group, folded across the wave at the end.
__global__ void maxpool_bwd_kernel(const bf16_t* __restrict__ gy, const uint8_t* __restrict__ idx,
                                   const bf16_t* __restrict__ xmask, bf16_t* __restrict__ gx,
                                   int B, int H, int W, int C, int Ho, int Wo, float* __restrict__ colsum,
                                   PoolDiv dv) {
  const int cg = C / 8;
  const int total = B * H * W * cg;
  float cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int pix = fdiv(t, dv.cg);
    const int g = t - pix * cg;
    const int t2 = fdiv(pix, dv.w);
    const int w = pix - t2 * W;
    const int b = fdiv(t2, dv.h);
    const int h = t2 - b * H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int hp = h + 1, wp = w + 1;  // padded coordinates
    const int ho_lo = max(0, (hp - 1) / 2), ho_hi = min(Ho - 1, hp / 2);
    const int wo_lo = max(0, (wp - 1) / 2), wo_hi = min(Wo - 1, wp / 2);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int r = hp - 2 * ho;
      if (r < 0 || r > 2) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int s = wp - 2 * wo;
        if (s < 0 || s > 2) continue;
        const long o = (((long)b * Ho + ho) * Wo + wo) * C + g * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        float gv[8];
        unpack8(*reinterpret_cast<const uint4*>(gy + o), gv);
        const uint8_t want = (uint8_t)(r * 3 + s);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t word = e < 4 ? pk.x : pk.y;
          const uint8_t id = (word >> (8 * (e & 3))) & 0xff;
          if (id == want) acc[e] += gv[e];
        }
      }
    }
    const long o = (long)pix * C + g * 8;
    if (xmask) {
      float mv[8];
      unpack8(*reinterpret_cast<const uint4*>(xmask + o), mv);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = mv[e] > 0.f ? acc[e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] += acc[e];
    *reinterpret_cast<uint4*>(gx + o) = pack8(acc);
  }
  if (colsum) {  // one partial row of C sums per wave (plain stores)
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = cg; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += __shfl_xor(cs[e], o, 64);
    if (lane < cg) {
      const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
      float4* dst = reinterpret_cast<float4*>(colsum + wave * C + lane * 8);
      dst[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
      dst[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
    }
  }
}
// Row-streaming forms (pool = 4): a wave owns WL = 64 / (C/8) output columns x all channel
// groups of one image and walks the output rows top to bottom.  Every input row is fetched
// once per wave (the per-output forms fetch the row shared by two vertically adjacent windows
// twice, and the two fetches land on different XCDs because neighbouring workgroups are
// dispatched round-robin over the 8 L2s), so the HBM traffic is one read of the input plus the
// outputs.  Forward: the horizontal 3-max (value + tap) of input row 2ho+1 is the bottom row of
// window ho and the top row of window ho+1, so it is carried to the next iteration; rows are
// combined top to bottom with strict '>' and taps left to right within a row, which keeps the
// first maximum in scan order (the per-output forms' tie rule).
template <int CG>
__global__ void __launch_bounds__(256) maxpool_fwd_stream_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                 uint8_t* __restrict__ idx, uint8_t* __restrict__ bits,
                                                                 int B, int H, int W, int Ho, int Wo) {
  constexpr int C = CG * 8, WL = 64 / CG;
  const int lane = threadIdx.x & 63, g = lane % CG, wl = lane / CG;
  const int bands = (Wo + WL - 1) / WL;
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= B * bands) return;
  const int b = wid / bands, wo = (wid - b * bands) * WL + wl;
  if (wo >= Wo) return;
  const bf16_t* xb = x + (long)b * H * W * C + g * 8;
  const int wi0 = 2 * wo - 1;
  // raw taps of input row hi, columns wi0 .. wi0 + 2: branch-free loads (address clamped into
  // the image, zero padding selected afterwards) so the next rows' loads can be issued ahead
  bool col_ok[3];
  int wcl[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int wi = wi0 + s;
    col_ok[s] = wi >= 0 && wi < W;
    wcl[s] = wi < 0 ? 0 : (wi >= W ? W - 1 : wi);
  }
  auto fetch = [&](int hi, uint4 (&r)[3]) {
    const bool row_ok = hi >= 0 && hi < H;
    const int hc = hi < 0 ? 0 : (hi >= H ? H - 1 : hi);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const uint4 v = *reinterpret_cast<const uint4*>(xb + ((long)hc * W + wcl[s]) * C);
      r[s] = (row_ok && col_ok[s]) ? v : make_uint4(0, 0, 0, 0);
    }
  };
  // horizontal max + first-max tap of one fetched row
  auto hmax = [&](const uint4 (&r)[3], float (&hv)[8], uint32_t (&hs)[8]) {
    float t[3][8];
#pragma unroll
    for (int s = 0; s < 3; ++s) unpack8(r[s], t[s]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = t[0][e];
      uint32_t s = 0;
      if (t[1][e] > v) { v = t[1][e]; s = 1; }
      if (t[2][e] > v) { v = t[2][e]; s = 2; }
      hv[e] = v; hs[e] = s;
    }
  };
  float tv[8];
  uint32_t ts[8];
  uint4 r1[3], r2[3];
  fetch(-1, r1);
  hmax(r1, tv, ts);   // the padding row above window 0
  fetch(0, r1);
  fetch(1, r2);
  for (int ho = 0; ho < Ho; ++ho) {
    float mv[8], bv[8];
    uint32_t ms[8], bs[8];
    hmax(r1, mv, ms);
    hmax(r2, bv, bs);
    if (ho + 1 < Ho) {   // rows of the next window in flight while this one is reduced and stored
      fetch(2 * ho + 2, r1);
      fetch(2 * ho + 3, r2);
    }
    float best[8];
    uint32_t code[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = tv[e]; code[e] = ts[e];
      if (mv[e] > best[e]) { best[e] = mv[e]; code[e] = 3 + ms[e]; }
      if (bv[e] > best[e]) { best[e] = bv[e]; code[e] = 6 + bs[e]; }
      tv[e] = bv[e]; ts[e] = bs[e];   // row 2ho+1 is the top row of window ho+1
    }
    const long o = (((long)b * Ho + ho) * Wo + wo) * C + g * 8;
    const uint4 yv = pack8(best);
    *reinterpret_cast<uint4*>(y + o) = yv;
    if (bits) bits[o >> 3] = (uint8_t)pos_bits8(yv);
    *reinterpret_cast<uint2*>(idx + o) =
        make_uint2(code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24),
                   code[4] | (code[5] << 8) | (code[6] << 16) | (code[7] << 24));
  }
}

// Backward, same wave shape: the lane owns input columns 2p, 2p+1 of one channel group and
// walks input row pairs (2q, 2q+1).  Exactly outputs (q..q+1, p..p+1) route gradient into the
// 2x2 block (row 2q: output row q tap r = 1; row 2q+1: output row q tap 2 and row q+1 tap 0;
// columns likewise), and output row q+1's (gy, idx) are carried as the next pair's row q, so
// every (gy, idx) row is read once per wave (the neighbour column p+1 comes from L1).
template <int CG>
__global__ void __launch_bounds__(256) maxpool_bwd_stream_kernel(const bf16_t* __restrict__ gy,
                                                                 const uint8_t* __restrict__ idx,
                                                                 const bf16_t* __restrict__ xmask,
                                                                 bf16_t* __restrict__ gx, int B, int H, int W,
                                                                 int Ho, int Wo, float* __restrict__ colsum) {
  constexpr int C = CG * 8, WL = 64 / CG;
  const int lane = threadIdx.x & 63, g = lane % CG, wl = lane / CG;
  const int Wq = (W + 1) / 2, Hq = (H + 1) / 2;
  const int bands = (Wq + WL - 1) / WL;
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= B * bands) return;   // (whole waves: the colsum row of such a wave is never read)
  const int b = wid / bands, p = (wid - b * bands) * WL + wl;
  float cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (p < Wq) {
    // raw (gy, idx) of output row ho at columns p, p + 1: branch-free loads (address clamped,
    // zero gradient / no-match taps outside the output) so the row after next is in flight
    // while this pair is scattered
    const bool okp1 = p + 1 < Wo;
    const int wo1 = okp1 ? p + 1 : Wo - 1;
    auto orow = [&](int ho, uint4 (&gr)[2], uint2 (&ir)[2]) {
      const bool rok = ho < Ho;
      const long rb = ((long)b * Ho + (rok ? ho : Ho - 1)) * Wo;
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const long o = (rb + (d ? wo1 : p)) * C + g * 8;
        const uint4 gv = *reinterpret_cast<const uint4*>(gy + o);
        const uint2 iv = *reinterpret_cast<const uint2*>(idx + o);
        const bool ok = rok && (d == 0 || okp1);
        gr[d] = ok ? gv : make_uint4(0, 0, 0, 0);
        ir[d] = ok ? iv : make_uint2(0xffffffffu, 0xffffffffu);   // matches no tap
      }
    };
    auto tap = [](const uint2& iv, int e) { return ((e < 4 ? iv.x : iv.y) >> (8 * (e & 3))) & 0xffu; };
    uint4 gq[2], gq1[2];   // output rows q and q + 1
    uint2 iq[2], iq1[2];
    orow(0, gq, iq);
    orow(1, gq1, iq1);
    for (int q = 0; q < Hq; ++q) {
      float ga[8], gb[8], gc[8], gd[8];   // (q, p), (q, p+1), (q+1, p), (q+1, p+1)
      unpack8(gq[0], ga); unpack8(gq[1], gb); unpack8(gq1[0], gc); unpack8(gq1[1], gd);
      const uint2 ia = iq[0], ib = iq[1], ic = iq1[0], id = iq1[1];
      gq[0] = gq1[0]; gq[1] = gq1[1]; iq[0] = iq1[0]; iq[1] = iq1[1];
      if (q + 1 < Hq) orow(q + 2, gq1, iq1);
      float acc[2][2][8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t ta = tap(ia, e), tb = tap(ib, e), tc = tap(ic, e), td = tap(id, e);
        // input (2q + a, 2p + c): from output (q, p) tap (a + 1, c + 1); (q, p+1) tap (a + 1, 0)
        // for c = 1; (q+1, p) tap (0, c + 1) for a = 1; (q+1, p+1) tap (0, 0) for a = c = 1
        acc[0][0][e] = ta == 4u ? ga[e] : 0.f;
        acc[0][1][e] = (ta == 5u ? ga[e] : 0.f) + (tb == 3u ? gb[e] : 0.f);
        acc[1][0][e] = (ta == 7u ? ga[e] : 0.f) + (tc == 1u ? gc[e] : 0.f);
        acc[1][1][e] = (ta == 8u ? ga[e] : 0.f) + (tb == 6u ? gb[e] : 0.f) + (tc == 2u ? gc[e] : 0.f) +
                       (td == 0u ? gd[e] : 0.f);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int h = 2 * q + a, w = 2 * p + c;
          if (h >= H || w >= W) continue;
          const long o = (((long)b * H + h) * W + w) * C + g * 8;
          if (xmask) {
            float mv[8];
            unpack8(*reinterpret_cast<const uint4*>(xmask + o), mv);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[a][c][e] = mv[e] > 0.f ? acc[a][c][e] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += acc[a][c][e];
          *reinterpret_cast<uint4*>(gx + o) = pack8(acc[a][c]);
        }
    }
  }
  if (colsum) {   // one partial row of C sums per wave
#pragma unroll
    for (int o = CG; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += __shfl_xor(cs[e], o, 64);
    if (wl == 0) {
      float4* dst = reinterpret_cast<float4*>(colsum + (long)wid * C + g * 8);
      dst[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
      dst[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
    }
  }
}

// Max-pool kernels: row-streaming forward and backward (one wave per image x column band) for
// the ResNet widths C = 64 / 128 / 256; the per-output forward and per-input-pixel backward
// for any other C % 8 == 0.  (Rejected after bench/pool.py A/B at b1024 @ 112x112x64,
// profiles/r1_pool_ab.json, and removed: 2- / 4-output strip forwards, 796 / 1000 us, and a
// 2x2-block backward, 628 us, against the streaming pair.)
static bool pool_stream(int C) { return C == 64 || C == 128 || C == 256; }
static long pool_stream_waves(int B, int cols, int C) {
  const int WL = 64 / (C / 8);
  return (long)B * ((cols + WL - 1) / WL);
}
static long pool_bwd_items(int B, int H, int W, int C) { return (long)B * H * W * C / 8; }
int maxpool_bwd_partial_rows(int B, int H, int W, int C) {
  if (pool_stream(C)) return (int)pool_stream_waves(B, (W + 1) / 2, C);
  return grid_for(pool_bwd_items(B, H, W, C)) * 4;
}

const char* maxpool_fwd_launch(const uint16_t* x, uint16_t* y, uint8_t* idx, uint8_t* bits, int B, int H, int W, int C, int Ho,
                               int Wo, hipStream_t s) {
  if (C % 8) return "maxpool: C % 8";
  if ((long)B * H * W * C / 8 >= (1L << 31) - (1L << 24)) return "maxpool: too many elements for 32-bit indexing";
  if (Ho != (H - 1) / 2 + 1 || Wo != (W - 1) / 2 + 1) return "maxpool: output must be the pad-1 3x3/s2 size";
  if (pool_stream(C)) {
    const int grid = (int)((pool_stream_waves(B, Wo, C) + 3) / 4);
#define POOL_F(CG_) hipLaunchKernelGGL(maxpool_fwd_stream_kernel<CG_>, dim3(grid), dim3(256), 0, s, x, y, idx, bits, B, H, W, Ho, Wo)
    if (C == 64) POOL_F(8); else if (C == 128) POOL_F(16); else POOL_F(32);
#undef POOL_F
  } else {
    const PoolDiv dv{fdiv_magic(C / 8), fdiv_magic(Wo), fdiv_magic(Ho)};
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for((long)B * Ho * Wo * C / 8)), dim3(256), 0, s, x, y, idx,
                       bits, B, H, W, C, Ho, Wo, dv);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* maxpool_bwd_launch(const uint16_t* gy, const uint8_t* idx, const uint16_t* xmask, uint16_t* gx, int B,
                               int H, int W, int C, int Ho, int Wo, float* colsum, hipStream_t s) {
  if (C % 8) return "maxpool: C % 8";
  if (colsum && (64 % (C / 8))) return "maxpool: fused colsum needs C/8 to divide 64";
  if ((long)B * H * W * C / 8 >= (1L << 31) - (1L << 24)) return "maxpool: too many elements for 32-bit indexing";
  if (Ho != (H - 1) / 2 + 1 || Wo != (W - 1) / 2 + 1) return "maxpool: output must be the pad-1 3x3/s2 size";
  const int grid = grid_for(pool_bwd_items(B, H, W, C));
  if (pool_stream(C)) {
    const int sgrid = (int)((pool_stream_waves(B, (W + 1) / 2, C) + 3) / 4);
#define POOL_B(CG_) \
  hipLaunchKernelGGL(maxpool_bwd_stream_kernel<CG_>, dim3(sgrid), dim3(256), 0, s, gy, idx, xmask, gx, B, H, W, Ho, Wo, colsum)
    if (C == 64) POOL_B(8); else if (C == 128) POOL_B(16); else POOL_B(32);
#undef POOL_B
  } else {
    const PoolDiv dv{fdiv_magic(C / 8), fdiv_magic(W), fdiv_magic(H)};
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid), dim3(256), 0, s, gy, idx, xmask, gx, B, H, W, C, Ho, Wo,
                       colsum, dv);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ------------------------------------------------------------------------------- GAP
__global__ void gap_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B, int HW, int C) {
  const int cg = C / 8;
  const long total = (long)B * cg;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int g = (int)(t % cg), b = (int)(t / cg);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < HW; ++i) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + ((long)b * HW + i) * C + g * 8), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
    const float inv = 1.f / HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    *reinterpret_cast<uint4*>(y + (long)b * C + g * 8) = pack8(acc);
  }
}
__global__ void gap_bwd_kernel(const bf16_t* __restrict__ gp, int ldgp, const bf16_t* __restrict__ ymask,
                               bf16_t* __restrict__ g, int B, int HW, int C, float* __restrict__ colsum) {
  const int cg = C / 8;
  const long total = (long)B * cg;
  const float inv = 1.f / HW;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int gg = (int)(t % cg), b = (int)(t / cg);
    float v[8], cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unpack8(*reinterpret_cast<const uint4*>(gp + (long)b * ldgp + gg * 8), v);
    for (int i = 0; i < HW; ++i) {
      const long row = (long)b * HW + i;
      float mv[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(ymask + row * C + gg * 8), mv);
#pragma unroll
      for (int e = 0; e < 8; ++e) { o[e] = mv[e] > 0.f ? v[e] * inv : 0.f; cs[e] += o[e]; }
      *reinterpret_cast<uint4*>(g + row * C + gg * 8) = pack8(o);
    }
    if (colsum) {  // partial row b (plain stores)
      float4* dst = reinterpret_cast<float4*>(colsum + (long)b * C + gg * 8);
      dst[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
      dst[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
    }
  }
}
const char* gap_fwd_launch(const uint16_t* x, uint16_t* y, int B, int HW, int C, hipStream_t s) {
  if (C % 8) return "gap: C % 8";
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(grid_for((long)B * C / 8)), dim3(256), 0, s, x, y, B, HW, C);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* gap_bwd_launch(const uint16_t* gp, int ldgp, const uint16_t* ymask, uint16_t* g, int B, int HW, int C,
                           float* colsum, hipStream_t s) {
  if (C % 8 || ldgp % 8) return "gap: C % 8";
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_for((long)B * C / 8)), dim3(256), 0, s, gp, ldgp, ymask, g, B,
                     HW, C, colsum);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ---------------------------------------------------------------------------- colsum
// out[c] += sum_m g[m, c].  Block = 256 threads = CG column groups (8 columns each) x RL row
// lanes; registers accumulate, LDS folds the row lanes, one atomic per column per block.
__global__ void colsum_kernel(const bf16_t* __restrict__ g, int M, int C, int ldg, int rows_per_block,
                              float* __restrict__ out) {
  __shared__ float red[256 * 8];
  const int G = C / 8;
  const int CG = G < 32 ? G : 32;
  const int RL = 256 / CG;
  const int t = threadIdx.x;
  const int cgi = t % CG, rl = t / CG;
  const int colg = blockIdx.x * CG + cgi;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (colg < G && rl < RL) {
    for (int r = r0 + rl; r < r1; r += RL) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(g + (long)r * ldg + colg * 8), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[t * 8 + e] = acc[e];
  __syncthreads();
  if (t < CG * 8) {
    const int cg2 = t / 8, e = t % 8;
    float s = 0.f;
    for (int l = 0; l < RL; ++l) s += red[((l * CG) + cg2) * 8 + e];
    const int col = (blockIdx.x * CG + cg2) * 8 + e;
    if (col < C) unsafeAtomicAdd(out + col, s);
  }
}
const char* colsum_launch(const uint16_t* g, int M, int C, int ldg, float* out, hipStream_t s) {
  if (C % 8 || ldg % 8) return "colsum: C % 8";
  const int G = C / 8, CG = G < 32 ? G : 32;
  const int gx = (G + CG - 1) / CG;
  int rpb = 512;
  int gy = (M + rpb - 1) / rpb;
  if ((long)gx * gy > 4096) { gy = (4096 + gx - 1) / gx; rpb = (M + gy - 1) / gy; gy = (M + rpb - 1) / rpb; }
  hipLaunchKernelGGL(colsum_kernel, dim3(gx, gy), dim3(256), 0, s, g, M, C, ldg, rpb, out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// Fold partial column-sum rows: grid (row chunks, layers).  A layer may fold a column range of
// wider rows (ColRedLayer::pad = row stride): the (sum g | sum g*(z-mu)) halves of a fused
// BN-backward dgrad land in two separate accumulators.
// The fold is bound by same-address atomics, not by bytes: atomics onto one column serialize
// at ~60-100 ns each, so 512-1024 row chunks per layer cost 30-100 us even for a 6 MB layer
// (the previous 256-thread, 512-chunk fold: 2.5 ms per train-BN b1024 step,
// profiles/r2_bntrain_b1024_summary.txt).  So: few chunks (COLRED_CHUNKS = 64, at least
// COLRED_MIN_ROWS rows each), and enough loads in flight per chunk to stream its rows anyway --
// 1024-thread blocks of RL row-lanes x NC float4 column lanes (NC <= 1024 float4 = 4096 columns
// per pass), 8 rows in flight per lane with independent accumulators (128 KiB per block), the
// row-lanes folded through LDS, one atomic per column per chunk.
// Vector path when C, the row stride and the offset are multiples of 4 floats (every engine
// table); scalar fallback otherwise.
constexpr int COLRED_MIN_ROWS = 32;
constexpr int COLRED_THREADS = 1024;
__global__ void __launch_bounds__(COLRED_THREADS) colsum_reduce_kernel(const float* __restrict__ part,
                                                                       const ColRedLayer* __restrict__ L,
                                                                       float* __restrict__ colsum) {
  __shared__ float4 red[COLRED_THREADS];
  const ColRedLayer l = L[blockIdx.y];
  const int eff = max(1, min((int)gridDim.x, l.rows / COLRED_MIN_ROWS));
  if ((int)blockIdx.x >= eff) return;
  const int r0 = (int)((long)l.rows * blockIdx.x / eff), r1 = (int)((long)l.rows * (blockIdx.x + 1) / eff);
  if (r0 >= r1) return;
  const int t = threadIdx.x;
  const long ld = l.pad > 0 ? l.pad : l.C;   // row stride (pad > 0: one column range of wider rows)
  if ((l.C & 3) == 0 && (ld & 3) == 0 && (l.part & 3) == 0) {
    const int C4 = l.C >> 2;
    const long ld4 = ld >> 2;
    const float4* base = reinterpret_cast<const float4*>(part + l.part);
    for (int cb = 0; cb < C4; cb += COLRED_THREADS) {
      const int nc = min(COLRED_THREADS, C4 - cb);
      const int RL = COLRED_THREADS / nc;
      const int c4 = cb + t % nc, rl = t / nc;
      float4 acc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rl < RL) {
        const float4* col = base + c4;
        int r = r0 + rl;
        for (; r < r1; r += 8 * RL) {   // 8 rows per lane in flight; rows past r1 re-read row r
          float4 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int rr = r + u * RL;
            const float4 x = col[(long)(rr < r1 ? rr : r) * ld4];
            v[u] = rr < r1 ? x : make_float4(0.f, 0.f, 0.f, 0.f);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) { acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w; }
        }
      }
      float4 s0 = acc[0];
#pragma unroll
      for (int u = 1; u < 8; ++u) { s0.x += acc[u].x; s0.y += acc[u].y; s0.z += acc[u].z; s0.w += acc[u].w; }
      red[t] = s0;
      __syncthreads();
      if (t < nc) {
        for (int i = 1; i < RL; ++i) {
          const float4 o = red[t + i * nc];
          s0.x += o.x; s0.y += o.y; s0.z += o.z; s0.w += o.w;
        }
        float* dst = colsum + l.out + 4 * c4;
        unsafeAtomicAdd(dst + 0, s0.x);
        unsafeAtomicAdd(dst + 1, s0.y);
        unsafeAtomicAdd(dst + 2, s0.z);
        unsafeAtomicAdd(dst + 3, s0.w);
      }
      __syncthreads();
    }
  } else {   // scalar fallback (unaligned column ranges)
    for (int c = t; c < l.C; c += blockDim.x) {
      float s = 0.f;
      for (int r = r0; r < r1; ++r) s += part[l.part + (long)r * ld + c];
      unsafeAtomicAdd(colsum + l.out + c, s);
    }
  }
}
int g_colred_chunks = 64;   // row-chunk cap per layer (knob colred_chunks)
const char* colsum_reduce_launch(const float* part, const ColRedLayer* layers_dev, int nlayers, float* colsum,
                                 hipStream_t s) {
  // up to g_colred_chunks row chunks per layer (at least COLRED_MIN_ROWS rows each): every CU
  // gets work for one large layer; chunks past a short layer's share exit at once
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3(g_colred_chunks, nlayers), dim3(COLRED_THREADS), 0, s, part, layers_dev, colsum);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ---------------------------------------------------------------------- softmax-xent
// One wave per example.  loss += logsumexp - logit[label]; dlogits = (softmax - onehot)*gscale
// written as bf16 into [B][ldd] (columns >= ncls zeroed: they are the K padding of the head
// dgrad); correct += (first argmax == label).
__global__ void softmax_xent_kernel(const float* __restrict__ logits, int ldl, const int64_t* __restrict__ labels,
                                    int B, int ncls, float gscale, bf16_t* __restrict__ dl, int ldd,
                                    float* __restrict__ loss_sum, float* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* row = logits + (long)b * ldl;
  float mx = -INFINITY; int amax = 0x7fffffff;
  for (int j = lane; j < ncls; j += 64) {
    const float v = row[j];
    if (v > mx) { mx = v; amax = j; }
  }
  // wave argmax (first index among equal maxima)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
  for (int j = lane; j < ncls; j += 64) se += __expf(row[j] - mx);
  se = warp_sum(se);
  const int lab = (int)labels[b];
  const float inv = 1.f / se;
  for (int j = lane; j < ldd; j += 64) {
    float d = 0.f;
    if (j < ncls) d = (__expf(row[j] - mx) * inv - (j == lab ? 1.f : 0.f)) * gscale;
    dl[(long)b * ldd + j] = f2bf(d);
  }
  if (lane == 0) {
    const float lse = mx + __logf(se);
    unsafeAtomicAdd(loss_sum, lse - row[lab]);
    unsafeAtomicAdd(correct, amax == lab ? 1.f : 0.f);
  }
}
const char* softmax_xent_launch(const float* logits, int ldl, const int64_t* labels, int B, int ncls, float gscale,
                                uint16_t* dlogits, int ldd, float* loss_sum, float* correct, hipStream_t s) {
  if (ldd < ncls) return "softmax_xent: ldd < ncls";
  hipLaunchKernelGGL(softmax_xent_kernel, dim3((B + 3) / 4), dim3(256), 0, s, logits, ldl, labels, B, ncls, gscale,
                     dlogits, ldd, loss_sum, correct);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ----------------------------------------------------------------------------- prep
// After each optimizer step: fp32 master -> bf16 forward weights [cout][kpad] (zero padded),
// bf16 dgrad weights W'[c][R-1-r][S-1-s][co] = a[co] * W[co][r][s][c], and the folded
// frozen-BN affine a = gamma / sqrt(var + eps), b = (bias - mean) * a + beta.
// (T = uint16_t: bf16 weights of the bf16 engine; T = float: the fp32 engine, whose forward
// convs read the fp32 master directly -- only the stem's space-to-depth copy and the dgrad
// weights are prepared)
template <typename T> __device__ __forceinline__ T wcvt(float v);
template <> __device__ __forceinline__ uint16_t wcvt<uint16_t>(float v) { return f2bf(v); }
template <> __device__ __forceinline__ float wcvt<float>(float v) { return v; }

template <typename T>
__global__ void prep_kernel(const float* __restrict__ prm, const PrepLayer* __restrict__ L, T* __restrict__ wbf,
                            float* __restrict__ scale, float* __restrict__ shift, float eps) {
  const PrepLayer l = L[blockIdx.y];
  const int RSC = l.R * l.S * l.cin;
  auto fold = [&](int co, float* a_out, float* b_out) {
    const float g = l.gamma_off >= 0 ? prm[l.gamma_off + co] : 1.f;
    const float var = l.var_off >= 0 ? prm[l.var_off + co] : 1.f - eps;
    const float mu = l.mean_off >= 0 ? prm[l.mean_off + co] : 0.f;
    const float be = l.beta_off >= 0 ? prm[l.beta_off + co] : 0.f;
    const float bi = l.bias_off >= 0 ? prm[l.bias_off + co] : 0.f;
    const float a = (l.gamma_off >= 0 || l.var_off >= 0) ? g * rsqrtf(var + eps) : 1.f;
    *a_out = a;
    *b_out = (bi - mu) * a + be;
  };
  if (l.mode == 1) {  // stem: scatter into the 4x4x16 space-to-depth layout (zeros stay zero)
    const int nf = l.cout * RSC;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nf; e += gridDim.x * blockDim.x) {
      const int co = e / RSC, k = e - co * RSC;
      const int r = k / (l.S * l.cin), rm = k - r * l.S * l.cin, s = rm / l.cin, c = rm - s * l.cin;
      wbf[l.wf_off + (long)co * l.kpad + s2d_col(r, s, c)] = wcvt<T>(prm[l.w_off + e]);
      if (k == 0) {
        float a, b;
        fold(co, &a, &b);
        scale[l.ch_off + co] = a;
        shift[l.ch_off + co] = b;
      }
    }
    return;
  }
  // every non-stem layer has kpad == R*S*cin: the forward copy is a flat fp32 -> bf16 cast
  if constexpr (sizeof(T) == 2) {
    const long nf = (long)l.cout * RSC;
    const long n4 = nf / 4;
    const float4* src = reinterpret_cast<const float4*>(prm + l.w_off);
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n4; e += (long)gridDim.x * blockDim.x) {
      const float4 w = src[e];
      uint2 o;
      o.x = pack2(w.x, w.y);
      o.y = pack2(w.z, w.w);
      *reinterpret_cast<uint2*>(wbf + l.wf_off + e * 4) = o;
    }
  }
  for (int co = blockIdx.x * blockDim.x + threadIdx.x; co < l.cout; co += gridDim.x * blockDim.x) {
    float a, b;
    fold(co, &a, &b);
    scale[l.ch_off + co] = a;
    shift[l.ch_off + co] = b;
  }
}

// dgrad weights W'[c][R-1-r][S-1-s][co] = a[co] * W[co][r][s][c]: per (layer, tap) a batch of
// [cout][cin] -> [cin][cout] transposes through a 64x64 LDS tile (coalesced both ways).
template <typename T>
__global__ void prep_dgrad_kernel(const float* __restrict__ prm, const PrepLayer* __restrict__ L,
                                  T* __restrict__ wbf, float eps) {
  __shared__ float tile[64][65];
  const PrepLayer l = L[blockIdx.y];
  if (l.wd_off < 0 || l.mode != 0) return;
  const int taps = l.R * l.S;
  const int tco = (l.cout + 63) / 64, tci = (l.cin + 63) / 64;
  const int ntiles = taps * tco * tci;
  const int RSC = taps * l.cin;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tap = t / (tco * tci), rem = t - tap * tco * tci;
    const int co0 = (rem / tci) * 64, c0 = (rem % tci) * 64;
    const int r = tap / l.S, s = tap - r * l.S;
    // load: thread -> (row co = co0 + i, col c = c0 + j), 16 rows per pass
    const int j = threadIdx.x & 63, i0 = threadIdx.x >> 6;
    for (int i = i0; i < 64; i += 4) {
      const int co = co0 + i, c = c0 + j;
      tile[i][j] = (co < l.cout && c < l.cin) ? prm[l.w_off + (long)co * RSC + tap * l.cin + c] : 0.f;
    }
    __syncthreads();
    // store: thread -> (row c = c0 + i, col co = co0 + j), scaled by the folded BN a[co]
    const int co = co0 + j;
    float a = 1.f;
    if (co < l.cout && (l.gamma_off >= 0 || l.var_off >= 0)) {
      const float g = l.gamma_off >= 0 ? prm[l.gamma_off + co] : 1.f;
      const float var = l.var_off >= 0 ? prm[l.var_off + co] : 1.f - eps;
      a = g * rsqrtf(var + eps);
    }
    for (int i = i0; i < 64; i += 4) {
      const int c = c0 + i;
      if (c < l.cin && co < l.cout) {
        const long d = (((long)c * l.R + (l.R - 1 - r)) * l.S + (l.S - 1 - s)) * l.cout_pad + co;
        wbf[l.wd_off + d] = wcvt<T>(a * tile[j][i]);
      }
    }
    __syncthreads();
  }
}

// Fused projection-block forward weights (FuseLayer): element (co, k) of [cout][k3 + k0] is
// a3[co] * W3[co][k] (k < k3) or a0[co] * W0[co][k - k3], rounded once to bf16; the fused affine
// is scale = 1, shift = b3 + b0 (both branches' frozen-BN shifts, summed before the ReLU).
__device__ __forceinline__ void bn_fold(const float* prm, int bias, int gamma, int beta, int mean, int var, int co,
                                        float eps, float* a, float* b) {
  const float g = gamma >= 0 ? prm[gamma + co] : 1.f;
  const float v = var >= 0 ? prm[var + co] : 1.f - eps;
  const float mu = mean >= 0 ? prm[mean + co] : 0.f;
  const float be = beta >= 0 ? prm[beta + co] : 0.f;
  const float bi = bias >= 0 ? prm[bias + co] : 0.f;
  *a = (gamma >= 0 || var >= 0) ? g * rsqrtf(v + eps) : 1.f;
  *b = (bi - mu) * *a + be;
}
__global__ void prep_fuse_kernel(const float* __restrict__ prm, const FuseLayer* __restrict__ L,
                                 uint16_t* __restrict__ wbf, float* __restrict__ scale, float* __restrict__ shift,
                                 float eps) {
  const FuseLayer l = L[blockIdx.y];
  const int K = l.k3 + l.k0;
  const long n = (long)l.cout * K;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int co = (int)(e / K), k = (int)(e - (long)co * K);
    float a, b;
    float w;
    if (k < l.k3) {
      bn_fold(prm, l.bias3, l.gamma3, l.beta3, l.mean3, l.var3, co, eps, &a, &b);
      w = prm[l.w3_off + (long)co * l.k3 + k];
    } else {
      bn_fold(prm, l.bias0, l.gamma0, l.beta0, l.mean0, l.var0, co, eps, &a, &b);
      w = prm[l.w0_off + (long)co * l.k0 + (k - l.k3)];
    }
    wbf[l.wf_off + e] = f2bf(a * w);
    if (k == 0) {
      float a3, b3, a0, b0;
      bn_fold(prm, l.bias3, l.gamma3, l.beta3, l.mean3, l.var3, co, eps, &a3, &b3);
      bn_fold(prm, l.bias0, l.gamma0, l.beta0, l.mean0, l.var0, co, eps, &a0, &b0);
      scale[l.ch_off + co] = 1.f;
      shift[l.ch_off + co] = b3 + b0;
    }
  }
}
const char* prep_fuse_launch(const float* params, const FuseLayer* layers_dev, int nlayers, int max_elems,
                             uint16_t* wbf, float* scale, float* shift, float eps, hipStream_t s) {
  int gx = (max_elems + 255) / 256;
  if (gx > 1024) gx = 1024;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(prep_fuse_kernel, dim3(gx, nlayers), dim3(256), 0, s, params, layers_dev, wbf, scale, shift, eps);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

const char* prep_launch(const float* params, const PrepLayer* layers_dev, int nlayers, int max_elems, uint16_t* wbf,
                        float* scale, float* shift, float eps, hipStream_t s, int parts) {
  // parts: bit 0 the forward weights + folded affine, bit 1 the dgrad weights (independent
  // passes over the master: the engine may run the second on its side stream, under the forward)
  int gx = (max_elems / 4 + 255) / 256;
  if (gx > 512) gx = 512;
  if (parts & 1)
    hipLaunchKernelGGL(prep_kernel<uint16_t>, dim3(gx, nlayers), dim3(256), 0, s, params, layers_dev, wbf, scale, shift,
                       eps);
  if (parts & 2)
    hipLaunchKernelGGL(prep_dgrad_kernel<uint16_t>, dim3(576, nlayers), dim3(256), 0, s, params, layers_dev, wbf, eps);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* prep_f32_launch(const float* params, const PrepLayer* layers_dev, int nlayers, float* wf32, float* scale,
                            float* shift, float eps, hipStream_t s) {
  hipLaunchKernelGGL(prep_kernel<float>, dim3(64, nlayers), dim3(256), 0, s, params, layers_dev, wf32, scale, shift, eps);
  hipLaunchKernelGGL(prep_dgrad_kernel<float>, dim3(576, nlayers), dim3(256), 0, s, params, layers_dev, wf32, eps);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// --------------------------------------------------------------------- wgrad finalize
// Per output row co of each layer in the table: dW[co] *= a[co] (the folded BN scale) and
// dgamma_raw[co] = <W[co], dW_raw[co]>.  One WAVE per row, 4 rows per 256-thread workgroup, rows
// streamed as 16-byte vectors (a row is 64-4608 floats): the pass is bound by reading
// W + dW and writing dW once, four 16-byte pairs per lane in flight (a one-row-per-workgroup
// form ran b32 at 16 us per block, 5x the bytes bound).  Rows whose offset or length is not a multiple of 4 floats (the stem, k = 147)
// take the scalar loop.
__global__ void __launch_bounds__(256) wgrad_finalize_kernel(const float* __restrict__ prm, float* __restrict__ grads,
                                                             const FinLayer* __restrict__ L,
                                                             const float* __restrict__ scale,
                                                             float* __restrict__ dgamma_raw) {
  const FinLayer l = L[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int co = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (co >= l.cout) return;
  const long base = l.w_off + (long)co * l.k;
  const float a = l.ch_off >= 0 ? scale[l.ch_off + co] : 1.f;
  float dot = 0.f;
  if (((base | l.k) & 3) == 0) {
    const float4* w = reinterpret_cast<const float4*>(prm + base);
    float4* dw = reinterpret_cast<float4*>(grads + base);
    const int n4 = l.k >> 2;
    int i = lane;
    for (; i + 192 < n4; i += 256) {   // four 16-byte pairs per lane in flight
      float4 wv[4], dv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { wv[u] = w[i + 64 * u]; dv[u] = dw[i + 64 * u]; }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dot += wv[u].x * dv[u].x + wv[u].y * dv[u].y + wv[u].z * dv[u].z + wv[u].w * dv[u].w;
        dw[i + 64 * u] = make_float4(dv[u].x * a, dv[u].y * a, dv[u].z * a, dv[u].w * a);
      }
    }
    for (; i < n4; i += 64) {
      const float4 w0 = w[i], d0 = dw[i];
      dot += w0.x * d0.x + w0.y * d0.y + w0.z * d0.z + w0.w * d0.w;
      dw[i] = make_float4(d0.x * a, d0.y * a, d0.z * a, d0.w * a);
    }
  } else {
    const float* w = prm + base;
    float* dw = grads + base;
    for (int k = lane; k < l.k; k += 64) {
      const float d = dw[k];
      dot += w[k] * d;
      dw[k] = d * a;
    }
  }
  dot = warp_sum(dot);
  if (lane == 0 && l.dg_off >= 0) dgamma_raw[l.dg_off + co] = dot;
}
const char* wgrad_finalize_launch(const float* params, float* grads, const FinLayer* layers_dev, int nlayers,
                                  const float* scale, float* dgamma_raw, hipStream_t s, int max_cout) {
  // rows of the widest layer in the table, 4 per workgroup (the table's other layers' surplus
  // rows exit at once): a stage-2 block's table is 256 rows wide, not 2048
  if (max_cout < 1 || max_cout > 65535 * 4) return "wgrad_finalize: max_cout out of range";
  hipLaunchKernelGGL(wgrad_finalize_kernel, dim3((max_cout + 3) / 4, nlayers), dim3(256), 0, s, params, grads, layers_dev,
                     scale, dgamma_raw);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// --------------------------------------------------------------------------- bn grads
__global__ void bn_grad_kernel(const float* __restrict__ prm, float* __restrict__ grads,
                               const BnGradLayer* __restrict__ L, const float* __restrict__ colsum,
                               const float* __restrict__ dgr, const float* __restrict__ scale, float eps) {
  const BnGradLayer l = L[blockIdx.y];
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < l.cout; c += gridDim.x * blockDim.x) {
    const float sg = colsum[l.colsum_off + c];
    const float a = l.ch_off >= 0 ? scale[l.ch_off + c] : 1.f;
    if (l.bias_off >= 0) grads[l.bias_off + c] = a * sg;
    if (l.beta_off >= 0) grads[l.beta_off + c] = sg;
    if (l.gamma_off >= 0) {
      const float mu = prm[l.mean_off + c], var = prm[l.var_off + c];
      const float bi = l.bias_off >= 0 ? prm[l.bias_off + c] : 0.f;
      grads[l.gamma_off + c] = (dgr[l.dg_off + c] + (bi - mu) * sg) * rsqrtf(var + eps);
    }
  }
}
const char* bn_grad_launch(const float* params, float* grads, const BnGradLayer* layers_dev, int nlayers,
                           const float* colsum, const float* dgamma_raw, const float* scale, float eps,
                           hipStream_t s) {
  hipLaunchKernelGGL(bn_grad_kernel, dim3(8, nlayers), dim3(256), 0, s, params, grads, layers_dev, colsum, dgamma_raw,
                     scale, eps);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ---------------------------------------------------------------------- synthetic data
// Deterministic synthetic ImageNet (data/datasets.py SyntheticImageNet): byte p of example i
// is a counter-based hash of (seed, i, p) -- the same example has the same pixels in every
// batch, shard and process.  Integer semantics follow the torch int64 reference exactly
// (wrapping multiplies, arithmetic right shifts).
__device__ __forceinline__ int64_t synth_mix(int64_t i, int64_t p, int64_t seed) {
  uint64_t u = (uint64_t)i * 0x9E3779B1ull + (uint64_t)p * 0x85EBCA77ull + (uint64_t)(seed + 1) * 0xC2B2AE3Dull;
  int64_t x = (int64_t)u;
  x ^= x >> 15;
  x = (int64_t)((uint64_t)x * 0x2C1B3C6Dull);
  x ^= x >> 12;
  x = (int64_t)((uint64_t)x * 0x297A2D39ull);
  x ^= x >> 15;
  return x;
}
__global__ void synth_kernel(const int64_t* __restrict__ idx, int n, long per, int64_t seed, int ncls,
                             uint8_t* __restrict__ img, int64_t* __restrict__ lab) {
  const long total4 = (long)n * per / 4;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total4; t += (long)gridDim.x * blockDim.x) {
    const long e0 = t * 4;
    const int b = (int)(e0 / per);
    const long p0 = e0 - (long)b * per;
    const int64_t i = idx[b];
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) w |= (uint32_t)(synth_mix(i, p0 + k, seed) & 255) << (8 * k);
    reinterpret_cast<uint32_t*>(img)[t] = w;
  }
  if (blockIdx.x == 0)
    for (int b = threadIdx.x; b < n; b += blockDim.x) {
      const uint64_t v = (uint64_t)idx[b] * 2654435761ull + (uint64_t)seed;
      lab[b] = (int64_t)(v % (uint64_t)ncls);
    }
}
const char* synth_launch(const int64_t* idx, int n, long per, int64_t seed, int ncls, uint8_t* img, int64_t* lab,
                         hipStream_t s) {
  if (per % 4) return "synth: bytes per example must be a multiple of 4";
  const long total4 = (long)n * per / 4;
  const int grid = (int)lmin((total4 + 255) / 256, 16384);
  hipLaunchKernelGGL(synth_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, idx, n, per, seed, ncls, img, lab);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
