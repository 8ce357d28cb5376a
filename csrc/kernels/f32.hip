// fp32 elementwise / reduction kernels of the reference-precision engine (models/engine_f32.py):
// the reference trains in float32 (imagenet-resnet50.py:56-62, no mixed-precision policy), so
// its max-pool, global-average-pool, softmax cross-entropy and the per-channel column sums run
// here on fp32 NHWC activations, 16 bytes (4 channels) per lane.
//   * maxpool_fwd_f32 : ZeroPadding2D(1) + MaxPooling2D(3, 2), first argmax in scan order -> idx
//   * maxpool_bwd_f32 : gather form (each input position sums the outputs whose argmax is it),
//                       fused with the ReLU mask of conv1's output (no atomics)
//   * gap_fwd_f32 / gap_bwd_f32 (+ ReLU mask of the last block's output, partial column sums)
//   * colsum_f32      : out[c] += sum_m g[m][c]
//   * softmax_xent_f32: softmax + sparse categorical CE + accuracy, fp32 dlogits
#include "common.h"
#include "kernels.h"

namespace pddl {

namespace {
int grid_f32(long n) { return (int)lmin((n + 255) / 256, 16384); }
const char* last_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
}  // namespace

// ------------------------------------------------------------------------------ maxpool
__global__ void maxpool_fwd_f32_kernel(const float* __restrict__ x, float* __restrict__ y, uint8_t* __restrict__ idx,
                                       int B, int H, int W, int C, int Ho, int Wo) {
  const int cg = C / 4;
  const long total = (long)B * Ho * Wo * cg;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int g = (int)(t % cg);
    long q = t / cg;
    const int wo = (int)(q % Wo);
    q /= Wo;
    const int ho = (int)(q % Ho), b = (int)(q / Ho);
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int am[4] = {0, 0, 0, 0};
    for (int r = 0; r < 3; ++r) {
      const int h = 2 * ho - 1 + r;
      for (int s = 0; s < 3; ++s) {
        const int w = 2 * wo - 1 + s;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);   // ZeroPadding2D: padded taps are real zeros
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
          v = *reinterpret_cast<const float4*>(x + (((long)b * H + h) * W + w) * C + 4 * g);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (vv[e] > mx[e]) { mx[e] = vv[e]; am[e] = r * 3 + s; }
      }
    }
    const long o = (((long)b * Ho + ho) * Wo + wo) * C + 4 * g;
    *reinterpret_cast<float4*>(y + o) = make_float4(mx[0], mx[1], mx[2], mx[3]);
    *reinterpret_cast<uchar4*>(idx + o) = make_uchar4(am[0], am[1], am[2], am[3]);
  }
}

__global__ void maxpool_bwd_f32_kernel(const float* __restrict__ gy, const uint8_t* __restrict__ idx,
                                       const float* __restrict__ xmask, float* __restrict__ gx, int B, int H, int W,
                                       int C, int Ho, int Wo) {
  const int cg = C / 4;
  const long total = (long)B * H * W * cg;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int g = (int)(t % cg);
    long q = t / cg;
    const int w = (int)(q % W);
    q /= W;
    const int h = (int)(q % H), b = (int)(q / H);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    // outputs whose window (rows 2ho-1 .. 2ho+1) covers h: ho in [h/2, (h+1)/2]
    const int ho0 = h / 2, ho1 = min((h + 1) / 2, Ho - 1), wo0 = w / 2, wo1 = min((w + 1) / 2, Wo - 1);
    for (int ho = ho0; ho <= ho1; ++ho)
      for (int wo = wo0; wo <= wo1; ++wo) {
        const int tap = (h - (2 * ho - 1)) * 3 + (w - (2 * wo - 1));
        const long o = (((long)b * Ho + ho) * Wo + wo) * C + 4 * g;
        const uchar4 id = *reinterpret_cast<const uchar4*>(idx + o);
        const float4 gv = *reinterpret_cast<const float4*>(gy + o);
        if (id.x == tap) acc[0] += gv.x;
        if (id.y == tap) acc[1] += gv.y;
        if (id.z == tap) acc[2] += gv.z;
        if (id.w == tap) acc[3] += gv.w;
      }
    const long i = (((long)b * H + h) * W + w) * C + 4 * g;
    const float4 mk = *reinterpret_cast<const float4*>(xmask + i);   // conv1's ReLU output
    *reinterpret_cast<float4*>(gx + i) = make_float4(mk.x > 0.f ? acc[0] : 0.f, mk.y > 0.f ? acc[1] : 0.f,
                                                     mk.z > 0.f ? acc[2] : 0.f, mk.w > 0.f ? acc[3] : 0.f);
  }
}

const char* maxpool_fwd_f32_launch(const float* x, float* y, uint8_t* idx, int B, int H, int W, int C, int Ho, int Wo,
                                   hipStream_t s) {
  if (C % 4) return "maxpool_f32: C % 4";
  hipLaunchKernelGGL(maxpool_fwd_f32_kernel, dim3(grid_f32((long)B * Ho * Wo * C / 4)), dim3(256), 0, s, x, y, idx, B,
                     H, W, C, Ho, Wo);
  return last_err();
}
const char* maxpool_bwd_f32_launch(const float* gy, const uint8_t* idx, const float* xmask, float* gx, int B, int H,
                                   int W, int C, int Ho, int Wo, hipStream_t s) {
  if (C % 4) return "maxpool_f32: C % 4";
  if (Ho != (H + 2 - 3) / 2 + 1 || Wo != (W + 2 - 3) / 2 + 1) return "maxpool_f32: output size";
  hipLaunchKernelGGL(maxpool_bwd_f32_kernel, dim3(grid_f32((long)B * H * W * C / 4)), dim3(256), 0, s, gy, idx, xmask,
                     gx, B, H, W, C, Ho, Wo);
  return last_err();
}

// ---------------------------------------------------------------------------------- GAP
__global__ void gap_fwd_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int HW, int C) {
  const int cg = C / 4;
  const long total = (long)B * cg;
  const float inv = 1.f / HW;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int g = (int)(t % cg), b = (int)(t / cg);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = 0; i < HW; ++i) {
      const float4 v = *reinterpret_cast<const float4*>(x + ((long)b * HW + i) * C + 4 * g);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    *reinterpret_cast<float4*>(y + (long)b * C + 4 * g) = make_float4(a.x * inv, a.y * inv, a.z * inv, a.w * inv);
  }
}
// g[b, i, c] = gp[b, c] / HW * (y[b, i, c] > 0); colsum_rows[b][c] = sum_i g[b, i, c] (partial rows)
__global__ void gap_bwd_f32_kernel(const float* __restrict__ gp, const float* __restrict__ ymask, float* __restrict__ g,
                                   int B, int HW, int C, float* __restrict__ colsum_rows) {
  const int cg = C / 4;
  const long total = (long)B * cg;
  const float inv = 1.f / HW;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int gg = (int)(t % cg), b = (int)(t / cg);
    const float4 v = *reinterpret_cast<const float4*>(gp + (long)b * C + 4 * gg);
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = 0; i < HW; ++i) {
      const long o = ((long)b * HW + i) * C + 4 * gg;
      const float4 m = *reinterpret_cast<const float4*>(ymask + o);
      const float4 r = make_float4(m.x > 0.f ? v.x * inv : 0.f, m.y > 0.f ? v.y * inv : 0.f,
                                   m.z > 0.f ? v.z * inv : 0.f, m.w > 0.f ? v.w * inv : 0.f);
      *reinterpret_cast<float4*>(g + o) = r;
      cs.x += r.x; cs.y += r.y; cs.z += r.z; cs.w += r.w;
    }
    if (colsum_rows) *reinterpret_cast<float4*>(colsum_rows + (long)b * C + 4 * gg) = cs;
  }
}
const char* gap_fwd_f32_launch(const float* x, float* y, int B, int HW, int C, hipStream_t s) {
  if (C % 4) return "gap_f32: C % 4";
  hipLaunchKernelGGL(gap_fwd_f32_kernel, dim3(grid_f32((long)B * C / 4)), dim3(256), 0, s, x, y, B, HW, C);
  return last_err();
}
const char* gap_bwd_f32_launch(const float* gp, const float* ymask, float* g, int B, int HW, int C, float* colsum_rows,
                               hipStream_t s) {
  if (C % 4) return "gap_f32: C % 4";
  hipLaunchKernelGGL(gap_bwd_f32_kernel, dim3(grid_f32((long)B * C / 4)), dim3(256), 0, s, gp, ymask, g, B, HW, C,
                     colsum_rows);
  return last_err();
}

// ------------------------------------------------------------------------------- colsum
// out[c] += sum_m g[m][c]: each block owns a contiguous row range; its 256 threads are CG
// column groups (4 columns) x RL row lanes; registers accumulate, LDS folds the row lanes,
// one atomic per column per block.
__global__ void colsum_f32_kernel(const float* __restrict__ g, long M, int C, int ldg, long rows_per_block,
                                  float* __restrict__ out) {
  __shared__ float4 red[256];
  const int cg = C / 4;
  const int CG = cg < 64 ? cg : 64, RL = 256 / CG;
  const int tid = threadIdx.x;
  const long r0 = blockIdx.x * rows_per_block, r1 = lmin(M, r0 + rows_per_block);
  for (int c0 = 0; c0 < cg; c0 += CG) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = c0 + tid % CG;
    if (tid < CG * RL && c < cg)
      for (long r = r0 + tid / CG; r < r1; r += RL) {
        const float4 v = *reinterpret_cast<const float4*>(g + r * ldg + 4 * c);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
    red[tid] = a;
    __syncthreads();
    if (tid < CG && c < cg) {
      float4 t = red[tid];
      for (int l = 1; l < RL; ++l) {
        const float4 u = red[l * CG + tid];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      unsafeAtomicAdd(out + 4 * c + 0, t.x);
      unsafeAtomicAdd(out + 4 * c + 1, t.y);
      unsafeAtomicAdd(out + 4 * c + 2, t.z);
      unsafeAtomicAdd(out + 4 * c + 3, t.w);
    }
    __syncthreads();
  }
}
// (any C: one thread per column, the rows split over blocks -- the Dense head with a class count
// that is not a multiple of 4)
__global__ void colsum_f32_scalar_kernel(const float* __restrict__ g, long M, int C, int ldg, long rows_per_block,
                                         float* __restrict__ out) {
  const long r0 = blockIdx.y * rows_per_block, r1 = lmin(M, r0 + rows_per_block);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    float a = 0.f;
    for (long r = r0; r < r1; ++r) a += g[r * ldg + c];
    unsafeAtomicAdd(out + c, a);
  }
}
const char* colsum_f32_launch(const float* g, long M, int C, int ldg, float* out, hipStream_t s) {
  if (C % 4 || ldg % 4) {
    const long rpb = 256, by = (M + rpb - 1) / rpb;
    hipLaunchKernelGGL(colsum_f32_scalar_kernel, dim3((C + 255) / 256, (int)lmin(by, 65535)), dim3(256), 0, s, g, M, C,
                       ldg, (M + lmin(by, 65535) - 1) / lmin(by, 65535), out);
    return last_err();
  }
  const long blocks = lmin((M + 255) / 256, 2048);
  const long rpb = (M + blocks - 1) / blocks;
  hipLaunchKernelGGL(colsum_f32_kernel, dim3((int)blocks), dim3(256), 0, s, g, M, C, ldg, rpb, out);
  return last_err();
}

// ------------------------------------------------------------------------- softmax-xent
// One wave per example (the bf16 engine's softmax_xent_kernel with fp32 dlogits).
__global__ void softmax_xent_f32_kernel(const float* __restrict__ logits, int ldl, const int64_t* __restrict__ labels,
                                        int B, int ncls, float gscale, float* __restrict__ dl, int ldd,
                                        float* __restrict__ loss_sum, float* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* row = logits + (long)b * ldl;
  float mx = -INFINITY;
  int amax = 0x7fffffff;
  for (int j = lane; j < ncls; j += 64) {
    const float v = row[j];
    if (v > mx) { mx = v; amax = j; }
  }
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
    dl[(long)b * ldd + j] = d;
  }
  if (lane == 0) {
    unsafeAtomicAdd(loss_sum, mx + __logf(se) - row[lab]);
    unsafeAtomicAdd(correct, amax == lab ? 1.f : 0.f);
  }
}
const char* softmax_xent_f32_launch(const float* logits, int ldl, const int64_t* labels, int B, int ncls, float gscale,
                                    float* dlogits, int ldd, float* loss_sum, float* correct, hipStream_t s) {
  if (ldd < ncls) return "softmax_xent_f32: ldd < ncls";
  hipLaunchKernelGGL(softmax_xent_f32_kernel, dim3((B + 3) / 4), dim3(256), 0, s, logits, ldl, labels, B, ncls, gscale,
                     dlogits, ldd, loss_sum, correct);
  return last_err();
}

}  // namespace pddl
