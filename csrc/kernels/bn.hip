// Train-mode BatchNormalization (batch statistics) for CDNA4 (gfx950).
//
// The reference calls the backbone with training=False (imagenet-resnet50.py:57),
// so its 53 BatchNormalization layers are per-channel affines that the frozen path folds into
// the conv epilogues.  `bn_mode=train` (Keras BN with training=True: FusedBatchNormV3 with
// batch statistics, momentum 0.99, epsilon 1.001e-5) runs here instead:
//
//   forward   conv igemm epilogue  -> z (bf16) + per-wave partial (sum z, sum z^2)   [igemm.hip]
//             colsum_reduce        -> per-channel (S, Q)                              [eltwise.hip]
//             bn_stats             -> mean, 1/sigma, scale = gamma/sigma, shift = beta - mean*scale,
//                                     moving statistics update (unbiased variance)
//             bn_apply             -> y = relu(z*scale + shift (+ residual | + bn(z0))) + ReLU bitmask
//   backward  bn_bwd_reduce        -> Sg = sum g, Sgx = sum g*(z - mean) (mean-centred: no cancellation)
//             bn_bwd_apply         -> dz = gamma/sigma * (g - Sg/M - (z-mean)/sigma^2 * Sgx/M),
//                                     dgamma = Sgx/sigma, dbeta = Sg, dbias = 0
//
// Every elementwise pass moves 8 channels per lane (16 bytes bf16, 32 bytes fp32: the kernels are
// templated on the activation type, the fp32 ones serve the reference-precision train-BN engine)
// and keeps one channel group per lane (grid stride a multiple of C/8), so its per-channel
// coefficients load once.
#include "common.h"
#include "kernels.h"

namespace pddl {

// 8 consecutive channels of one row: bf16 activations (one 16-byte load) or fp32 ones (the
// reference-precision engine, models/engine_f32.py: two 16-byte loads).  store() returns the
// ReLU bitmask of the stored values (bit e: value e > 0).
template <class T> struct Vec8;
template <> struct Vec8<bf16_t> {
  uint4 q;
  __device__ __forceinline__ void load(const bf16_t* p, long t) { q = reinterpret_cast<const uint4*>(p)[t]; }
  __device__ __forceinline__ void get(float* v) const { unpack8(q, v); }
  __device__ static __forceinline__ uint32_t store(bf16_t* p, long t, const float* v) {
    const uint4 k = pack8(v);
    reinterpret_cast<uint4*>(p)[t] = k;
    return pos_bits8(k);
  }
};
template <> struct Vec8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p, long t) {
    a = reinterpret_cast<const float4*>(p)[2 * t];
    b = reinterpret_cast<const float4*>(p)[2 * t + 1];
  }
  __device__ __forceinline__ void get(float* v) const {
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ static __forceinline__ uint32_t store(float* p, long t, const float* v) {
    reinterpret_cast<float4*>(p)[2 * t] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[2 * t + 1] = make_float4(v[4], v[5], v[6], v[7]);
    uint32_t m = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) m |= (v[e] > 0.f ? 1u : 0u) << e;
    return m;
  }
};

// ~8 blocks of 256 lanes per CU; lanes loop so their per-channel setup is amortized
// Grid caps of the streaming BN kernels (bench/bn.py sweep at b256, profiles/r1_bn_kernels_b256.json):
// 512 blocks of 256 lanes for < 4M channel groups, 1024 above (2048 was 1.2-2x slower on the
// 7x7 / 14x14 layers); 0 = this heuristic, > 0 forces a cap.
int g_bn_apply_blocks = 0;
int g_bn_red_blocks = 0;        // bn_bwd_reduce block cap: 0 = heuristic (see the launcher)
static int bn_grid(long n) {
  const long cap = g_bn_apply_blocks > 0 ? g_bn_apply_blocks : (n >= (4L << 20) ? 1024 : 512);
  return (int)lmin((n + 255) / 256, cap);
}

// ------------------------------------------------------------------------------ stats
__global__ void bn_stats_kernel(const float* __restrict__ acc, const BnStatLayer* __restrict__ L, int training,
                                float* __restrict__ prm, float* __restrict__ mean, float* __restrict__ inv,
                                float* __restrict__ scale, float* __restrict__ shift, float eps, float momentum) {
  const BnStatLayer l = L[blockIdx.y];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= l.C) return;
  float mu, var;
  if (training) {
    const double S = acc[l.sum_off + c], Q = acc[l.sq_off + c], n = l.count;
    const double m = S / n;
    double v = Q / n - m * m;
    v = v > 0.0 ? v : 0.0;
    mu = (float)m; var = (float)v;
    // Keras moving statistics: mean and Bessel-corrected variance, momentum 0.99
    float& mm = prm[l.mm_off + c];
    float& mv = prm[l.mv_off + c];
    mm = mm * momentum + (1.f - momentum) * mu;
    mv = mv * momentum + (1.f - momentum) * (float)(v * n / (n > 1.0 ? n - 1.0 : 1.0));
  } else {
    mu = prm[l.mm_off + c]; var = prm[l.mv_off + c];
  }
  const float is = rsqrtf(var + eps);
  const float a = prm[l.gamma_off + c] * is;
  mean[l.ch + c] = mu;
  inv[l.ch + c] = is;
  scale[l.ch + c] = a;
  shift[l.ch + c] = prm[l.beta_off + c] - mu * a;
}

const char* bn_stats_launch(const float* acc, const BnStatLayer* layers_dev, int nlayers, int max_c, int training,
                            float* params, float* mean, float* inv, float* scale, float* shift, float eps,
                            float momentum, hipStream_t s) {
  hipLaunchKernelGGL(bn_stats_kernel, dim3((max_c + 255) / 256, nlayers), dim3(256), 0, s, acc, layers_dev, training,
                     params, mean, inv, scale, shift, eps, momentum);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ------------------------------------------------------------------------------ apply
// y = act(z*a + b (+ r | + r*a2 + b2)); bits (nullable) = ReLU bitmask of the stored y.
template <class T>
__global__ void bn_apply_kernel(const T* __restrict__ z, const float* __restrict__ a, const float* __restrict__ b,
                                const T* __restrict__ r, const float* __restrict__ a2, const float* __restrict__ b2,
                                int relu, T* __restrict__ y, uint8_t* __restrict__ bits, long M, int C) {
  // the grid stride is a multiple of C/8 (a power of two <= 256): every lane keeps one
  // channel group, so its per-channel coefficients are loaded once
  const int cg = C >> 3;
  const long total = M * cg;
  const long t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int c0 = (int)(t0 % cg) * 8;
  float sa[8], sb[8], ra[8], rb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sa[e] = a[c0 + e]; sb[e] = b[c0 + e];
    ra[e] = a2 ? a2[c0 + e] : 1.f; rb[e] = a2 ? b2[c0 + e] : 0.f;
  }
  // two items per iteration, both loads issued before either is used (memory-level
  // parallelism: one item per lane left these streaming kernels at ~3.4 TB/s)
  const long stride = (long)gridDim.x * blockDim.x;
  for (long t = t0; t < total; t += 2 * stride) {
    const bool two = t + stride < total;
    Vec8<T> zq0, zq1, rq0, rq1;
    zq0.load(z, t);
    zq1 = zq0;
    if (two) zq1.load(z, t + stride);
    if (r) {
      rq0.load(r, t);
      rq1 = rq0;
      if (two) rq1.load(r, t + stride);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      float v[8];
      (u ? zq1 : zq0).get(v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * sa[e] + sb[e];
      if (r) {
        float rv[8];
        (u ? rq1 : rq0).get(rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rv[e] * ra[e] + rb[e];
      }
      if (relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      const long tu = t + u * stride;
      const uint32_t m = Vec8<T>::store(y, tu, v);
      if (bits) bits[tu] = (uint8_t)m;
    }
  }
}

template <class T>
static const char* bn_apply_any(const T* z, const float* a, const float* b, const T* r, const float* a2,
                                const float* b2, int relu, T* y, uint8_t* bits, long M, int C, hipStream_t s) {
  if (C % 8 || 256 % (C / 8)) return "bn_apply: C/8 must divide 256";
  hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(bn_grid(M * (C / 8))), dim3(256), 0, s, z, a, b, r, a2, b2, relu, y,
                     bits, M, C);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* bn_apply_launch(const uint16_t* z, const float* a, const float* b, const uint16_t* r, const float* a2,
                            const float* b2, int relu, uint16_t* y, uint8_t* bits, long M, int C, hipStream_t s) {
  return bn_apply_any<bf16_t>(reinterpret_cast<const bf16_t*>(z), a, b, reinterpret_cast<const bf16_t*>(r), a2, b2,
                              relu, reinterpret_cast<bf16_t*>(y), bits, M, C, s);
}
const char* bn_apply_launch(const float* z, const float* a, const float* b, const float* r, const float* a2,
                            const float* b2, int relu, float* y, uint8_t* bits, long M, int C, hipStream_t s) {
  return bn_apply_any<float>(z, a, b, r, a2, b2, relu, y, bits, M, C, s);
}

// ----------------------------------------------------------------------- bwd reduce
// Per channel: Sg += sum_m g, Sgx += sum_m g*(z - mean), Sgx2 += sum_m g*(z2 - mean2).
// A block takes a contiguous row range; lane (row-slot, column-group) keeps 8 channels in
// registers, the row slots are folded through LDS and one fp32 atomic per channel and block
// lands in the per-step workspace.
template <class T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const T* __restrict__ g, const T* __restrict__ z,
                                                            const T* __restrict__ z2,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ mean2, long M, int C,
                                                            float* __restrict__ sg, float* __restrict__ sgx,
                                                            float* __restrict__ sg2, float* __restrict__ sgx2) {
  __shared__ float red[3][256 * 8 / 1];   // [sum][slot * G + col-group][e] folded below
  const int G = C >> 3;                 // column groups (<= 256)
  const int RPI = 256 / G;              // row slots per iteration
  const int tid = threadIdx.x;
  const int cgi = tid % G, slot = tid / G;
  const long rows_per = (M + gridDim.x - 1) / gridDim.x;
  const long r0 = blockIdx.x * rows_per, r1 = lmin(M, r0 + rows_per);
  float s0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], mu2[8];
  const int c0 = cgi * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) { mu[e] = mean[c0 + e]; mu2[e] = z2 ? mean2[c0 + e] : 0.f; }
  if (slot < RPI) {
    for (long row = r0 + slot; row < r1; row += 2 * RPI) {   // two rows in flight per lane
      const bool two = row + RPI < r1;
      const long o = row * G + cgi, o1 = two ? o + (long)RPI * G : o;
      Vec8<T> gq0, gq1, zq0, zq1, wq0, wq1;
      gq0.load(g, o); gq1.load(g, o1);
      zq0.load(z, o); zq1.load(z, o1);
      if (z2) { wq0.load(z2, o); wq1.load(z2, o1); }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        float gv[8], zv[8];
        (u ? gq1 : gq0).get(gv);
        (u ? zq1 : zq0).get(zv);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s0[e] += gv[e]; s1[e] += gv[e] * (zv[e] - mu[e]); }
        if (z2) {
          (u ? wq1 : wq0).get(zv);
#pragma unroll
          for (int e = 0; e < 8; ++e) s2[e] += gv[e] * (zv[e] - mu2[e]);
        }
      }
    }
  }
  // fold the row slots: red[k][slot*G*8 + cgi*8 + e] (RPI * G <= 256 lanes -> <= 2048 floats)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][tid * 8 + e] = s0[e];
    red[1][tid * 8 + e] = s1[e];
    red[2][tid * 8 + e] = s2[e];
  }
  __syncthreads();
  // thread t < C finalizes channel t: sum over slots of red[k][(slot*G + t/8)*8 + t%8]
  for (int c = tid; c < C; c += 256) {
    const int cg2 = c >> 3, e = c & 7;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int sl = 0; sl < RPI; ++sl) {
      const int idx = (sl * G + cg2) * 8 + e;
      a0 += red[0][idx]; a1 += red[1][idx]; a2 += red[2][idx];
    }
    unsafeAtomicAdd(sg + c, a0);
    unsafeAtomicAdd(sgx + c, a1);
    if (z2) {   // the projection shortcut's BN sees the same gradient
      unsafeAtomicAdd(sg2 + c, a0);
      unsafeAtomicAdd(sgx2 + c, a2);
    }
  }
}

template <class T>
static const char* bn_bwd_reduce_any(const T* g, const T* z, const T* z2, const float* mean, const float* mean2,
                                     long M, int C, float* sg, float* sgx, float* sg2, float* sgx2, hipStream_t s) {
  if (C % 8 || C > 2048) return "bn_bwd_reduce: C must be a multiple of 8 and <= 2048";
  const int G = C / 8, rpi = 256 / G;
  // >= 8 row iterations per lane
  long nb = M / ((long)rpi * 8);
  // About one block per CU (bench/bn.py sweep, profiles/r1_bn_kernels_b256.json): more blocks
  // only add per-block LDS folds and same-address atomics (2048 blocks ran the 56x56x64
  // reduce at 3.2 TB/s, 256 blocks at 6.0); the largest layers take 512.
  const long cap = g_bn_red_blocks > 0 ? g_bn_red_blocks : (M * C > (1L << 27) ? 512 : 256);
  nb = nb < 1 ? 1 : (nb > cap ? cap : nb);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3((int)nb), dim3(256), 0, s, g, z, z2, mean, mean2, M, C, sg,
                     sgx, sg2, sgx2);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* bn_bwd_reduce_launch(const uint16_t* g, const uint16_t* z, const uint16_t* z2, const float* mean,
                                 const float* mean2, long M, int C, float* sg, float* sgx, float* sg2,
                                 float* sgx2, hipStream_t s) {
  return bn_bwd_reduce_any<bf16_t>(reinterpret_cast<const bf16_t*>(g), reinterpret_cast<const bf16_t*>(z),
                                   reinterpret_cast<const bf16_t*>(z2), mean, mean2, M, C, sg, sgx, sg2, sgx2, s);
}
const char* bn_bwd_reduce_launch(const float* g, const float* z, const float* z2, const float* mean,
                                 const float* mean2, long M, int C, float* sg, float* sgx, float* sg2,
                                 float* sgx2, hipStream_t s) {
  return bn_bwd_reduce_any<float>(g, z, z2, mean, mean2, M, C, sg, sgx, sg2, sgx2, s);
}

// ------------------------------------------------------------------------ bwd apply
// Per channel (one thread each): dz = A*g + B*z + C with A = gamma/sigma,
// B = -A/sigma^2 * Sgx/M (Sgx = sum g*(z-mean)), C = -A*Sg/M - B*mean; and the parameter
// gradients dgamma = Sgx/sigma, dbeta = Sg, dbias = 0 (BN removes any per-channel shift).
__global__ void bn_bwd_coef_kernel(BnBwdLayer l, const float* __restrict__ prm, const float* __restrict__ mean,
                                   const float* __restrict__ inv, const float* __restrict__ sg,
                                   const float* __restrict__ sgx, float* __restrict__ coef, int ldc,
                                   float* __restrict__ grads) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= l.C) return;
  const int k = l.ch + c;
  const float is = inv[k], s0 = sg[k], s1 = sgx[k], rn = 1.f / l.count;
  const float A = prm[l.gamma_off + c] * is;
  const float B = -A * is * is * s1 * rn;
  coef[k] = A;
  coef[ldc + k] = B;
  coef[2 * ldc + k] = -A * s0 * rn - B * mean[k];
  grads[l.gamma_off + c] = s1 * is;
  grads[l.beta_off + c] = s0;
  if (l.bias_off >= 0) grads[l.bias_off + c] = 0.f;
}

__device__ __forceinline__ void load8(const float* p, float* v) {
  *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(p);
  *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(p + 4);
}

// dz = A*g + B*z + C (and dz2 from z2 with the second layer's coefficients; same g).
// dz / dz2 may alias g (each lane reads its g before writing).  The grid stride is a
// multiple of C/8, so a lane's 24 (or 48) coefficients are loaded once.
template <class T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* g, const T* __restrict__ z,
                                                           const T* __restrict__ z2,
                                                           const float* __restrict__ c1, const float* __restrict__ c2,
                                                           int ldc, T* dz, T* dz2, long M, int C) {
  const int cg = C >> 3;
  const long total = M * cg;
  const long t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int c0 = (int)(t0 % cg) * 8;
  float A[8], B[8], Cc[8], A2[8], B2[8], C2[8];
  load8(c1 + c0, A); load8(c1 + ldc + c0, B); load8(c1 + 2 * ldc + c0, Cc);
  if (z2) { load8(c2 + c0, A2); load8(c2 + ldc + c0, B2); load8(c2 + 2 * ldc + c0, C2); }
  const long stride = (long)gridDim.x * blockDim.x;
  for (long t = t0; t < total; t += 2 * stride) {   // two items in flight per lane (see bn_apply)
    const bool two = t + stride < total;
    Vec8<T> gq0, zq0, gq1, zq1, wq0, wq1;
    gq0.load(g, t);
    zq0.load(z, t);
    gq1 = gq0;
    zq1 = zq0;
    if (two) { gq1.load(g, t + stride); zq1.load(z, t + stride); }
    if (z2) {
      wq0.load(z2, t);
      wq1 = wq0;
      if (two) wq1.load(z2, t + stride);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      float gv[8], zv[8], o[8];
      (u ? gq1 : gq0).get(gv);
      (u ? zq1 : zq0).get(zv);
      const long tu = t + u * stride;
      if (z2) {
        float wv[8], o2[8];
        (u ? wq1 : wq0).get(wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o2[e] = A2[e] * gv[e] + B2[e] * wv[e] + C2[e];
        Vec8<T>::store(dz2, tu, o2);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = A[e] * gv[e] + B[e] * zv[e] + Cc[e];
      Vec8<T>::store(dz, tu, o);
    }
  }
}

template <class T>
static const char* bn_bwd_apply_any(const T* g, const T* z, const T* z2, const BnBwdLayer& l, const BnBwdLayer& l2,
                                    const float* params, const float* mean, const float* inv, const float* sg,
                                    const float* sgx, float* coef, int ldc, T* dz, T* dz2, float* grads, long M,
                                    hipStream_t s) {
  if (l.C % 8 || 256 % (l.C / 8)) return "bn_bwd_apply: C/8 must divide 256";
  if (z2 && (l2.C != l.C || !dz2)) return "bn_bwd_apply: second source must match";
  const int cb = (l.C + 255) / 256;
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3(cb), dim3(256), 0, s, l, params, mean, inv, sg, sgx, coef, ldc, grads);
  if (z2)
    hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3(cb), dim3(256), 0, s, l2, params, mean, inv, sg, sgx, coef, ldc,
                       grads);
  hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(bn_grid(M * (l.C / 8))), dim3(256), 0, s, g, z, z2, coef + l.ch,
                     coef + l2.ch, ldc, dz, dz2, M, l.C);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* bn_bwd_apply_launch(const uint16_t* g, const uint16_t* z, const uint16_t* z2, const BnBwdLayer& l,
                                const BnBwdLayer& l2, const float* params, const float* mean, const float* inv,
                                const float* sg, const float* sgx, float* coef, int ldc, uint16_t* dz, uint16_t* dz2,
                                float* grads, long M, hipStream_t s) {
  return bn_bwd_apply_any<bf16_t>(reinterpret_cast<const bf16_t*>(g), reinterpret_cast<const bf16_t*>(z),
                                  reinterpret_cast<const bf16_t*>(z2), l, l2, params, mean, inv, sg, sgx, coef, ldc,
                                  reinterpret_cast<bf16_t*>(dz), reinterpret_cast<bf16_t*>(dz2), grads, M, s);
}
const char* bn_bwd_apply_launch(const float* g, const float* z, const float* z2, const BnBwdLayer& l,
                                const BnBwdLayer& l2, const float* params, const float* mean, const float* inv,
                                const float* sg, const float* sgx, float* coef, int ldc, float* dz, float* dz2,
                                float* grads, long M, hipStream_t s) {
  return bn_bwd_apply_any<float>(g, z, z2, l, l2, params, mean, inv, sg, sgx, coef, ldc, dz, dz2, grads, M, s);
}

}  // namespace pddl
