// Fused optimizers over the flat fp32 parameter buffer (gfx950).
//
// Adam follows TF/Keras ResourceApplyAdam exactly (reference: `optimizer='adam'` at
// imagenet-resnet50.py:62, `keras.optimizers.Adam(learning_rate=0.1*hvd.size())` at
// imagenet-resnet50-hvd.py:99): the bias correction is folded into the step
// size ("epsilon hat"):  lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t),
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;  p -= lr_t * m / (sqrt(v) + eps).
// SGD with momentum follows keras.optimizers.SGD:  v = mu v - lr g;  p += v  (Nesterov:
// p += mu v - lr g), with optional L2 weight decay folded into g.
// One launch updates all 25.6M parameters; 16-byte loads/stores per lane.
#include "common.h"
#include "kernels.h"

namespace pddl {

// Device-resident step hyper-parameters hs = {t, lr, lr_t}: one thread advances the step
// counter and derives the step size, so a captured training step (HIP graph) replays with
// the right bias correction and with learning-rate changes the host writes between replays.
__global__ void opt_hparams_kernel(float* hs, float b1, float b2, int adam) {
  const float t = hs[0] + 1.f;
  hs[0] = t;
  hs[2] = adam ? hs[1] * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t)) : hs[1];
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long n4, float lr_t, float b1, float b2, float eps, float gs,
                            const float* __restrict__ hs) {
  if (hs) lr_t = hs[2];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
#define ADAM1(c)                                              \
  {                                                           \
    const float gr = gg.c * gs;                               \
    mm.c = b1 * mm.c + (1.f - b1) * gr;                       \
    vv.c = b2 * vv.c + (1.f - b2) * gr * gr;                  \
    pp.c -= lr_t * mm.c / (sqrtf(vv.c) + eps);                \
  }
    ADAM1(x) ADAM1(y) ADAM1(z) ADAM1(w)
#undef ADAM1
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
}

// Parameter-server form with the bf16 wire (--ps-wire bf16): the gradient arrives in bf16
// (the worker's mailbox push) and the update also writes the bf16 snapshot of the new
// parameters that the pulls copy (half the xGMI bytes both ways; the PS keeps fp32 master
// weights and Adam slots).  Same arithmetic as adam_kernel.
__global__ void adam_bf16_wire_kernel(float* __restrict__ p, const uint16_t* __restrict__ g, float* __restrict__ m,
                                      float* __restrict__ v, uint16_t* __restrict__ snap, long n4, float lr_t,
                                      float b1, float b2, float eps) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const uint2 gb = reinterpret_cast<const uint2*>(g)[i];
    const float4 gg = make_float4(__uint_as_float(gb.x << 16), __uint_as_float(gb.x & 0xffff0000u),
                                  __uint_as_float(gb.y << 16), __uint_as_float(gb.y & 0xffff0000u));
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
#define ADAM1(c)                                              \
  {                                                           \
    const float gr = gg.c;                                    \
    mm.c = b1 * mm.c + (1.f - b1) * gr;                       \
    vv.c = b2 * vv.c + (1.f - b2) * gr * gr;                  \
    pp.c -= lr_t * mm.c / (sqrtf(vv.c) + eps);                \
  }
    ADAM1(x) ADAM1(y) ADAM1(z) ADAM1(w)
#undef ADAM1
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    reinterpret_cast<uint2*>(snap)[i] = make_uint2(pack2(pp.x, pp.y), pack2(pp.z, pp.w));
  }
}

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ mom, long n4,
                           float lr, float mu, float wd, int nesterov, float gs, const float* __restrict__ hs) {
  if (hs) lr = hs[2];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 vv = reinterpret_cast<float4*>(mom)[i];
#define SGD1(c)                                               \
  {                                                           \
    const float gr = gg.c * gs + wd * pp.c;                   \
    vv.c = mu * vv.c - lr * gr;                               \
    pp.c += nesterov ? (mu * vv.c - lr * gr) : vv.c;          \
  }
    SGD1(x) SGD1(y) SGD1(z) SGD1(w)
#undef SGD1
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(mom)[i] = vv;
  }
}

__global__ void scale_kernel(float* __restrict__ x, long n, float a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= a;
}
__global__ void cast_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = f2bf(x[i]);
}
__global__ void cast_f32_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = bf2f(x[i]);
}

static int grid_of(long n) { return (int)lmin((n + 255) / 256, 4096); }
#define LAUNCH_RET                                        \
  {                                                       \
    hipError_t e = hipGetLastError();                     \
    return e == hipSuccess ? nullptr : hipGetErrorString(e); \
  }

const char* opt_hparams_launch(float* hs, float b1, float b2, int adam, hipStream_t s) {
  hipLaunchKernelGGL(opt_hparams_kernel, dim3(1), dim3(1), 0, s, hs, b1, b2, adam);
  LAUNCH_RET
}
const char* adam_launch(float* p, const float* g, float* m, float* v, long n, float lr_t, float b1, float b2,
                        float eps, float gscale, const float* hs, hipStream_t s) {
  if (n % 4) return "adam: n must be a multiple of 4";
  hipLaunchKernelGGL(adam_kernel, dim3(grid_of(n / 4)), dim3(256), 0, s, p, g, m, v, n / 4, lr_t, b1, b2, eps, gscale,
                     hs);
  LAUNCH_RET
}
const char* sgd_launch(float* p, const float* g, float* mom, long n, float lr, float momentum, float wd, int nesterov,
                       float gscale, const float* hs, hipStream_t s) {
  if (n % 4) return "sgd: n must be a multiple of 4";
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_of(n / 4)), dim3(256), 0, s, p, g, mom, n / 4, lr, momentum, wd, nesterov,
                     gscale, hs);
  LAUNCH_RET
}
const char* scale_launch(float* x, long n, float a, hipStream_t s) {
  hipLaunchKernelGGL(scale_kernel, dim3(grid_of(n)), dim3(256), 0, s, x, n, a);
  LAUNCH_RET
}
const char* adam_bf16_wire_launch(float* p, const uint16_t* g, float* m, float* v, uint16_t* snap, long n, float lr_t,
                                  float b1, float b2, float eps, hipStream_t s) {
  if (n % 4) return "adam_bf16_wire: n must be a multiple of 4";
  hipLaunchKernelGGL(adam_bf16_wire_kernel, dim3(grid_of(n / 4)), dim3(256), 0, s, p, g, m, v, snap, n / 4, lr_t, b1,
                     b2, eps);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}
const char* cast_bf16_launch(const float* x, uint16_t* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_of(n)), dim3(256), 0, s, x, y, n);
  LAUNCH_RET
}
const char* cast_f32_launch(const uint16_t* x, float* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_kernel, dim3(grid_of(n)), dim3(256), 0, s, x, y, n);
  LAUNCH_RET
}

}  // namespace pddl
