// Shared device helpers for the CDNA4 (gfx950 / MI355X) kernels of pddl.
//
// Storage convention: bf16 tensors are raw `uint16_t` buffers (torch.bfloat16
// bit pattern); every kernel computes in fp32 and rounds once on store.
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <mutex>
#include <stdint.h>

namespace pddl {

typedef uint16_t bf16_t;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even via the hardware convert (keeps NaN a NaN; see
// MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// ReLU bitmask of 8 packed bf16 values: bit e = (value e > 0), i.e. nonzero with a clear
// sign bit.  Derived from the stored (rounded) values so it matches a bf16 mask exactly.
// Branch- and compare-free (19 VALU, was 31 with per-half compares and selects): per word,
// t = ((w & 0x7fff7fff) + 0x7fff7fff) & ~w has bit 15 / 31 set exactly when the low / high
// half is positive (magnitude nonzero, sign clear; no carry crosses the halves); v_perm's
// sign-replicate selectors 8-11 turn those bits of two words into 0x00 / 0xff bytes, and a
// dot4 against 1,1,1,1 of the bytes masked with 1,2,4,8 packs each group into a nibble.
__device__ __forceinline__ uint32_t pos_bits8(const uint4& u) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t t[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) t[e] = ((w[e] & 0x7fff7fffu) + 0x7fff7fffu) & ~w[e];
  const uint32_t s01 = __builtin_amdgcn_perm(t[1], t[0], 0x0b0a0908u);
  const uint32_t s23 = __builtin_amdgcn_perm(t[3], t[2], 0x0b0a0908u);
  const uint32_t n01 = __builtin_amdgcn_udot4(s01 & 0x08040201u, 0x01010101u, 0u, false);
  const uint32_t n23 = __builtin_amdgcn_udot4(s23 & 0x08040201u, 0x01010101u, 0u, false);
  return n01 | (n23 << 4);
}

// ReLU of 8 packed bf16 values in the integer domain: a bf16 orders like a sign-magnitude
// int16, so max_i16(x, 0) zeroes exactly the negatives (and -0): 4 v_pk_max_i16 instead of 8
// v_max_f32 before the pack.  Rounding is monotonic, so relu(round(v)) == round(relu(v)).
__device__ __forceinline__ uint32_t relu_pk2(uint32_t u) {
  typedef short v2s __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(v2s, u), v2s{0, 0}));
}
__device__ __forceinline__ uint4 relu_pk8(uint4 u) {
  typedef short v2s __attribute__((ext_vector_type(2)));
  const v2s z = {0, 0};
  const v2s a = __builtin_elementwise_max(__builtin_bit_cast(v2s, u.x), z);
  const v2s b = __builtin_elementwise_max(__builtin_bit_cast(v2s, u.y), z);
  const v2s c = __builtin_elementwise_max(__builtin_bit_cast(v2s, u.z), z);
  const v2s d = __builtin_elementwise_max(__builtin_bit_cast(v2s, u.w), z);
  return make_uint4(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, c),
                    __builtin_bit_cast(uint32_t, d));
}

// Buffer offset past every descriptor's range (record counts are clamped below 2 GiB; large
// activations are reached through per-tile rebased descriptors, make_rsrc_at): the buffer
// unit returns zeros for it.
constexpr uint32_t OOB_OFF = 0x80000000u;

// 16-byte-per-lane buffer LDS-DMA (buffer_load_dwordx4 ... lds): LDS destination = M0 base
// (wave-uniform dst) + lane * 16; out-of-range offsets load zeros.
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, __attribute__((address_space(3))) void* dst,
                                          uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

// 64 bytes of zeros: the source of every out-of-bounds LDS-DMA lane (padding
// rows of the implicit-GEMM gather, tile overhang).  LDS-DMA cannot write a
// literal, so invalid lanes read from here instead.  One copy per translation
// unit (no relocatable device code needed).
static __device__ __attribute__((aligned(64))) uint4 g_zero_page[4];

__host__ __device__ __forceinline__ long lmin(long a, long b) { return a < b ? a : b; }
__host__ __device__ __forceinline__ long lmax(long a, long b) { return a > b ? a : b; }

// Descriptor over elements [e0, e_end) of a bf16 tensor, rebased at e0 with 64-bit pointer
// arithmetic: a workgroup's lane offsets (relative to the first image / row its tile reads)
// stay 32-bit at any batch, and the record count is clamped below OOB_OFF so that marker
// still reads zeros.  This is what lets one GPU train at b2048 (stage-1 activations > 2 GiB).
// (An empty range -- e_end <= e0 -- gives a zero-size descriptor: every access reads zeros / is dropped.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_at(const uint16_t* base, long e0, long e_end) {
  const long bytes = (e_end - e0) * 2;
  return make_rsrc(base + e0, (int)(bytes <= 0 ? 0 : lmin(bytes, 0x7fffffffL)));
}

// Division by a runtime divisor d as one 64-bit multiply + shift: exact for
// 0 <= x < 2^40 / d (every row index of the ResNet-50 GEMMs: x < 2^26, d < 2^14).
__host__ __device__ __forceinline__ uint64_t fdiv_magic(int d) { return ((1ull << 40) + d - 1) / (uint64_t)d; }
__device__ __forceinline__ int fdiv(int x, uint64_t magic) { return (int)(((uint64_t)(uint32_t)x * magic) >> 40); }

// Bijective XCD-aware remap of the linear workgroup id (cdna_hip_programming
// §5 "XCD swizzle must be bijective"): consecutive logical tiles land on the
// same XCD so blocks sharing an operand panel share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = b & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Per-device one-time launch setup (hipFuncSetAttribute is per device, so a process-wide flag
// would leave devices >= 1 unconfigured): runs `setup` the first time it is reached on the
// current device for this `done` mask (one bit per device).  The bit is published only after
// `setup` has returned, under a lock, so a second thread launching on the same device (replica
// threads of a 1-GPU Mirrored rehearsal) waits for the attributes instead of racing past them.
template <class F>
inline void once_per_device(std::atomic<unsigned long long>& done, F&& setup) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 63;
  const unsigned long long bit = 1ull << dev;
  if (done.load(std::memory_order_acquire) & bit) return;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (done.load(std::memory_order_relaxed) & bit) return;
  setup();
  done.fetch_or(bit, std::memory_order_release);
}

}  // namespace pddl
