// 64-channel 3x3 convolution for the stage-2 bottlenecks (ResNet-50 conv2_block*_2: 56x56x64 -> 64,
// pad 1, stride 1), forward and data gradient, plus its weight gradient (gfx950).
//
// The generic implicit GEMM (igemm.hip) gathers every one of the nine taps of a 256-row tile
// from L2: 9 x 32 KiB of A per tile for 2 x 256 x 64 x 576 FLOP, plus the 72 KiB weight matrix
// per tile, and runs these layers at 620-690 TF/s (0.87 / 0.95 ms at b2560, forward / dgrad)
// while their HBM floor -- read 1 GB, write 1 GB -- is ~0.4 ms.  Here a tile is 4 output rows of
// one image, computed from the zero-padded 6-row x 64-slot input window of rows h0 - 1 .. h0 + 4
// (48 KiB, LDS-DMA'd straight from HBM; padding taps read the zeros the out-of-range DMA wrote, so
// no tap masks): every tap is a shifted read of that window, so each input row crosses L2 -> LDS
// 1.5 times instead of nine.  One workgroup per CU walks a contiguous range of tiles with the
// windows double-buffered (tile t + 1 loads while tile t computes).  The MFMAs run with the
// weights as the A operand, so a lane ends with 4 consecutive output channels of one pixel: the
// epilogue (BN scale/shift + ReLU + ReLU bits forward; ReLU-bit mask + per-channel column sums
// for the data gradient) runs in fp32 registers and is staged as bf16 through a per-wave LDS
// slice into contiguous row stores.
// Reference: the Keras Conv2D(64, 3, padding='same') of every conv2 bottleneck block behind
// keras.applications.ResNet50 (imagenet-resnet50.py:56).
#include "common.h"
#include "kernels.h"

namespace pddl {

namespace {
constexpr int CR_WIN = 6 * 64 * 128;                // 49,152 B per input window
}  // namespace

// LDS staging of the epilogue as inline asm: a compiler-visible LDS access after an LDS-DMA makes
// the compiler drain every DMA in flight first (s_waitcnt vmcnt(0)), which would stall each
// tile's epilogue on the next tile's window load.  Callers wait on lgkmcnt themselves.
__device__ __forceinline__ void c64_wr8(char* p, uint2 v) {
  asm volatile("ds_write_b64 %0, %1" : : "v"((uint32_t)(uintptr_t)LDS_PTR(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint4 c64_rd16(const char* p) {
  uint4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}

// Logical 16-byte chunk `c` of LDS row `row` ([rows][128 B] images) sits at chunk c ^ f(row):
// 16 consecutive rows at one logical chunk hit 16 distinct 16-B slots (igemm.hip sw_chunk).
__device__ __forceinline__ int c64_sw(int row) { return (row >> 1) & 7; }

// Forward / data gradient: 8 waves in two channel halves -- wave w computes output row h0 + (w & 3)
// as 64 pixel slots (slots >= W are padding, not stored), channels 32 (w >> 2) .. + 31.  The
// wave's half of the weight matrix for taps < R8_TR lives in registers as MFMA A fragments (80
// VGPRs), taps >= R8_TR in LDS (read like the igemm B images), so two waves fit per SIMD: one
// wave's epilogue, window-DMA issue and fragment-read latency overlap the other's MFMAs.  (The
// round-4 first form ran 4 waves with the whole weight matrix per wave, one wave per SIMD, MFMA
// busy 39 %: 767 / 739 us forward / dgrad at b2560 against 695 / 679 us here,
// profiles/r4_c64_row8.txt; a 12-slot row ring that DMAs only the 4 new rows per tile measured
// no gain and was dropped.)  The pixel fragments are read by both halves, per lane at
// precomputed offsets (the window row of tap r is an immediate offset).
namespace {
constexpr int R8_TR = 5;                             // taps 0..4 in registers, 5..8 in LDS
constexpr int R8_WL = (9 - R8_TR) * 8192;
constexpr int R8_STAGE = 1024;                       // per wave: 16 pixels x 64 B
constexpr int R8_LDS = 2 * CR_WIN + R8_WL + 8 * R8_STAGE;
static_assert(R8_LDS <= 163840, "LDS budget");
__device__ __forceinline__ int r8_sw(int row) { return (row >> 2) & 3; }   // 64-B rows: 16 rows, 4 chunks
}  // namespace

template <int MODE>
__global__ void __launch_bounds__(512, 1) conv3x3c64_row8_kernel(C64Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wave & 3, hf = wave >> 2;
  char* wl = smem + 2 * CR_WIN;
  char* stage = smem + 2 * CR_WIN + R8_WL + wave * R8_STAGE;
  const int RT = (p.H + 3) / 4;
  const int T = p.N * RT;
  const int G = gridDim.x, gb = blockIdx.x;
  const int t_begin = (int)((long)gb * T / G), t_end = (int)((long)(gb + 1) * T / G);
  if (t_begin >= t_end) return;
  const long img = (long)p.H * p.W * 64;
  const int r16 = lane & 15, kq = lane >> 4, cq = 4 * kq;

  // window DMA of tile t into buffer b: 6 rows x 8 pieces, 6 per wave
  auto load_tile = [&](int t, int b) {
    const bool live = t < t_end;
    const int tt = live ? t : t_begin;
    const int n = tt / RT, h0 = (tt - n * RT) * 4;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc_at(p.x, n * img, (n + 1) * img);
    char* base = smem + b * CR_WIN;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int pc = wave * 6 + q;
      const int slot = pc * 8 + (lane >> 3);
      const int rr = slot >> 6, j = slot & 63;
      const int h = h0 - 1 + rr, w = j - 1;
      const bool ok = live && h >= 0 && h < p.H && w >= 0 && w < p.W;
      const int ch = (lane & 7) ^ c64_sw(slot);
      buf_lds16(rx, LDS_PTR(base + pc * 1024), ok ? (uint32_t)(((h * p.W + w) * 64 + ch * 8) * 2) : OOB_OFF, 0);
    }
  };

  // weights of taps >= TR -> LDS ([tap - TR][n][128 B], chunk swizzled by n): 32 pieces, 4 per wave
  {
    const __amdgpu_buffer_rsrc_t rw_ = make_rsrc(p.w, 64 * 576 * 2);
#pragma unroll
    for (int q = 0; q < (9 - R8_TR); ++q) {
      const int pc = wave * (9 - R8_TR) + q;
      const int tl = pc >> 3, nn = (pc & 7) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ c64_sw(nn);
      buf_lds16(rw_, LDS_PTR(wl + pc * 1024), (uint32_t)((nn * 576 + (R8_TR + tl) * 64 + ch * 8) * 2), 0);
    }
  }
  // this half's weights of taps < TR as A fragments: wf[tap][kh][jl] = W[16 (2 hf + jl) + r16][tap * 64 + kh * 32 + 8 kq ..]
  v8bf wf[R8_TR][2][2];
#pragma unroll
  for (int tap = 0; tap < R8_TR; ++tap)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int jl = 0; jl < 2; ++jl)
        wf[tap][kh][jl] = *reinterpret_cast<const v8bf*>(p.w + (16 * (2 * hf + jl) + r16) * 576 + tap * 64 + kh * 32 + 8 * kq);
  int aoff[4][3][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int sx = 0; sx < 3; ++sx)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int sl = 16 * i + r16 + sx;
        aoff[i][sx][kh] = sl * 128 + (((kh * 4 + kq) ^ c64_sw(sl)) << 4);
      }
  float sc[2][4], sh[2][4];
  if (MODE == C64_FWD) {
#pragma unroll
    for (int jl = 0; jl < 2; ++jl) {
      const float4 a = *reinterpret_cast<const float4*>(p.scale + 16 * (2 * hf + jl) + cq);
      const float4 b = *reinterpret_cast<const float4*>(p.shift + 16 * (2 * hf + jl) + cq);
      sc[jl][0] = a.x; sc[jl][1] = a.y; sc[jl][2] = a.z; sc[jl][3] = a.w;
      sh[jl][0] = b.x; sh[jl][1] = b.y; sh[jl][2] = b.z; sh[jl][3] = b.w;
    }
  }
  float csum[2][4];
#pragma unroll
  for (int jl = 0; jl < 2; ++jl)
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[jl][e] = 0.f;
  const bool bits_st = MODE == C64_FWD && p.bits_out != nullptr;

  load_tile(t_begin, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = t_begin; t < t_end; ++t) {
    const int b = (t - t_begin) & 1;
    if (t > t_begin) {
      // this tile's window landed (only the previous tile's 4 / 8 stores may be outstanding), and
      // every wave finished the previous tile (its window buffer takes tile t + 1)
      if (bits_st) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const int n = t / RT, h = (t - n * RT) * 4 + rw;   // this wave's output row
    const bool row_ok = h < p.H;
    const long mrow = ((long)n * p.H + (row_ok ? h : 0)) * p.W;
    uint32_t mbits[4];
    if (MODE == C64_DGRAD) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int wpx = 16 * i + r16;
        const long m = mrow + (wpx < p.W ? wpx : p.W - 1);
        mbits[i] = *reinterpret_cast<const uint32_t*>(p.bits_mask + m * 8 + 4 * hf);
      }
    }
    load_tile(t + 1, b ^ 1);                     // (past the range: zeros into the idle buffer)
    const char* xw = smem + b * CR_WIN + rw * 8192;

    v4f acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jl = 0; jl < 2; ++jl) acc[i][jl] = v4f{0.f, 0.f, 0.f, 0.f};
    v8bf ra[2][4], rwt[2][2];
    auto load_step = [&](int st, int set) {
      const int tap = st >> 1, kh = st & 1, r = tap / 3, sx = tap % 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) ra[set][i] = *reinterpret_cast<const v8bf*>(xw + r * 8192 + aoff[i][sx][kh]);
      if (tap >= R8_TR) {
#pragma unroll
        for (int jl = 0; jl < 2; ++jl) {
          const int nn = 16 * (2 * hf + jl) + r16;
          rwt[set][jl] = *reinterpret_cast<const v8bf*>(wl + (tap - R8_TR) * 8192 + nn * 128 +
                                                         (((kh * 4 + kq) ^ c64_sw(nn)) << 4));
        }
      }
    };
    auto mfma_step = [&](int st, int set) {
      const int tap = st >> 1, kh = st & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jl = 0; jl < 2; ++jl)
          acc[i][jl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tap < R8_TR ? wf[tap < R8_TR ? tap : 0][kh][jl] : rwt[set][jl],
                                                               ra[set][i], acc[i][jl], 0, 0, 0);
    };
    load_step(0, 0);
#pragma unroll
    for (int st = 0; st < 18; st += 2) {
      load_step(st + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      mfma_step(st, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (st + 2 < 18) load_step(st + 2, 0);
      __builtin_amdgcn_sched_barrier(0);
      mfma_step(st + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: acc[i][jl][e] = out[pixel slot 16 i + r16][channel 32 hf + 16 jl + cq + e]
    if (MODE == C64_DGRAD) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // mbits (the window DMA may fly)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool px_ok = row_ok && 16 * i + r16 < p.W;
#pragma unroll
      for (int jl = 0; jl < 2; ++jl) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[i][jl][e];
          if (MODE == C64_FWD) {
            x = x * sc[jl][e] + sh[jl][e];   // (ReLU on the packed pairs below)
          } else {
            x = ((mbits[i] >> (16 * jl + cq + e)) & 1u) ? x : 0.f;
            if (px_ok) csum[jl][e] += x;
          }
          v[e] = x;
        }
        const int chunk = 2 * jl + (kq >> 1);
        uint2 pv = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if (MODE == C64_FWD) pv = make_uint2(relu_pk2(pv.x), relu_pk2(pv.y));
        c64_wr8(stage + r16 * 64 + ((chunk ^ r8_sw(r16)) << 4) + 8 * (kq & 1), pv);
      }
      const int rr = lane >> 2, c = lane & 3;
      const uint4 pk = c64_rd16(stage + rr * 64 + ((c ^ r8_sw(rr)) << 4));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (also orders the next i's writes after this read)
      __builtin_amdgcn_sched_barrier(0);
      const int wpx = 16 * i + rr;
      if (row_ok && wpx < p.W) {
        const long mo = mrow + wpx;
        *reinterpret_cast<uint4*>(p.out + mo * 64 + 32 * hf + c * 8) = pk;
        if (bits_st) p.bits_out[mo * 8 + 4 * hf + c] = (uint8_t)pos_bits8(pk);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (MODE == C64_DGRAD && p.colsum) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int jl = 0; jl < 2; ++jl)
#pragma unroll
        for (int e = 0; e < 4; ++e) csum[jl][e] += __shfl_xor(csum[jl][e], o, 64);
    if (r16 == 0) {
      float* rowp = p.colsum + (long)(gb * 4 + rw) * 64 + 32 * hf;
#pragma unroll
      for (int jl = 0; jl < 2; ++jl)
        *reinterpret_cast<float4*>(rowp + 16 * jl + cq) = make_float4(csum[jl][0], csum[jl][1], csum[jl][2], csum[jl][3]);
    }
  }
}

int g_c64_grid = 0;   // test knob: cap on the workgroup count (0: one per CU), so that small
                      // problems still run many tiles per workgroup
// the partial column-sum rows are 4 per workgroup (one per output row of a tile), so a caller
// sizes them from the CU count alone
int conv3x3c64_partial_rows(int M) { return num_cus() * 4; }

const char* conv3x3c64_launch(const C64Params& p_in, int mode, hipStream_t s) {
  C64Params p = p_in;
  if (p.M <= 0 || p.M != p.N * p.H * p.W) return "conv3x3c64: M must be N * H * W";
  if (p.W + 2 > 64) return "conv3x3c64: image rows wider than 62 pixels";
  if ((long)p.M * 64 >= (1L << 40)) return "conv3x3c64: too many pixels";
  if (mode == C64_FWD && (!p.scale || !p.shift)) return "conv3x3c64: forward needs scale / shift";
  if (mode == C64_DGRAD && !p.bits_mask) return "conv3x3c64: data gradient needs the ReLU bits";
  p.mg_hw = fdiv_magic(p.H * p.W);
  p.mg_w = fdiv_magic(p.W);
  static std::atomic<unsigned long long> attr{0};
  once_per_device(attr, [&] {
    (void)hipFuncSetAttribute((const void*)conv3x3c64_row8_kernel<C64_FWD>, hipFuncAttributeMaxDynamicSharedMemorySize, R8_LDS);
    (void)hipFuncSetAttribute((const void*)conv3x3c64_row8_kernel<C64_DGRAD>, hipFuncAttributeMaxDynamicSharedMemorySize, R8_LDS);
    (void)hipGetLastError();   // (a refused attribute call must not read as the launch's error)
  });
  const int T = p.N * ((p.H + 3) / 4);
  int G = num_cus();
  if (g_c64_grid > 0 && g_c64_grid < G) G = g_c64_grid;
  if (G > T) G = T;
  // (rows of workgroups the grid leaves out stay zero for the reduction; no zero-byte memset: a
  // HIP graph capture rejects it as an invalid argument -- the Mirrored entry script's first,
  // captured step with the full 256-workgroup grid)
  if (p.colsum && G < num_cus())
    (void)hipMemsetAsync(p.colsum + (long)G * 4 * 64, 0, (size_t)(num_cus() - G) * 4 * 64 * sizeof(float), s);
  if (mode == C64_FWD) hipLaunchKernelGGL(conv3x3c64_row8_kernel<C64_FWD>, dim3(G), dim3(512), R8_LDS, s, p);
  else hipLaunchKernelGGL(conv3x3c64_row8_kernel<C64_DGRAD>, dim3(G), dim3(512), R8_LDS, s, p);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// ---------------------------------------------------------------------------------------------
// Weight gradient of the same conv: dW[co][tap][ci] = sum_m g[m][co] x[m + tap][ci].
// Row tiles: a tile is 4 output rows (h0 .. h0 + 3) of one image, each as 64 pixel slots (slot w,
// w >= W zero): 256 slots of g (32 KiB) and the 6 x 64 zero-padded input rows h0 - 1 .. h0 + 4
// (slot j <-> w = j - 1; padding rows / columns are zeros straight from the LDS-DMA's out-of-range
// loads), so every tap of every slot is a plain shifted read -- no tap masks.  Two such buffers
// (2 x 80 KiB) alternate: tile t + 1 is DMA'd while tile t computes.  A wave owns 16 input channels
// x 32 output channels for all 9 taps (acc[9][2]) for the workgroup's whole range and adds them
// once at the end (row-contiguous fp32 atomics).  The
// reduction runs over pixels, so both operands are read with ds_read_b64_tr_b16.
// Reference: the Conv2D kernel gradient of conv2_block*_2 (tf.GradientTape in model.fit,
// imagenet-resnet50.py:67).
namespace {
constexpr int CW_XS = 6 * 64;                       // input-window slots
constexpr int CW_BUF = (CW_XS + 256) * 128;         // 81,920 B per buffer
constexpr int CW_LDS = 2 * CW_BUF;
static_assert(CW_LDS <= 163840, "LDS budget");
}  // namespace

// 16-channel pair-preserving swizzle: chunk pairs (2c, 2c + 1) move together, so a 4-row x 32-B
// transposed read of 8 consecutive slots hits 8 distinct 32-B bank segments
__device__ __forceinline__ int cw_sw(int slot) { return ((slot >> 1) & 3) << 1; }
// Inline asm, not the builtin: with the builtin the compiler drains the next tile's LDS-DMA
// (vmcnt(0)) before every read (wgrad.hip).  The asm results are invisible to its wait insertion,
// so the loop waits itself (lgkmcnt(0)) and pins the MFMAs behind that wait with a scheduling
// barrier -- without it an MFMA consuming a fragment can be hoisted above the wait.
__device__ __forceinline__ v4bf cw_tr(const char* p) {
  v4bf r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}

// 8 waves: wave w owns input-channel block w & 3 for output channels 32 (w >> 2) .. + 31
// (acc[9][2]), so two waves fit per SIMD and one wave's fragment reads overlap the other's MFMAs;
// the x fragments are read by both halves.  (The first form, 4 waves with all 64 output channels
// each and one wave per SIMD, ran 680-700 us at b2560 against 654 us: profiles/r4_c64_row8.txt.)
__global__ void __launch_bounds__(512, 1) conv3x3c64_wgrad_kernel(C64WgradParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PPW = 10, NI = 2;   // DMA pieces per wave (80 / 8 waves), output-channel blocks per wave
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave & 3, i0 = (wave >> 2) * NI;   // ci block, first co block
  const int RT = (p.H + 3) / 4;                 // row tiles per image
  const int T = p.N * RT;
  const int G = gridDim.x, gb = blockIdx.x;
  const int t_begin = (int)((long)gb * T / G), t_end = (int)((long)(gb + 1) * T / G);
  if (t_begin >= t_end) return;
  const long img = (long)p.H * p.W * 64;        // elements per image

  // DMA of tile t into buffer b: 48 x-window pieces then 32 g pieces (8 slots each), 10 per wave
  auto load_tile = [&](int t, int b) {
    const bool live = t < t_end;
    const int tt = live ? t : t_begin;
    const int n = tt / RT, h0 = (tt - n * RT) * 4;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc_at(p.x, n * img, (n + 1) * img);
    const __amdgpu_buffer_rsrc_t rg = make_rsrc_at(p.g, n * img, (n + 1) * img);
    char* base = smem + b * CW_BUF;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int pc = wave * PPW + q;            // 0..79
      const bool isx = pc < 48;
      const int sp0 = (isx ? pc : pc - 48) * 8;                 // first slot of the piece
      const int slot = sp0 + (lane >> 3);
      const int rr = slot >> 6, j = slot & 63;
      const int h = isx ? h0 - 1 + rr : h0 + rr;
      const int w = isx ? j - 1 : j;
      const bool ok = live && h >= 0 && h < p.H && w >= 0 && w < p.W;
      const int ch = (lane & 7) ^ cw_sw(slot);
      const uint32_t off = ok ? (uint32_t)(((h * p.W + w) * 64 + ch * 8) * 2) : OOB_OFF;
      char* dst = base + (isx ? 0 : CW_XS * 128) + sp0 * 128;
      buf_lds16(isx ? rx : rg, LDS_PTR(dst), off, 0);
    }
  };

  v4f acc[9][NI];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[t][i] = v4f{0.f, 0.f, 0.f, 0.f};

  // ds_read_b64_tr_b16: lane 4 q + pp of each 16-lane group addresses slot row q, channels 4 pp .. +3
  // of a 16-channel block; lane i of the group then holds channel i for the 4 slots
  const int gq = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  load_tile(t_begin, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = t_begin; t < t_end; ++t) {
    const int b = (t - t_begin) & 1;
    load_tile(t + 1, b ^ 1);                    // (past the range: zeros into the idle buffer)
    const char* xw = smem + b * CW_BUF;
    const char* gt = xw + CW_XS * 128;
    // 8 k-steps of 32 slots; each step's 26 transposed reads (4 g + 9 x fragments, two halves)
    // are issued during the previous step's MFMAs, in two batches of 13 (the LDS counter tracks
    // at most 15 reads in flight), behind explicit waits and scheduling barriers (asm reads)
    v8bf af[2][NI], bfr[2][9];
    auto rd_a = [&](int ks, int set) {
      const int rl = ks >> 1, w0 = (ks & 1) * 32;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int sg = rl * 64 + w0 + 8 * gq + 4 * hh + q;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const v4bf r = cw_tr(gt + sg * 128 + (((2 * (i0 + i) + (pp >> 1)) ^ cw_sw(sg)) << 4) + (pp & 1) * 8);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[set][i][4 * hh + e] = r[e];
        }
      }
    };
    auto rd_b = [&](int ks, int set, int t0, int t1) {
      const int rl = ks >> 1, w0 = (ks & 1) * 32;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int ws = w0 + 8 * gq + 4 * hh + q;
#pragma unroll
        for (int tap = t0; tap < t1; ++tap) {
          const int sx = (rl + tap / 3) * 64 + ws + tap % 3;
          const v4bf r = cw_tr(xw + sx * 128 + (((2 * cb + (pp >> 1)) ^ cw_sw(sx)) << 4) + (pp & 1) * 8);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[set][tap][4 * hh + e] = r[e];
        }
      }
    };
    auto mm = [&](int set, int t0, int t1) {
#pragma unroll
      for (int tap = t0; tap < t1; ++tap)
#pragma unroll
        for (int i = 0; i < NI; ++i)
          acc[tap][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[set][i], bfr[set][tap], acc[tap][i], 0, 0, 0);
    };
    rd_a(0, 0);
    rd_b(0, 0, 0, 9);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int cs = ks & 1, ns = cs ^ 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // step ks's fragments
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < 8) { rd_a(ks + 1, ns); rd_b(ks + 1, ns, 0, 3); }   // 8 + 6 reads
      __builtin_amdgcn_sched_barrier(0);
      mm(cs, 0, 5);
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < 8) rd_b(ks + 1, ns, 3, 9);                         // 12 reads
      __builtin_amdgcn_sched_barrier(0);
      mm(cs, 5, 9);
      __builtin_amdgcn_sched_barrier(0);
    }
    // tile t + 1 landed; every wave is done with buffer b (tile t + 2 goes there next)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // D[co][ci] of tap: co = 16 (i0 + i) + 4 (lane >> 4) + e, ci = 16 cb + (lane & 15)
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = 16 * (i0 + i) + 4 * gq + e, ci = 16 * cb + (lane & 15);
        atomicAdd(p.dw + (long)co * p.ld_dw + tap * 64 + ci, acc[tap][i][e]);
      }
}

int g_c64w_grid = 0;   // test knob: workgroup cap of the weight-gradient kernel (0: one per CU)
const char* conv3x3c64_wgrad_launch(const C64WgradParams& p, hipStream_t s) {
  if (p.N <= 0 || p.H <= 0 || p.W <= 0) return "conv3x3c64_wgrad: empty";
  if (p.W + 2 > 64) return "conv3x3c64_wgrad: image rows wider than 62 pixels";
  if ((long)p.H * p.W * 64 * 2 >= (1L << 31)) return "conv3x3c64_wgrad: image too large";
  if (p.ld_dw < 576) return "conv3x3c64_wgrad: ld_dw";
  const int T = p.N * ((p.H + 3) / 4);
  int G = num_cus();
  if (g_c64w_grid > 0 && g_c64w_grid < G) G = g_c64w_grid;
  if (G > T) G = T;
  static std::atomic<unsigned long long> attr{0};
  once_per_device(attr, [&] {
    (void)hipFuncSetAttribute((const void*)conv3x3c64_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, CW_LDS);
    (void)hipGetLastError();
  });
  hipLaunchKernelGGL(conv3x3c64_wgrad_kernel, dim3(G), dim3(512), CW_LDS, s, p);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
