// fp32 convolution on the fp32 matrix cores (v_mfma_f32_16x16x4_f32) for the reference's
// precision (imagenet-resnet50.py:56-62 builds and trains the Keras model in float32 with no
// mixed-precision policy).  NHWC activations, OHWI weights, fp32 accumulate AND fp32 operands.
//
//   conv_f32_kernel:   y[m][n] = epi(sum_k im2col(x)[m][k] * w[n][k])   (forward, and the data
//                      gradient as a forward conv of dy with flipped/transposed weights), with
//                      the fused epilogues of ConvF32Params (frozen BN + bias + residual + ReLU;
//                      residual-gradient add + ReLU mask + stride-2 scatter + column sums)
//   wgrad_f32_kernel:  dw[n][k] += sum_m dy[m][n] * im2col(x)[m][k]           (weight gradient,
//                      m split over workgroups, fp32 atomics into dw)
//
// Both: 256 threads = 4 waves as 2 x 2 wave tiles of 32 x 32 (2 x 2 MFMA tiles), block tile
// 64 x 64, reduction step 16.  The 16x16x4 fp32 MFMA takes ONE operand element per lane
// (row lane % 16, reduction index lane / 16); the reduction order inside a 16-step is free, so
// lane group g owns reduction indices 4g .. 4g+3 and reads its four MFMA operands with one
// ds_read_b128 from a [row][16 (+4 pad)] LDS image.  Global loads for step t+1 are issued into
// registers before step t's MFMAs and stored to the other LDS buffer after them: one barrier per
// step.  VEC: C % 4 == 0, so a 4-wide reduction chunk is 4 channels of one tap (float4 gathers);
// otherwise (the 3-channel stem) elements are gathered one by one.
#include "common.h"
#include "kernels.h"

namespace pddl {

namespace {
constexpr int F_BM = 64, F_BN = 64, F_BK = 16, F_LD = F_BK + 4;   // LDS row: 16 floats + 4 pad

__device__ __forceinline__ v4f mfma4(const float4& a, const float4& b, v4f c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
  return c;
}

// im2col element / 4-chunk of row geometry (n, hi0 = ho*stride - pad, wi0) at reduction index k
template <bool VEC>
__device__ __forceinline__ float4 gather4(const ConvF32Params& p, int n, int hi0, int wi0, bool mok, int k,
                                          int S, int C) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!mok) return v;
  if (VEC) {
    if (k < p.K) {
      const int rs = k / C, c = k - rs * C, r = rs / S, s = rs - r * S;
      const int hi = hi0 + r, wi = wi0 + s;
      if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
        v = *reinterpret_cast<const float4*>(p.x + ((long)(n * p.H + hi) * p.W + wi) * C + c);
    }
  } else {
    float e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      e[q] = 0.f;
      const int kk = k + q;
      if (kk < p.K) {
        const int rs = kk / C, c = kk - rs * C, r = rs / S, s = rs - r * S;
        const int hi = hi0 + r, wi = wi0 + s;
        if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
          e[q] = p.x[((long)(n * p.H + hi) * p.W + wi) * C + c];
      }
    }
    v = make_float4(e[0], e[1], e[2], e[3]);
  }
  return v;
}
}  // namespace

template <bool VEC>
__global__ void __launch_bounds__(256) conv_f32_kernel(ConvF32Params p) {
  __shared__ __attribute__((aligned(16))) float As[2][F_BM * F_LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][F_BN * F_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int mt = (p.M + F_BM - 1) / F_BM, nt = (p.Cout + F_BN - 1) / F_BN;
  const int wg = xcd_remap(blockIdx.x, mt * nt);
  const int tn = wg % nt, tm = wg / nt;
  const int m0 = tm * F_BM, n0 = tn * F_BN;
  // loader: thread -> (row tid/4, reduction chunk (tid%4)*4) of both tiles
  const int lrow = tid >> 2, lk = (tid & 3) * 4;
  const int m = m0 + lrow;
  const bool mok = m < p.M;
  int n = 0, hi0 = 0, wi0 = 0;
  if (mok) {
    n = fdiv(m, p.mg_howo);
    const int rem = m - n * p.Ho * p.Wo, ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
    hi0 = ho * p.stride - p.pad;
    wi0 = wo * p.stride - p.pad;
  }
  const int wrow = n0 + lrow;
  const bool wok = wrow < p.Cout;
  auto load_b = [&](int k) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (wok) {
      if (VEC) {
        if (k < p.K) v = *reinterpret_cast<const float4*>(p.w + (long)wrow * p.K + k);
      } else {
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = (k + q < p.K) ? p.w[(long)wrow * p.K + k + q] : 0.f;
        v = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
    return v;
  };
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int nk = (p.K + F_BK - 1) / F_BK;
  float4 ra = gather4<VEC>(p, n, hi0, wi0, mok, lk, p.S, p.C);
  float4 rb = load_b(lk);
  *reinterpret_cast<float4*>(&As[0][lrow * F_LD + lk]) = ra;
  *reinterpret_cast<float4*>(&Bs[0][lrow * F_LD + lk]) = rb;
  __syncthreads();
  const int fr = lane & 15, g = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      ra = gather4<VEC>(p, n, hi0, wi0, mok, (t + 1) * F_BK + lk, p.S, p.C);
      rb = load_b((t + 1) * F_BK + lk);
    }
    float4 af[2], bf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *reinterpret_cast<const float4*>(&As[cur][(wm * 32 + i * 16 + fr) * F_LD + 4 * g]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bf[j] = *reinterpret_cast<const float4*>(&Bs[cur][(wn * 32 + j * 16 + fr) * F_LD + 4 * g]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(af[i], bf[j], acc[i][j]);
    if (t + 1 < nk) {
      *reinterpret_cast<float4*>(&As[cur ^ 1][lrow * F_LD + lk]) = ra;
      *reinterpret_cast<float4*>(&Bs[cur ^ 1][lrow * F_LD + lk]) = rb;
    }
    __syncthreads();
  }
  // Epilogue: D fragments (lane: rows 4g .. 4g+3 of column lane % 16) -> LDS tile -> each
  // thread owns one 4-column group and 4 rows: 16-byte loads of the epilogue operands and
  // 16-byte stores; per-m-tile partial column sums folded through the same LDS tile.
  __shared__ __attribute__((aligned(16))) float Cs[F_BM * (F_BN + 4)];
  constexpr int CLD = F_BN + 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wm * 32 + i * 16 + 4 * g + e) * CLD + wn * 32 + j * 16 + fr] = acc[i][j][e];
  __syncthreads();
  const int c4 = (tid & 15) * 4, col = n0 + c4;
  const bool vec = col + 3 < p.Cout;                 // (a ragged last column group: scalar path)
  float sc[4] = {1.f, 1.f, 1.f, 1.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (col + e < p.Cout) {
      if (p.epi == F32_EPI_FWD) { sc[e] = p.scale[col + e]; sh[e] = p.shift[col + e]; }
      else if (p.epi == F32_EPI_PLAIN && p.bias) sh[e] = p.bias[col + e];
    }
  }
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int rl = (tid >> 4) + 16 * it, row = m0 + rl;
    if (row >= p.M || col >= p.Cout) continue;
    const float4 q = *reinterpret_cast<const float4*>(&Cs[rl * CLD + c4]);
    float v[4] = {q.x, q.y, q.z, q.w};
    long orow = row;
    if (p.epi == F32_EPI_DGRAD && p.up2) {
      const int nn = fdiv(row, p.mg_howo), rem = row - nn * p.Ho * p.Wo, ii = fdiv(rem, p.mg_wo), jj = rem - ii * p.Wo;
      orow = ((long)nn * p.Hf + 2 * ii) * p.Wf + 2 * jj;
    }
    const long o = orow * p.Cout + col;
    const long oa = p.up2 ? (long)row * p.Cout + col : o;   // (up2: `add` is indexed by the GEMM row)
    if (vec) {
      if (p.epi == F32_EPI_FWD) {
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.res) r = *reinterpret_cast<const float4*>(p.res + o);
        const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = v[e] * sc[e] + sh[e] + rv[e];
          if (p.relu) v[e] = fmaxf(v[e], 0.f);
        }
      } else if (p.epi == F32_EPI_DGRAD) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), mk = make_float4(1.f, 1.f, 1.f, 1.f);
        if (p.add) a = *reinterpret_cast<const float4*>(p.add + oa);
        if (p.mask) mk = *reinterpret_cast<const float4*>(p.mask + o);
        const float av[4] = {a.x, a.y, a.z, a.w}, mv[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = mv[e] > 0.f ? v[e] + av[e] : 0.f;
          cs[e] += v[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += sh[e];
      }
      *reinterpret_cast<float4*>(p.y + o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (col + e >= p.Cout) break;
        float x = v[e];
        if (p.epi == F32_EPI_FWD) {
          x = x * sc[e] + sh[e] + (p.res ? p.res[o + e] : 0.f);
          if (p.relu) x = fmaxf(x, 0.f);
        } else if (p.epi == F32_EPI_DGRAD) {
          x = (!p.mask || p.mask[o + e] > 0.f) ? x + (p.add ? p.add[oa + e] : 0.f) : 0.f;
          cs[e] += x;
        } else {
          x += sh[e];
        }
        p.y[o + e] = x;
      }
    }
  }
  if (p.epi == F32_EPI_DGRAD && p.colsum) {
    // fold the 16 row groups of each 4-column group: lanes l, l+16, l+32, l+48 of a wave, then
    // the 4 waves through LDS; one plain-store partial row per m-tile (colsum_reduce folds them)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      cs[e] += __shfl_xor(cs[e], 16, 64);
      cs[e] += __shfl_xor(cs[e], 32, 64);
    }
    __syncthreads();
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[wave * CLD + c4 + e] = cs[e];
    }
    __syncthreads();
    if (tid < 16) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = Cs[c4 + e] + Cs[CLD + c4 + e] + Cs[2 * CLD + c4 + e] + Cs[3 * CLD + c4 + e];
        if (col + e < p.Cout) p.colsum[(long)tm * p.Cout + col + e] = t;
      }
    }
  }
}

// dw[n][k] += sum over this workgroup's m range of dy[m][n] * im2col(x)[m][k]
template <bool VEC>
__global__ void __launch_bounds__(256) wgrad_f32_kernel(ConvF32Params p, int m_per_split) {
  __shared__ __attribute__((aligned(16))) float Gs[2][F_BM * F_LD];   // [n][m]
  __shared__ __attribute__((aligned(16))) float Xs[2][F_BN * F_LD];   // [k][m]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tnn = (p.Cout + F_BM - 1) / F_BM, tkk = (p.K + F_BN - 1) / F_BN, ntiles = tnn * tkk;
  const int splits = (p.M + m_per_split - 1) / m_per_split;
  const int wg = xcd_remap(blockIdx.x, ntiles * splits);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int n0 = (tile % tnn) * F_BM, k0 = (tile / tnn) * F_BN;
  const int mbeg = split * m_per_split, mend = min(p.M, mbeg + m_per_split);
  // loader: thread -> (m row tid/16 of the 16-row step, 4 columns (tid%16)*4) of both tiles
  const int lm = tid >> 4, lc = (tid & 15) * 4;
  const int gcol = n0 + lc;
  const int kq = k0 + lc;
  auto load = [&](int mb, float4& gv, float4& xv) {
    const int mm = mb + lm;
    const bool ok = mm < mend;
    gv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok && gcol + 3 < p.Cout) {
      gv = *reinterpret_cast<const float4*>(p.y + (long)mm * p.Cout + gcol);
    } else if (ok && gcol < p.Cout) {   // ragged last column group (Dense head, classes % 4 != 0)
      const float* r = p.y + (long)mm * p.Cout + gcol;
      gv = make_float4(r[0], gcol + 1 < p.Cout ? r[1] : 0.f, gcol + 2 < p.Cout ? r[2] : 0.f, 0.f);
    }
    int n = 0, hi0 = 0, wi0 = 0;
    if (ok) {
      n = fdiv(mm, p.mg_howo);
      const int rem = mm - n * p.Ho * p.Wo, ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
      hi0 = ho * p.stride - p.pad;
      wi0 = wo * p.stride - p.pad;
    }
    xv = gather4<VEC>(p, n, hi0, wi0, ok, kq, p.S, p.C);
  };
  auto store = [&](int buf, const float4& gv, const float4& xv) {   // transposed: [col][m]
    Gs[buf][(lc + 0) * F_LD + lm] = gv.x;
    Gs[buf][(lc + 1) * F_LD + lm] = gv.y;
    Gs[buf][(lc + 2) * F_LD + lm] = gv.z;
    Gs[buf][(lc + 3) * F_LD + lm] = gv.w;
    Xs[buf][(lc + 0) * F_LD + lm] = xv.x;
    Xs[buf][(lc + 1) * F_LD + lm] = xv.y;
    Xs[buf][(lc + 2) * F_LD + lm] = xv.z;
    Xs[buf][(lc + 3) * F_LD + lm] = xv.w;
  };
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (mend - mbeg + F_BK - 1) / F_BK;
  if (nsteps <= 0) return;   // (block-uniform, before any barrier)
  float4 gv, xv;
  load(mbeg, gv, xv);
  store(0, gv, xv);
  __syncthreads();
  const int fr = lane & 15, g = lane >> 4;
  for (int t = 0; t < nsteps; ++t) {
    const int cur = t & 1;
    if (t + 1 < nsteps) load(mbeg + (t + 1) * F_BK, gv, xv);
    float4 af[2], bf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *reinterpret_cast<const float4*>(&Gs[cur][(wm * 32 + i * 16 + fr) * F_LD + 4 * g]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bf[j] = *reinterpret_cast<const float4*>(&Xs[cur][(wn * 32 + j * 16 + fr) * F_LD + 4 * g]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(af[i], bf[j], acc[i][j]);
    if (t + 1 < nsteps) store(cur ^ 1, gv, xv);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = k0 + wn * 32 + j * 16 + fr;
    if (col >= p.K) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = n0 + wm * 32 + i * 16 + 4 * g + e;
        if (row < p.Cout) unsafeAtomicAdd(p.dw + (long)row * p.K + col, acc[i][j][e]);
      }
  }
}

// ------------------------------------------------------------------------------------------
// 128 x BN tiles (round 4; BN = 128, or 64 for the 64-channel layers and small grids): 4 waves
// as 2 x 2 wave tiles of 64 x BN/2 (4 x BN/32 MFMA tiles of 16x16x4 f32), reduction step 16
// floats, a 3-stage LDS pipeline fed by buffer LDS-DMA (16 B per lane straight from HBM / L2 into
// LDS, no register staging).  The gather geometry of each tile row (image, top-left input pixel,
// bitmask of its in-bounds taps) is computed once per tile; the k walk (tap r, s and channel
// offset: C % 16 == 0, so a 16-wide step never crosses a tap) is scalar, so the k loop carries no
// divides.  LDS images are chunk-major ([4 chunks][rows][16 B]: one DMA piece = one chunk column
// of 64 rows), which makes every ds_read_b128 fragment read conflict-free.  The fragment reads
// are inline asm: the compiler's own LDS loads after an LDS-DMA make it drain every DMA in flight
// (s_waitcnt vmcnt(0)), which would serialise the pipeline; the asm reads wait on lgkmcnt only,
// behind a scheduling barrier so no MFMA is hoisted above the wait.
// The epilogue is the 64 x 64 kernel's, run over the tile's two 64-row halves through the
// pipeline's LDS (partial column sums: one row per 64-row half, the same layout).
namespace {
constexpr int G_BM = 128;

__device__ __forceinline__ v4f mfma4v(const float4& a, const float4& b, v4f c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ float4 f32_read16(const char* p) {
  float4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)LDS_PTR(p)) : "memory");
  return r;
}
}  // namespace

template <int BN>
__device__ __forceinline__ void f32_big_epilogue(const ConvF32Params& p, v4f (&acc)[4][BN / 32], int m0, int n0,
                                                 int tm, char* smem, int half = -1);

template <int BN>
__global__ void __launch_bounds__(256, 2) conv_f32_big_kernel(ConvF32Params p) {
  constexpr int A_CH = G_BM * 16, B_CH = BN * 16;   // bytes of one 16-byte chunk column
  constexpr int B_BASE = 4 * A_CH, STAGE = 4 * (A_CH + B_CH);
  constexpr int NB = BN / 64;                        // B DMA pieces per lane per step
  constexpr int TJ = BN / 32;                        // MFMA column tiles per wave
  constexpr int CLD = BN + 4;
  static_assert(64 * CLD * 4 <= 3 * STAGE, "epilogue tile must fit the pipeline's LDS");
  __shared__ __attribute__((aligned(16))) char smem[3 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int mt = (p.M + G_BM - 1) / G_BM, nt = (p.Cout + BN - 1) / BN;
  const int ks = p.ksplit > 1 ? p.ksplit : 1;   // split-K: slice `slice` of the tile's K steps
  const int wg = xcd_remap(blockIdx.x, mt * nt * ks);
  const int tile = wg % (mt * nt), slice = wg / (mt * nt);
  const int tn = tile % nt, tm = tile / nt;
  const int m0 = tm * G_BM, n0 = tn * BN;
  const int HoWo = p.Ho * p.Wo;
  // descriptors: A from the first image of the tile (lane offsets span a few images at any batch)
  const int n_first = fdiv(m0, p.mg_howo);
  const long HWC = (long)p.H * p.W * p.C;
  const __amdgpu_buffer_rsrc_t ra =
      make_rsrc(p.x + n_first * HWC, (int)lmin((long)(p.N - n_first) * HWC * 4, 0x7fffffffL));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.w, (int)lmin((long)p.Cout * p.K * 4, 0x7fffffffL));
  // this lane's two A rows (pieces rh = 0, 1: rows rh * 64 + lane) and NB B rows, chunk = wave
  uint32_t a_off[2], a_taps[2], b_off[NB];
#pragma unroll
  for (int rh = 0; rh < 2; ++rh) {
    const int m = m0 + rh * 64 + lane;
    a_off[rh] = OOB_OFF;
    a_taps[rh] = 0;
    if (m < p.M) {
      const int n = fdiv(m, p.mg_howo), rem = m - n * HoWo;
      const int ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
      const int hi = ho * p.stride - p.pad, wi = wo * p.stride - p.pad;
      const int pix = ((n - n_first) * p.H + hi) * p.W + wi;
      a_off[rh] = (uint32_t)((pix * p.C + 4 * wave) * 4);
      uint32_t t = 0;
      for (int r = 0; r < p.R; ++r)
        for (int s2 = 0; s2 < p.S; ++s2)
          if ((unsigned)(hi + r) < (unsigned)p.H && (unsigned)(wi + s2) < (unsigned)p.W) t |= 1u << (r * p.S + s2);
      a_taps[rh] = t;
    }
  }
#pragma unroll
  for (int rh = 0; rh < NB; ++rh) {
    const int nn = n0 + rh * 64 + lane;
    b_off[rh] = nn < p.Cout ? (uint32_t)((nn * p.K + 4 * wave) * 4) : OOB_OFF;
  }
  const int KT_all = p.K / 16;
  const int t_begin = (int)((long)KT_all * slice / ks), t_end = (int)((long)KT_all * (slice + 1) / ks);
  // (16-float steps never straddle a tap: C % 16 == 0)
  int ld_k = t_begin * 16, ld_r, ld_s, ld_c0;
  {
    const int tap = ld_k / p.C;
    ld_c0 = ld_k - tap * p.C;
    ld_r = tap / p.S;
    ld_s = tap - ld_r * p.S;
  }
  auto load_step = [&](int buf) {
    char* base = smem + buf * STAGE;
    const int tap = ld_r * p.S + ld_s;
    const int delta = ((ld_r * p.W + ld_s) * p.C + ld_c0) * 4;
#pragma unroll
    for (int rh = 0; rh < 2; ++rh) {
      const uint32_t off = ((a_taps[rh] >> tap) & 1u) ? a_off[rh] + (uint32_t)delta : OOB_OFF;
      buf_lds16(ra, LDS_PTR(base + wave * A_CH + rh * 1024), off, 0);
    }
#pragma unroll
    for (int rh = 0; rh < NB; ++rh) buf_lds16(rb, LDS_PTR(base + B_BASE + wave * B_CH + rh * 1024), b_off[rh], ld_k * 4);
    ld_k += 16;
    ld_c0 += 16;
    if (ld_c0 == p.C) {
      ld_c0 = 0;
      if (++ld_s == p.S) { ld_s = 0; ++ld_r; }
    }
  };
  v4f acc[4][TJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int KT = t_end - t_begin;
  load_step(0);
  if (KT > 1) load_step(1);
  const int fr = lane & 15, g = lane >> 4;
  const int a_rd = g * A_CH + (wm * 64 + fr) * 16, b_rd = B_BASE + g * B_CH + (wn * (BN / 2) + fr) * 16;
  for (int t = 0; t < KT; ++t) {
    // step t landed (step t+1 stays in flight across the raw barrier), and every wave finished
    // step t-1, whose buffer takes step t+2
    if (t + 1 < KT) {
      if constexpr (NB == 2) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    const int cur = t % 3;
    if (t + 2 < KT) load_step((t + 2) % 3);
    const char* st = smem + cur * STAGE;
    float4 af[4], bf[TJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = f32_read16(st + a_rd + i * 256);
#pragma unroll
    for (int j = 0; j < TJ; ++j) bf[j] = f32_read16(st + b_rd + j * 256);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = mfma4v(af[i], bf[j], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (ks > 1) {   // split-K slice: the fp32 partial tile in fragment order, combined by conv_f32_splitk_kernel
    float4* dst = reinterpret_cast<float4*>(p.slab) + (long)(tile * ks + slice) * (4 * TJ) * 256 + tid;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) dst[(i * TJ + j) * 256] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    return;
  }
  __syncthreads();   // every fragment read done: the epilogue reuses the pipeline's LDS
  f32_big_epilogue<BN>(p, acc, m0, n0, tm, smem);
}

// Fused epilogue of the 128 x BN fp32 tiles (conv_f32_big_kernel, conv_f32_splitk_kernel): the
// accumulator fragments through LDS into 16-byte row stores.
template <int BN>
__device__ __forceinline__ void f32_big_epilogue(const ConvF32Params& p, v4f (&acc)[4][BN / 32], int m0, int n0,
                                                 int tm, char* smem, int half) {
  // half < 0: the whole 128-row tile, wave (wm, wn) holding rows wm * 64 + [0, 64); half 0 / 1:
  // only that 64-row half, its fragments in waves 0 / 1 (as wn), waves 2 / 3 holding none
  constexpr int TJ = BN / 32, CLD = BN + 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = half < 0 ? wave >> 1 : (wave < 2 ? half : -1), wn = wave & 1;
  const int fr = lane & 15, g = lane >> 4;
  const int HoWo = p.Ho * p.Wo;
  // epilogue: thread -> one 4-column group (CG groups across the tile) and every RPI-th row
  constexpr int CG = BN / 4, RPI = 256 / CG;
  float* Cs = reinterpret_cast<float*>(smem);
  const int c4 = (tid % CG) * 4, col = n0 + c4;
  const bool vec = col + 3 < p.Cout;
  float sc[4] = {1.f, 1.f, 1.f, 1.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (col + e < p.Cout) {
      if (p.epi == F32_EPI_FWD) { sc[e] = p.scale[col + e]; sh[e] = p.shift[col + e]; }
      else if (p.epi == F32_EPI_PLAIN && p.bias) sh[e] = p.bias[col + e];
    }
  }
  const int h_lo = half < 0 ? 0 : half, h_hi = half < 0 ? 2 : half + 1;
  for (int h = h_lo; h < h_hi; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) Cs[(i * 16 + 4 * g + e) * CLD + wn * (BN / 2) + j * 16 + fr] = acc[i][j][e];
    }
    __syncthreads();
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int rl = tid / CG + RPI * it, row = m0 + h * 64 + rl;
      if (row >= p.M || col >= p.Cout) continue;
      const float4 q = *reinterpret_cast<const float4*>(&Cs[rl * CLD + c4]);
      float v[4] = {q.x, q.y, q.z, q.w};
      long orow = row;
      if (p.epi == F32_EPI_DGRAD && p.up2) {
        const int nn = fdiv(row, p.mg_howo), rem = row - nn * HoWo, ii = fdiv(rem, p.mg_wo), jj = rem - ii * p.Wo;
        orow = ((long)nn * p.Hf + 2 * ii) * p.Wf + 2 * jj;
      }
      const long o = orow * p.Cout + col;
      const long oa = p.up2 ? (long)row * p.Cout + col : o;
      if (vec) {
        if (p.epi == F32_EPI_FWD) {
          float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
          if (p.res) r = *reinterpret_cast<const float4*>(p.res + o);
          const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = v[e] * sc[e] + sh[e] + rv[e];
            if (p.relu) v[e] = fmaxf(v[e], 0.f);
          }
        } else if (p.epi == F32_EPI_DGRAD) {
          float4 a = make_float4(0.f, 0.f, 0.f, 0.f), mk = make_float4(1.f, 1.f, 1.f, 1.f);
          if (p.add) a = *reinterpret_cast<const float4*>(p.add + oa);
          if (p.mask) mk = *reinterpret_cast<const float4*>(p.mask + o);
          const float av[4] = {a.x, a.y, a.z, a.w}, mv[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = mv[e] > 0.f ? v[e] + av[e] : 0.f;
            cs[e] += v[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += sh[e];
        }
        *reinterpret_cast<float4*>(p.y + o) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (col + e >= p.Cout) break;
          float x = v[e];
          if (p.epi == F32_EPI_FWD) {
            x = x * sc[e] + sh[e] + (p.res ? p.res[o + e] : 0.f);
            if (p.relu) x = fmaxf(x, 0.f);
          } else if (p.epi == F32_EPI_DGRAD) {
            x = (!p.mask || p.mask[o + e] > 0.f) ? x + (p.add ? p.add[oa + e] : 0.f) : 0.f;
            cs[e] += x;
          } else {
            x += sh[e];
          }
          p.y[o + e] = x;
        }
      }
    }
    if (p.epi == F32_EPI_DGRAD && p.colsum) {
      // fold the row groups of each 4-column group: lanes l, l + CG, ... of a wave, then the 4 waves
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[e] += __shfl_xor(cs[e], 32, 64);
        if (CG == 16) cs[e] += __shfl_xor(cs[e], 16, 64);
      }
      __syncthreads();
      if (lane < CG) {
#pragma unroll
        for (int e = 0; e < 4; ++e) Cs[wave * CLD + c4 + e] = cs[e];
      }
      __syncthreads();
      if (tid < CG && m0 + h * 64 < p.M) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = Cs[c4 + e] + Cs[CLD + c4 + e] + Cs[2 * CLD + c4 + e] + Cs[3 * CLD + c4 + e];
          if (col + e < p.Cout) p.colsum[(long)(tm * 2 + h) * p.Cout + col + e] = t;
        }
      }
    }
    __syncthreads();   // (the next half overwrites Cs)
  }
}

// Split-K combine of the fp32 tiles: one workgroup per 64-row half of a 128 x BN tile (the
// combines run ~100 tiles at small batches: one workgroup per tile measured bound by its two-half
// epilogue), waves 0 / 1 summing the fragments of the half's two slice waves over the slices
// (16-byte loads, two slices in flight), then the fused epilogue of that half.
template <int BN>
__global__ void __launch_bounds__(256) conv_f32_splitk_kernel(ConvF32Params p) {
  constexpr int TJ = BN / 32, F = 4 * TJ;
  __shared__ __attribute__((aligned(16))) char smem[64 * (BN + 4) * 4];
  const int nt = (p.Cout + BN - 1) / BN;
  const int tile = blockIdx.x >> 1, half = blockIdx.x & 1, tn = tile % nt, tm = tile / nt;
  const int tid = threadIdx.x;
  v4f acc[4][TJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  // (slice wave 2 * half + w wrote rows half * 64 + [0, 64) of the tile; w = this wave, 0 or 1)
  const float4* src = reinterpret_cast<const float4*>(p.slab) + (long)tile * p.ksplit * F * 256 + half * 128 + tid;
  auto add = [&](const float4* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const float4 q = v[i * TJ + j];
        acc[i][j][0] += q.x; acc[i][j][1] += q.y; acc[i][j][2] += q.z; acc[i][j][3] += q.w;
      }
  };
  int sl = tid < 128 ? 0 : p.ksplit;   // (waves 2 / 3 hold no fragments)
  for (; sl + 1 < p.ksplit; sl += 2) {
    float4 v0[F], v1[F];
#pragma unroll
    for (int f = 0; f < F; ++f) { v0[f] = src[((long)sl * F + f) * 256]; v1[f] = src[((long)(sl + 1) * F + f) * 256]; }
    add(v0);
    add(v1);
  }
  if (sl < p.ksplit) {
    float4 v0[F];
#pragma unroll
    for (int f = 0; f < F; ++f) v0[f] = src[((long)sl * F + f) * 256];
    add(v0);
  }
  f32_big_epilogue<BN>(p, acc, tm * G_BM, tn * BN, tm, smem, half);
}
int g_conv_f32_variant = 1;
int g_conv_f32_sk_elig = 1;   // ... for problems of fewer than this many tiles per CU (knob conv_f32_sk_elig)
int g_conv_f32_splitk = 4;    // split-K of the underfilled fp32 conv / dgrad problems: slice workgroups aimed
                              // at this many per CU (knob conv_f32_splitk, 0 off)   // 0: 64 x 64 register-staged kernels only; 1: the LDS-DMA kernels where they
                              // apply (C % 16 == 0: 128 x 64 conv tiles; the 128 x 128 weight-gradient
                              // tiles where both GEMM sides are >= 128 wide); 2: 128 x 128 conv tiles and
                              // the 128 x 128 weight gradient wherever they apply

// Weight gradient on 128 (Cout) x 128 (K) tiles, reduction over m in steps of 16 rows, the same
// 3-stage LDS-DMA pipeline.  Both operands arrive row-major ([m][n] / [m][k] rows of 128 floats,
// one DMA piece = 2 m-rows, pieces padded by 64 B so the fragment reads spread over the banks) and
// are read as single floats (ds_read_b32: the MFMA reduction index is m, which is the row).  The
// k geometry of a lane's 16-byte chunk (tap r, s and channel) is fixed for the tile; the pixel
// of its m-row is recomputed per step (magic-number division).  dW accumulates in registers over
// the workgroup's m range and is added once with fp32 atomics.
namespace {
constexpr int W_PIECE = 1024 + 64, W_TILE = 8 * W_PIECE, W_STAGE = 2 * W_TILE;
}
__global__ void __launch_bounds__(256, 2) wgrad_f32_big_kernel(ConvF32Params p, int m_per_split) {
  __shared__ __attribute__((aligned(16))) char smem[3 * W_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tnn = (p.Cout + 127) / 128, tkk = (p.K + 127) / 128, ntiles = tnn * tkk;
  const int splits = (p.M + m_per_split - 1) / m_per_split;
  const int wg = xcd_remap(blockIdx.x, ntiles * splits);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int n0 = (tile % tnn) * 128, k0 = (tile / tnn) * 128;
  const int mbeg = split * m_per_split, mend = min(p.M, mbeg + m_per_split);
  const int nsteps = (mend - mbeg + 15) / 16;
  if (nsteps <= 0) return;   // (block-uniform, before any barrier)
  const int HoWo = p.Ho * p.Wo;
  // descriptors over the whole tensors (offsets of one split stay below 2 GiB: the launcher
  // bounds a split's span), rebased at the split's first image for x
  const int n_first = fdiv(mbeg, p.mg_howo);
  const long HWC = (long)p.H * p.W * p.C;
  const __amdgpu_buffer_rsrc_t rx =
      make_rsrc(p.x + n_first * HWC, (int)lmin((long)(p.N - n_first) * HWC * 4, 0x7fffffffL));
  const __amdgpu_buffer_rsrc_t rg =
      make_rsrc(p.y + (long)mbeg * p.Cout, (int)lmin((long)(mend - mbeg) * p.Cout * 4, 0x7fffffffL));
  // this lane's chunk: 4 consecutive columns (n for the gradient, k for x) of m-row (lane >> 5)
  // of every piece; each wave issues pieces 2 wave, 2 wave + 1 of both tiles
  const int cc = (lane & 31) * 4;
  const int gcol = n0 + cc;
  const bool g_ok = gcol < p.Cout;   // (Cout % 4 == 0: checked by the launcher)
  const int kq = k0 + cc;
  const bool k_ok = kq < p.K;
  int kr = 0, ks = 0, kc = 0;
  if (k_ok) {
    const int rs = kq / p.C;
    kc = kq - rs * p.C;
    kr = rs / p.S;
    ks = rs - kr * p.S;
  }
  auto load_step = [&](int buf, int mb) {
    char* base = smem + buf * W_STAGE;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int piece = 2 * wave + q;
      const int m = mb + 2 * piece + (lane >> 5);
      const bool ok = m < mend;
      const uint32_t goff = (ok && g_ok) ? (uint32_t)(((m - mbeg) * p.Cout + gcol) * 4) : OOB_OFF;
      buf_lds16(rg, LDS_PTR(base + piece * W_PIECE), goff, 0);
      uint32_t xoff = OOB_OFF;
      if (ok && k_ok) {
        const int n = fdiv(m, p.mg_howo), rem = m - n * HoWo;
        const int ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
        const int hi = ho * p.stride - p.pad + kr, wi = wo * p.stride - p.pad + ks;
        if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
          xoff = (uint32_t)(((((n - n_first) * p.H + hi) * p.W + wi) * p.C + kc) * 4);
      }
      buf_lds16(rx, LDS_PTR(base + W_TILE + piece * W_PIECE), xoff, 0);
    }
  };
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  load_step(0, mbeg);
  if (nsteps > 1) load_step(1, mbeg + 16);
  const int fr = lane & 15, g = lane >> 4;
  // fragment element e of lane (fr, g): m-row 4 g + e = piece 2 g + (e >> 1), half e & 1
  const int a_rd = 2 * g * W_PIECE + (wm * 64 + fr) * 4, b_rd = W_TILE + 2 * g * W_PIECE + (wn * 64 + fr) * 4;
  for (int t = 0; t < nsteps; ++t) {
    if (t + 1 < nsteps) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int cur = t % 3;
    if (t + 2 < nsteps) load_step((t + 2) % 3, mbeg + (t + 2) * 16);
    const char* st = smem + cur * W_STAGE;
    float4 af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* a = reinterpret_cast<const float*>(st + a_rd + i * 64);
      af[i] = make_float4(a[0], a[128], a[W_PIECE / 4], a[W_PIECE / 4 + 128]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* b = reinterpret_cast<const float*>(st + b_rd + j * 64);
      bf[j] = make_float4(b[0], b[128], b[W_PIECE / 4], b[W_PIECE / 4 + 128]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma4v(af[i], bf[j], acc[i][j]);
  }
  // dW[n][k] += D: lane holds D[n = 16 i + 4 g + e][k = 16 j + fr] of the wave's 64 x 64
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = k0 + wn * 64 + j * 16 + fr;
    if (col >= p.K) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = n0 + wm * 64 + i * 16 + 4 * g + e;
        if (row < p.Cout) unsafeAtomicAdd(p.dw + (long)row * p.K + col, acc[i][j][e]);
      }
  }
}

static const char* check_f32(const ConvF32Params& p) {
  if (p.M <= 0 || p.Cout <= 0 || p.K <= 0) return "conv_f32: empty problem";
  if (p.epi == F32_EPI_FWD && (!p.scale || !p.shift)) return "conv_f32: forward epilogue needs scale and shift";
  if (p.epi == F32_EPI_DGRAD && p.up2 && (p.Hf < 2 * p.Ho - 1 || p.Wf < 2 * p.Wo - 1))
    return "conv_f32: up2 grid smaller than the scattered rows";
  if (p.epi != F32_EPI_PLAIN && p.epi != F32_EPI_FWD && p.epi != F32_EPI_DGRAD) return "conv_f32: unknown epilogue";
  if (p.K != p.R * p.S * p.C) return "conv_f32: K must be R*S*C";
  if ((long)p.N * p.H * p.W * p.C >= (1L << 31) || (long)p.M * p.Cout >= (1L << 31))
    return "conv_f32: tensor too large for 32-bit row indexing";
  return nullptr;
}

const char* conv_f32_launch(ConvF32Params p, hipStream_t stream) {
  if (const char* e = check_f32(p)) return e;
  p.mg_howo = fdiv_magic(p.Ho * p.Wo);
  p.mg_wo = fdiv_magic(p.Wo);
  if (g_conv_f32_variant >= 1 && p.C % 16 == 0 && p.R * p.S <= 32) {
    const int mt = (p.M + G_BM - 1) / G_BM;
    // 128 x 64 tiles unless forced: 4 workgroups per CU (36 KB of LDS, 76 VGPRs) against the wide
    // tile's 3, equal or faster on every ResNet-50 layer (bench/f32.py, profiles/r4_fp32.txt)
    const bool wide = g_conv_f32_variant == 2;
    const int BN = wide ? 128 : 64;
    const int T = mt * ((p.Cout + BN - 1) / BN);
    // split-K where the tiles leave CUs idle (small batches: b32 stage 5 is 104 tiles of a
    // 288-step K loop on 256 CUs): slices aimed at 4 workgroups per CU, >= 8 K steps each, <= 8
    const long C = num_cus(), KT = p.K / 16;
    long ks = 1;
    if (g_conv_f32_splitk > 0 && T < (long)g_conv_f32_sk_elig * C) {
      ks = ((long)g_conv_f32_splitk * C + T - 1) / T;
      if (ks > 8) ks = 8;
      if (ks > KT / 8) ks = KT / 8;
    }
    if (ks >= 2 && p.slab && p.slab_floats >= (long)T * ks * G_BM * BN) {
      p.ksplit = (int)ks;
      if (wide) {
        hipLaunchKernelGGL(conv_f32_big_kernel<128>, dim3(T * ks), dim3(256), 0, stream, p);
        hipLaunchKernelGGL(conv_f32_splitk_kernel<128>, dim3(2 * T), dim3(256), 0, stream, p);
      } else {
        hipLaunchKernelGGL(conv_f32_big_kernel<64>, dim3(T * ks), dim3(256), 0, stream, p);
        hipLaunchKernelGGL(conv_f32_splitk_kernel<64>, dim3(2 * T), dim3(256), 0, stream, p);
      }
    } else {
      p.ksplit = 1;
      if (wide) hipLaunchKernelGGL(conv_f32_big_kernel<128>, dim3(T), dim3(256), 0, stream, p);
      else hipLaunchKernelGGL(conv_f32_big_kernel<64>, dim3(T), dim3(256), 0, stream, p);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? nullptr : hipGetErrorString(e);
  }
  const int grid = ((p.M + F_BM - 1) / F_BM) * ((p.Cout + F_BN - 1) / F_BN);
  if (p.C % 4 == 0) hipLaunchKernelGGL(conv_f32_kernel<true>, dim3(grid), dim3(256), 0, stream, p);
  else hipLaunchKernelGGL(conv_f32_kernel<false>, dim3(grid), dim3(256), 0, stream, p);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

// Workgroups per CU of the 64- / 128-wide fp32 weight gradients (knobs wgrad_f32_wpc64 / _wpc128).
// Measured whole fp32 step at b256 (round 5, gpurun_out/ks45-ks47): {4, 3} 64.18 ms; fewer splits
// (the atomic epilogue shrinks) lose -- {4, 2} 65.11, {4, 1} 69.63, {2, 3} 65.73; more win:
// {8, 3} 63.27, {16, 3} 63.02, {4, 6} 63.14, {16, 6} 62.09, {24, 8} 62.24, {32, 12} 62.20.  The
// kernels are MFMA-bound and the surplus workgroups keep every CU fed to the end of the launch.
// Round 6, weight gradients on the side stream of the two-stream backward (models/engine_f32.py):
// {16, 6} 58.34-58.50, {8, 4} 58.39-58.48, {4, 3} 58.95-58.99, {16, 3} 58.14-58.29 ms -- the
// 128-wide ones now share the CUs with the data-gradient chain.
int g_wgrad_f32_wpc[2] = {16, 3};
const char* wgrad_f32_launch(ConvF32Params p, hipStream_t stream) {
  if (const char* e = check_f32(p)) return e;
  p.mg_howo = fdiv_magic(p.Ho * p.Wo);
  p.mg_wo = fdiv_magic(p.Wo);
  const int ntiles = ((p.Cout + F_BM - 1) / F_BM) * ((p.K + F_BN - 1) / F_BN);
  // ~16 workgroups per CU, each reducing at least 256 rows of m
  int splits = (g_wgrad_f32_wpc[0] * num_cus() + ntiles - 1) / ntiles;
  const int cap = (p.M + 255) / 256;
  if (splits > cap) splits = cap;
  if (splits < 1) splits = 1;
  int mps = ((p.M + splits - 1) / splits + F_BK - 1) / F_BK * F_BK;
  splits = (p.M + mps - 1) / mps;
  // the 128 x 128 weight-gradient tiles run half empty on 64-wide sides (Cout or K = 64, or
  // K = 576 = 4.5 tiles): those layers keep the 64 x 64 kernel unless forced
  const bool big_fits = p.Cout >= 128 && p.K >= 128 && (p.K % 128 == 0 || p.K >= 1024);
  if (g_conv_f32_variant >= 1 && p.C % 4 == 0 && p.Cout % 4 == 0 && (big_fits || g_conv_f32_variant >= 2)) {
    const int bt = ((p.Cout + 127) / 128) * ((p.K + 127) / 128);
    int bs = (g_wgrad_f32_wpc[1] * num_cus() + bt - 1) / bt;   // ~6 workgroups per CU
    const int bcap = (p.M + 511) / 512;                      // each reducing >= 512 rows of m
    bs = bs > bcap ? bcap : (bs < 1 ? 1 : bs);
    const int bmps = ((p.M + bs - 1) / bs + 15) / 16 * 16;
    bs = (p.M + bmps - 1) / bmps;
    hipLaunchKernelGGL(wgrad_f32_big_kernel, dim3(bt * bs), dim3(256), 0, stream, p, bmps);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? nullptr : hipGetErrorString(e);
  }
  if (p.C % 4 == 0) hipLaunchKernelGGL(wgrad_f32_kernel<true>, dim3(ntiles * splits), dim3(256), 0, stream, p, mps);
  else hipLaunchKernelGGL(wgrad_f32_kernel<false>, dim3(ntiles * splits), dim3(256), 0, stream, p, mps);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
