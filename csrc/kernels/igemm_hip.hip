#include "hip/hip_runtime.h"
// Implicit-GEMM convolution on MFMA for CDNA4 (gfx950): forward and data-gradient.
//
//   C[m, n] = sum_k A[m, k] * B[n, k]
//   A = im2col(x) gathered on the fly from an NHWC bf16 tensor (k = (r, s, c), c fastest),
//   B = weights [Nn][K] (K contiguous; OHWI for forward, transposed+scaled for dgrad).
//
// One kernel serves every conv of ResNet-50 (reference: the 53 Keras Conv2D layers behind
// keras.applications.ResNet50 called at imagenet-resnet50.py:56; SURVEY.md §2.5 lists the
// shapes) in both directions:
//   * forward:  y = act(acc * scale[n] + shift[n] (+ residual))      (frozen-BN folded, Q3)
//   * dgrad:    g = (acc (+ add)) * (mask > 0)  with an optional stride-2 scatter ("up2")
//     that also writes the zero rows a strided 1x1 conv leaves in the input gradient.
//   * fp32:     logits = acc * scale + shift (the Dense head)
// Two A sources may be concatenated along K (projection-block dgrad: dx = g1*W1' + gp*Wp')
// and two outputs split along N (conv1 + projection shortcut read x once).
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §5):
//   * 256 threads = 4 waves, wave tile 64x64 (or 64x32) of 16x16x32 bf16 MFMAs.
//   * BK = 64: one k-tile never crosses an (r, s) tap because C % 64 == 0, so the im2col
//     gather needs only per-row (n, ho, wo) bookkeeping plus uniform (r, s, c0) scalars.
//   * Tiles are staged global->LDS with 16-byte LDS-DMA (global_load_lds_dwordx4); the LDS
//     image is lane-linear, so the bank-conflict XOR swizzle is applied to the SOURCE
//     address and the same involution on the ds_read_b128 address (rule 21).
//   * Out-of-bounds lanes (padding taps, tile overhang) read a 64-byte zero page.
//   * Double-buffered LDS, XCD-aware bijective tile remap, LDS-staged epilogue that turns
//     the MFMA fragment layout into 16-byte row-contiguous stores.
#include "common.h"
#include "kernels.h"

namespace pddl {

template <int BM, int BN, int WTM, int WTN, int NSTAGE>
__global__ void __launch_bounds__(256, 2) igemm_kernel(IgemmParams p) {
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int WAVES_N = BN / WTN;
  static_assert((BM / WTM) * (BN / WTN) == 4, "4 waves per block");
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = BM / 32, BI = BN / 32;  // 1 KiB LDS-DMA pieces per wave per tile
  constexpr int EPI_LD = WTN + 4;
  constexpr int EPI_BYTES = 4 * 32 * EPI_LD * 4;
  constexpr int SMEM = (NSTAGE * STAGE > EPI_BYTES) ? NSTAGE * STAGE : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Nn + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, mt * nt);
  const int tn = wg % nt, tm = wg / nt;
  const int m0 = tm * BM, n0 = tn * BN;
  const int HoWo = p.Ho * p.Wo;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero_page);

  // Per-lane constant source chunk: LDS position (lane & 7) of row (lane >> 3) holds the
  // logical 16-byte chunk (lane & 7) ^ (row & 7).
  const int chunk_sw = (lane & 7) ^ ((lane >> 3) & 7);

  // A-row bookkeeping (fixed over the k loop): the element offset of the row's tap (0, 0)
  // in each source; a k-tile then only adds a wave-uniform (r*W + s)*C + c0.
  int a_hi[AI], a_wi[AI], a_o1[AI], a_o2[AI];
  const bool no_halo = p.R == 1 && p.S == 1 && p.pad == 0;   // 1x1: only the row itself can be invalid
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (wave * AI + i) * 8 + (lane >> 3);
    if (m < p.M) {
      const int n = m / HoWo, rem = m - n * HoWo;
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      a_hi[i] = ho * p.stride - p.pad;
      a_wi[i] = wo * p.stride - p.pad;
      const int pix = (n * p.H + a_hi[i]) * p.W + a_wi[i];
      a_o1[i] = pix * p.C1 + chunk_sw * 8;
      a_o2[i] = pix * p.C2 + chunk_sw * 8;
    } else {
      a_hi[i] = -(1 << 28); a_wi[i] = 0; a_o1[i] = 0; a_o2[i] = 0;
    }
  }
  const bf16_t* b_row[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + (wave * BI + i) * 8 + (lane >> 3);
    b_row[i] = (n < p.Nn) ? p.b + (long)n * p.ldb + chunk_sw * 8 : nullptr;
  }

  auto load_tile = [&](int t, int buf) {
    const int kk0 = t * 64;
    const bf16_t* src; int C, kr;
    const bool first = kk0 < p.K1;
    if (first) { src = p.a1; C = p.C1; kr = kk0; }
    else { src = p.a2; C = p.C2; kr = kk0 - p.K1; }
    const int rs = kr / C, c0 = kr - rs * C;
    const int r = rs / p.S, s = rs - r * p.S;
    const int delta = (r * p.W + s) * C + c0;
    char* abase = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bool ok = no_halo ? a_hi[i] >= 0
                              : ((unsigned)(a_hi[i] + r) < (unsigned)p.H) && ((unsigned)(a_wi[i] + s) < (unsigned)p.W);
      const bf16_t* g = ok ? src + ((first ? a_o1[i] : a_o2[i]) + delta) : zero;
      __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(abase + (wave * AI + i) * 1024), 16, 0, 0);
    }
    char* bbase = abase + A_BYTES;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const bf16_t* g = b_row[i] ? b_row[i] + kk0 : zero;
      __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(bbase + (wave * BI + i) * 1024), 16, 0, 0);
    }
  };

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int KT = p.K / 64;
  const int a_off = (wm * WTM + (lane & 15)) * 128;
  const int b_off = (wn * WTN + (lane & 15)) * 128;
  load_tile(0, 0);
  if (NSTAGE == 3 && KT > 1) load_tile(1, 1);
  if (NSTAGE != 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < KT; ++t) {
    int cur;
    if (NSTAGE == 3) {
      // 3-deep ring: tile t landed (tile t+1 may stay in flight across the barrier), every
      // wave finished reading tile t-1, so its buffer can take tile t+2.  Raw s_barrier: a
      // __syncthreads() here would drain the LDS-DMA queue (vmcnt(0)).
      if (t + 1 < KT) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(AI + BI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      cur = t % 3;
      if (t + 2 < KT) load_tile(t + 2, (t + 2) % 3);
    } else {
      cur = NSTAGE == 2 ? (t & 1) : 0;
      if (NSTAGE == 2 && t + 1 < KT) load_tile(t + 1, cur ^ 1);
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int pos = (((kh * 4) + (lane >> 4)) ^ (lane & 7)) * 16;
      v8bf af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const v8bf*>(As + a_off + i * 16 * 128 + pos);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const v8bf*>(Bs + b_off + j * 16 * 128 + pos);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (NSTAGE == 1 && t + 1 < KT) {
      __syncthreads();            // every wave is done reading the single buffer
      load_tile(t + 1, 0);
    }
    if (NSTAGE != 3) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if (NSTAGE == 3) __syncthreads();   // all LDS reads done before the epilogue reuses LDS

  // ---------------- epilogue: fragments -> LDS (fp32) -> 16-byte row stores -------------
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * EPI_LD);
  constexpr int LPR = WTN / 8;   // lanes per row (8 columns each)
  constexpr int RPI = 64 / LPR;  // rows per iteration
  const int c8 = lane % LPR, rr = lane / LPR;
  const int gn = n0 + wn * WTN + c8 * 8;
  const bool col_ok = gn < p.Nn;
  float sc[8], sh[8];
  bool relu = p.relu != 0;
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  int ldo = p.ldo, col = gn;
  bool seg0 = true;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (p.mode != EPI_DGRAD && col_ok) {
    const float4* s4 = reinterpret_cast<const float4*>(p.scale + gn);
    const float4* h4 = reinterpret_cast<const float4*>(p.shift + gn);
    float4 a = s4[0], b = s4[1], c = h4[0], d = h4[1];
    sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
    sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w; sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
    if (p.out2 && gn >= p.n_split) {
      out = reinterpret_cast<bf16_t*>(p.out2); ldo = p.ldo2; relu = p.relu2 != 0; col = gn - p.n_split;
      seg0 = false;
    }
  }
#pragma unroll
  for (int pass = 0; pass < TM / 2; ++pass) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          stage[(i2 * 16 + (lane >> 4) * 4 + jj) * EPI_LD + j * 16 + (lane & 15)] = acc[pass * 2 + i2][j][jj];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int rl = it * RPI + rr;
      const int gm = m0 + wm * WTM + pass * 32 + rl;
      if (gm < p.M && col_ok) {
        const float4* sp = reinterpret_cast<const float4*>(stage + rl * EPI_LD + c8 * 8);
        float4 q0 = sp[0], q1 = sp[1];
        float v[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        if (p.mode == EPI_FWD) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[e] + sh[e];
          if (p.res) {
            float rv[8];
            unpack8(*reinterpret_cast<const uint4*>(p.res + (long)gm * p.ld_res + gn), rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += rv[e];
          }
          if (relu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          const uint4 pk = pack8(v);
          *reinterpret_cast<uint4*>(out + (long)gm * ldo + col) = pk;
          if (p.bits_out && seg0) {
            p.bits_out[(long)gm * p.ld_bits_out + (col >> 3)] = (uint8_t)pos_bits8(pk);
          }
        } else if (p.mode == EPI_F32) {
          float* o = reinterpret_cast<float*>(p.out) + (long)gm * p.ldo + gn;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[e] + sh[e];
          reinterpret_cast<float4*>(o)[0] = make_float4(v[0], v[1], v[2], v[3]);
          reinterpret_cast<float4*>(o)[1] = make_float4(v[4], v[5], v[6], v[7]);
        } else {  // EPI_DGRAD
          long row = gm;
          int n = 0, i = 0, j = 0;
          if (p.up2) {
            n = gm / HoWo; const int rem = gm - n * HoWo; i = rem / p.Wo; j = rem - i * p.Wo;
            row = ((long)n * p.Hf + 2 * i) * p.Wf + 2 * j;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            long rq = row;
            if (q > 0) {
              if (!p.up2) break;
              const int hh = 2 * i + (q >> 1), ww = 2 * j + (q & 1);
              if (hh >= p.Hf || ww >= p.Wf) continue;
              rq = ((long)n * p.Hf + hh) * p.Wf + ww;
            }
            float w[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = (q == 0) ? v[e] : 0.f;
            if (p.add) {
              float av[8];
              unpack8(*reinterpret_cast<const uint4*>(p.add + rq * p.ld_add + gn), av);
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] += av[e];
            }
            if (p.mask) {
              float mv[8];
              unpack8(*reinterpret_cast<const uint4*>(p.mask + rq * p.ld_mask + gn), mv);
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] = (mv[e] > 0.f) ? w[e] : 0.f;
            } else if (p.bits_mask) {
              const uint32_t byte = p.bits_mask[rq * p.ld_bits_mask + (gn >> 3)];
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] = ((byte >> e) & 1u) ? w[e] : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) csum[e] += w[e];
            *reinterpret_cast<uint4*>(out + rq * p.ldo + gn) = pack8(w);
          }
        }
      }
    }
    __syncthreads();
  }
  // Fused per-channel column sums of the written gradient (BN beta / conv bias grads):
  // fold the lanes that share columns, then each wave stores ONE partial row (plain
  // stores; atomics from every workgroup onto the same 64-2048 addresses serialize).
  // Rows are indexed (m-tile, wave-row); colsum_reduce folds them.
  if (p.colsum) {
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) csum[e] += __shfl_xor(csum[e], o, 64);
    if (rr == 0 && col_ok) {
      float4* dst = reinterpret_cast<float4*>(p.colsum + (long)(tm * (BM / WTM) + wm) * p.Nn + gn);
      dst[0] = make_float4(csum[0], csum[1], csum[2], csum[3]);
      dst[1] = make_float4(csum[4], csum[5], csum[6], csum[7]);
    }
  }
}

int igemm_partial_rows(int M, int Nn) {
  const int BM = Nn <= 64 ? 256 : 128;
  return ((M + BM - 1) / BM) * (BM / 64);
}

int g_igemm_variant = 0;   // 0 = heuristic; 1, 2, 3 = forced pipeline depth
int g_igemm_deep = 2;      // depth the heuristic uses for K >= 256

static bool igemm_check(const IgemmParams& p, const char** why) {
  if (p.K % 64 || p.K1 % 64) { *why = "K must be a multiple of 64"; return false; }
  // A k-tile (64 elements) must be contiguous in memory: C % 64 == 0, or the "window" form
  // S * C == 64 with stride 1 / pad 0 (space-to-depth stem: 4 taps x 16 channels).
  const bool window = (p.C1 * p.S == 64) && p.stride == 1 && p.pad == 0 && !p.a2;
  if ((p.C1 % 64 && !window) || (p.a2 && p.C2 % 64)) { *why = "channels must be multiples of 64"; return false; }
  if (p.a2 && (p.K - p.K1) % 64) { *why = "second source K must be a multiple of 64"; return false; }
  if (p.Nn % 8 || p.ldb % 8 || p.ldo % 8) { *why = "N / ldb / ldo must be multiples of 8"; return false; }
  if (p.M <= 0 || p.Nn <= 0 || p.K <= 0) { *why = "empty problem"; return false; }
  if ((long)p.N * p.H * p.W * (p.C1 > p.C2 ? p.C1 : p.C2) >= (1L << 31)) { *why = "input too large for 32-bit offsets"; return false; }
  return true;
}

const char* igemm_launch(const IgemmParams& p, hipStream_t stream) {
  const char* why = nullptr;
  if (!igemm_check(p, &why)) return why;
  // short K (<= 2 k-tiles) is memory-bound: single LDS stage for twice the resident blocks
  // Pipeline depth by K (variant knob for A/B timing: 0 = heuristic, 1/2/3 = forced stages)
  const int KT = p.K / 64;
  int ns = g_igemm_variant;
  if (ns == 0) ns = KT <= 2 ? 1 : (KT >= 4 ? g_igemm_deep : 2);
  if (ns == 3 && KT < 3) ns = 2;
#define IG_LAUNCH(BM_, BN_)                                                                                 \
  {                                                                                                        \
    const int nwg = ((p.M + BM_ - 1) / BM_) * ((p.Nn + BN_ - 1) / BN_);                                     \
    if (ns == 1) hipLaunchKernelGGL((igemm_kernel<BM_, BN_, 64, 64, 1>), dim3(nwg), dim3(256), 0, stream, p); \
    else if (ns == 2) hipLaunchKernelGGL((igemm_kernel<BM_, BN_, 64, 64, 2>), dim3(nwg), dim3(256), 0, stream, p); \
    else hipLaunchKernelGGL((igemm_kernel<BM_, BN_, 64, 64, 3>), dim3(nwg), dim3(256), 0, stream, p);      \
  }
  if (p.Nn <= 64) IG_LAUNCH(256, 64) else IG_LAUNCH(128, 128)
#undef IG_LAUNCH
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
