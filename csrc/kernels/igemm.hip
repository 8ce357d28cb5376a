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
//   * Tiles are staged global->LDS with 16-byte buffer LDS-DMA (buffer_load_dwordx4 ... lds);
//     the LDS image is lane-linear, so the bank-conflict XOR swizzle is applied to the SOURCE
//     address and the same involution on the ds_read_b128 address (rule 21).
//   * Out-of-bounds lanes (padding taps, tile overhang) use an out-of-range buffer offset,
//     which the buffer unit turns into zeros; the k-tile shift is a scalar soffset.
//   * Double-buffered LDS, XCD-aware bijective tile remap, LDS-staged epilogue that turns
//     the MFMA fragment layout into 16-byte row-contiguous stores.
#include "common.h"
#include "kernels.h"

namespace pddl {

// A-operand gather modes (compile-time, so the k loop carries no mode branches):
//   AM_DIRECT: every tap of every valid row is in bounds (1x1 / pad 0, the s2d stem window):
//              the per-lane buffer offset is loop-invariant and the k-tile's (r, s, c0) shift
//              rides in the scalar soffset -> no vector work per load.
//   AM_HALO:   padded convs (3x3 / pad 1): a per-row bitmask of the valid taps selects between
//              the row's offset and an out-of-range offset (buffer loads return zeros there).
//   AM_DUAL:   two AM_DIRECT sources concatenated along K (projection-block dgrad).
enum { AM_DIRECT = 0, AM_HALO = 1, AM_DUAL = 2 };

// Blocks per CU the 4-wave tiles are register-budgeted for (launch-bounds minimum).
#ifndef IGEMM_MIN_BLOCKS
#define IGEMM_MIN_BLOCKS 2
#endif

// LDS bank swizzle of the [rows][128 B] operand tiles (the XOR involution is applied to the
// DMA SOURCE chunk and to the ds_read_b128 address, cdna_hip_programming §5.4 rule 21).
// ds_read_b128 serves 16 lanes (16 consecutive rows, same logical chunk) per 256-byte bank
// row of two 128-byte LDS rows: slot = (row & 1) * 8 + (chunk ^ f(row)).  f(row) = (row >> 1) & 7
// gives 8 distinct chunks to the 8 rows of each parity -> 16 distinct slots, conflict-free
// (f(row) = row & 7 would put rows r and r + 8 on the same banks: 2-way conflicts).
// sw_chunk: logical chunk carried by lane-linear position (lane & 7) of DMA piece `i` (pieces
// are 8 rows, consecutive pieces of a wave alternate parity, so (row >> 1) & 7 =
// 4 * (i & 1) + lane / 16).  sw_read: byte position of logical chunk kh * 4 + lane / 16 for
// a lane reading row 16 * j + (lane & 15).
__device__ __forceinline__ int sw_chunk(int lane, int i) { return (lane & 7) ^ ((4 * (i & 1) + (lane >> 4)) & 7); }
__device__ __forceinline__ int sw_read(int lane, int kh) { return (((kh * 4) + (lane >> 4)) ^ ((lane >> 1) & 7)) * 16; }

// Bitmask of the in-bounds taps (bit r * S + s) of an output row whose window starts at input
// (hi, wi).  The 3x3 case (every padded conv of ResNet-50) is unrolled: the generic runtime-R/S
// loops cost ~45 instructions and three branches per staged row in every tile's prologue.
__device__ __forceinline__ uint32_t halo_taps(const IgemmParams& p, int hi, int wi) {
  if (p.R == 3 && p.S == 3) {
    const uint32_t cols = ((unsigned)wi < (unsigned)p.W ? 1u : 0u) | ((unsigned)(wi + 1) < (unsigned)p.W ? 2u : 0u) |
                          ((unsigned)(wi + 2) < (unsigned)p.W ? 4u : 0u);
    return ((unsigned)hi < (unsigned)p.H ? cols : 0u) | ((unsigned)(hi + 1) < (unsigned)p.H ? cols << 3 : 0u) |
           ((unsigned)(hi + 2) < (unsigned)p.H ? cols << 6 : 0u);
  }
  uint32_t rows = 0, cols = 0, mk = 0;
  for (int r = 0; r < p.R; ++r) rows |= (uint32_t)((unsigned)(hi + r) < (unsigned)p.H) << r;
  for (int s = 0; s < p.S; ++s) cols |= (uint32_t)((unsigned)(wi + s) < (unsigned)p.W) << s;
  for (int r = 0; r < p.R; ++r) mk |= ((rows >> r) & 1u) ? cols << (r * p.S) : 0u;
  return mk;
}

// Epilogue of one wave sub-tile of TM x TN 16x16 fragments at global rows [mb, mb + 16*TM)
// and columns [nb, nb + 16*TN): fragments -> LDS (fp32, per-wave `stage` of 32 x (16*TN + 4))
// -> 16-byte row stores with the fused FWD / F32 / DGRAD operations; the column sums (dgrad)
// and batch statistics (train-mode BN forward) go to partial row `prow`.
// PF: the per-element epilogue operand of the whole sub-tile is loaded into registers before
// the accumulators are staged, so its HBM latency overlaps the staging.
// The per-element epilogue operand rows of a wave sub-tile (forward residual / dgrad `add`, plus
// the dgrad ReLU bits), 32-row passes [pass0, pass0 + npass) into dst / bits.  Branch-free loads
// (row and column clamped into the tensor, the value zeroed afterwards): under an exec branch
// the compiler completes each load (and everything issued before it) inside the branch, which
// serialises the prefetch into one HBM round trip per row.  Both loads are issued whenever
// either operand is in use (an unused one reads the output tensor's first element) so that
// neither sits under a uniform branch either.
template <int TM, int TN>
__device__ __forceinline__ void igemm_epi_load(const IgemmParams& p, int mb, int nb, int lane, int pass0, int npass,
                                               uint4* dst, uint32_t* bits) {
  constexpr int WTN = 16 * TN, LPR = WTN / 8, RPI = 64 / LPR, NIT = 32 / RPI;
  const int c8 = lane % LPR, rr = lane / LPR;
  const int gn = nb + c8 * 8;
  const bool col_ok = gn < p.Nn;
  const bool pf_bits = p.mode == EPI_DGRAD && !p.up2 && !p.mask && p.bits_mask;
  const bool pre_on = (p.mode == EPI_FWD && p.res) || (p.mode == EPI_DGRAD && p.add && !p.up2);
  const bf16_t* pre_src = p.mode == EPI_FWD ? p.res : p.add;
  const int pre_ld = p.mode == EPI_FWD ? p.ld_res : p.ld_add;
  const int gn_c = col_ok ? gn : 0;
  const bf16_t* psrc = pre_on ? pre_src : reinterpret_cast<const bf16_t*>(p.out);
  const long pld = pre_on ? pre_ld : 0;
  const int pcol = pre_on ? gn_c : 0;
  const uint8_t* bsrc = pf_bits ? p.bits_mask : reinterpret_cast<const uint8_t*>(p.out);
  const long bld = pf_bits ? p.ld_bits_mask : 0;
  const int bcol = pf_bits ? (gn_c >> 3) : 0;
#pragma unroll
  for (int q = 0; q < npass; ++q)
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int gm = mb + (pass0 + q) * 32 + it * RPI + rr;
      const bool ok = gm < p.M && col_ok;
      const long gr = gm < p.M ? gm : p.M - 1;
      long rr_res = gr;
      if (p.mode == EPI_FWD && p.up2) {   // residual on the 2x finer grid, read at the stride-2 positions
        const int n = fdiv((int)gr, p.mg_howo), rem = (int)gr - n * p.Ho * p.Wo, i = fdiv(rem, p.mg_wo);
        rr_res = ((long)n * p.Hf + 2 * i) * p.Wf + 2 * (rem - i * p.Wo);
      }
      const uint4 v = *reinterpret_cast<const uint4*>(psrc + rr_res * pld + pcol);
      const uint32_t b = bsrc[gr * bld + bcol];
      dst[q * NIT + it] = (ok && pre_on) ? v : make_uint4(0, 0, 0, 0);
      bits[q * NIT + it] = (ok && pf_bits) ? b : 0u;
    }
}

template <int TM, int TN, bool PF, bool BNZ = false>
__device__ __forceinline__ void igemm_epilogue(const IgemmParams& p, v4f (&acc)[TM][TN], int mb, int nb, int prow,
                                               float* stage, int lane) {
  constexpr int WTN = 16 * TN;
  constexpr int EPI_LD = WTN + 4;
  const int HoWo = p.Ho * p.Wo;
  constexpr int LPR = WTN / 8;   // lanes per row (8 columns each)
  constexpr int RPI = 64 / LPR;  // rows per iteration
  const int c8 = lane % LPR, rr = lane / LPR;
  const int gn = nb + c8 * 8;
  const bool col_ok = gn < p.Nn;
  float sc[8], sh[8];
  bool relu = p.relu != 0;
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  int ldo = p.ldo, col = gn;
  bool seg0 = true;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float csq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // FWD stats: sum of squares; DGRAD: sum g*(z-mu)
  // sc: FWD / F32 scale, or (BNZ: DGRAD + bn_z) the batch mean of the BN whose output
  // gradient this is.  BNZ is a separate kernel instantiation: the fused sums cost the
  // default kernels' register budget 30 VGPRs (occupancy 3 -> 2) when compiled in.
  if ((p.mode != EPI_DGRAD || BNZ) && col_ok) {
    const float4* s4 = reinterpret_cast<const float4*>((p.mode == EPI_DGRAD ? p.bn_mean : p.scale) + gn);
    const float4* h4 = reinterpret_cast<const float4*>((p.mode == EPI_DGRAD ? p.bn_mean : p.shift) + gn);
    float4 a = s4[0], b = s4[1], c = h4[0], d = h4[1];
    sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
    sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w; sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
    if (p.out2 && gn >= p.n_split) {
      out = reinterpret_cast<bf16_t*>(p.out2); ldo = p.ldo2; relu = p.relu2 != 0; col = gn - p.n_split;
      seg0 = false;
    }
  }
  constexpr int NIT = 32 / RPI;
  // The per-element operand (forward residual / dgrad `add` + ReLU bits) is loaded ahead of
  // the stores that consume it: PF for the whole sub-tile before the staging, otherwise one
  // 32-row pass at a time at the top of the pass.  (Loaded inside the store loop, each load
  // would wait behind the previous iteration's store -- `out` may alias `add` as far as the
  // compiler knows -- and the pass would pay NIT serialised HBM round trips.)
  uint4 pre[PF ? (TM / 2) * NIT : NIT];
  uint32_t pre_bits[PF ? (TM / 2) * NIT : NIT];
  const bool pf_bits = p.mode == EPI_DGRAD && !p.up2 && !p.mask && p.bits_mask;
  const bool pre_on = (p.mode == EPI_FWD && p.res) || (p.mode == EPI_DGRAD && p.add && !p.up2);
  if (PF && (pre_on || pf_bits)) igemm_epi_load<TM, TN>(p, mb, nb, lane, 0, TM / 2, pre, pre_bits);
#pragma unroll
  for (int pass = 0; pass < TM / 2; ++pass) {
    if (!PF && (pre_on || pf_bits)) igemm_epi_load<TM, TN>(p, mb, nb, lane, pass, 1, pre, pre_bits);
    const uint4* ppre = PF ? pre + pass * NIT : pre;
    const uint32_t* pbits = PF ? pre_bits + pass * NIT : pre_bits;
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
      const int gm = mb + pass * 32 + rl;
      if (gm < p.M && col_ok) {
        const float4* sp = reinterpret_cast<const float4*>(stage + rl * EPI_LD + c8 * 8);
        float4 q0 = sp[0], q1 = sp[1];
        float v[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        if (p.mode == EPI_FWD) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[e] + sh[e];
          if (p.res) {
            float rv[8];
            const uint4 r4 = ppre[it];
            unpack8(r4, rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += rv[e];
          }
          uint4 pk = pack8(v);
          if (relu) pk = relu_pk8(pk);
          *reinterpret_cast<uint4*>(out + (long)gm * ldo + col) = pk;
          if (p.bits_out && seg0) {
            p.bits_out[(long)gm * p.ld_bits_out + (col >> 3)] = (uint8_t)pos_bits8(pk);
          }
          if (p.stats) {   // batch statistics of exactly the values the BN-apply pass will read
            float rv[8];
            unpack8(pk, rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) { csum[e] += rv[e]; csq[e] += rv[e] * rv[e]; }
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
            n = fdiv(gm, p.mg_howo); const int rem = gm - n * HoWo; i = fdiv(rem, p.mg_wo); j = rem - i * p.Wo;
            row = ((long)n * p.Hf + 2 * i) * p.Wf + 2 * j;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            long rq = row;
            if (q > 0) {
              if (p.up2 != 1) break;   // up2 == 2: the caller's tensor is zero off the grid already
              const int hh = 2 * i + (q >> 1), ww = 2 * j + (q & 1);
              if (hh >= p.Hf || ww >= p.Wf) continue;
              rq = ((long)n * p.Hf + hh) * p.Wf + ww;
            }
            float w[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = (q == 0) ? v[e] : 0.f;
            if (p.add) {
              float av[8];
              uint4 a4;   // (if/else, not ?: -- an lvalue select would force `pre` into scratch)
              if (!p.up2) a4 = ppre[it];
              else a4 = *reinterpret_cast<const uint4*>(p.add + rq * p.ld_add + gn);
              unpack8(a4, av);
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] += av[e];
            }
            const long rm = p.up2 == 3 ? (long)gm : rq;   // (up2 3: the mask is on the compact grid)
            if (p.mask) {
              float mv[8];
              unpack8(*reinterpret_cast<const uint4*>(p.mask + rm * p.ld_mask + gn), mv);
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] = (mv[e] > 0.f) ? w[e] : 0.f;
            } else if (p.bits_mask) {
              uint32_t byte;
              if (pf_bits) byte = pbits[it];
              else byte = p.bits_mask[rm * p.ld_bits_mask + (gn >> 3)];
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] = ((byte >> e) & 1u) ? w[e] : 0.f;
            }
            const uint4 pk = pack8(w);
            if constexpr (BNZ) {
              // train-mode BN backward reduction fused here (stats rows; no up2): sums of exactly
              // the stored bf16 gradient, as bn_bwd_apply will read it
              float zv[8], wr[8];
              unpack8(*reinterpret_cast<const uint4*>(p.bn_z + rq * p.ldo + gn), zv);
              unpack8(pk, wr);
#pragma unroll
              for (int e = 0; e < 8; ++e) { csum[e] += wr[e]; csq[e] += wr[e] * (zv[e] - sc[e]); }
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) csum[e] += w[e];
            }
            *reinterpret_cast<uint4*>(out + rq * p.ldo + gn) = pk;
            // compact copy of the stride-2 positions (the only nonzero rows of the scatter):
            // the consumers of a downsampling block's input gradient run at a quarter of M on it
            if (q == 0 && p.up2 && p.out2)
              *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.out2) + (long)gm * p.ldo2 + gn) = pk;
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
      float4* dst = reinterpret_cast<float4*>(p.colsum + (long)prow * p.Nn + gn);
      dst[0] = make_float4(csum[0], csum[1], csum[2], csum[3]);
      dst[1] = make_float4(csum[4], csum[5], csum[6], csum[7]);
    }
  }
  // Train-mode BN: per-wave partial (sum, sum of squares) rows of the forward output, same
  // row indexing as the column sums; colsum_reduce folds them and bn_stats finalizes.  In a
  // dgrad with bn_z the rows are (sum g, sum g*(z - mean)) for bn_bwd_apply.
  if (p.stats) {
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        csum[e] += __shfl_xor(csum[e], o, 64);
        csq[e] += __shfl_xor(csq[e], o, 64);
      }
    if (rr == 0 && col_ok) {
      float* row = p.stats + (long)prow * 2 * p.Nn;
      float4* d1 = reinterpret_cast<float4*>(row + gn);
      float4* d2 = reinterpret_cast<float4*>(row + p.Nn + gn);
      d1[0] = make_float4(csum[0], csum[1], csum[2], csum[3]);
      d1[1] = make_float4(csum[4], csum[5], csum[6], csum[7]);
      d2[0] = make_float4(csq[0], csq[1], csq[2], csq[3]);
      d2[1] = make_float4(csq[4], csq[5], csq[6], csq[7]);
    }
  }
}

// Block tile BM x BN (128x128 or 256x64) of 4 waves, each wave a 64x64 tile of 16x16x32 MFMAs.
//   NSTAGE 1: one LDS buffer, 3 resident blocks per CU overlap each other's load and MFMA phases.
//   NSTAGE 2: double buffer, the next k-tile's LDS-DMA overlaps this tile's MFMAs.
// (Rejected and removed after per-layer A/B: an 8-wave 256x128 3-stage ring, an 8-wave 256x256
// 2-stage tile, a 2-stage pipeline with the next tile's LDS-DMA interleaved into the MFMA groups,
// an early epilogue-operand prefetch and a register-direct epilogue -- all neutral or slower,
// profiles/r1_kbench_b1024_interleaved_issue.json, profiles/r3_hbm_bytes_per_layer.txt.  The
// wide long-K layers run on igemm8_kernel below.)
// PF: the epilogue's per-element operand (forward residual / dgrad residual-gradient `add`,
// plus the dgrad ReLU bitmask) of the whole wave tile is loaded into registers before the
// accumulators are staged through LDS, so its HBM latency overlaps the staging instead of
// stalling every store iteration (short-K 1x1 layers are epilogue-bound).
// SK: split-K slice instantiation (separate, so the unsplit kernels keep their register budget:
// the slice bookkeeping compiled into every instantiation cost 33 VGPRs, occupancy 3 -> 2).
template <int BM, int BN, int NSTAGE, int AM, bool PF = false, bool BNZ = false, bool SK = false>
__global__ void __launch_bounds__(256, IGEMM_MIN_BLOCKS) igemm_kernel(IgemmParams p) {
  constexpr int NW = 4, WTM = 64, WTN = 64;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int WAVES_N = BN / WTN;
  static_assert((BM / WTM) * (BN / WTN) == NW, "wave grid must cover the block tile");
  static_assert(NSTAGE == 1 || NSTAGE == 2, "1- or 2-stage LDS pipeline");
  constexpr int NS = NSTAGE;   // LDS buffers
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW);  // 1 KiB LDS-DMA pieces per wave per tile
  static_assert(AI * 8 * NW == BM && BI * 8 * NW == BN, "tile rows must split evenly over the waves");
  constexpr int EPI_LD = WTN + 4;
  constexpr int EPI_BYTES = NW * 32 * EPI_LD * 4;
  constexpr int SMEM = (NS * STAGE > EPI_BYTES) ? NS * STAGE : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably uniform: M0 from SGPRs
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int mt = (p.M - p.m_begin + BM - 1) / BM, nt = (p.Nn + BN - 1) / BN;
  // split-K: the K loop of every tile is cut into `ks` slices run by adjacent workgroups (same
  // XCD after the remap); each slice leaves its fp32 partial tile in the workspace and
  // igemm_splitk_reduce_kernel sums them and runs the fused epilogue
  const int ks = SK ? p.ksplit : 1;
  const int wgs = xcd_remap(blockIdx.x, mt * nt * ks);
  const int slice = wgs % ks, wg = wgs / ks;
  const int tn = wg % nt, tm = wg / nt;
  const int m0 = p.m_begin + tm * BM, n0 = tn * BN;
  const int HoWo = p.Ho * p.Wo;
  const int KT_all = p.K / 64;
  const int kt0 = (int)((long)slice * KT_all / ks);
  const int KT = (int)((long)(slice + 1) * KT_all / ks) - kt0;

  // Buffer descriptors (wave-uniform values only, so no waterfall loops).  The A descriptors
  // start at the first image this tile's rows read (n_first), so lane offsets span only the
  // tile's few images, whatever the batch.
  const int n_first = fdiv(m0, p.mg_howo);
  const long HW = (long)p.H * p.W, pix0 = n_first * HW, pix_end = p.N * HW;
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc_at(p.a1, pix0 * p.C1, pix_end * p.C1);
  const int C2r = AM == AM_DUAL ? p.C2 : p.C1;
  // (the second source may have its own geometry: the fused projection shortcut reads the block
  // input at H2 x W2 with stride2 next to conv3's stride-1 operand)
  const long HW2 = AM == AM_DUAL ? (long)p.H2 * p.W2 : HW;
  const __amdgpu_buffer_rsrc_t ra2 =
      make_rsrc_at(AM == AM_DUAL ? p.a2 : p.a1, n_first * HW2 * C2r, p.N * HW2 * C2r);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.b, p.Nn * p.ldb * 2);

  // Per-lane constant source chunk: LDS position (lane & 7) of row (lane >> 3) holds the
  // logical 16-byte chunk (lane & 7) ^ (row & 7).
  // LDS-DMA piece i of a wave holds rows 8*(piece) + lane/8 (piece parity = i & 1); its lane-linear
  // 16-byte chunk (lane & 7) carries logical chunk (lane & 7) ^ ((row >> 1) & 7) (sw_chunk).

  // A-row bookkeeping (fixed over the k loop): byte offset of the row's tap (0, 0) in each
  // source (OOB_OFF for rows past M) and, for AM_HALO, the bitmask of its in-bounds taps.
  uint32_t a_o1[AI], a_o2[AI], a_taps[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (wave * AI + i) * 8 + (lane >> 3);
    a_o1[i] = OOB_OFF; a_o2[i] = OOB_OFF; a_taps[i] = 0;
    if (m < p.M) {
      const int n = fdiv(m, p.mg_howo), rem = m - n * HoWo;
      const int ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
      const int hi = ho * p.stride - p.pad, wi = wo * p.stride - p.pad;
      const int pix = ((n - n_first) * p.H + hi) * p.W + wi;
      a_o1[i] = (uint32_t)((pix * p.C1 + sw_chunk(lane, i) * 8) * 2);
      if (AM == AM_DUAL) {
        const int pix2 = ((n - n_first) * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2;
        a_o2[i] = (uint32_t)((pix2 * p.C2 + sw_chunk(lane, i) * 8) * 2);
      }
      if (AM == AM_HALO) a_taps[i] = halo_taps(p, hi, wi);
    }
  }
  uint32_t b_o[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + (wave * BI + i) * 8 + (lane >> 3);
    b_o[i] = (n < p.Nn) ? (uint32_t)((n * p.ldb + sw_chunk(lane, i) * 8) * 2) : OOB_OFF;
  }

  // k-tile walk state (scalar): the next tile to load is tap (r, s), channels [c0, c0 + 64)
  // of source `src2`; a "window" tile (C * S == 64) spans all S taps of one r.
  int ld_r = 0, ld_s = 0, ld_c0 = 0, ld_src2 = 0, ld_k = 0;
  const bool window = p.C1 * p.S == 64 && p.C1 < 64;
  if (SK && kt0 > 0) {   // (split-K slices: single source, C1 % 64 == 0 -- igemm_launch guarantees)
    ld_k = kt0 * 64;
    ld_c0 = ld_k % p.C1;
    const int tq = ld_k / p.C1;
    ld_s = tq % p.S;
    ld_r = tq / p.S;
  }
  // piece j (< AI: A rows, else B rows) of the current walk position into LDS buffer buf
  auto tile_delta = [&]() { return ((ld_r * p.W + ld_s) * (ld_src2 ? p.C2 : p.C1) + ld_c0) * 2; };   // bytes
  auto load_piece = [&](int buf, int j, int delta) {
    char* abase = smem + buf * STAGE;
    if (j < AI) {
      const int i = j;
      void __attribute__((address_space(3)))* dst = LDS_PTR(abase + (wave * AI + i) * 1024);
      if (AM == AM_HALO) {
        const int tap = ld_r * p.S + ld_s;
        const uint32_t off = ((a_taps[i] >> tap) & 1u) ? a_o1[i] + (uint32_t)delta : OOB_OFF;
        buf_lds16(ra1, dst, off, 0);
      } else if (AM == AM_DUAL && ld_src2) {
        buf_lds16(ra2, dst, a_o2[i], delta);
      } else {
        buf_lds16(ra1, dst, a_o1[i], delta);
      }
    } else {
      const int i = j - AI;
      buf_lds16(rb, LDS_PTR(abase + A_BYTES + (wave * BI + i) * 1024), b_o[i], ld_k * 2);
    }
  };
  // advance the walk to the next k-tile
  auto advance = [&]() {
    const int C = ld_src2 ? p.C2 : p.C1;
    ld_k += 64;
    if (window && !ld_src2) {
      ++ld_r;
    } else {
      ld_c0 += 64;
      if (ld_c0 == C) {
        ld_c0 = 0;
        if (++ld_s == p.S) { ld_s = 0; ++ld_r; }
      }
    }
    if (AM == AM_DUAL && !ld_src2 && ld_k == p.K1) { ld_src2 = 1; ld_r = ld_s = ld_c0 = 0; }
  };
  auto load_tile = [&](int buf) {
    const int delta = tile_delta();
#pragma unroll
    for (int j = 0; j < AI + BI; ++j) load_piece(buf, j, delta);
    advance();
  };

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int a_off = (wm * WTM + (lane & 15)) * 128;
  const int b_off = (wn * WTN + (lane & 15)) * 128;
  load_tile(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < KT; ++t) {
    const int cur = NS == 2 ? (t & 1) : 0;
    if (NSTAGE == 2 && t + 1 < KT) load_tile(cur ^ 1);
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int pos = sw_read(lane, kh);
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
      load_tile(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (SK) {   // split-K slice: the fp32 partial tile in fragment order (16-byte coalesced stores)
    float4* dst = reinterpret_cast<float4*>(p.slab) + ((long)(wg * ks + slice) * NW + wave) * (TM * TN) * 64 + lane;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        dst[(i * TN + j) * 64] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    return;   // igemm_splitk_reduce_kernel combines
  }

  // ---------------- epilogue: fragments -> LDS (fp32) -> 16-byte row stores -------------
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * (WTN + 4));
  igemm_epilogue<TM, TN, PF, BNZ>(p, acc, m0 + wm * WTM, n0 + wn * WTN, p.prow_begin + tm * (BM / WTM) + wm, stage,
                                  lane);
}


// Persistent ring implicit GEMM for the short-K 1x1 layers (K = 64 * KT, KT <= 8): the
// expansion 1x1s of every block in forward, whose epilogue streams the residual, and the 1x1
// dgrads with their residual-gradient add and ReLU bits (cdna_hip_programming §5.6, loader
// ring).  The single-stage tiles run those layers at 3.4-4.8 TB/s: each block is a serial chain
// load -> MFMA -> load ... -> residual load -> store, overlapped only across 3 resident blocks.
//
// One launch of #CUs x (LDS / ring) workgroups; each owns a contiguous range of 128x128 output
// tiles (column tiles fastest: consecutive tiles re-read the same A rows from L2; the XCD remap
// keeps neighbouring ranges on one XCD).  A tile is SPT = KT (+1) RING STEPS of 32 KiB: its KT
// k-steps (A | B operand tiles) and, when the epilogue has a per-element operand, one OPERAND
// step (the residual / residual-gradient tile, plus its ReLU-bit rows or, forward, the tile's
// scale / shift columns: the epilogue issues no global load at all).  Every step is
// LDS-DMA; step s + NB - 1 is issued right after step s landed, so NB - 1 steps are always in
// flight ACROSS tile boundaries: while a tile's epilogue runs, the next tile's operands and
// residual are already on their way.  The epilogue is register direct (the igemm_epilogue_rd
// shuffles) and reads its operand from the ring slot; its stores are branch-free buffer stores
// (out-of-range rows / columns get the out-of-range offset, which the hardware drops).
//
// vmcnt bookkeeping (loads, stores and LDS-DMA share one in-order counter): a k-step is exactly
// PPS = 8 LDS-DMA pieces per wave, an operand step op_n (8 residual pieces + 2 four-byte ReLU-bit
// pieces, or 1 scale / shift piece), a tile epilogue e_n stores; steps past the block's range are issued anyway (zeros
// from out-of-range offsets into a slot nobody reads), so every count is a launch constant and
// the wait for step s counts exactly the younger operations (rounded down: a lower bound only
// makes the wait stricter).  AM_DIRECT only (1x1, any stride); no stride-2 scatter, no split
// outputs, no train-BN sums (those layers keep igemm_kernel).
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int cdiv_signed(int a, int b) { return a >= 0 ? (a + b - 1) / b : -((-a) / b); }
// LDS chunk swizzle of the operand tile ([128 rows][16 chunks of 16 B], row-major): the RD
// epilogue's ds_read_b128 serves 8 rows x 2 chunks per 16 lanes; XOR-ing the chunk with
// (row & 3) | (row & 4) << 1 keeps those 16 positions distinct (conflict-free).
__device__ __forceinline__ int pk_sw(int row) { return (row & 3) | ((row & 4) << 1); }

// DUAL: two A sources concatenated along K (the projection block's conv3 + shortcut conv,
// K = K1 + K2): k-steps [0, K1 / 64) read the first source, the rest the second at its own
// geometry (H2 x W2, stride2) -- the same ring, the same B walk over the concatenated weights.
template <int KT, int NB, bool OPS, bool FWD, bool DUAL = false>
__global__ void __launch_bounds__(256, NB == 2 ? 2 : 1) igemm_pk_kernel(IgemmParams p) {
  constexpr int BM = 128, BN = 128, NW = 4, TM = 4, TN = 4, WAVES_N = 2;
  constexpr int A_BYTES = BM * 128, STAGE = A_BYTES + BN * 128;   // 32 KiB: A | B, or the operand tile
  constexpr int BITS_BYTES = BM * 16;                             // ReLU-bit rows of one tile
  constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW), PPS = AI + BI;
  constexpr int SPT = KT + (OPS ? 1 : 0);
  static_assert(NB >= 2 && NB * (STAGE + (OPS ? BITS_BYTES : 0)) <= 160 * 1024, "ring must fit the LDS");
  __shared__ __attribute__((aligned(16))) char smem[NB * STAGE + (OPS ? NB * BITS_BYTES : 1)];
  char* bits_lds = smem + NB * STAGE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int mt = (p.M - p.m_begin + BM - 1) / BM, nt = (p.Nn + BN - 1) / BN;
  const int T = mt * nt, G = gridDim.x;
  // tiles bq, bq + G, bq + 2G, ...: at any moment the co-resident workgroups of one XCD (consecutive
  // bq after the remap) work on consecutive tiles, i.e. on all column tiles of a few row tiles,
  // so each A row block is fetched once and shared through that XCD's L2 (a contiguous range
  // per workgroup re-fetched A for every column tile: measured 2.4x the fabric reads)
  const int bq = xcd_remap(blockIdx.x, G);
  if (bq >= T) return;   // (whole workgroup)
  const int t_begin = bq, t_end = T;
  const long HW = (long)p.H * p.W, pix_end = p.N * HW;
  const long HW2 = DUAL ? (long)p.H2 * p.W2 : 0;
  const int KT1 = DUAL ? p.K1 / 64 : KT;   // k-steps of the first source
  const int HoWo = p.Ho * p.Wo;
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.b, p.Nn * p.ldb * 2);

  // launch-uniform epilogue configuration and the vector-memory op counts it implies
  // (FWD: one instantiation per epilogue mode, so neither carries the other's code)
  constexpr bool is_fwd = FWD;
  const uint16_t* opnd = is_fwd ? p.res : p.add;
  const int ld_op = is_fwd ? p.ld_res : p.ld_add;
  const bool res_on = OPS && opnd != nullptr;
  const bool bits_in = OPS && !is_fwd && p.bits_mask != nullptr;
  const bool bits_out = is_fwd && p.bits_out != nullptr;
  const bool csum_on = !is_fwd && p.colsum != nullptr;
  const int op_n = (res_on ? 8 : 0) + (bits_in ? 2 : 0) + (is_fwd ? 1 : 0);
  const int e_n = 2 * TM * (bits_out ? 2 : 1) + (csum_on ? 2 : 0);

  // ---- loader: LDS-DMA of ring step (ld_t, ld_j) ----
  int ld_t = t_begin, ld_j = 0;
  uint32_t a_o[AI], a_o2[DUAL ? AI : 1], b_o[BI];
  __amdgpu_buffer_rsrc_t ra, ra2;
  auto set_tile = [&](int t) {
    const int m0 = p.m_begin + (t / nt) * BM, n0 = (t % nt) * BN;
    const int n_first = fdiv(m0, p.mg_howo);
    ra = make_rsrc_at(p.a1, n_first * HW * p.C1, pix_end * p.C1);
    if (DUAL) ra2 = make_rsrc_at(p.a2, n_first * HW2 * p.C2, p.N * HW2 * p.C2);
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int m = m0 + (wave * AI + i) * 8 + (lane >> 3);
      a_o[i] = OOB_OFF;
      if (DUAL) a_o2[i] = OOB_OFF;
      if (m < p.M) {
        const int n = fdiv(m, p.mg_howo), rem = m - n * HoWo;
        const int ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
        const int pix = ((n - n_first) * p.H + ho * p.stride) * p.W + wo * p.stride;
        a_o[i] = (uint32_t)((pix * p.C1 + sw_chunk(lane, i) * 8) * 2);
        if (DUAL) {
          const int pix2 = ((n - n_first) * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2;
          a_o2[i] = (uint32_t)((pix2 * p.C2 + sw_chunk(lane, i) * 8) * 2);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int n = n0 + (wave * BI + i) * 8 + (lane >> 3);
      b_o[i] = (n < p.Nn) ? (uint32_t)((n * p.ldb + sw_chunk(lane, i) * 8) * 2) : OOB_OFF;
    }
  };
  set_tile(t_begin);
  auto issue = [&](int buf) {
    const bool live = ld_t < t_end;    // (uniform) past the range: zeros into a slot nobody reads
    char* base = smem + buf * STAGE;
    if (!OPS || ld_j < KT) {           // k-step: channels [64 ld_j, 64 ld_j + 64) of the rows
      const int kofs = ld_j * 128;
      if (DUAL && ld_j >= KT1) {       // (uniform) the second source's channels [64 (ld_j - KT1), +64)
#pragma unroll
        for (int i = 0; i < AI; ++i)
          buf_lds16(ra2, LDS_PTR(base + (wave * AI + i) * 1024), live ? a_o2[i] : OOB_OFF, kofs - KT1 * 128);
      } else {
#pragma unroll
        for (int i = 0; i < AI; ++i) buf_lds16(ra, LDS_PTR(base + (wave * AI + i) * 1024), live ? a_o[i] : OOB_OFF, kofs);
      }
#pragma unroll
      for (int i = 0; i < BI; ++i)
        buf_lds16(rb, LDS_PTR(base + A_BYTES + (wave * BI + i) * 1024), live ? b_o[i] : OOB_OFF, kofs);
    } else {                           // operand step: rows 32 wave + 4 i + lane / 16, chunk (lane & 15)
      const int lt = live ? ld_t : t_begin;   // (past the range: a valid tile's descriptors, zero reads)
      const int m0 = p.m_begin + (lt / nt) * BM, n0 = (lt % nt) * BN;
      if (res_on) {
        const __amdgpu_buffer_rsrc_t ro = make_rsrc_at(opnd, (long)m0 * ld_op, (long)p.M * ld_op);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = wave * 32 + i * 4 + (lane >> 4);
          const int ch = (lane & 15) ^ pk_sw(row);
          const int col = n0 + ch * 8;
          const bool ok = live && m0 + row < p.M && col < p.Nn;
          buf_lds16(ro, LDS_PTR(base + (wave * 32 + i * 4) * 256), ok ? (uint32_t)((row * ld_op + col) * 2) : OOB_OFF, 0);
        }
      }
      if (is_fwd) {                    // the tile's 128 scale | 128 shift values: one 256 B piece per wave
        const float* src = wave < 2 ? p.scale : p.shift;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, p.Nn * 4);
        const int col = n0 + (wave & 1) * 64 + lane;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(bits_lds + buf * BITS_BYTES + wave * 256), 4,
                                                 live && col < p.Nn ? (uint32_t)(col * 4) : OOB_OFF, 0, 0, 0);
      }
      if (bits_in) {                   // 16 bytes (128 columns) per row, 4 bytes per lane
        const int ldb8 = p.ld_bits_mask;
        const __amdgpu_buffer_rsrc_t rbm =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.bits_mask) + (long)m0 * ldb8, (short)0,
                                              (int)lmin(((long)p.M - m0) * ldb8, 0x7fffffffL), 0x00020000);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int row = wave * 32 + q * 16 + (lane >> 2);
          const int byte = (n0 >> 3) + (lane & 3) * 4;
          const bool ok = live && m0 + row < p.M && byte * 8 < p.Nn;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbm, LDS_PTR(bits_lds + buf * BITS_BYTES + (wave * 32 + q * 16) * 16), 4,
                                                   ok ? (uint32_t)(row * ldb8 + byte) : OOB_OFF, 0, 0, 0);
        }
      }
    }
    if (++ld_j == SPT) {
      ld_j = 0;
      ld_t += G;
      if (ld_t < t_end) set_tile(ld_t);
    }
  };
  // wait until step s landed in every wave's view: `younger` = vector-memory ops this wave issued
  // after it (a lower bound is safe); vmcnt takes an immediate, so buckets of 4
  auto wait_barrier = [&](int younger) {
    switch ((younger > 63 ? 63 : younger) >> 2) {
#define PK_W(n, c) case n: asm volatile("s_waitcnt vmcnt(" #c ") lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      PK_W(1, 4) PK_W(2, 8) PK_W(3, 12) PK_W(4, 16) PK_W(5, 20) PK_W(6, 24) PK_W(7, 28) PK_W(8, 32) PK_W(9, 36)
      PK_W(10, 40) PK_W(11, 44) PK_W(12, 48) PK_W(13, 52) PK_W(14, 56) PK_W(15, 60)
#undef PK_W
      default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
  };

#pragma unroll
  for (int j = 0; j < NB - 1; ++j) issue(j);   // prologue: ring steps 0 .. NB-2
  int cur = 0;                                   // ring slot of the current step
  const int a_off = (wm * 64 + (lane & 15)) * 128;
  const int b_off = (wn * 64 + (lane & 15)) * 128;
  const int g = lane >> 4, r = lane & 15, r8 = r & 7;
  const int lc = wn * 64 + 32 * (r >> 3) + 16 * (g & 1) + 8 * (g >> 1);   // this lane's 8 columns in the tile
  for (int t = t_begin, u = 0; t < t_end; t += G, ++u) {
    const int m0 = p.m_begin + (t / nt) * BM, n0 = (t % nt) * BN;
    v4f acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    int op_slot = 0;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      // younger than step s = u * SPT + j: steps s+1 .. s+NB-2, and the epilogues of tiles
      // v in [u - 1 + cdiv(j - NB + 2, SPT), u - 1] (issued after step s was)
      int y = 0;
#pragma unroll
      for (int x = 1; x <= NB - 2; ++x) y += (OPS && (j + x) % SPT == KT) ? op_n : PPS;
      int ce = 1 - cdiv_signed(j - NB + 2, SPT);
      ce = ce < 0 ? 0 : (ce > u ? u : ce);
      wait_barrier(y + ce * e_n);
      issue(cur == 0 ? NB - 1 : cur - 1);        // step s + NB - 1 into the slot step s - 1 used
      if (!OPS || j < KT) {
        const char* As = smem + cur * STAGE;
        const char* Bs = As + A_BYTES;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const int pos = sw_read(lane, kh);
          v8bf af[TM], bfr[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const v8bf*>(As + a_off + i * 16 * 128 + pos);
#pragma unroll
          for (int jn = 0; jn < TN; ++jn) bfr[jn] = *reinterpret_cast<const v8bf*>(Bs + b_off + jn * 16 * 128 + pos);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jn = 0; jn < TN; ++jn)
              acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[jn], af[i], acc[i][jn], 0, 0, 0);
        }
      } else {
        op_slot = cur;
      }
      cur = cur + 1 == NB ? 0 : cur + 1;
    }

    // ---------------- epilogue (register direct; operand from the ring slot) ----------------
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * q][jj]),
                                                           __float_as_uint(acc[i][2 * q + 1][jj]), false, false);
          acc[i][2 * q][jj] = __uint_as_float(sw[0]);
          acc[i][2 * q + 1][jj] = __uint_as_float(sw[1]);
        }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int c0 = __float_as_int(acc[i][j][jj]), c1 = __float_as_int(acc[i][2 + j][jj]);
          acc[i][j][jj] = __int_as_float(__builtin_amdgcn_update_dpp(c0, c1, 0x128, 0xf, 0xc, false));
          acc[i][2 + j][jj] = __int_as_float(__builtin_amdgcn_update_dpp(c1, c0, 0x128, 0xf, 0x3, false));
        }
    }
    const int gn = n0 + lc;
    const bool col_ok = gn < p.Nn;
    const char* bits_base = bits_lds + op_slot * BITS_BYTES;
    float sc[8], sh[8];
    if (is_fwd) {
      // from the operand step (no global load whose wait would drain the ring), read as inline
      // asm: the compiler drains the LDS-DMA queue (vmcnt(0)) before a ds_read it cannot tell
      // apart from the four-byte DMA targets
      float4 a, b, c, d;
      const uint32_t sa = (uint32_t)(uintptr_t)LDS_PTR(bits_base + lc * 4);
      asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
                   "ds_read_b128 %2, %4 offset:512\n\tds_read_b128 %3, %4 offset:528\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(sa) : "memory");   // (early clobber: the
                                                                                  // address must survive)
      sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
      sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w; sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
    }
    const __amdgpu_buffer_rsrc_t rout = make_rsrc_at(reinterpret_cast<const uint16_t*>(p.out), (long)m0 * p.ldo,
                                                     (long)p.M * p.ldo);
    const __amdgpu_buffer_rsrc_t rbo =
        __builtin_amdgcn_make_buffer_rsrc(bits_out ? p.bits_out + (long)m0 * p.ld_bits_out : reinterpret_cast<uint8_t*>(p.out),
                                          (short)0, bits_out ? (int)lmin(((long)p.M - m0) * p.ld_bits_out, 0x7fffffffL) : 0,
                                          0x00020000);
    char* op_w = smem + op_slot * STAGE;
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // Every LDS access of the epilogue is inline asm: the compiler cannot tell these addresses
    // from the LDS-DMA targets still in flight and would otherwise drain the ring (vmcnt(0))
    // before the first one.  Chunk k = 2i + h: row wm*64 + 16i + 8h + r8, this lane's 8 columns.
    uint32_t la[2 * TM];
#pragma unroll
    for (int k = 0; k < 2 * TM; ++k) {
      const int row = wm * 64 + 8 * k + r8;
      la[k] = (uint32_t)(uintptr_t)LDS_PTR(op_w + row * 256 + (((lc >> 3) ^ pk_sw(row)) << 4));
    }
    v4u_t ov4[2 * TM];
    uint32_t bytes[2 * TM];
    if (res_on) {
      asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %10\n\tds_read_b128 %3, %11\n\t"
                   "ds_read_b128 %4, %12\n\tds_read_b128 %5, %13\n\tds_read_b128 %6, %14\n\tds_read_b128 %7, %15\n\t"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&v"(ov4[0]), "=&v"(ov4[1]), "=&v"(ov4[2]), "=&v"(ov4[3]), "=&v"(ov4[4]), "=&v"(ov4[5]),
                     "=&v"(ov4[6]), "=&v"(ov4[7])
                   : "v"(la[0]), "v"(la[1]), "v"(la[2]), "v"(la[3]), "v"(la[4]), "v"(la[5]), "v"(la[6]), "v"(la[7])
                   : "memory");
    } else {
#pragma unroll
      for (int k = 0; k < 2 * TM; ++k) ov4[k] = v4u_t{0u, 0u, 0u, 0u};
    }
    if (bits_in) {
      uint32_t ba[2 * TM];
#pragma unroll
      for (int k = 0; k < 2 * TM; ++k)
        ba[k] = (uint32_t)(uintptr_t)LDS_PTR(bits_base + (wm * 64 + 8 * k + r8) * 16 + (lc >> 3));
      asm volatile("ds_read_u8 %0, %8\n\tds_read_u8 %1, %9\n\tds_read_u8 %2, %10\n\tds_read_u8 %3, %11\n\t"
                   "ds_read_u8 %4, %12\n\tds_read_u8 %5, %13\n\tds_read_u8 %6, %14\n\tds_read_u8 %7, %15\n\t"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&v"(bytes[0]), "=&v"(bytes[1]), "=&v"(bytes[2]), "=&v"(bytes[3]), "=&v"(bytes[4]), "=&v"(bytes[5]),
                     "=&v"(bytes[6]), "=&v"(bytes[7])
                   : "v"(ba[0]), "v"(ba[1]), "v"(ba[2]), "v"(ba[3]), "v"(ba[4]), "v"(ba[5]), "v"(ba[6]), "v"(ba[7])
                   : "memory");
    }
    // 1. fused element-wise work in the register layout; each lane writes its result chunk over
    //    the operand chunk it read (same LDS address: no other lane's data is touched)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * i + h;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] = acc[i][2 * h][e]; v[4 + e] = acc[i][2 * h + 1][e]; }
        float ov[8];
        unpack8(make_uint4(ov4[k].x, ov4[k].y, ov4[k].z, ov4[k].w), ov);
        uint4 pk;
        if constexpr (is_fwd) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[e] + sh[e] + ov[e];
          pk = pack8(v);
          if (p.relu) pk = relu_pk8(pk);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += ov[e];
          if (bits_in) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = ((bytes[k] >> e) & 1u) ? v[e] : 0.f;
          }
          pk = pack8(v);
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += v[e];   // (rows / columns outside the problem are zero)
        }
        const v4u_t pkv = {pk.x, pk.y, pk.z, pk.w};
        asm volatile("ds_write_b128 %0, %1" ::"v"(la[k]), "v"(pkv) : "memory");
      }
    // 2. row-contiguous stores of the wave's 64 x 64 region from the slot: 8 consecutive lanes
    //    cover one row's 128 B, so each store instruction writes whole 128 B lines (the register
    //    layout puts consecutive lanes on different rows: 16 B partial-line writes, which the
    //    counters show as a second read + write of the whole output through the fabric)
    uint32_t ra2[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = wm * 64 + it * 8 + (lane >> 3), c = wn * 8 + (lane & 7);
      ra2[it] = (uint32_t)(uintptr_t)LDS_PTR(op_w + row * 256 + ((c ^ pk_sw(row)) << 4));
    }
    v4u_t so[8];
    asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %10\n\tds_read_b128 %3, %11\n\t"
                 "ds_read_b128 %4, %12\n\tds_read_b128 %5, %13\n\tds_read_b128 %6, %14\n\tds_read_b128 %7, %15\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(so[0]), "=&v"(so[1]), "=&v"(so[2]), "=&v"(so[3]), "=&v"(so[4]), "=&v"(so[5]), "=&v"(so[6]),
                   "=&v"(so[7])
                 : "v"(ra2[0]), "v"(ra2[1]), "v"(ra2[2]), "v"(ra2[3]), "v"(ra2[4]), "v"(ra2[5]), "v"(ra2[6]), "v"(ra2[7])
                 : "memory");
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = wm * 64 + it * 8 + (lane >> 3), c = wn * 8 + (lane & 7);
      const int gc = n0 + c * 8;
      const bool ok = m0 + row < p.M && gc < p.Nn;
      __builtin_amdgcn_raw_buffer_store_b128(so[it], rout, ok ? (uint32_t)((row * p.ldo + gc) * 2) : OOB_OFF, 0, 0);
      if (bits_out)
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)pos_bits8(make_uint4(so[it].x, so[it].y, so[it].z, so[it].w)), rbo,
                                             ok ? (uint32_t)(row * p.ld_bits_out + (gc >> 3)) : OOB_OFF, 0, 0);
    }
    if (csum_on) {   // fold the 8 lanes (r8) sharing this lane's columns; lane r8 == 0 stores
#pragma unroll
      for (int o = 1; o < 8; o <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += __shfl_xor(csum[e], o, 64);
      const int prow = p.prow_begin + ((m0 - p.m_begin) / BM) * (BM / 64) + wm;
      const __amdgpu_buffer_rsrc_t rcs = __builtin_amdgcn_make_buffer_rsrc(p.colsum + (long)prow * p.Nn, (short)0,
                                                                           p.Nn * 4, 0x00020000);
      const bool w_ok = r8 == 0 && col_ok;
      typedef float v4fl __attribute__((ext_vector_type(4)));
      const v4fl c0 = {csum[0], csum[1], csum[2], csum[3]}, c1 = {csum[4], csum[5], csum[6], csum[7]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, c0), rcs, w_ok ? (uint32_t)(gn * 4) : OOB_OFF, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, c1), rcs, w_ok ? (uint32_t)(gn * 4 + 16) : OOB_OFF,
                                             0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring's trailing (zero) steps land before exit
}

// Split-K combine: one 4-wave workgroup per 64x64 wave sub-tile (4 per output tile, so a
// small-M layer's few tiles still spread over the chip), each wave owning one 16-column
// fragment group: it sums that group's 4 fragments over the `ksplit` fp32 partial tiles its
// slices left in the workspace (same fragment order: 16-byte vectors of the slices' own
// accumulator registers, four slices' loads in flight) and runs the fused epilogue on its 64 x 16
// columns.  (Round 6: the single-wave form -- one wave pulling all 16 fragments of every slice,
// two slices in flight -- was bound by that one wave's memory-level parallelism: 493 us of the
// 3.75 ms b32 step.  Here no LDS reduction is needed: the fragment groups are disjoint, and the
// fused column sums still land as one partial row per 64-row wave tile.)
// A separate launch instead of an in-launch last-arriver reduction (cdna_hip_programming §5,
// "In-launch split-K reduction"): built and measured in round 6 -- each slice published its
// 64 KiB partial with one agent-scope release and drew a ticket, the tile's last arriver summed
// the slices and ran the epilogue -- the b32 step went from 3.72-3.73 to 4.31 ms: the partials
// are 4-8 x 64 KiB per tile (10x the guide's "few tens of KB"), so one workgroup's serial
// read of them and the per-slice L2 write-back cost far more than the boundary saved.
template <int BM, int BN>
__global__ void __launch_bounds__(256) igemm_splitk_reduce_kernel(IgemmParams p) {
  constexpr int NW = 4, WTM = 64, WTN = 64, TM = 4, TN = 4, WAVES_N = BN / WTN, F = TM * TN;
  constexpr int EPI_LD = 16 + 4;
  __shared__ __attribute__((aligned(16))) float smem[4][32 * EPI_LD];
  const int lane = threadIdx.x & 63;
  const int jw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // this wave's fragment column group
  const int sub = blockIdx.x % NW;
  const int wm = sub / WAVES_N, wn = sub % WAVES_N;
  const int nt = (p.Nn + BN - 1) / BN;
  const int tile = blockIdx.x / NW, tn = tile % nt, tm = tile / nt;
  v4f acc[TM][1];
#pragma unroll
  for (int i = 0; i < TM; ++i) acc[i][0] = v4f{0.f, 0.f, 0.f, 0.f};
  // fragment f = i * TN + jw of slice sl
  const float4* src = reinterpret_cast<const float4*>(p.slab) + ((long)tile * p.ksplit * NW + sub) * F * 64 + jw * 64 + lane;
  const long sstride = (long)NW * F * 64;
  auto add = [&](const float4 (&v)[TM]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      acc[i][0][0] += v[i].x; acc[i][0][1] += v[i].y; acc[i][0][2] += v[i].z; acc[i][0][3] += v[i].w;
    }
  };
  int sl = 0;
  for (; sl + 3 < p.ksplit; sl += 4) {
    float4 v[4][TM];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < TM; ++i) v[u][i] = src[(sl + u) * sstride + i * TN * 64];
#pragma unroll
    for (int u = 0; u < 4; ++u) add(v[u]);
  }
  for (; sl < p.ksplit; ++sl) {
    float4 v[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) v[i] = src[sl * sstride + i * TN * 64];
    add(v);
  }
  igemm_epilogue<TM, 1, false>(p, acc, p.m_begin + tm * BM + wm * WTM, tn * BN + wn * WTN + jw * 16,
                               p.prow_begin + tm * (BM / WTM) + wm, smem[jw], lane);
}

// ---------------------------------------------------------------------------------------
// 8-phase 256x256 implicit GEMM (cdna_hip_programming.md §5 "The 256² 8-phase template",
// T3+T4): 8 waves, one 128 KiB block per CU, BK = 64, two LDS buffers of four 16 KiB
// half-tiles {A rows 0-127, B cols 0-127, B cols 128-255, A rows 128-255} ("parts" 0..3).
//
// Every K-tile is computed in 4 phases, one 128x128 block QUADRANT per phase in snake order
// Q(0,0) Q(0,1) Q(1,1) Q(1,0); all 8 waves work on the phase's quadrant (wave (wm, wn) owns a
// 64x32 sub-tile of every quadrant = 16 MFMAs 16x16x32 per phase), so a phase reads exactly
// one A half and one B half, and the snake reuses the A (or B) fragments of the previous
// phase: 12, 4, 8, 4 ds_read_b128 per phase.
//
// Staging runs LEAD = 5 half-tiles ahead of the phase counter (one half = 2 LDS-DMA pieces
// per wave, issued by every phase), in first-use order (part 0, 1, 2, 3 of K-tile t are first
// read in phases 0, 0, 1, 2 of t).  RAW: before the FIRST barrier of the phase preceding a
// half's first use, each wave waits with a COUNTED vmcnt (2 x halves issued after it: 6 in
// steady state, never 0 inside the loop); the raw s_barrier then publishes every wave's
// pieces.  WAR: a half is restaged >= 1 phase after the phase that last read it (the
// reading phase's lgkmcnt retires its ds_reads before that phase's second barrier).
// STAGGER: the wave row wm = 1 (the second wave on every SIMD) runs one barrier behind, so
// one wave's ds_reads / DMA issue overlap the other's MFMAs; the barrier rules above hold for
// that offset because every wait sits one phase ahead of its first read.
template <int AM, bool STAGGER>
__global__ void __launch_bounds__(512, 1) igemm8_kernel(IgemmParams p) {
  constexpr int BM = 256, BN = 256, HALF = 16384, BUF = 4 * HALF, LEAD = 5;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int mt = (p.M - p.m_begin + BM - 1) / BM, nt = (p.Nn + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, mt * nt);
  const int tn = wg % nt, tm = wg / nt;
  const int m0 = p.m_begin + tm * BM, n0 = tn * BN;
  const int HoWo = p.Ho * p.Wo;
  const int n_first = fdiv(m0, p.mg_howo);   // A descriptors rebased at the tile's first image
  const long HW = (long)p.H * p.W, pix0 = n_first * HW, pix_end = p.N * HW;
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc_at(p.a1, pix0 * p.C1, pix_end * p.C1);
  const int C2r = AM == AM_DUAL ? p.C2 : p.C1;
  // (the second source may have its own geometry: the fused projection shortcut reads the block
  // input at H2 x W2 with stride2 next to conv3's stride-1 operand)
  const long HW2 = AM == AM_DUAL ? (long)p.H2 * p.W2 : HW;
  const __amdgpu_buffer_rsrc_t ra2 =
      make_rsrc_at(AM == AM_DUAL ? p.a2 : p.a1, n_first * HW2 * C2r, p.N * HW2 * C2r);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.b, p.Nn * p.ldb * 2);
  // LDS-DMA piece i of a wave holds rows 8*(piece) + lane/8 (piece parity = i & 1); its lane-linear
  // 16-byte chunk (lane & 7) carries logical chunk (lane & 7) ^ ((row >> 1) & 7) (sw_chunk).

  // Rows this lane stages: A/B half h, piece i (of the wave's 2) -> tile row 128h + (2*wave+i)*8 + lane/8.
  uint32_t a_o1[4], a_o2[4], a_taps[4], b_o[4];
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    const int r = 128 * (hi >> 1) + (2 * wave + (hi & 1)) * 8 + (lane >> 3);
    const int m = m0 + r;
    a_o1[hi] = OOB_OFF; a_o2[hi] = OOB_OFF; a_taps[hi] = 0;
    if (m < p.M) {
      const int n = fdiv(m, p.mg_howo), rem = m - n * HoWo;
      const int ho = fdiv(rem, p.mg_wo), wo = rem - ho * p.Wo;
      const int hi_ = ho * p.stride - p.pad, wi = wo * p.stride - p.pad;
      const int pix = ((n - n_first) * p.H + hi_) * p.W + wi;
      a_o1[hi] = (uint32_t)((pix * p.C1 + sw_chunk(lane, hi) * 8) * 2);
      if (AM == AM_DUAL) {
        const int pix2 = ((n - n_first) * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2;
        a_o2[hi] = (uint32_t)((pix2 * p.C2 + sw_chunk(lane, hi) * 8) * 2);
      }
      if (AM == AM_HALO) a_taps[hi] = halo_taps(p, hi_, wi);
    }
    const int n = n0 + r;
    b_o[hi] = (n < p.Nn) ? (uint32_t)((n * p.ldb + sw_chunk(lane, hi) * 8) * 2) : OOB_OFF;
  }

  // scalar k-walk of the NEXT K-tile to stage (same walk as igemm_kernel)
  int ld_r = 0, ld_s = 0, ld_c0 = 0, ld_src2 = 0, ld_k = 0;
  auto tile_delta = [&]() { return ((ld_r * p.W + ld_s) * (ld_src2 ? p.C2 : p.C1) + ld_c0) * 2; };
  auto advance = [&]() {
    const int C = ld_src2 ? p.C2 : p.C1;
    ld_k += 64;
    ld_c0 += 64;
    if (ld_c0 == C) {
      ld_c0 = 0;
      if (++ld_s == p.S) { ld_s = 0; ++ld_r; }
    }
    if (AM == AM_DUAL && !ld_src2 && ld_k == p.K1) { ld_src2 = 1; ld_r = ld_s = ld_c0 = 0; }
  };
  const int KT = p.K / 64;
  const int NH = 4 * KT;              // half-tiles of the whole K loop
  // stage half-tile j = 4*kt + part (part: 0 A rows 0-127, 1 B cols 0-127, 2 B cols 128-255, 3 A rows 128-255)
  auto stage_half = [&](int j, int part) {
    char* base = smem + ((j >> 2) & 1) * BUF;
    const int delta = tile_delta();
    if (part == 0 || part == 3) {
      const int h = part == 0 ? 0 : 1;
      char* hb = base + (part == 0 ? 0 : 3) * HALF;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        auto dst = LDS_PTR(hb + (2 * wave + i) * 1024);
        const int hi = 2 * h + i;
        if (AM == AM_HALO) {
          const int tap = ld_r * p.S + ld_s;
          const uint32_t off = ((a_taps[hi] >> tap) & 1u) ? a_o1[hi] + (uint32_t)delta : OOB_OFF;
          buf_lds16(ra1, dst, off, 0);
        } else if (AM == AM_DUAL && ld_src2) {
          buf_lds16(ra2, dst, a_o2[hi], delta);
        } else {
          buf_lds16(ra1, dst, a_o1[hi], delta);
        }
      }
    } else {
      const int h = part == 1 ? 0 : 1;
      char* hb = base + part * HALF;
#pragma unroll
      for (int i = 0; i < 2; ++i) buf_lds16(rb, LDS_PTR(hb + (2 * wave + i) * 1024), b_o[2 * h + i], ld_k * 2);
    }
    if (part == 3) advance();
  };
  // counted wait: half `need` complete while the halves issued after it (up to `last`) fly
#define IG8_WAIT_BARRIER(need, last)                                                              \
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

  // prologue: halves 0 .. LEAD-1, then halves 0 and 1 (phase 0's) landed and published
#pragma unroll
  for (int j = 0; j < LEAD; ++j)      // (unrolled: the part selects registers at compile time)
    if (j < NH) stage_half(j, j & 3);
  {
    const int last = (LEAD < NH ? LEAD : NH) - 1;
    IG8_WAIT_BARRIER(1, last)
  }
  if (STAGGER && wm == 1) asm volatile("s_barrier" ::: "memory");

  v8bf af[2][4], bfr[2][2];
  const int a_row = (wm * 64 + (lane & 15)) * 128;
  const int b_row = (wn * 32 + (lane & 15)) * 128;
  int pos[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) pos[kh] = sw_read(lane, kh);

  for (int t = 0; t < KT; ++t) {
    const char* buf = smem + (t & 1) * BUF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qm = (q == 0 || q == 1) ? 0 : 1;
      const int qn = (q == 0 || q == 3) ? 0 : 1;
      const bool loadA = (q == 0 || q == 2), loadB = (q != 2);
      if (loadB) {
        const char* Bs = buf + (qn == 0 ? 1 : 2) * HALF + b_row;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int j = 0; j < 2; ++j) bfr[kh][j] = *reinterpret_cast<const v8bf*>(Bs + j * 16 * 128 + pos[kh]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (loadA) {
        const char* As = buf + (qm == 0 ? 0 : 3) * HALF + a_row;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 4; ++i) af[kh][i] = *reinterpret_cast<const v8bf*>(As + i * 16 * 128 + pos[kh]);
      }
      const int js = 4 * t + q + LEAD;                 // half staged by this phase
      if (js < NH) stage_half(js, (q + LEAD) & 3);
      const int last = (js < NH ? js : NH - 1);
      // wait for the half(s) the NEXT phase reads first: q0 -> part 2 of t; q1 -> part 3 of t;
      // q3 -> parts 0, 1 of t+1; q2 -> none (phase 3 re-reads A1 / B0)
      if (q == 0) IG8_WAIT_BARRIER(4 * t + 2, last)
      else if (q == 1) IG8_WAIT_BARRIER(4 * t + 3, last)
      else if (q == 3 && t + 1 < KT) IG8_WAIT_BARRIER(4 * t + 5, last)
      else asm volatile("s_barrier" ::: "memory");
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
#undef IG8_WAIT_BARRIER
  if (STAGGER && wm == 0) asm volatile("s_barrier" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();   // every wave is done with the LDS tiles before the epilogue stages through them

  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * (32 + 4));
  const int pr = p.prow_begin + tm * 4;
  igemm_epilogue<4, 2, false>(p, acc[0][0], m0 + wm * 64, n0 + wn * 32, pr + wm, stage, lane);
  igemm_epilogue<4, 2, false>(p, acc[0][1], m0 + wm * 64, n0 + 128 + wn * 32, pr + wm, stage, lane);
  igemm_epilogue<4, 2, false>(p, acc[1][0], m0 + 128 + wm * 64, n0 + wn * 32, pr + 2 + wm, stage, lane);
  igemm_epilogue<4, 2, false>(p, acc[1][1], m0 + 128 + wm * 64, n0 + 128 + wn * 32, pr + 2 + wm, stage, lane);
}

int g_igemm_variant = 0;   // 0 = heuristic; 1, 2 = forced pipeline depth (4-wave tiles)
int g_igemm_deep = 2;      // depth the heuristic uses for K >= 256 (3-stage measured slower: removed;
                           // round 6 again for the split-K layers at b32 as a counted-vmcnt 3-stage
                           // tile with asm fragment reads: split slices 3.92-3.95 ms, unsplit
                           // 4.04 ms vs 3.73-3.74 -- its 96 KiB of LDS leaves one block per CU)
int g_igemm_pf = 1;        // epilogue-operand prefetch (PF variant) for 1x1 layers with a residual / add
int g_igemm8 = 2;          // 8-phase 256x256 kernel (igemm8_kernel) for Nn >= 256, K >= 256, Nn < 4K:
                           // 0 off, 1 on, 2 on with the wave-row stagger (default: b1024 end to end
                           // 18.82k -> 19.00k img/s; stagger beats 1 on every layer, kbench)
int g_igemm_ns1_kt = 1000; // single-stage tile for K <= 64 * this (default: every K).  b1024 end to
                           // end 2/4/8/16/36 -> 20.11k/20.42k/20.53k/20.76k/20.87k img/s: three
                           // resident single-buffer blocks per CU overlap each other's load and MFMA
                           // phases better than one block's double buffer does
int g_igemm8_min_n = 512;  // ... and only for GEMM widths Nn >= this (with single-stage 128x128
                           // tiles the 8-phase kernel wins only the stage-5 layers, kbench)
int g_igemm8_min_tiles = 128;   // ... when the problem has at least this many 256x256 tiles
int g_igemm_n64 = 1;       // see igemm_config (1: conv2_block1 c1+c0 fwd 831 -> 765 us; 2: no further gain)

static bool igemm_no_halo(const IgemmParams& p) {
  return p.pad == 0 && (p.Ho - 1) * p.stride + p.R <= p.H && (p.Wo - 1) * p.stride + p.S <= p.W;
}

static bool igemm_check(const IgemmParams& p, const char** why) {
  if (p.K % 64 || p.K1 % 64) { *why = "K must be a multiple of 64"; return false; }
  // A k-tile (64 elements) must be contiguous in memory: C % 64 == 0, or the "window" form
  // S * C == 64 with stride 1 / pad 0 (space-to-depth stem: 4 taps x 16 channels).
  const bool window = (p.C1 * p.S == 64) && p.stride == 1 && p.pad == 0 && !p.a2;
  if ((p.C1 % 64 && !window) || (p.a2 && p.C2 % 64)) { *why = "channels must be multiples of 64"; return false; }
  if (p.a2 && (p.K - p.K1) % 64) { *why = "second source K must be a multiple of 64"; return false; }
  if (p.a2 && !igemm_no_halo(p)) { *why = "two A sources need an unpadded (1x1) gather"; return false; }
  if (!igemm_no_halo(p) && p.R * p.S > 32) { *why = "padded convs support at most 32 taps"; return false; }
  if (p.Nn % 8 || p.ldb % 8 || p.ldo % 8) { *why = "N / ldb / ldo must be multiples of 8"; return false; }
  if (p.M <= 0 || p.Nn <= 0 || p.K <= 0) { *why = "empty problem"; return false; }
  if (p.bn_z && (p.mode != EPI_DGRAD || p.a2 || p.up2 || !p.stats)) {
    *why = "bn_z: fused BN-backward sums need a single-source dgrad without scatter, with stats rows"; return false;
  }
  if ((long)p.M * p.Ho * p.Wo >= (1L << 40)) { *why = "too many output rows for the magic-number row decode"; return false; }
  // buffer offsets are 32-bit byte offsets with 0x80000000 reserved as "out of range"; the A
  // descriptors are rebased per tile, so only the images one 256-row tile spans must fit
  // (and every element index below is an int: < 2^31 elements per tensor)
  const long span = 256 / (p.Ho * p.Wo) + 2, cmax = p.C1 > p.C2 ? p.C1 : p.C2;
  const long hwmax = (long)p.H * p.W > (long)p.H2 * p.W2 ? (long)p.H * p.W : (long)p.H2 * p.W2;
  if (p.a2 && ((p.Ho - 1) * p.stride2 >= p.H2 || (p.Wo - 1) * p.stride2 >= p.W2 || p.stride2 < 1)) {
    *why = "second source geometry does not cover the output rows"; return false;
  }
  if (span * hwmax * cmax * 2 >= (1L << 31) || (long)p.Nn * p.ldb * 2 >= (1L << 31)) {
    *why = "operand too large for 31-bit buffer offsets"; return false;
  }
  if ((long)p.N * hwmax * cmax >= (1L << 31) || (long)p.M * (p.ldo > p.Nn ? p.ldo : p.Nn) >= (1L << 31)) {
    *why = "tensor has more than 2^31 elements"; return false;
  }
  return true;
}

// Tile configuration of a problem: 0 = 256x64 / 4 waves (Nn <= 64), 1 = 128x128 / 4 waves,
// 4 = the 8-phase 256x256 kernel (igemm8_kernel; wide, long-K layers).
static int igemm_config(int M, int Nn, int K) {
  if (Nn <= 64) return 0;
  // A/B knob: 256x64 tiles for widths that are not a multiple of 128 (1: conv2_block1's
  // c1 + shortcut, Nn = 320, whose third 128-column tile is half empty) or for every short-K
  // (K = 64) layer (2)
  if (g_igemm_n64 == 1 && Nn % 128 && Nn % 64 == 0) return 0;
  if (g_igemm_n64 == 2 && K <= 64 && Nn % 64 == 0) return 0;
  // 8-phase 256x256 for wide, long-K GEMMs -- not the expansion 1x1s (Nn >= 4K: conv3 forward,
  // conv1 dgrad), whose short K loop is dominated by an epilogue that streams a residual /
  // residual gradient: measured 30-40% slower there than the 2-block 128x128 tile with the
  // epilogue-operand prefetch (per-layer A/B, profiles/r2_igemm8_per_layer_ab.txt)
  // (widths that are not a multiple of 256 stay on the 128x128 tile: conv3_block1 c1 + shortcut,
  // Nn = 640, measured 680 us on 8-phase tiles vs 588 us on five 128-wide tiles)
  if (g_igemm8 && Nn >= g_igemm8_min_n && K >= 256 && Nn < 4 * K && Nn % 256 == 0 &&
      (long)((M + 255) / 256) * ((Nn + 255) / 256) >= g_igemm8_min_tiles)
    return 4;
  return 1;
}
static int igemm_bm(int cfg) { return cfg == 1 ? 128 : 256; }

// partial column-sum rows of m output rows: one per 64-row wave group (cfg 4: 64-row groups too)
static int igemm_rows_of(int cfg, int m) {
  const int BM = igemm_bm(cfg);
  return ((m + BM - 1) / BM) * (BM / 64);
}

int num_cus() {
  static int cached[64] = {0};   // (per device; a benign race writes the same value)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// Launch plan: rows [0, split) with `cfg`, rows [split, M) with the 128x128 tile.  The 8-phase
// kernel runs one 256x256 block per CU, so its tiles come in rounds of #CUs; a last round
// that fills at most half of the chip is handed to the 4x finer 128x128 tile (2 blocks per
// CU) instead of leaving CUs idle for a whole 256x256 tile time (b1024 stage 4: 784 tiles on
// 256 CUs = 3 full rounds + 16 tiles).
struct IgemmPlan { int cfg, split, ks; };

int g_igemm_splitk = 1;
// Split-K plan knobs (igemm_sk_fill / _cap / _elig): slice workgroups aimed at fill x #CUs, at
// most cap slices, and only problems with elig x tiles <= #CUs (plus the long-K exception).
int g_igemm_sk_fill = 2, g_igemm_sk_cap = 8, g_igemm_sk_elig = 2;
int g_igemm_pk = 2;        // persistent ring kernel (igemm_pk_kernel) for the short-K 1x1 layers:
                           // 0 off, else the ring depth NB (2: two 68 KiB blocks per CU; 3, 4: one
                           // 128 KiB+ block per CU, measured 5-7 % slower end to end)
int g_igemm_pk_all = 0;    // 0: only where it measured faster (dgrads with a residual-gradient add:
                           // -10..-18 % per layer; forwards with a residual and K >= 128: -4..-10 %);
                           // 1: every eligible layer (K = 64 forwards +5 %, no-residual ones +5..8 %)

// Split-K for layers with too few output tiles to fill the chip (small batches, small spatial
// stages: stage 5 at batch 32-256, crop 160): the 4-wave tiles stay resident 2-3 per CU, so a
// problem with at most #CUs / 2 tiles leaves most CUs idle for its whole K loop.  Slices keep
// >= 4 k-tiles each (the LDS pipeline's prologue / epilogue amortised) and at most 8, aiming at
// ~2 x #CUs slice workgroups.
static int igemm_splitk_slices(int M, int Nn, int K, int cfg) {
  if (!g_igemm_splitk || (cfg != 0 && cfg != 1)) return 1;
  const int KT = K / 64;
  const int BM = igemm_bm(cfg), BN = cfg == 0 ? 64 : 128;
  const long T = (long)((M + BM - 1) / BM) * ((Nn + BN - 1) / BN);
  if (g_igemm_splitk >= 2) return KT >= 2 ? (g_igemm_splitk < KT ? g_igemm_splitk : KT) : 1;
  // Split only problems that fill at most half the CUs: measured per layer at b32 / b256-crop160
  // (profiles/r3_splitk_b32_per_layer.txt), 52-98 tiles gain 20-60 us per layer while 196-490
  // tiles LOSE 4-16 us (the slab round trip + the combine launch outweigh the fill gained)
  // Long-K layers (K >= 2048: the stage-4/5 3x3s) also split up to 2 x #CUs tiles: their K loop
  // is long enough that the slab round trip is a few % of the layer (b256 crop 160: the stage-5
  // 3x3 runs 200 tiles = 200 lone 4-wave blocks on 256 CUs at 340 TF/s unsplit).
  const long C = num_cus();
  const long target = (long)g_igemm_sk_fill * C;
  if (KT < 8) return 1;
  if ((long)g_igemm_sk_elig * T > C && !(T < target && KT >= 32)) return 1;
  long ks = (target + T - 1) / T;
  if (ks > KT / 4) ks = KT / 4;
  if (ks > g_igemm_sk_cap) ks = g_igemm_sk_cap;   // (a cap of 4 measured +0.5 %, 2 +7 % on the b32 step, round 6)
  return ks >= 2 ? (int)ks : 1;
}

static IgemmPlan igemm_plan(int M, int Nn, int K, bool bnz = false) {
  IgemmPlan pl{igemm_config(M, Nn, K), M, 1};
  if (bnz) {   // fused BN-backward sums: only the 4-wave single-stage tiles carry that epilogue
    if (pl.cfg != 0) pl.cfg = 1;
    return pl;
  }
  // (the split decision depends on the shape only -- never on the workspace -- so the partial
  // column-sum row count igemm_partial_rows reports always matches the launch)
  {
    const int c = pl.cfg == 4 ? 1 : pl.cfg;
    const int ks = igemm_splitk_slices(M, Nn, K, c);
    if (ks > 1) {
      pl.cfg = c;
      pl.ks = ks;
      return pl;
    }
  }
  if (pl.cfg != 4) return pl;
  const int nt = (Nn + 255) / 256, mt = (M + 255) / 256;
  const long T = (long)mt * nt, C = num_cus();
  const long F = T / C, r = T % C;
  // the tail's 4r 128x128 tiles fit one round (2 per CU) when 2r <= C: it then costs about one
  // 128x128 tile time instead of a whole 256x256 round; a bigger tail runs as a full round
  if (r == 0 || 2 * r > C) return pl;
  if (F == 0) { pl.cfg = 1; return pl; }
  const long full_m_tiles = (F * C) / nt;
  pl.split = (int)lmin((long)M, full_m_tiles * 256);
  return pl;
}

void igemm_plan_query(int M, int Nn, int K, int* cfg, int* split, int* ksplit) {
  const IgemmPlan pl = igemm_plan(M, Nn, K);
  *cfg = pl.cfg;
  *split = pl.split;
  if (ksplit) *ksplit = pl.ks;
}

long igemm_splitk_floats(int M, int Nn, int K) {
  const IgemmPlan pl = igemm_plan(M, Nn, K);
  if (pl.ks <= 1) return 0;
  const int BM = igemm_bm(pl.cfg), BN = pl.cfg == 0 ? 64 : 128;
  return (long)((M + BM - 1) / BM) * ((Nn + BN - 1) / BN) * pl.ks * BM * BN;
}

int igemm_partial_rows(int M, int Nn, int K, bool bnz) {
  const IgemmPlan pl = igemm_plan(M, Nn, K, bnz);
  return igemm_rows_of(pl.cfg, pl.split) + (pl.split < M ? igemm_rows_of(1, M - pl.split) : 0);
}

static void igemm_launch_cfg(const IgemmParams& p, int cfg, hipStream_t stream);

// The dual-source (projection block conv3 + shortcut) forward on the persistent ring: the
// fused c3 + c0 launches of the four projection blocks (K = 128 / 384 / 768 / 1536).  The
// one-block-per-CU 8-phase tiles and the 2-stage 128x128 tiles both serialise each tile's
// 32-128 KiB output store behind its K loop (35-56 % of the measured-bytes bound,
// profiles/r6_roofline_b2560.txt); here the next tile's operands stream in during the
// epilogue.  Ring depth 2 only.
int g_igemm_pk_dual = 2;    // largest K / 64 run on the ring (0: off): K = 128 (conv2_block1) only --
                            // the longer-K blocks ran 3-16 % slower there than on their tiles (ring
                            // fills of 32 KiB per k-step cannot feed the MFMAs from L2: profiles/r6_pk_dual.txt)
static bool igemm_pk_dual_launch(const IgemmParams& p, hipStream_t stream) {
  const int KT = p.K / 64;
  if (!g_igemm_pk_dual || KT > g_igemm_pk_dual || g_igemm_pk != 2) return false;
  if (p.mode != EPI_FWD || !p.scale || !p.shift || p.res || p.up2 || p.out2 || p.stats || p.bn_z) return false;
  if (p.R != 1 || p.S != 1 || p.pad != 0 || p.C1 != p.K1 || p.C2 != p.K - p.K1 || !igemm_no_halo(p)) return false;
  if (p.Nn % 32) return false;
  const long T = (long)((p.M - p.m_begin + 127) / 128) * ((p.Nn + 127) / 128);
  long G = (long)num_cus() * 2;
  if (G > T) G = T;
#define PKD_GO(KT_) hipLaunchKernelGGL((igemm_pk_kernel<KT_, 2, true, true, true>), dim3((unsigned)G), dim3(256), 0, stream, p)
  if (KT == 2) PKD_GO(2);
  else if (KT == 6) PKD_GO(6);
  else if (KT == 12) PKD_GO(12);
  else if (KT == 24) PKD_GO(24);
  else return false;
#undef PKD_GO
  return true;
}

// The persistent ring kernel for a short-K 1x1 problem (false: not eligible, nothing launched).
static bool igemm_pk_launch(const IgemmParams& p, hipStream_t stream) {
  const int KT = p.K / 64;
  if (p.a2) return igemm_pk_dual_launch(p, stream);
  if (p.R != 1 || p.S != 1 || p.pad != 0 || p.C1 != p.K || !igemm_no_halo(p)) return false;
  if (KT != 1 && KT != 2 && KT != 4 && KT != 8) return false;
  if (p.mode != EPI_FWD && p.mode != EPI_DGRAD) return false;
  if (p.up2 || p.out2 || p.stats || p.bn_z || p.mask || p.Nn % 32) return false;
  if (p.mode == EPI_FWD && (!p.scale || !p.shift)) return false;
  const bool ops = p.mode == EPI_FWD || p.add || p.bits_mask;
  if (!ops) return false;   // (the epilogue stages its stores through the operand step's slot)
  if (!g_igemm_pk_all && !((p.mode == EPI_DGRAD && p.add) || (p.mode == EPI_FWD && p.res && KT >= 2))) return false;
  const long T = (long)((p.M - p.m_begin + 127) / 128) * ((p.Nn + 127) / 128);
  const int nb = g_igemm_pk;
  long G = (long)num_cus() * (nb == 2 ? 2 : 1);
  if (G > T) G = T;
#define PK_GO(KT_, NB_)                                                                                      \
  {                                                                                                          \
    if (p.mode == EPI_FWD) hipLaunchKernelGGL((igemm_pk_kernel<KT_, NB_, true, true>), dim3((unsigned)G), dim3(256), 0, stream, p); \
    else hipLaunchKernelGGL((igemm_pk_kernel<KT_, NB_, true, false>), dim3((unsigned)G), dim3(256), 0, stream, p); \
  }
#define PK_NB(KT_)                          \
  {                                         \
    if (nb == 2) PK_GO(KT_, 2)              \
    else if (nb == 3) PK_GO(KT_, 3)         \
    else PK_GO(KT_, 4)                      \
  }
  if (KT == 1) PK_NB(1) else if (KT == 2) PK_NB(2) else if (KT == 4) PK_NB(4) else PK_NB(8)
#undef PK_NB
#undef PK_GO
  return true;
}

const char* igemm_launch(const IgemmParams& p_in, hipStream_t stream) {
  const char* why = nullptr;
  if (!igemm_check(p_in, &why)) return why;
  IgemmParams p = p_in;
  p.mg_howo = fdiv_magic(p.Ho * p.Wo);
  p.mg_wo = fdiv_magic(p.Wo);
  p.m_begin = 0;
  p.prow_begin = 0;
  p.ksplit = 1;
  const IgemmPlan pl = igemm_plan(p.M, p.Nn, p.K, p.bn_z != nullptr);
  // (a forward dual-source problem goes to the ring whatever tile the plan picked: it has no
  // column sums, so the partial-row layout of the plan does not apply)
  if (g_igemm_pk && pl.ks == 1 && ((pl.split >= p.M && pl.cfg == 1) || p.a2) && igemm_pk_launch(p, stream)) {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? nullptr : hipGetErrorString(e);
  }
  const bool window = (p.C1 * p.S == 64) && p.C1 < 64;
  if (pl.ks > 1 && !p.a2 && !window && p.C1 % 64 == 0 && p.slab && !(p.mode == EPI_FWD && p.up2) &&
      p.slab_floats >= igemm_splitk_floats(p.M, p.Nn, p.K)) {
    // slices -> workspace, then the combine + fused epilogue (without a workspace the same
    // tile config runs unsplit, so the partial-row layout does not change)
    p.ksplit = pl.ks;
    const int BM = igemm_bm(pl.cfg), BN = pl.cfg == 0 ? 64 : 128;
    const int tiles = ((p.M + BM - 1) / BM) * ((p.Nn + BN - 1) / BN);
    igemm_launch_cfg(p, pl.cfg, stream);
    if (pl.cfg == 0) hipLaunchKernelGGL((igemm_splitk_reduce_kernel<256, 64>), dim3(tiles * 4), dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((igemm_splitk_reduce_kernel<128, 128>), dim3(tiles * 4), dim3(256), 0, stream, p);
  } else if (pl.split < p.M) {
    IgemmParams head = p, tail = p;
    head.M = pl.split;
    tail.m_begin = pl.split;
    tail.prow_begin = igemm_rows_of(pl.cfg, pl.split);
    igemm_launch_cfg(head, pl.cfg, stream);
    igemm_launch_cfg(tail, 1, stream);
  } else {
    igemm_launch_cfg(p, pl.cfg, stream);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

static void igemm_launch_cfg(const IgemmParams& p, int cfg, hipStream_t stream) {
  // Pipeline depth by K: short K (<= 2 k-tiles) is memory-bound -> single LDS stage for
  // twice the resident blocks (variant knob for A/B timing: 0 = heuristic, 1/2 = forced).
  const int KT = p.K / 64;
  int ns = g_igemm_variant;
  if (ns == 0) ns = KT <= g_igemm_ns1_kt ? 1 : 2;
  const int am = p.a2 ? AM_DUAL : (igemm_no_halo(p) ? AM_DIRECT : AM_HALO);
  // (explicit launches per instantiation: taking kernel addresses through a conditional
  // expression leaves the host stubs uninstantiated with this compiler)
#define IG_GO(BM_, BN_, NS_, AM_) \
  hipLaunchKernelGGL((igemm_kernel<BM_, BN_, NS_, AM_>), dim3(nwg), dim3(256), 0, stream, p)
#define IG_MODES(BM_, BN_, NS_)                                 \
  {                                                             \
    if (am == AM_DIRECT) IG_GO(BM_, BN_, NS_, AM_DIRECT);       \
    else if (am == AM_HALO) IG_GO(BM_, BN_, NS_, AM_HALO);      \
    else IG_GO(BM_, BN_, NS_, AM_DUAL);                         \
  }
  const int BM = igemm_bm(cfg), BN = cfg == 0 ? 64 : (cfg == 4 ? 256 : 128);
  const int nwg = ((p.M - p.m_begin + BM - 1) / BM) * ((p.Nn + BN - 1) / BN) * (p.ksplit > 1 ? p.ksplit : 1);
  // PF where the prefetched operand exists for every element (forward residual; dgrad
  // residual-gradient without the stride-2 scatter).  Measured (bench/epilogue.py, b1024,
  // profiles/r1_epilogue_prefetch_ab.json): forward +3-20% on every stage; dgrad +10-14% for
  // K >= 256 but -8-10% for the single-stage K <= 128 tiles, whose occupancy the 24 extra
  // VGPRs cut from 3 to 2 waves per SIMD -- so dgrad uses it only on 2-stage tiles.
  if (p.ksplit > 1) {   // split-K slices (cfg 0 / 1, single source; igemm_launch)
#define IG_SK(BM_, BN_, NS_, AM_) \
  hipLaunchKernelGGL((igemm_kernel<BM_, BN_, NS_, AM_, false, false, true>), dim3(nwg), dim3(256), 0, stream, p)
    if (cfg == 1) {
      if (ns == 1) { if (am == AM_DIRECT) IG_SK(128, 128, 1, AM_DIRECT); else IG_SK(128, 128, 1, AM_HALO); }
      else { if (am == AM_DIRECT) IG_SK(128, 128, 2, AM_DIRECT); else IG_SK(128, 128, 2, AM_HALO); }
    } else {
      if (ns == 1) { if (am == AM_DIRECT) IG_SK(256, 64, 1, AM_DIRECT); else IG_SK(256, 64, 1, AM_HALO); }
      else { if (am == AM_DIRECT) IG_SK(256, 64, 2, AM_DIRECT); else IG_SK(256, 64, 2, AM_HALO); }
    }
#undef IG_SK
    return;
  }
  const bool pf = g_igemm_pf && am == AM_DIRECT && cfg <= 1 &&
                  ((p.mode == EPI_FWD && p.res) || (p.mode == EPI_DGRAD && p.add && !p.up2 && (ns == 2 || g_igemm_pf == 2)));
  if (p.bn_z) {   // (igemm_check: DGRAD, no dual source; plan: cfg 0 / 1)
#define IG_Z(BM_, BN_, AM_) \
  hipLaunchKernelGGL((igemm_kernel<BM_, BN_, 1, AM_, false, true>), dim3(nwg), dim3(256), 0, stream, p)
    if (cfg == 0) {
      if (am == AM_DIRECT) IG_Z(256, 64, AM_DIRECT); else IG_Z(256, 64, AM_HALO);
    } else {
      if (am == AM_DIRECT) IG_Z(128, 128, AM_DIRECT); else IG_Z(128, 128, AM_HALO);
    }
#undef IG_Z
  } else if (cfg == 4) {
#define IG_8(AM_)                                                                                         \
  {                                                                                                       \
    if (g_igemm8 == 2) hipLaunchKernelGGL((igemm8_kernel<AM_, true>), dim3(nwg), dim3(512), 0, stream, p); \
    else hipLaunchKernelGGL((igemm8_kernel<AM_, false>), dim3(nwg), dim3(512), 0, stream, p);             \
  }
    if (am == AM_DIRECT) IG_8(AM_DIRECT)
    else if (am == AM_HALO) IG_8(AM_HALO)
    else IG_8(AM_DUAL)
#undef IG_8
  } else if (pf) {
#define IG_PF(BM_, BN_, NS_) \
  hipLaunchKernelGGL((igemm_kernel<BM_, BN_, NS_, AM_DIRECT, true>), dim3(nwg), dim3(256), 0, stream, p)
    if (cfg == 1) {
      if (ns == 1) IG_PF(128, 128, 1); else IG_PF(128, 128, 2);
    } else {
      if (ns == 1) IG_PF(256, 64, 1); else IG_PF(256, 64, 2);
    }
#undef IG_PF
  } else if (cfg == 1) {
    if (ns == 1) IG_MODES(128, 128, 1) else IG_MODES(128, 128, 2)
  } else {
    if (ns == 1) IG_MODES(256, 64, 1) else IG_MODES(256, 64, 2)
  }
#undef IG_MODES
#undef IG_GO
}

}  // namespace pddl
