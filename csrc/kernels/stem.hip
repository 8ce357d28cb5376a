// Fused stem forward (gfx950): conv1 (7x7/s2 as the 4x4/s1 space-to-depth window GEMM, K = 256)
// + frozen BN + ReLU + ZeroPadding2D(1) + MaxPooling2D(3, 2), in one launch.  The conv output
// (N x 112 x 112 x 64 bf16 at crop 224: 1.6 MB per image) never reaches HBM: the workgroup keeps
// the conv rows a pool row needs in LDS and writes only the pool output, its argmax taps and its
// ReLU bits -- what the backward uses (the max-pool backward routes by the argmax tap, and
// conv2_block1's dgrad masks with the pool output's bits).  Reference: the Keras ResNet50 stem
// behind imagenet-resnet50.py:56.
//
// Workgroup = (image, block of PB pool rows), 256 threads (4 waves), two workgroups per CU.
// Per pool row p: conv rows 2p and 2p+1 (and 2p-1 for the block's first row) are computed as
// 16-pixel x 64-channel MFMA tiles (v_mfma_f32_16x16x32_bf16 with the weights as the A operand,
// held in registers for the whole launch, and the im2col pixels as the B operand, read from a
// ring of eight space-to-depth input rows in LDS: 16 B per lane = 8 channels of one tap, rows of
// a 16-pixel tile are consecutive pixels, conflict-free); the epilogue (scale / shift / ReLU /
// bf16, exactly the igemm forward epilogue's expression) writes 4 channels x 1 pixel per lane
// into a 3-row conv buffer (8-byte chunks XOR-swizzled by the pixel column so the stores and the
// 16-byte pool reads are conflict-free; index 0 of a row is a zero pixel).  After a barrier the
// workgroup pools row p (first maximum in scan order, padding taps are zeros, as
// maxpool_fwd_kernel) while the next rows' input is already in flight (global loads issued
// before the MFMA phase, written to the ring after it).
// (Round 6 also measured a one-workgroup-per-CU form with the roles split over the waves -- four
// waves computing conv rows beside four pooling the previous row, input rows loaded four rows
// ahead -- at 1.77 ms against 1.68 ms for this one at b2560: with one wave per SIMD per role both
// roles were latency-bound.)
#include "common.h"
#include "kernels.h"

namespace pddl {

namespace {

constexpr int SP_THREADS = 256;

__device__ __forceinline__ uint32_t swz_chunk(int chunk, int x) { return (uint32_t)(chunk ^ (x & 14)); }

}  // namespace

template <bool BITS>
__global__ void __launch_bounds__(SP_THREADS, 2) stem_pool_fwd_kernel(StemPoolParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int SLOT = p.Ws * 32;
  // conv row buffer: pixel x at index x + 1, index 0 a zero pixel (the pool's left padding tap
  // reads it like any other: no per-tap bounds selects)
  const int CROW = (p.W1 + 1) * 128;
  uint8_t* ring = lds;
  uint8_t* cbuf = lds + 8 * SLOT;
  const int b = blockIdx.x / p.nblk;
  const int blk = blockIdx.x - b * p.nblk;
  const int P0 = blk * p.PB;
  const int P1 = min(P0 + p.PB, p.H2);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // (uniform: the tile walk in SGPRs)
  const int lr = lane & 15, lg = lane >> 4;

  // ---- weights as A fragments: co = 16 nt + lr, k = 32 t + 8 lg + j (held for the whole launch)
  // wave w owns output channels [32 (w & 1), + 32) of every tile and tiles w >> 1, +2, ...: 7 tiles
  // per wave per pool row with half the weight registers (the round-4 first form, whole tiles per
  // wave, ran 2.14 ms against 1.88 ms at b2560: profiles/r4_fused_stem_ab.txt)
  constexpr int NTW = 2;
  const int nt0 = 2 * (wave & 1);
  v8bf wa[NTW][8];
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
    for (int t = 0; t < 8; ++t)
      wa[nt][t] = *reinterpret_cast<const v8bf*>(p.w + (16 * (nt0 + nt) + lr) * 256 + 32 * t + 8 * lg);
  // folded BN (scale | shift of the 64 output channels) in LDS: read per epilogue, so the
  // weight fragments keep the register file
  float* bn = reinterpret_cast<float*>(cbuf + 3 * CROW);
  if (tid < 128) bn[tid] = tid < 64 ? p.scale[tid] : p.shift[tid - 64];
  if (tid < 24) *reinterpret_cast<uint4*>(cbuf + (tid >> 3) * CROW + (tid & 7) * 16) = make_uint4(0, 0, 0, 0);

  const uint4* x2b = reinterpret_cast<const uint4*>(p.x2 + (long)b * p.Hs * p.Ws * 16);
  const int RCH = p.Ws * 2;   // 16-byte chunks per input row

  // ---- initial ring fill: input rows [2 P0 - 1, 2 P0 + 5) (the first pool row's conv rows
  //      2 P0 - 1 .. 2 P0 + 1 read input rows up to 2 P0 + 4)
  for (int yy = max(2 * P0 - 1, 0); yy < min(2 * P0 + 5, p.Hs); ++yy) {
    uint4* dst = reinterpret_cast<uint4*>(ring + (yy & 7) * SLOT);
    for (int c = tid; c < RCH; c += SP_THREADS) dst[c] = x2b[(long)yy * RCH + c];
  }
  // wait for the weights here (an empty asm reading them): left pending into the row loop, the
  // compiler's in-order vmcnt waits before their MFMAs also wait for every pool row's prefetch
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
    for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(wa[nt][t]));
  __syncthreads();
  float bsc[NTW][4], bsh[NTW][4];   // this lane's folded BN: channels 16 (nt0 + ntl) + 4 lg + i
#pragma unroll
  for (int ntl = 0; ntl < NTW; ++ntl) {
    const float4 a = *reinterpret_cast<const float4*>(bn + 16 * (nt0 + ntl) + 4 * lg);
    const float4 c = *reinterpret_cast<const float4*>(bn + 64 + 16 * (nt0 + ntl) + 4 * lg);
    bsc[ntl][0] = a.x; bsc[ntl][1] = a.y; bsc[ntl][2] = a.z; bsc[ntl][3] = a.w;
    bsh[ntl][0] = c.x; bsh[ntl][1] = c.y; bsh[ntl][2] = c.z; bsh[ntl][3] = c.w;
  }

  const int nct = (p.W1 + 15) >> 4;
  for (int pr = P0; pr < P1; ++pr) {
    // ---- prefetch the two input rows the next pool row adds (2 pr + 5, 2 pr + 6)
    constexpr int PFN = 2;   // 2 rows x RCH chunks <= 2 x 256 for Ws <= 128 (checked by the launcher)
    uint4 pf[PFN];
    const bool more = pr + 1 < P1;
#pragma unroll
    for (int k = 0; k < PFN; ++k) {
      const int c = tid + k * SP_THREADS;
      const int yy = 2 * pr + 5 + (c >= RCH ? 1 : 0), cc = c >= RCH ? c - RCH : c;
      pf[k] = make_uint4(0, 0, 0, 0);
      if (more && c < 2 * RCH && yy < p.Hs) pf[k] = x2b[(long)yy * RCH + cc];
    }
    // ---- conv rows of this iteration: 2pr, 2pr+1 (and 2pr-1 on the block's first pool row)
    const int ylo = (pr == P0 && pr > 0) ? 2 * pr - 1 : 2 * pr;
    const int nrows = 2 * pr + 2 - ylo;
    const int ntiles = nrows * nct;
    for (int ti = wave >> 1; ti < ntiles; ti += 2) {
      const int y = ylo + ti / nct, x0 = (ti % nct) * 16;
      v4f acc[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) acc[nt] = (v4f){0.f, 0.f, 0.f, 0.f};
      const int xl = x0 + lr;   // this lane's pixel (B-operand column)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        // k = 32 t + 8 lg + j: tap (R, S) = (t >> 1, 2 (t & 1) + (lg >> 1)), channels 8 (lg & 1) + j
        const int R = t >> 1, S = 2 * (t & 1) + (lg >> 1);
        const uint8_t* src = ring + ((y + R) & 7) * SLOT + (xl + S) * 32 + (lg & 1) * 16;
        const v8bf bx = *reinterpret_cast<const v8bf*>(src);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nt][t], bx, acc[nt], 0, 0, 0);
      }
      // epilogue: lane holds D[co = 16 nt + 4 lg + i][px = lr]
      if (xl < p.W1) {
        uint8_t* crow = cbuf + (y % 3) * CROW + (xl + 1) * 128;
#pragma unroll
        for (int ntl = 0; ntl < NTW; ++ntl) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[ntl][i] * bsc[ntl][i] + bsh[ntl][i];
          const uint2 pk = make_uint2(relu_pk2(pack2(v[0], v[1])), relu_pk2(pack2(v[2], v[3])));
          *reinterpret_cast<uint2*>(crow + swz_chunk(4 * (nt0 + ntl) + lg, xl + 1) * 8) = pk;
        }
      }
    }
    // ---- the prefetched rows into their ring slots (rows this iteration no longer reads)
    if (more) {
#pragma unroll
      for (int k = 0; k < PFN; ++k) {
        const int c = tid + k * SP_THREADS;
        if (c < 2 * RCH) {
          const int yy = 2 * pr + 5 + (c >= RCH ? 1 : 0), cc = c >= RCH ? c - RCH : c;
          if (yy < p.Hs) reinterpret_cast<uint4*>(ring + (yy & 7) * SLOT)[cc] = pf[k];
        }
      }
    }
    __syncthreads();
    // ---- pool row pr: window rows 2pr-1 .. 2pr+1, columns 2q-1 .. 2q+1; item = (q, 8-channel group)
    const long orow = ((long)b * p.H2 + pr) * p.W2;
    // branch-free: the conv rows are ReLU outputs (relu_pk2 leaves no sign bit, -0 included),
    // so bf16 bit patterns order like unsigned integers; key = bits << 16 | (15 - tap), one byte
    // permute per element, and one unsigned max per tap keeps the largest value and, among equal
    // values, the first tap in scan order -- the float compare's winner.  Every key starts as a
    // zero at tap 0 (15): a padding tap (zero) never beats it, so the top padding row is skipped
    // (uniform branch) and the left one reads the zero pixel at index 0.  (Round 5 built the keys
    // with shifts / masks and bounds-selected every tap: 280 VALU per item, 150 now.)
    const int rs0 = pr > 0 ? ((2 * pr - 1) % 3) * CROW : 0, rs1 = ((2 * pr) % 3) * CROW, rs2 = ((2 * pr + 1) % 3) * CROW;
    for (int it = tid; it < p.W2 * 8; it += SP_THREADS) {
      const int q = it >> 3, cg = it & 7;
      uint32_t key[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) key[e] = 15u;   // (tap 0 of a zero)
      auto tap_row = [&](int roff, uint32_t cbase) __attribute__((always_inline)) {   // window row r: cbase = 15 - 3 r
#pragma unroll
        for (int sx = 0; sx < 3; ++sx) {
          const int xi = 2 * q + sx;                   // buffer index of conv pixel 2q - 1 + sx
          const uint4 u = *reinterpret_cast<const uint4*>(cbuf + roff + xi * 128 + swz_chunk(2 * cg, xi) * 8);
          const uint32_t c = cbase - (uint32_t)sx;
          const uint32_t d[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            key[2 * h] = max(key[2 * h], __builtin_amdgcn_perm(d[h], c, 0x05040100u));       // lo << 16 | c
            key[2 * h + 1] = max(key[2 * h + 1], __builtin_amdgcn_perm(d[h], c, 0x07060100u));   // hi | c
          }
        }
      };
      if (pr > 0) tap_row(rs0, 15u);
      tap_row(rs1, 12u);
      tap_row(rs2, 9u);
      const long o = (orow + q) * 64 + cg * 8;
      const uint4 yv = make_uint4((key[0] >> 16) | (key[1] & 0xffff0000u), (key[2] >> 16) | (key[3] & 0xffff0000u),
                                  (key[4] >> 16) | (key[5] & 0xffff0000u), (key[6] >> 16) | (key[7] & 0xffff0000u));
      *reinterpret_cast<uint4*>(p.pool + o) = yv;
      if (BITS) p.bits[o >> 3] = (uint8_t)pos_bits8(yv);
      uint32_t cd[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) cd[e] = 15u - (key[e] & 15u);
      *reinterpret_cast<uint2*>(p.idx + o) =
          make_uint2(cd[0] | (cd[1] << 8) | (cd[2] << 16) | (cd[3] << 24), cd[4] | (cd[5] << 8) | (cd[6] << 16) | (cd[7] << 24));
    }
    __syncthreads();   // the next rows' epilogue overwrites conv rows 2pr-1 / 2pr
  }
}

// ------------------------------------------------------------------------------------------
// Fused stem backward: max-pool backward (route each pool-output gradient to its argmax tap) +
// conv1 weight gradient dW2[co][k] = sum_px gc1[px][co] * im2col(x2)[px][k] (s2d domain, K = 256)
// + the stem's per-channel gradient sums, in one launch.  conv1's output gradient gc1 (4.1 GB at
// b2560) never reaches HBM: per conv row pair (2p, 2p+1) -- fed by pool rows p (taps r = 1, 2)
// and p+1 (tap r = 0), so pool-row blocks partition the conv rows with no halo -- the workgroup
// routes the pool gradient into an LDS image [2 rows][128 px][64 ch] (16-byte chunks XOR-swizzled
// by the pixel), then runs the weight-gradient MFMAs with BOTH operands read back transposed by
// ds_read_b64_tr_b16 (the reduction runs over pixels): A = gc1^T (co x px) from that image, B =
// the im2col pixels from the ring of space-to-depth input rows.  Each wave owns 4 taps (64 of the
// 256 k columns) x all 64 output channels in registers for the whole launch and adds them once at
// the end with row-contiguous fp32 atomics.  Padding pixels of a 32-pixel step carry zero
// gradient and read a clamped (finite) input pixel.
// (the builtin, not inline asm: with asm the compiler may schedule an MFMA that consumes the
// result before a hand-placed s_waitcnt lgkmcnt)
__device__ __forceinline__ v4bf sp_tr_read(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(p));
}
// gc1 image: pixel x of row a at a * 128 * 128 + x * 128; its 8-channel chunk c at (c ^ swz(x)) * 16
__device__ __forceinline__ int gimg_off(int a, int x, int chunk) {
  return a * 16384 + x * 128 + ((chunk ^ (x & 7) ^ ((x >> 3) & 1) * 4) << 4);
}

__global__ void __launch_bounds__(SP_THREADS, 2) stem_pool_bwd_kernel(StemPoolBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int SLOT = p.Ws * 32;
  uint8_t* ring = lds;
  uint8_t* gimg = lds + 8 * SLOT;                              // 2 x 128 px x 128 B
  float* csum = reinterpret_cast<float*>(gimg + 2 * 16384);   // [4 waves][64]
  const int b = blockIdx.x / p.nblk;
  const int blk = blockIdx.x - b * p.nblk;
  const int P0 = blk * p.PB;
  const int P1 = min(P0 + p.PB, p.H2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int W1 = p.W1;
  const int nst = (W1 + 31) >> 5;                              // 32-pixel steps per conv row

  // zero the image's padding pixels [W1, 32 nst) once (never written by the router)
  for (int i = tid; i < 2 * (32 * nst - W1) * 8; i += SP_THREADS) {
    const int a = i / ((32 * nst - W1) * 8), r = i - a * (32 * nst - W1) * 8;
    const int x = W1 + (r >> 3), c = r & 7;
    *reinterpret_cast<uint4*>(gimg + gimg_off(a, x, c)) = make_uint4(0, 0, 0, 0);
  }
  const uint4* x2b = reinterpret_cast<const uint4*>(p.x2 + (long)b * p.Hs * p.Ws * 16);
  const int RCH = p.Ws * 2;
  for (int yy = 2 * P0; yy < min(2 * P0 + 5, p.Hs); ++yy) {
    uint4* dst = reinterpret_cast<uint4*>(ring + (yy & 7) * SLOT);
    for (int c = tid; c < RCH; c += SP_THREADS) dst[c] = x2b[(long)yy * RCH + c];
  }

  v4f acc[4][4];   // [co16 tile][tap of this wave]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = (v4f){0.f, 0.f, 0.f, 0.f};
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // ds_read_b64_tr_b16: lane 4 q + pp of each 16-lane group addresses block row q, columns 4 pp .. +3
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const long gbase = (long)b * p.H2 * p.W2;
  const int Wq = W1 / 2;   // conv column pairs (= W2)
  // The router's operands (pool gradient + argmax taps of pool rows rp, rp + 1 at the item's two
  // column pairs) are loaded one row pair AHEAD, during the previous row pair's MFMAs: loaded at
  // the top of the router, every row pair paid a dependent HBM round trip before any MFMA.
  // Raw values only (clamped, always-valid addresses); the bounds masks are applied at use, so
  // no select makes the compiler wait for a load early.  Items it = tid + 256 k, k < RI.
  constexpr int RI = 2;   // (W2 * 8 <= 512 items: checked by the launcher)
  uint4 rgv[RI][2][2];
  uint2 riv[RI][2][2];
  auto router_load = [&](int rp) {
#pragma unroll
    for (int k = 0; k < RI; ++k) {
      const int it = tid + k * SP_THREADS;
      const int qq = min(it >> 3, Wq - 1), cg = it & 7;
#pragma unroll
      for (int dr = 0; dr < 2; ++dr)
#pragma unroll
        for (int dc = 0; dc < 2; ++dc) {
          const int pr = min(rp + dr, p.H2 - 1), pc = min(qq + dc, p.W2 - 1);
          const long o = (gbase + (long)pr * p.W2 + pc) * 64 + cg * 8;
          rgv[k][dr][dc] = *reinterpret_cast<const uint4*>(p.gpool + o);
          riv[k][dr][dc] = *reinterpret_cast<const uint2*>(p.idx + o);
        }
    }
  };
  router_load(P0);
  __syncthreads();

  for (int rp = P0; rp < P1; ++rp) {
    // ---- prefetch the input rows the next row pair adds (2 rp + 5, 2 rp + 6)
    constexpr int PFN = 2;
    uint4 pf[PFN];
    const bool more = rp + 1 < P1;
#pragma unroll
    for (int k = 0; k < PFN; ++k) {
      const int c = tid + k * SP_THREADS;
      const int yy = 2 * rp + 5 + (c >= RCH ? 1 : 0), cc = c >= RCH ? c - RCH : c;
      pf[k] = make_uint4(0, 0, 0, 0);
      if (more && c < 2 * RCH && yy < p.Hs) pf[k] = x2b[(long)yy * RCH + cc];
    }
    // ---- route pool rows rp (taps r = 1, 2) and rp + 1 (tap r = 0) into conv rows 2rp, 2rp+1:
    //      item = (column pair qq, 8-channel group cg), as maxpool_bwd_stream_kernel
#pragma unroll
    for (int k = 0; k < RI; ++k) {
      const int it = tid + k * SP_THREADS;
      if (it >= Wq * 8) continue;
      const int qq = it >> 3, cg = it & 7;
      uint4 gv[2][2];
      uint2 iv[2][2];
#pragma unroll
      for (int dr = 0; dr < 2; ++dr)
#pragma unroll
        for (int dc = 0; dc < 2; ++dc) {
          const bool ok = rp + dr < p.H2 && qq + dc < p.W2;
          gv[dr][dc] = ok ? rgv[k][dr][dc] : make_uint4(0, 0, 0, 0);
          iv[dr][dc] = ok ? riv[k][dr][dc] : make_uint2(0xffffffffu, 0xffffffffu);
        }
      float ga[8], gb[8], gc[8], gd[8];
      unpack8(gv[0][0], ga); unpack8(gv[0][1], gb); unpack8(gv[1][0], gc); unpack8(gv[1][1], gd);
      auto tap = [](const uint2& v, int e) { return ((e < 4 ? v.x : v.y) >> (8 * (e & 3))) & 0xffu; };
      float o4[2][2][8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t ta = tap(iv[0][0], e), tb = tap(iv[0][1], e), tc = tap(iv[1][0], e), td = tap(iv[1][1], e);
        o4[0][0][e] = ta == 4u ? ga[e] : 0.f;
        o4[0][1][e] = (ta == 5u ? ga[e] : 0.f) + (tb == 3u ? gb[e] : 0.f);
        o4[1][0][e] = (ta == 7u ? ga[e] : 0.f) + (tc == 1u ? gc[e] : 0.f);
        o4[1][1][e] = (ta == 8u ? ga[e] : 0.f) + (tb == 6u ? gb[e] : 0.f) + (tc == 2u ? gc[e] : 0.f) +
                      (td == 0u ? gd[e] : 0.f);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += o4[a][c][e];   // (fp32, as maxpool_bwd's fused sums)
          *reinterpret_cast<uint4*>(gimg + gimg_off(a, 2 * qq + c, cg)) = pack8(o4[a][c]);
        }
    }
    if (more) {
#pragma unroll
      for (int k = 0; k < PFN; ++k) {
        const int c = tid + k * SP_THREADS;
        if (c < 2 * RCH) {
          const int yy = 2 * rp + 5 + (c >= RCH ? 1 : 0), cc = c >= RCH ? c - RCH : c;
          if (yy < p.Hs) reinterpret_cast<uint4*>(ring + (yy & 7) * SLOT)[cc] = pf[k];
        }
      }
    }
    __syncthreads();
    if (more) router_load(rp + 1);   // (lands during this row pair's MFMAs)
    // ---- weight-gradient MFMAs over the row pair: 2 rows x nst steps of 32 pixels
    for (int a = 0; a < 2; ++a) {
      const int y = 2 * rp + a;
      for (int st = 0; st < nst; ++st) {
        const int x0 = 32 * st;
        v8bf af[4], bfr[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int px = x0 + 8 * g + 4 * h + q;   // this lane's block row (pixel)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            // A block: pixels px0..px0+3 x channels 16 i + 4 pp .. +3 -> chunk 2 i + (pp >> 1), half pp & 1
            const v4bf r = sp_tr_read(gimg + gimg_off(a, px, 2 * i + (pp >> 1)) + (pp & 1) * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) af[i][4 * h + j] = r[j];
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int T = 4 * wave + t, R = T >> 2, S = T & 3;
            const int xs = min(px + S, p.Ws - 1);
            const v4bf r = sp_tr_read(ring + ((y + R) & 7) * SLOT + xs * 32 + pp * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[t][4 * h + j] = r[j];
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[t], acc[i][t], 0, 0, 0);
      }
    }
    __syncthreads();   // the next row pair's router overwrites the image and ring slots
  }
  // ---- dW2 += acc: lane holds D[co = 16 i + 4 g + e][k = 16 T + (lane & 15)]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = 16 * i + 4 * g + e, k = 16 * (4 * wave + t) + (lane & 15);
        unsafeAtomicAdd(p.dw + co * 256 + k, acc[i][t][e]);
      }
  // ---- the workgroup's partial column sums: thread (it & 7) owns channels 8 (it & 7) .. +7
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] += __shfl_xor(cs[e], 8, 64);
    cs[e] += __shfl_xor(cs[e], 16, 64);
    cs[e] += __shfl_xor(cs[e], 32, 64);
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[wave * 64 + lane * 8 + e] = cs[e];
  }
  __syncthreads();
  if (tid < 64) {
    const float t = csum[tid] + csum[64 + tid] + csum[128 + tid] + csum[192 + tid];
    p.colsum[(long)blockIdx.x * 64 + tid] = t;
  }
}

int stem_pool_bwd_lds_bytes(int Ws) { return 8 * Ws * 32 + 2 * 16384 + 4 * 64 * 4; }

// Pool rows per backward workgroup: whole images at large batches; at small ones the largest block
// that still gives ~2 workgroups per CU.  Every workgroup ends with 64 x 256 fp32 atomics into dW,
// so the one-row blocks of the forward heuristic (4 per CU) cost b32 1,792 x 16 Ki atomics: 150 us
// of a 4.2 ms step (profiles/r4_b32_timeline.txt).
static int stem_pool_rows(int B, int H2, int PB) {
  if (PB > 0) return PB;
  const long want = 2L * num_cus();
  long pb = (long)B * H2 / want;
  return (int)(pb < 1 ? 1 : (pb > H2 ? H2 : pb));
}
int stem_pool_bwd_partial_rows(int B, int H2, int PB) {
  const int pb = stem_pool_rows(B, H2, PB);
  return B * ((H2 + pb - 1) / pb);
}

const char* stem_pool_bwd_launch(StemPoolBwdParams p, hipStream_t s) {
  if (p.H1 != p.Hs - 3 || p.W1 != p.Ws - 3) return "stem_pool_bwd: conv1 output must be the s2d input minus 3";
  if (p.H1 % 2 || p.W1 % 2) return "stem_pool_bwd: even conv1 output (even crop) expected";
  if (p.H2 != p.H1 / 2 || p.W2 != p.W1 / 2) return "stem_pool_bwd: pool output must be the pad-1 3x3/s2 size";
  if (p.Ws > 128 || p.W1 > 128) return "stem_pool_bwd: rows wider than the image / prefetch cover (crop <= 250)";
  if (p.W2 * 8 > 2 * SP_THREADS) return "stem_pool_bwd: more router items per row than the prefetch registers cover";
  const int lds = stem_pool_bwd_lds_bytes(p.Ws);
  if (lds > 80 * 1024) return "stem_pool_bwd: LDS per workgroup above the two-per-CU budget";
  p.PB = stem_pool_rows(p.B, p.H2, p.PB);
  p.nblk = (p.H2 + p.PB - 1) / p.PB;
  static std::atomic<unsigned long long> attr{0};
  once_per_device(attr, [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_pool_bwd_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  });
  hipLaunchKernelGGL(stem_pool_bwd_kernel, dim3((unsigned)((long)p.B * p.nblk)), dim3(SP_THREADS), lds, s, p);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

int stem_pool_lds_bytes(int Ws, int W1) { return 8 * Ws * 32 + 3 * (W1 + 1) * 128 + 512; }

const char* stem_pool_fwd_launch(StemPoolParams p, hipStream_t s) {
  if (p.H1 != p.Hs - 3 || p.W1 != p.Ws - 3) return "stem_pool: conv1 output must be the s2d input minus 3";
  if (p.H1 % 2 || p.W1 % 2) return "stem_pool: even conv1 output (even crop) expected";
  if (p.H2 != p.H1 / 2 || p.W2 != p.W1 / 2) return "stem_pool: pool output must be the pad-1 3x3/s2 size";
  if (p.Ws > 128) return "stem_pool: input rows wider than the prefetch covers (crop <= 250)";
  const int lds = stem_pool_lds_bytes(p.Ws, p.W1);
  if (lds > 80 * 1024) return "stem_pool: LDS per workgroup above the two-per-CU budget";
  if ((long)p.B * p.H2 * p.W2 * 64 >= (1L << 40)) return "stem_pool: output too large";
  if (p.PB <= 0) {   // pool rows per workgroup: whole images when the batch fills the chip
    const long want = 4L * num_cus();
    int pb = p.H2;
    while (pb > 2 && (long)p.B * ((p.H2 + pb - 1) / pb) < want) pb = (pb + 1) / 2;
    p.PB = pb;
  }
  p.nblk = (p.H2 + p.PB - 1) / p.PB;
  static std::atomic<unsigned long long> attr{0};
  once_per_device(attr, [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_pool_fwd_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_pool_fwd_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  });
  const dim3 grid((unsigned)((long)p.B * p.nblk));
  if (p.bits) hipLaunchKernelGGL((stem_pool_fwd_kernel<true>), grid, dim3(SP_THREADS), lds, s, p);
  else hipLaunchKernelGGL((stem_pool_fwd_kernel<false>), grid, dim3(SP_THREADS), lds, s, p);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

}  // namespace pddl
