// Host-visible parameter blocks and launchers of the pddl HIP kernels.
// This header is included by the kernel translation units and by the torch bindings;
// it deliberately has no torch dependency so the .hip files compile in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pddl {

enum EpiMode { EPI_FWD = 0, EPI_DGRAD = 1, EPI_F32 = 2 };

struct IgemmParams {
  // A operand: NHWC bf16 tensor(s), gathered as im2col rows.
  const uint16_t* a1; int C1;      // first source, channels (multiple of 64)
  const uint16_t* a2; int C2;      // optional second source (concatenated along K), 1x1 pad 0:
  int H2, W2, stride2;             //   its own spatial dims and stride (= H, W, stride when shared)
  int N, H, W;                     // input dims of the first source (the second's batch N too)
  int R, S, stride, pad;
  int Ho, Wo, M;                   // GEMM rows = N * Ho * Wo
  int K1, K;                       // K1 = R*S*C1, K = K1 + R*S*C2
  // B operand: [Nn][ldb] bf16, K contiguous.
  const uint16_t* b; int ldb; int Nn;
  // epilogue
  int mode;
  const float* scale; const float* shift;           // per output column (FWD / F32)
  const uint16_t* res; int ld_res;                  // FWD residual (added before act)
  const uint16_t* mask; int ld_mask;                // DGRAD: multiply by (mask > 0)
  const uint16_t* add; int ld_add;                  // DGRAD: added before the mask
  void* out; int ldo; int relu;
  void* out2; int ldo2; int relu2; int n_split;     // FWD: columns >= n_split -> out2
  int up2; int Hf, Wf;                              // DGRAD: scatter to a 2x finer grid (1: zero-fill the
                                                    //   off-grid positions; 2: write grid positions only;
                                                    //   3: as 2, the ReLU mask on the compact grid)
                                                    // FWD (up2 != 0): the residual is the Hf x Wf finer
                                                    //   grid, read at the output rows' stride-2 positions
  float* colsum;                                    // DGRAD: per-wave partial column sums [rows][Nn]
  // ReLU masks as bitmasks (bit e of byte [row][c/8] = value[row][8*(c/8)+e] > 0):
  uint8_t* bits_out; int ld_bits_out;               // FWD: write the mask of the (segment-0) output
  const uint8_t* bits_mask; int ld_bits_mask;       // DGRAD: multiply by the bit instead of (mask > 0)
  float* stats;                                     // FWD: per-wave partial [rows][2*Nn]: sum | sum of squares
                                                    //      of the stored outputs (train-mode BN batch statistics)
                                                    // DGRAD (with bn_z): sum g | sum g * (z - bn_mean) of the
                                                    //      stored gradient (train-mode BN backward reduction)
  const uint16_t* bn_z; const float* bn_mean;       // DGRAD: the BN input z ([rows][ldo]) and its batch mean
  uint64_t mg_howo, mg_wo;                          // set by igemm_launch: magic divisors (fdiv)
  int m_begin, prow_begin;                          // set by igemm_launch: this launch covers GEMM rows
                                                    // [m_begin, M); its partial rows start at prow_begin
  float* slab; long slab_floats;                    // split-K workspace (fp32 partial tiles), optional
  int ksplit;                                       // set by igemm_launch: K slices per tile (1 = none)
};
const char* igemm_launch(const IgemmParams& p, hipStream_t stream);
int igemm_partial_rows(int M, int Nn, int K, bool bnz = false);   // rows of the partial column-sum buffer
                                                    // (bnz: a launch with the fused BN-backward sums)
void igemm_plan_query(int M, int Nn, int K, int* cfg, int* split, int* ksplit = nullptr);   // tile config;
                                                    // rows >= split: 128x128 tail; ksplit: K slices (split-K)
long igemm_splitk_floats(int M, int Nn, int K);     // split-K workspace a problem wants (0: no split)
extern int g_igemm8, g_igemm8_min_tiles, g_igemm8_min_n, g_igemm_ns1_kt, g_wgrad8, g_wgrad1;
int num_cus();   // compute units of the current device (cached)
extern int g_wgrad_f32_wpc[2];
extern int g_igemm_sk_fill, g_igemm_sk_cap, g_igemm_sk_elig;   // split-K plan knobs (igemm.hip)
extern int g_igemm_splitk, g_wgrad8_min_rows, g_igemm_pk, g_igemm_pk_all, g_igemm_pk_dual;   // split-K: 0 off, 1 heuristic (default), >= 2 forced slices (where legal)
extern int g_stem_variant, g_igemm_n64, g_igemm_variant, g_igemm_deep, g_igemm_pf, g_bn_red_blocks, g_bn_apply_blocks, g_pool_blocks, g_colred_chunks;   // tuning knobs (A/B timing)

struct WgradParams {
  const uint16_t* x; int N, H, W, C;   // conv input, NHWC (or [M][ldx] rows for 1x1/s1)
  int ldx;
  int R, S, stride, pad, Ho, Wo, M;
  const uint16_t* g; int ldg;          // output gradient [M][ldg]
  const uint16_t* g2; int ldg2; int co_split;  // optional second gradient for rows >= co_split
  int Cout, K;                         // dW is [Cout][K]
  float* dw; int ld_dw;                // fp32, accumulated with atomics
  int splits;                          // split of M across workgroups (0 = auto)
};
const char* wgrad_launch(const WgradParams& p, hipStream_t stream);

// Fused backward of a stride-1 1x1 conv with (CO, CI) = (256, 64) or (512, 128) output / input
// channels (bwd1x1.hip): out = bits * (g . Wd) with partial column sums, dw += g^T . x, from one
// HBM read of g.
struct Bwd1x1Params {
  const uint16_t* g;                   // output gradient [M][CO]
  const uint16_t* x;                   // conv input [M][CI]
  const uint16_t* wd; int ld_wd;       // data-gradient weights [CI][ld_wd >= CO]
  const uint8_t* bits;                 // ReLU bits of x [M][CI / 8]
  uint16_t* out;                       // input gradient [M][CI]
  float* colsum;                       // partial column sums [bwd1x1_partial_rows(M, CO, CI)][CI]
  float* dw; int ld_dw;                // fp32 [CO][ld_dw >= CI], accumulated with atomics
  int M, CO, CI;
  // stride-2 form (the block feeds a downsampling block): g has the M = N * Hc * Wc compact rows,
  // x / out / bits are full resolution N x Hf x Wf (out written at the grid pixels only, into a
  // pre-zeroed tensor), out2 gets the compact copy
  int s2, N, Hf, Wf, Hc, Wc;
  uint16_t* out2;
  uint64_t mg_hwc, mg_wc;              // set by bwd1x1_launch
  // "pre" form (stage 2, not stride-2): g is not read from HBM but computed per tile from the next
  // block's conv1 gradient -- g = bit(gmask) * (g1 . w1d^T + g) with g the shortcut gradient --
  // and written out (gx) with its per-channel partial sums (colsum_gx, rows as colsum, CO columns)
  const uint16_t* g1;                  // [M][64] gradient of the next block's conv1 output
  const uint16_t* w1d;                 // [CO][64] its data-gradient weights
  const uint8_t* gmask;                // [M][CO / 8] ReLU bits of this block's output
  uint16_t* gx;                        // [M][CO]
  float* colsum_gx;                    // [bwd1x1_partial_rows][CO]
};
const char* bwd1x1_launch(const Bwd1x1Params& p, hipStream_t stream);
int bwd1x1_partial_rows(int M, int CO, int CI);

// ---- fp32 convolution on the fp32 matrix cores (conv_f32.hip): the reference-precision path ----
struct ConvF32Params {
  const float* x; int N, H, W, C;      // NHWC input (im2col source)
  int R, S, stride, pad, Ho, Wo, M;    // M = N * Ho * Wo
  const float* w; const float* bias;   // forward: w [Cout][K] (OHWI), optional bias [Cout]
  int Cout, K;                         // K = R * S * C
  float* y;                            // forward: output [M][Cout]; wgrad: the output gradient (read)
  float* dw;                           // wgrad: [Cout][K], accumulated with atomics
  uint64_t mg_howo, mg_wo;             // (set by the launchers)
  // fused epilogue of conv_f32 (the fp32 engine, models/engine_f32.py), staged through LDS into
  // 16-byte row stores:
  //   F32_EPI_PLAIN: y = acc (+ bias)
  //   F32_EPI_FWD:   y = act(acc * scale[n] + shift[n] (+ res))          (frozen BN + bias folded)
  //   F32_EPI_DGRAD: y = (acc (+ add)) * (mask > 0), optional stride-2 grid scatter (up2: GEMM
  //                  row (n, i, j) -> output row (n, 2i, 2j) of an Hf x Wf grid; the caller's
  //                  buffer holds zeros off the grid; `add` is then indexed by the GEMM row,
  //                  `mask` by the output row), and per-m-tile partial column sums
  int epi;
  const float* scale; const float* shift; const float* res; int relu;
  const float* add; const float* mask; int up2, Hf, Wf;
  float* colsum;                       // [ceil(M / 64)][Cout] partial column sums (DGRAD, optional)
  float* slab; long slab_floats;       // split-K workspace (the engine's, bindings' splitk_use); null: unsplit
  int ksplit;                          // (set by the launcher)
};
enum { F32_EPI_PLAIN = 0, F32_EPI_FWD = 1, F32_EPI_DGRAD = 2 };
const char* conv_f32_launch(ConvF32Params p, hipStream_t stream);
extern int g_conv_f32_variant, g_conv_f32_splitk, g_conv_f32_sk_elig;   // 0: 64 x 64 register-staged fp32 kernels; 1: LDS-DMA 128 x {64, 128} by model (default); 2: 128 x 128; 3: 128 x 64
const char* wgrad_f32_launch(ConvF32Params p, hipStream_t stream);
// fp32 elementwise kernels of the fp32 engine (f32.hip)
const char* maxpool_fwd_f32_launch(const float* x, float* y, uint8_t* idx, int B, int H, int W, int C, int Ho, int Wo,
                                   hipStream_t s);
const char* maxpool_bwd_f32_launch(const float* gy, const uint8_t* idx, const float* xmask, float* gx, int B, int H,
                                   int W, int C, int Ho, int Wo, hipStream_t s);
const char* gap_fwd_f32_launch(const float* x, float* y, int B, int HW, int C, hipStream_t s);
const char* gap_bwd_f32_launch(const float* gp, const float* ymask, float* g, int B, int HW, int C, float* colsum_rows,
                               hipStream_t s);
const char* colsum_f32_launch(const float* g, long M, int C, int ldg, float* out, hipStream_t s);
const char* softmax_xent_f32_launch(const float* logits, int ldl, const int64_t* labels, int B, int ncls, float gscale,
                                    float* dlogits, int ldd, float* loss_sum, float* correct, hipStream_t s);

// ---- elementwise / reduction kernels (eltwise.hip) ----
struct StemParams {
  const void* in; int in_u8;          // [B, Hin, Win, 3] uint8 or fp32 (0..255)
  int B, Hin, Win;
  int Hc, Wc;                         // preprocessed (cropped / resized) size
  int mode;                           // 0 identity, 1 bilinear resize, 2 crop at (oy, ox)
  int oy, ox;
  const int32_t* crop_dev;            // optional device {oy, ox} (overrides oy/ox; HIP-graph replays)
  const uint8_t* flip;                // per-image horizontal flip flags (nullable)
  float scale;                        // Rescaling(1/255)
  uint16_t* out; int Hs, Ws;          // space-to-depth image [B][Hs][Ws][16], Hs = (Hc + 6) / 2
};
// Preprocess + ZeroPadding2D(3) + 2x2 space-to-depth: channel (dy*2+dx)*4 + c of pixel (i, j)
// is the padded preprocessed pixel (2i+dy-3, 2j+dx-3, c) (c = 3 is zero).  The 7x7/s2 stem
// conv then becomes a 4x4/s1 "window" implicit GEMM with K = 4*4*16 = 256.
const char* stem_s2d_launch(const StemParams& p, hipStream_t s);
const char* stem_s2d_f32_launch(const StemParams& p, float* out, hipStream_t s);   // fp32 image (out ignored)
// Fold the s2d-domain stem weight gradient [64][256] back to [64][7][7][3] (added into dw).
const char* stem_wgrad_fold_launch(const float* g2, float* dw, int cout, hipStream_t s);

// Fused stem forward (stem.hip): conv1 on the s2d input + frozen BN + ReLU + the 3x3/s2 max-pool,
// writing only the pool output, its argmax taps and (nullable) ReLU bits -- conv1's output never
// reaches HBM.  PB = pool rows per workgroup (<= 0: chosen by the launcher; nblk is set by it).
struct StemPoolParams {
  const uint16_t* x2;                 // [B][Hs][Ws][16] space-to-depth input
  const uint16_t* w;                  // [64][256] bf16 forward weights (s2d k order)
  const float* scale; const float* shift;   // folded frozen BN of conv1 (64 each)
  uint16_t* pool; uint8_t* idx; uint8_t* bits;   // [B][H2][W2][64], same, [B][H2][W2][8]
  int B, Hs, Ws, H1, W1, H2, W2;
  int PB, nblk;
};
const char* stem_pool_fwd_launch(StemPoolParams p, hipStream_t s);
// Fused stem backward (stem.hip): max-pool backward into LDS + conv1 weight gradient
// dw[64][256] += sum gc1^T im2col(x2) (fp32 atomics) + per-workgroup partial column sums of gc1
// ([stem_pool_bwd_partial_rows][64]); conv1's output gradient never reaches HBM.
struct StemPoolBwdParams {
  const uint16_t* x2;                 // [B][Hs][Ws][16]
  const uint16_t* gpool;              // [B][H2][W2][64] pool-output gradient
  const uint8_t* idx;                 // [B][H2][W2][64] argmax taps of the forward
  float* dw;                          // [64][256] s2d-domain weight gradient (accumulated)
  float* colsum;                      // partial rows [grid][64]
  int B, Hs, Ws, H1, W1, H2, W2;
  int PB, nblk;
};
// Persistent row-tile 3x3 / pad 1 / stride 1 convolution, 64 -> 64 channels (conv3x3c64.hip).
enum { C64_FWD = 0, C64_DGRAD = 1 };
struct C64Params {
  const uint16_t* x;          // [M][64] NHWC input (forward) / output gradient (dgrad)
  const uint16_t* w;          // [64][576] OHWI weights (dgrad: transposed + flipped, as igemm's B)
  const float* scale;         // forward: folded BN scale / shift (ReLU always applied)
  const float* shift;
  const uint8_t* bits_mask;   // dgrad: [M][8] ReLU bits of the layer input
  uint16_t* out;              // [M][64]
  uint8_t* bits_out;          // forward, optional: [M][8] ReLU bits of out
  float* colsum;              // dgrad, optional: partial rows [grid * 4][64]
  int N, H, W, M;
  uint64_t mg_hw, mg_w;
};
const char* conv3x3c64_launch(const C64Params& p, int mode, hipStream_t s);
int conv3x3c64_partial_rows(int M);
extern int g_c64_grid, g_c64w_grid;
struct C64WgradParams {
  const uint16_t* x;          // [N][H][W][64] conv input
  const uint16_t* g;          // [N][H][W][64] output gradient
  float* dw; int ld_dw;       // [64][ld_dw >= 576] fp32, accumulated with atomics
  int N, H, W;
};
const char* conv3x3c64_wgrad_launch(const C64WgradParams& p, hipStream_t s);

// Fused 64-channel bottleneck boundary (c3c1.hip): block b's conv3 (+ residual, or the fused
// projection with a second A source) and block b + 1's conv1, one launch.
struct C3C1Params {
  const uint16_t* a;           // [M][64] conv3 input (block b's conv2 output)
  const uint16_t* w3;          // [256][64] conv3 weights
  const float* scale3; const float* shift3;   // [256]
  const uint16_t* res;         // optional [M][256] residual (plain blocks)
  uint16_t* out;               // [M][256] block-b output
  uint8_t* bits3;              // optional [M][32] its ReLU bits
  const uint16_t* w1;          // [64][256] block b+1 conv1 weights
  const float* scale1; const float* shift1;   // [64]
  uint16_t* y1;                // [M][64] block b+1 conv1 output
  uint8_t* bits1;              // optional [M][8]
  int M;
};
const char* c3c1_launch(const C3C1Params& p, hipStream_t s);
const char* stem_pool_bwd_launch(StemPoolBwdParams p, hipStream_t s);
int stem_pool_bwd_partial_rows(int B, int H2, int PB);
int stem_pool_lds_bytes(int Ws, int W1);

const char* maxpool_fwd_launch(const uint16_t* x, uint16_t* y, uint8_t* idx, uint8_t* bits, int B, int H, int W, int C,
                               int Ho, int Wo, hipStream_t s);
const char* maxpool_bwd_launch(const uint16_t* gy, const uint8_t* idx, const uint16_t* xmask, uint16_t* gx,
                               int B, int H, int W, int C, int Ho, int Wo, float* colsum, hipStream_t s);
const char* gap_fwd_launch(const uint16_t* x, uint16_t* y, int B, int HW, int C, hipStream_t s);
const char* gap_bwd_launch(const uint16_t* gp, int ldgp, const uint16_t* ymask, uint16_t* g, int B, int HW, int C,
                           float* colsum, hipStream_t s);
const char* colsum_launch(const uint16_t* g, int M, int C, int ldg, float* out, hipStream_t s);
// Partial column sums written by the fused producers (igemm dgrad, maxpool_bwd, gap_bwd):
// colsum[l.out + c] += sum_t part[l.part + t * C + c] for every layer of the table.
struct ColRedLayer { long part; int rows, C, out; int pad; };   // pad > 0: row stride (floats)
const char* colsum_reduce_launch(const float* part, const ColRedLayer* layers_dev, int nlayers, float* colsum,
                                 hipStream_t s);
int maxpool_bwd_partial_rows(int B, int H, int W, int C);
const char* softmax_xent_launch(const float* logits, int ldl, const int64_t* labels, int B, int ncls,
                                float gscale, uint16_t* dlogits, int ldd, float* loss_sum, float* correct,
                                hipStream_t s);

// Per-layer parameter preparation after every optimizer step (one launch for all layers).
struct PrepLayer {
  int w_off;          // offset of the fp32 kernel [Cout][R][S][Cin] in the flat param buffer
  int cout, R, S, cin;
  int kpad;           // forward bf16 row length (>= R*S*cin, multiple of 64)
  long wf_off;        // offset (elements) of the forward bf16 weights
  long wd_off;        // offset of the dgrad bf16 weights [cin][R][S][cout_pad] (-1: none)
  int cout_pad;
  int bias_off, gamma_off, beta_off, mean_off, var_off;   // -1 when absent
  int ch_off;         // offset of this layer's folded scale/shift (per output channel)
  int mode;           // 0: dense [cout][kpad] rows; 1: stem in the 4x4x16 space-to-depth layout
};
// Fused projection-block forward (conv3 + projection shortcut as one dual-source GEMM): the
// bf16 weights [cout][k3 + k0] = [a3 * W3 | a0 * W0] with both frozen-BN scales folded in, and
// the epilogue affine scale = 1, shift = b3 + b0 (prep_fuse_kernel).
struct FuseLayer {
  int cout, k3, k0;
  int w3_off, w0_off;                                   // fp32 kernels [cout][k3], [cout][k0]
  int bias3, gamma3, beta3, mean3, var3;                // BN of conv3 (-1: absent)
  int bias0, gamma0, beta0, mean0, var0;                // BN of the shortcut conv
  int ch_off;                                           // fused scale / shift slots
  long wf_off;                                          // bf16 destination
};
const char* prep_fuse_launch(const float* params, const FuseLayer* layers_dev, int nlayers, int max_elems,
                             uint16_t* wbf, float* scale, float* shift, float eps, hipStream_t s);
const char* prep_f32_launch(const float* params, const PrepLayer* layers_dev, int nlayers, float* wf32, float* scale,
                            float* shift, float eps, hipStream_t s);   // fp32 stem s2d + dgrad weights
const char* prep_launch(const float* params, const PrepLayer* layers_dev, int nlayers, int max_elems,
                        uint16_t* wbf, float* scale, float* shift, float eps, hipStream_t s, int parts = 3);

// dW finalize: dgamma_raw[c] = sum_k W[c,k] * dWraw[c,k]; dW[c,k] *= a[c] (in place).
struct FinLayer {
  int w_off; int cout; int k;   // flat offsets of W (params) / dW (grads), rows x k
  int ch_off;                   // folded scale index
  int dg_off;                   // output offset for dgamma_raw (per channel, -1: none)
};
const char* wgrad_finalize_launch(const float* params, float* grads, const FinLayer* layers_dev, int nlayers,
                                  const float* scale, float* dgamma_raw, hipStream_t s, int max_cout = 2048);

// Per-channel BN/bias grads from column sums and dgamma_raw.
struct BnGradLayer {
  int cout, ch_off;
  int bias_off, gamma_off, beta_off, mean_off, var_off;   // -1 when absent (grads written into `grads`)
  int colsum_off, dg_off;
};
const char* bn_grad_launch(const float* params, float* grads, const BnGradLayer* layers_dev, int nlayers,
                           const float* colsum, const float* dgamma_raw, const float* scale, float eps,
                           hipStream_t s);

// ---- train-mode BatchNormalization (bn.hip) ----
// Batch statistics of one BN layer from the reduced (sum, sum of squares) of its conv output.
struct BnStatLayer {
  int C;
  int sum_off, sq_off;     // offsets of the reduced sums in `acc`
  int ch;                  // offset in the per-channel mean / inv / scale / shift arrays
  int gamma_off, beta_off, mm_off, mv_off;   // flat parameter offsets
  float count;             // N * H * W
  int pad;
};
// training: batch statistics + moving-statistics update; else the moving statistics.
const char* bn_stats_launch(const float* acc, const BnStatLayer* layers_dev, int nlayers, int max_c, int training,
                            float* params, float* mean, float* inv, float* scale, float* shift, float eps,
                            float momentum, hipStream_t s);
// y = act(z*a + b (+ r*a2 + b2 | + r)) over [M][C] bf16 or fp32; bits (nullable) = ReLU bitmask of y.
const char* bn_apply_launch(const uint16_t* z, const float* a, const float* b, const uint16_t* r, const float* a2,
                            const float* b2, int relu, uint16_t* y, uint8_t* bits, long M, int C, hipStream_t s);
const char* bn_apply_launch(const float* z, const float* a, const float* b, const float* r, const float* a2,
                            const float* b2, int relu, float* y, uint8_t* bits, long M, int C, hipStream_t s);   // fp32
// sg[c] += sum g, sgx[c] += sum g*(z-mean[c]) (sg2/sgx2 for z2/mean2, nullable).
const char* bn_bwd_reduce_launch(const uint16_t* g, const uint16_t* z, const uint16_t* z2, const float* mean,
                                 const float* mean2, long M, int C, float* sg, float* sgx, float* sg2, float* sgx2,
                                 hipStream_t s);
const char* bn_bwd_reduce_launch(const float* g, const float* z, const float* z2, const float* mean,
                                 const float* mean2, long M, int C, float* sg, float* sgx, float* sg2, float* sgx2,
                                 hipStream_t s);   // fp32
struct BnBwdLayer {
  int C, ch;                             // channels, per-channel array offset
  int gamma_off, beta_off, bias_off;     // flat offsets (params for gamma, grads for all)
  float count;
};
// dz = gamma/sigma * (g - Sg/M - (z - mean)/sigma^2 * Sgx/M); BN/bias parameter grads.
// coef: scratch [3][ldc] per-channel (A, B, C) indexed by the layers' channel offsets.
const char* bn_bwd_apply_launch(const uint16_t* g, const uint16_t* z, const uint16_t* z2, const BnBwdLayer& l,
                                const BnBwdLayer& l2, const float* params, const float* mean, const float* inv,
                                const float* sg, const float* sgx, float* coef, int ldc, uint16_t* dz, uint16_t* dz2,
                                float* grads, long M, hipStream_t s);
const char* bn_bwd_apply_launch(const float* g, const float* z, const float* z2, const BnBwdLayer& l,
                                const BnBwdLayer& l2, const float* params, const float* mean, const float* inv,
                                const float* sg, const float* sgx, float* coef, int ldc, float* dz, float* dz2,
                                float* grads, long M, hipStream_t s);   // fp32

// ---- range gather / scatter (pack.hip) ----
struct RangeRow { long flat, packed, len; };   // rows laid end to end: packed[i + 1] = packed[i] + len[i]
// scatter = 0: dst[packed + i] = src[flat + i]; 1: dst[flat + i] = src[packed + i].
const char* range_copy_launch(const float* src, float* dst, const RangeRow* rows_dev, int nrows, int scatter,
                              hipStream_t s);
const char* range_copy_cvt_launch(const void* src, void* dst, const RangeRow* rows_dev, int nrows, int scatter,
                                  hipStream_t s);   // gather: fp32 -> bf16 packed; scatter: bf16 packed -> fp32
const char* comm_proxy_launch(const float* src, float* scratch, long n, int passes, long ticks, int nch,
                              hipStream_t s);

// Deterministic synthetic images / labels for example ids idx[0..n) (uint8 [n][per], int64 [n]).
const char* synth_launch(const int64_t* idx, int n, long per, int64_t seed, int ncls, uint8_t* img, int64_t* lab,
                         hipStream_t s);

// ---- optimizers (optim.hip) ----
// hs (nullable): device {t, lr, lr_t}; when given, the step size is read from hs[2].
const char* opt_hparams_launch(float* hs, float b1, float b2, int adam, hipStream_t s);
const char* adam_launch(float* p, const float* g, float* m, float* v, long n, float lr_t, float b1, float b2,
                        float eps, float gscale, const float* hs, hipStream_t s);
const char* sgd_launch(float* p, const float* g, float* mom, long n, float lr, float momentum, float wd,
                       int nesterov, float gscale, const float* hs, hipStream_t s);
const char* adam_bf16_wire_launch(float* p, const uint16_t* g, float* m, float* v, uint16_t* snap, long n, float lr_t,
                                  float b1, float b2, float eps, hipStream_t s);
const char* scale_launch(float* x, long n, float a, hipStream_t s);
const char* cast_bf16_launch(const float* x, uint16_t* y, long n, hipStream_t s);
const char* cast_f32_launch(const uint16_t* x, float* y, long n, hipStream_t s);

}  // namespace pddl
