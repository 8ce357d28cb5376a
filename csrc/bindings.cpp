// torch bindings of the pddl HIP kernels (module `_pddl_native`).
//
// Every op launches on the caller's current HIP stream and raises on a bad shape or a
// launch error; the Python layer (pddl.ops) never silently falls back to eager PyTorch on
// a GPU tensor.
#include <torch/extension.h>

#include <atomic>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/util/Optional.h>

#include "kernels/kernels.h"

using torch::Tensor;
using OptT = c10::optional<Tensor>;
namespace py = pybind11;

#define PCHECK(cond, msg) TORCH_CHECK(cond, "pddl: ", msg)

namespace {

// Kernel knobs (set_variant) are process-global launch configuration shared by every device and
// replica thread: they are fixed once the first kernel has been issued (every launching binding
// takes its stream from cur_stream), so no replica can see a plan change mid-step.  Tuning code
// (A/B tests, micro-benchmarks) opts in with allow_knob_changes(True).
std::atomic<bool> g_launched{false};
std::atomic<bool> g_knob_tuning{false};
hipStream_t cur_stream() {
  if (!g_launched.load(std::memory_order_relaxed)) g_launched.store(true, std::memory_order_relaxed);
  return at::hip::getCurrentHIPStream().stream();
}

void ok(const char* err, const char* what) { TORCH_CHECK(err == nullptr, "pddl ", what, ": ", err ? err : ""); }

const uint16_t* bfp(const Tensor& t) {
  PCHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16, "expected a bf16 GPU tensor");
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
uint16_t* bfpm(const Tensor& t) { return const_cast<uint16_t*>(bfp(t)); }
const uint16_t* obfp(const OptT& t) { return t.has_value() ? bfp(*t) : nullptr; }
float* f32p(const Tensor& t) {
  PCHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32, "expected an fp32 GPU tensor");
  return t.data_ptr<float>();
}
const float* of32p(const OptT& t) { return t.has_value() ? f32p(*t) : nullptr; }
// Row stride of a row-major [..., C] view (innermost dim contiguous).
int ld(const Tensor& t) {
  PCHECK(t.stride(-1) == 1, "innermost dim must be contiguous");
  return t.dim() >= 2 ? (int)t.stride(-2) : (int)t.size(-1);
}
int old(const OptT& t) { return t.has_value() ? ld(*t) : 0; }

// Split-K workspace (fp32 partial tiles of the small-M layers, igemm.hip), owned by the
// calling engine and made current for the calling THREAD (`splitk_use`): two engines whose
// launches interleave on one device (Mirrored replicas driven from threads, rehearsals) must
// never share one -- replica B's slices would overwrite replica A's partials between A's
// slices and A's combine.  Nothing is allocated inside a launch, so graph capture bakes the
// engine's own buffer into its kernels.
thread_local Tensor tls_splitk;
void splitk_use(OptT ws) {
  if (ws.has_value()) PCHECK(ws->is_cuda() && ws->scalar_type() == torch::kFloat32 && ws->is_contiguous(),
                             "split-K workspace: contiguous fp32 GPU tensor");
  tls_splitk = ws.has_value() ? *ws : Tensor();
}
int64_t splitk_default_floats(int64_t device) {   // the heuristic's bound: tiles x slices < (fill + 2) x #CUs tiles of 16384 floats
  c10::hip::HIPGuardMasqueradingAsCUDA g((int)device);
  return (long)(pddl::g_igemm_sk_fill + 2) * pddl::num_cus() * 16384;
}

// Generic implicit-GEMM (conv forward / dgrad / fp32 dense).
void igemm_impl(Tensor a1, OptT a2, int64_t H, int64_t W, int64_t R, int64_t S, int64_t stride, int64_t pad,
                int64_t Ho, int64_t Wo, Tensor b, int64_t mode, OptT scale, OptT shift, OptT res, OptT mask,
                OptT add, Tensor out, int64_t relu, OptT out2, int64_t relu2, int64_t n_split, int64_t up2,
                int64_t Hf, int64_t Wf, OptT colsum, OptT bits_out, OptT stats, OptT bn_z = c10::nullopt,
                OptT bn_mean = c10::nullopt) {
  pddl::IgemmParams p{};
  PCHECK(a1.is_contiguous(), "A source must be contiguous NHWC");
  p.a1 = bfp(a1);
  p.C1 = (int)a1.size(-1);
  p.N = (int)a1.size(0);
  p.H = (int)H; p.W = (int)W;
  PCHECK(a1.numel() == (int64_t)p.N * H * W * p.C1, "A source numel does not match N*H*W*C");
  p.R = (int)R; p.S = (int)S; p.stride = (int)stride; p.pad = (int)pad;
  p.Ho = (int)Ho; p.Wo = (int)Wo; p.M = p.N * (int)Ho * (int)Wo;
  p.K1 = (int)(R * S * p.C1);
  p.K = p.K1;
  p.H2 = p.H; p.W2 = p.W; p.stride2 = p.stride;
  if (a2.has_value()) {
    PCHECK(a2->is_contiguous() && a2->size(0) == a1.size(0), "second A source shape");
    p.a2 = bfp(*a2);
    p.C2 = (int)a2->size(-1);
    if (a2->dim() == 4 && (a2->size(1) != H || a2->size(2) != W)) {
      // a second source with its own geometry (fused projection shortcut: the block input at
      // stride 1 or 2 next to conv3's operand): 1x1 / pad 0, stride from the spatial ratio
      PCHECK(R == 1 && S == 1 && pad == 0, "a second source of other dims needs a 1x1 / pad 0 gather");
      p.H2 = (int)a2->size(1); p.W2 = (int)a2->size(2);
      p.stride2 = (int)((p.H2 + Ho - 1) / Ho);
      PCHECK(p.stride2 >= 1 && (Ho - 1) * p.stride2 < p.H2 && (Wo - 1) * p.stride2 < p.W2 &&
                 (p.H2 - 1) / p.stride2 + 1 == Ho && (p.W2 - 1) / p.stride2 + 1 == Wo,
             "second A source dims do not map onto the output grid");
    }
    PCHECK(a2->numel() == (int64_t)p.N * p.H2 * p.W2 * p.C2, "second A source numel");
    p.K += (int)(R * S * p.C2);
  }
  PCHECK(b.dim() == 2 && b.size(1) >= p.K, "B must be [Nn][>=K]");
  p.b = bfp(b); p.ldb = ld(b); p.Nn = (int)b.size(0);
  p.mode = (int)mode;
  if (mode != pddl::EPI_DGRAD) {
    PCHECK(scale.has_value() && shift.has_value(), "forward epilogue needs scale and shift");
    PCHECK(scale->numel() >= p.Nn && shift->numel() >= p.Nn, "scale/shift too short");
  }
  p.scale = of32p(scale); p.shift = of32p(shift);
  p.res = obfp(res); p.ld_res = old(res);
  if (mask.has_value() && mask->scalar_type() == torch::kUInt8) {
    // bitmask [rows][Nn/8]: bit e of byte c/8 is (x[row][c] > 0)
    PCHECK(mode == pddl::EPI_DGRAD && mask->is_cuda() && mask->size(-1) * 8 >= p.Nn, "bitmask mask shape");
    p.bits_mask = mask->data_ptr<uint8_t>(); p.ld_bits_mask = ld(*mask);
  } else {
    p.mask = obfp(mask); p.ld_mask = old(mask);
  }
  if (bits_out.has_value()) {
    PCHECK(mode == pddl::EPI_FWD && bits_out->scalar_type() == torch::kUInt8 && bits_out->is_cuda(),
           "bits_out must be a uint8 tensor of a forward epilogue");
    const int64_t seg0 = out2.has_value() ? n_split : p.Nn;
    PCHECK(bits_out->size(-1) * 8 >= seg0 && bits_out->numel() / bits_out->size(-1) >= p.M, "bits_out too small");
    p.bits_out = bits_out->data_ptr<uint8_t>(); p.ld_bits_out = ld(*bits_out);
  }
  p.add = obfp(add); p.ld_add = old(add);
  if (mode == pddl::EPI_F32) p.out = f32p(out); else p.out = bfpm(out);
  p.ldo = ld(out);
  p.relu = (int)relu;
  if (out2.has_value()) {
    p.out2 = bfpm(*out2); p.ldo2 = ld(*out2);
    if (mode == pddl::EPI_DGRAD)   // dgrad: compact copy of the stride-2 scatter's rows
      PCHECK(up2 && out2->numel() / std::max<int64_t>(1, out2->size(-1)) >= p.M && out2->size(-1) >= p.Nn,
             "dgrad out2 is the compact [N*Ho*Wo][Nn] copy of an up2 scatter");
  }
  p.relu2 = (int)relu2; p.n_split = (int)n_split;
  PCHECK(up2 >= 0 && up2 <= 3, "up2: 0 none, 1 scatter + zero fill, 2 grid positions only, 3 as 2 + compact mask");
  if (mode == pddl::EPI_FWD && up2) {
    // forward: a residual on the 2x finer grid, read at the output's stride-2 positions
    PCHECK(res.has_value() && (Hf - 1) / 2 + 1 == Ho && (Wf - 1) / 2 + 1 == Wo &&
               res->numel() >= (int64_t)p.N * Hf * Wf * p.Nn && !out2.has_value() && !stats.has_value(),
           "forward up2: residual [N][Hf][Wf][Nn] with Ho = ceil(Hf / 2), no second output / stats");
  } else {
    PCHECK(mode == pddl::EPI_DGRAD || !up2, "up2 is a dgrad scatter or a forward stride-2 residual");
  }
  p.up2 = (int)up2; p.Hf = (int)Hf; p.Wf = (int)Wf;
  p.colsum = colsum.has_value() ? f32p(*colsum) : nullptr;
  if (p.colsum)
    PCHECK(colsum->numel() >= (int64_t)pddl::igemm_partial_rows(p.M, p.Nn, p.K) * p.Nn, "colsum partial buffer too short");
  if (bn_z.has_value()) {
    PCHECK(mode == pddl::EPI_DGRAD && stats.has_value() && bn_mean.has_value() && !up2,
           "bn_z: fused BN-backward sums of a dgrad (stats rows, bn_mean; no stride-2 scatter)");
    PCHECK(bn_z->scalar_type() == torch::kBFloat16 && ld(*bn_z) == ld(out) &&
               bn_z->numel() / std::max<int64_t>(1, bn_z->size(-1)) >= p.M && bn_mean->numel() >= p.Nn,
           "bn_z must be bf16 [M][ldo] like the output, bn_mean [Nn]");
    p.bn_z = bfp(*bn_z);
    p.bn_mean = f32p(*bn_mean);
  }
  if (stats.has_value()) {
    PCHECK(mode == pddl::EPI_FWD || p.bn_z, "BN statistics are a forward-epilogue output (or a bn_z dgrad)");
    p.stats = f32p(*stats);
    PCHECK(stats->numel() >= (int64_t)pddl::igemm_partial_rows(p.M, p.Nn, p.K, p.bn_z != nullptr) * 2 * p.Nn,
           "stats partial buffer too short");
  }
  const int64_t rows_out = (up2 && mode == pddl::EPI_DGRAD) ? (int64_t)p.N * Hf * Wf : (int64_t)p.M;
  PCHECK(out.numel() / std::max<int64_t>(1, out.size(-1)) >= (out2.has_value() ? p.M : rows_out) ||
             out.dim() >= 2,
         "output too small");
  if (tls_splitk.defined() && tls_splitk.device() == a1.device()) {
    p.slab = tls_splitk.data_ptr<float>();
    p.slab_floats = tls_splitk.numel();
  }
  ok(pddl::igemm_launch(p, cur_stream()), "igemm");
}

void igemm(Tensor a1, OptT a2, int64_t H, int64_t W, int64_t R, int64_t S, int64_t stride, int64_t pad,
           int64_t Ho, int64_t Wo, Tensor b, int64_t mode, OptT scale, OptT shift, OptT res, OptT mask, OptT add,
           Tensor out, int64_t relu, OptT out2, int64_t relu2, int64_t n_split, int64_t up2, int64_t Hf,
           int64_t Wf, OptT colsum, OptT bits_out) {
  igemm_impl(a1, a2, H, W, R, S, stride, pad, Ho, Wo, b, mode, scale, shift, res, mask, add, out, relu, out2, relu2,
             n_split, up2, Hf, Wf, colsum, bits_out, c10::nullopt);
}

// ---- train-mode BatchNormalization (bn.hip)
int64_t rows_of(const Tensor& t) { return t.numel() / std::max<int64_t>(1, t.size(-1)); }
void bn_stats(Tensor acc, Tensor table, int64_t nlayers, int64_t max_c, bool training, Tensor params, Tensor mean,
              Tensor inv, Tensor scale, Tensor shift, double eps, double momentum) {
  PCHECK(table.is_cuda() && table.numel() == nlayers * (int64_t)sizeof(pddl::BnStatLayer), "bn_stats table size");
  ok(pddl::bn_stats_launch(f32p(acc), reinterpret_cast<const pddl::BnStatLayer*>(table.data_ptr()), (int)nlayers,
                           (int)max_c, training ? 1 : 0, f32p(params), f32p(mean), f32p(inv), f32p(scale),
                           f32p(shift), (float)eps, (float)momentum, cur_stream()),
     "bn_stats");
}
void bn_apply(Tensor z, Tensor a, Tensor b, OptT r, OptT a2, OptT b2, bool relu, Tensor y, OptT bits) {
  PCHECK(z.is_contiguous() && y.is_contiguous(), "bn_apply: contiguous [.., C] tensors");
  const int C = (int)z.size(-1);
  const int64_t M = rows_of(z);
  PCHECK(y.numel() == z.numel() && a.numel() >= C && b.numel() >= C, "bn_apply shapes");
  if (r.has_value()) PCHECK(r->is_contiguous() && r->numel() == z.numel(), "bn_apply residual shape");
  PCHECK(a2.has_value() == b2.has_value(), "bn_apply: a2 and b2 go together");
  if (bits.has_value())
    PCHECK(bits->scalar_type() == torch::kUInt8 && bits->is_contiguous() && bits->numel() * 8 >= z.numel(),
           "bn_apply bits");
  uint8_t* bp = bits.has_value() ? bits->data_ptr<uint8_t>() : nullptr;
  if (z.scalar_type() == torch::kFloat32)   // (the fp32 train-BN engine)
    ok(pddl::bn_apply_launch(f32p(z), f32p(a), f32p(b), r.has_value() ? f32p(*r) : nullptr, of32p(a2), of32p(b2),
                             relu ? 1 : 0, f32p(y), bp, M, C, cur_stream()),
       "bn_apply");
  else
    ok(pddl::bn_apply_launch(bfp(z), f32p(a), f32p(b), obfp(r), of32p(a2), of32p(b2), relu ? 1 : 0, bfpm(y), bp, M,
                             C, cur_stream()),
       "bn_apply");
}
void bn_bwd_reduce(Tensor g, Tensor z, OptT z2, Tensor mean, OptT mean2, Tensor sg, Tensor sgx, OptT sg2,
                   OptT sgx2) {
  PCHECK(g.is_contiguous() && z.is_contiguous() && g.numel() == z.numel(), "bn_bwd_reduce shapes");
  const int64_t C = z.size(-1);
  PCHECK(mean.numel() >= C && sg.numel() >= C && sgx.numel() >= C, "bn_bwd_reduce per-channel arrays");
  if (z2.has_value())
    PCHECK(z2->is_contiguous() && z2->numel() == z.numel() && mean2.has_value() && sg2.has_value() &&
               sgx2.has_value() && mean2->numel() >= C && sg2->numel() >= C && sgx2->numel() >= C,
           "bn_bwd_reduce z2");
  float* o2 = sg2.has_value() ? f32p(*sg2) : nullptr;
  float* ox2 = sgx2.has_value() ? f32p(*sgx2) : nullptr;
  if (z.scalar_type() == torch::kFloat32)
    ok(pddl::bn_bwd_reduce_launch(f32p(g), f32p(z), z2.has_value() ? f32p(*z2) : nullptr, f32p(mean), of32p(mean2),
                                  rows_of(z), (int)C, f32p(sg), f32p(sgx), o2, ox2, cur_stream()),
       "bn_bwd_reduce");
  else
    ok(pddl::bn_bwd_reduce_launch(bfp(g), bfp(z), obfp(z2), f32p(mean), of32p(mean2), rows_of(z), (int)C, f32p(sg),
                                  f32p(sgx), o2, ox2, cur_stream()),
       "bn_bwd_reduce");
}
pddl::BnBwdLayer bn_layer(const std::vector<double>& v) {
  PCHECK(v.size() == 6, "BN layer: (C, ch, gamma_off, beta_off, bias_off, count)");
  pddl::BnBwdLayer l{};
  l.C = (int)v[0]; l.ch = (int)v[1]; l.gamma_off = (int)v[2]; l.beta_off = (int)v[3]; l.bias_off = (int)v[4];
  l.count = (float)v[5];
  return l;
}
void bn_bwd_apply(Tensor g, Tensor z, OptT z2, std::vector<double> l, std::vector<double> l2, Tensor params,
                  Tensor mean, Tensor inv, Tensor sg, Tensor sgx, Tensor dz, OptT dz2, Tensor grads, Tensor coef) {
  PCHECK(g.is_contiguous() && z.is_contiguous() && dz.is_contiguous() && g.numel() == z.numel() &&
             dz.numel() == z.numel(),
         "bn_bwd_apply shapes");
  const pddl::BnBwdLayer L1 = bn_layer(l);
  PCHECK(L1.C == z.size(-1), "bn_bwd_apply: layer channels");
  pddl::BnBwdLayer L2 = L1;
  if (z2.has_value()) {
    PCHECK(z2->is_contiguous() && z2->numel() == z.numel() && dz2 && dz2->numel() == z.numel(), "bn_bwd_apply z2");
    L2 = bn_layer(l2);
  }
  const int64_t ldc = coef.numel() / 3;
  PCHECK(ldc >= mean.numel() && ldc >= L1.ch + L1.C && ldc >= L2.ch + L2.C, "bn_bwd_apply: coef is [3][>= channels]");
  PCHECK(mean.numel() >= L1.ch + L1.C && mean.numel() >= L2.ch + L2.C && inv.numel() == mean.numel() &&
             sg.numel() >= mean.numel() && sgx.numel() >= mean.numel(),
         "bn_bwd_apply: per-channel arrays too short for the layer offsets");
  if (z.scalar_type() == torch::kFloat32)
    ok(pddl::bn_bwd_apply_launch(f32p(g), f32p(z), z2.has_value() ? f32p(*z2) : nullptr, L1, L2, f32p(params),
                                 f32p(mean), f32p(inv), f32p(sg), f32p(sgx), f32p(coef), (int)ldc, f32p(dz),
                                 dz2.has_value() ? f32p(*dz2) : nullptr, f32p(grads), rows_of(z), cur_stream()),
       "bn_bwd_apply");
  else
    ok(pddl::bn_bwd_apply_launch(bfp(g), bfp(z), obfp(z2), L1, L2, f32p(params), f32p(mean), f32p(inv), f32p(sg),
                                 f32p(sgx), f32p(coef), (int)ldc, bfpm(dz), dz2.has_value() ? bfpm(*dz2) : nullptr,
                                 f32p(grads), rows_of(z), cur_stream()),
       "bn_bwd_apply");
}

void wgrad(Tensor x, int64_t H, int64_t W, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Ho,
           int64_t Wo, Tensor g, OptT g2, int64_t co_split, Tensor dw, int64_t K, int64_t splits) {
  pddl::WgradParams p{};
  PCHECK(x.is_contiguous() && g.stride(-1) == 1, "wgrad operand layout");
  p.x = bfp(x); p.N = (int)x.size(0); p.H = (int)H; p.W = (int)W; p.C = (int)x.size(-1);
  p.ldx = p.C;
  p.R = (int)R; p.S = (int)S; p.stride = (int)stride; p.pad = (int)pad; p.Ho = (int)Ho; p.Wo = (int)Wo;
  p.M = p.N * (int)Ho * (int)Wo;
  p.g = bfp(g); p.ldg = ld(g);
  PCHECK(g.numel() / g.size(-1) == p.M || g.dim() == 2, "gradient rows != N*Ho*Wo");
  if (g2.has_value()) { p.g2 = bfp(*g2); p.ldg2 = ld(*g2); p.co_split = (int)co_split; }
  p.Cout = (int)dw.size(0); p.K = (int)K;
  p.dw = f32p(dw); p.ld_dw = ld(dw);
  PCHECK(dw.size(1) >= K, "dw too narrow");
  p.splits = (int)splits;
  ok(pddl::wgrad_launch(p, cur_stream()), "wgrad");
}

// Fused stride-1 1x1 conv backward (bwd1x1.hip): g [.., CO], x [.., CI], wd [CI][>=CO] bf16,
// bits [.., CI/8] uint8, out [.., CI] bf16, colsum fp32 >= partial rows x CI, dw fp32 [CO][>=CI];
// (CO, CI) = (256, 64) or (512, 128).
void bwd1x1(Tensor g, Tensor x, Tensor wd, Tensor bits, Tensor out, Tensor colsum, Tensor dw, OptT out2, OptT g1,
            OptT w1d, OptT gmask, OptT gx, OptT colsum_gx) {
  pddl::Bwd1x1Params p{};
  if (g1.has_value()) {   // pre form: g = bit(gmask) * (g1 . w1d^T + g) computed per tile, written to gx
    PCHECK(!out2.has_value() && w1d.has_value() && gmask.has_value() && gx.has_value() && colsum_gx.has_value(),
           "bwd1x1 pre form: g1, w1d, gmask, gx, colsum_gx together, stride-1 only");
    PCHECK(g.size(-1) == 256 && g1->size(-1) == 64 && g1->is_contiguous() && rows_of(*g1) == rows_of(g),
           "bwd1x1 pre form: g1 [M,64] next to g [M,256]");
    PCHECK(w1d->dim() == 2 && w1d->size(0) == 256 && w1d->size(1) == 64 && w1d->is_contiguous(), "bwd1x1: w1d [256,64]");
    PCHECK(gmask->scalar_type() == torch::kUInt8 && gmask->numel() == rows_of(g) * 32, "bwd1x1: gmask [M,32] uint8");
    PCHECK(gx->sizes() == g.sizes() && gx->is_contiguous() && gx->scalar_type() == torch::kBFloat16, "bwd1x1: gx like g");
    PCHECK(colsum_gx->numel() >= (int64_t)pddl::bwd1x1_partial_rows((int)rows_of(g), 256, 64) * 256,
           "bwd1x1: colsum_gx too small");
    p.g1 = bfp(*g1); p.w1d = bfp(*w1d); p.gmask = gmask->data_ptr<uint8_t>(); p.gx = bfpm(*gx);
    p.colsum_gx = f32p(*colsum_gx);
  }
  PCHECK(g.is_contiguous() && x.is_contiguous() && out.is_contiguous() && bits.is_contiguous(), "bwd1x1: contiguous operands");
  const int64_t CO = g.size(-1), CI = x.size(-1);
  PCHECK((CO == 256 && CI == 64) || (CO == 512 && CI == 128), "bwd1x1: (CO, CI) must be (256, 64) or (512, 128)");
  PCHECK(out.size(-1) == CI && bits.size(-1) == CI / 8, "bwd1x1: out / bits channel counts");
  const int64_t M = rows_of(g);
  if (out2.has_value()) {   // stride-2 form: g / out2 on the compact grid of x / out / bits
    PCHECK(g.dim() == 4 && x.dim() == 4 && out.sizes() == x.sizes() && out2->is_contiguous() && rows_of(*out2) == M &&
               out2->size(-1) == CI && g.size(0) == x.size(0) && g.size(1) == (x.size(1) + 1) / 2 &&
               g.size(2) == (x.size(2) + 1) / 2 && rows_of(bits) == rows_of(x),
           "bwd1x1: stride-2 form needs g [N,Hc,Wc,CO], x / out [N,Hf,Wf,CI], bits [.., CI/8] at x's rows, out2 [N,Hc,Wc,CI]");
    p.s2 = 1; p.N = (int)x.size(0); p.Hf = (int)x.size(1); p.Wf = (int)x.size(2); p.Hc = (int)g.size(1);
    p.Wc = (int)g.size(2); p.out2 = bfpm(*out2);
    PCHECK((int64_t)p.N * p.Hf * p.Wf * CI < (1LL << 31), "bwd1x1: more than 2^31 elements");
  } else {
    PCHECK(rows_of(x) == M && rows_of(out) == M && rows_of(bits) == M, "bwd1x1: row counts differ");
  }
  PCHECK(bits.is_cuda() && bits.scalar_type() == torch::kUInt8, "bwd1x1: bits must be a uint8 GPU tensor");
  PCHECK(wd.dim() == 2 && wd.size(0) == CI && wd.size(1) >= CO, "bwd1x1: wd must be [CI][>=CO]");
  PCHECK(dw.dim() == 2 && dw.size(0) == CO && dw.size(1) >= CI, "bwd1x1: dw must be [CO][>=CI]");
  PCHECK(colsum.is_contiguous() && colsum.numel() >= (int64_t)pddl::bwd1x1_partial_rows((int)M, (int)CO, (int)CI) * CI,
         "bwd1x1: colsum too small");
  p.g = bfp(g); p.x = bfp(x); p.wd = bfp(wd); p.ld_wd = ld(wd); p.bits = bits.data_ptr<uint8_t>();
  p.out = bfpm(out); p.colsum = f32p(colsum); p.dw = f32p(dw); p.ld_dw = ld(dw);
  p.M = (int)M; p.CO = (int)CO; p.CI = (int)CI;
  ok(pddl::bwd1x1_launch(p, cur_stream()), "bwd1x1");
}
int64_t bwd1x1_partial_rows(int64_t M, int64_t CO, int64_t CI) {
  return pddl::bwd1x1_partial_rows((int)M, (int)CO, (int)CI);
}

// fp32 convolution (reference precision): y[N,Ho,Wo,Cout] = conv(x[N,H,W,C], w[Cout, R*S*C]) (+ bias)
// the calling engine's split-K workspace (splitk_use) for the fp32 conv launcher's small-M slices
static void f32_splitk(pddl::ConvF32Params& p, const Tensor& x) {
  if (tls_splitk.defined() && tls_splitk.device() == x.device()) {
    p.slab = tls_splitk.data_ptr<float>();
    p.slab_floats = tls_splitk.numel();
  }
}

void conv_f32(Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, Tensor w, OptT bias, Tensor y) {
  pddl::ConvF32Params p{};
  PCHECK(x.is_contiguous() && x.dim() == 4 && w.is_contiguous() && y.is_contiguous() && y.dim() == 4,
         "conv_f32: contiguous NHWC x / y and [Cout, K] w");
  p.x = f32p(x); p.N = (int)x.size(0); p.H = (int)x.size(1); p.W = (int)x.size(2); p.C = (int)x.size(3);
  p.R = (int)R; p.S = (int)S; p.stride = (int)stride; p.pad = (int)pad;
  p.Ho = (int)y.size(1); p.Wo = (int)y.size(2); p.M = p.N * p.Ho * p.Wo;
  PCHECK(y.size(0) == p.N && p.Ho == (p.H + 2 * p.pad - p.R) / p.stride + 1 &&
         p.Wo == (p.W + 2 * p.pad - p.S) / p.stride + 1, "conv_f32: output shape");
  p.w = f32p(w); p.Cout = (int)w.size(0); p.K = (int)w.size(1);
  PCHECK(y.size(3) == p.Cout && p.K == p.R * p.S * p.C, "conv_f32: weight shape");
  if (bias.has_value()) { PCHECK(bias->numel() == p.Cout, "conv_f32: bias"); p.bias = f32p(*bias); }
  p.y = f32p(y);
  f32_splitk(p, x);
  ok(pddl::conv_f32_launch(p, cur_stream()), "conv_f32");
}

// conv_f32 with a fused epilogue (the fp32 engine): epi 1 = FWD (scale/shift [+res] [relu]),
// epi 2 = DGRAD ([+add] * (mask > 0), up2 grid scatter into y of [N, Hf, Wf, Cout], partial
// column sums [ceil(M/64)][Cout]).  x / y NHWC fp32; w [Cout][K] rows with row stride K.
void conv_f32_epi(Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Ho, int64_t Wo, Tensor w,
                  int64_t epi, OptT scale, OptT shift, OptT res, int64_t relu, OptT add, OptT mask, int64_t up2,
                  Tensor y, OptT colsum) {
  pddl::ConvF32Params p{};
  PCHECK(x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.is_contiguous() && x.dim() == 4,
         "conv_f32_epi: contiguous fp32 NHWC x");
  PCHECK(w.is_contiguous() && w.dim() == 2 && y.is_contiguous() && y.dim() == 4, "conv_f32_epi: w [Cout][K], NHWC y");
  p.x = f32p(x); p.N = (int)x.size(0); p.H = (int)x.size(1); p.W = (int)x.size(2); p.C = (int)x.size(3);
  p.R = (int)R; p.S = (int)S; p.stride = (int)stride; p.pad = (int)pad;
  p.Ho = (int)Ho; p.Wo = (int)Wo; p.M = p.N * p.Ho * p.Wo;
  PCHECK(p.Ho == (p.H + 2 * p.pad - p.R) / p.stride + 1 && p.Wo == (p.W + 2 * p.pad - p.S) / p.stride + 1,
         "conv_f32_epi: output size");
  p.w = f32p(w); p.Cout = (int)w.size(0); p.K = (int)w.size(1);
  PCHECK(p.K == p.R * p.S * p.C, "conv_f32_epi: K must be R*S*C");
  PCHECK(y.size(0) == p.N && y.size(3) == p.Cout, "conv_f32_epi: output batch / channels");
  if (up2) {
    PCHECK(epi == pddl::F32_EPI_DGRAD, "conv_f32_epi: up2 is a dgrad scatter");
    p.Hf = (int)y.size(1); p.Wf = (int)y.size(2);
  } else {
    PCHECK(y.size(1) == p.Ho && y.size(2) == p.Wo, "conv_f32_epi: output shape");
  }
  const int64_t out_el = y.numel();
  auto same = [&](const OptT& t, const char* what) {
    PCHECK(!t.has_value() || (t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous() &&
                              t->numel() == out_el), what);
  };
  same(res, "conv_f32_epi: res must match y");
  if (up2) {
    PCHECK(!add.has_value() || (add->is_contiguous() && add->scalar_type() == torch::kFloat32 &&
                                add->numel() == (int64_t)p.M * p.Cout),
           "conv_f32_epi: with up2, add is the compact [N, Ho, Wo, Cout] tensor");
  } else {
    same(add, "conv_f32_epi: add must match y");
  }
  same(mask, "conv_f32_epi: mask must match y");
  p.epi = (int)epi;
  if (epi == pddl::F32_EPI_FWD) {
    PCHECK(scale.has_value() && shift.has_value() && scale->numel() >= p.Cout && shift->numel() >= p.Cout,
           "conv_f32_epi: forward scale / shift");
  }
  p.scale = of32p(scale); p.shift = of32p(shift);
  p.res = of32p(res); p.relu = (int)relu;
  p.add = of32p(add); p.mask = of32p(mask); p.up2 = (int)up2;
  if (colsum.has_value()) {
    PCHECK(epi == pddl::F32_EPI_DGRAD && colsum->numel() >= (int64_t)((p.M + 63) / 64) * p.Cout,
           "conv_f32_epi: colsum partial rows [ceil(M/64)][Cout] of a dgrad");
    p.colsum = f32p(*colsum);
  }
  p.y = f32p(y);
  f32_splitk(p, x);
  ok(pddl::conv_f32_launch(p, cur_stream()), "conv_f32_epi");
}

void maxpool_fwd_f32(Tensor x, Tensor y, Tensor idx) {
  PCHECK(x.dim() == 4 && y.dim() == 4 && x.is_contiguous() && y.is_contiguous() && idx.numel() == y.numel() &&
             idx.scalar_type() == torch::kUInt8, "maxpool_fwd_f32 shapes");
  ok(pddl::maxpool_fwd_f32_launch(f32p(x), f32p(y), idx.data_ptr<uint8_t>(), (int)x.size(0), (int)x.size(1),
                                  (int)x.size(2), (int)x.size(3), (int)y.size(1), (int)y.size(2), cur_stream()),
     "maxpool_fwd_f32");
}
void maxpool_bwd_f32(Tensor gy, Tensor idx, Tensor xmask, Tensor gx) {
  PCHECK(gx.dim() == 4 && gy.dim() == 4 && gx.is_contiguous() && gy.is_contiguous() && xmask.numel() == gx.numel() &&
             idx.numel() == gy.numel(), "maxpool_bwd_f32 shapes");
  ok(pddl::maxpool_bwd_f32_launch(f32p(gy), idx.data_ptr<uint8_t>(), f32p(xmask), f32p(gx), (int)gx.size(0),
                                  (int)gx.size(1), (int)gx.size(2), (int)gx.size(3), (int)gy.size(1), (int)gy.size(2),
                                  cur_stream()),
     "maxpool_bwd_f32");
}
void gap_fwd_f32(Tensor x, Tensor y) {
  PCHECK(x.dim() == 4 && x.is_contiguous() && y.numel() == x.size(0) * x.size(3), "gap_fwd_f32 shapes");
  ok(pddl::gap_fwd_f32_launch(f32p(x), f32p(y), (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(3),
                              cur_stream()), "gap_fwd_f32");
}
void gap_bwd_f32(Tensor gp, Tensor ymask, Tensor g, OptT colsum_rows) {
  PCHECK(g.dim() == 4 && g.is_contiguous() && ymask.numel() == g.numel() && gp.numel() == g.size(0) * g.size(3),
         "gap_bwd_f32 shapes");
  if (colsum_rows.has_value()) PCHECK(colsum_rows->numel() >= gp.numel(), "gap_bwd_f32 colsum rows [B][C]");
  ok(pddl::gap_bwd_f32_launch(f32p(gp), f32p(ymask), f32p(g), (int)g.size(0), (int)(g.size(1) * g.size(2)),
                              (int)g.size(3), colsum_rows.has_value() ? f32p(*colsum_rows) : nullptr, cur_stream()),
     "gap_bwd_f32");
}
void colsum_f32(Tensor g, int64_t C, Tensor out) {
  PCHECK(g.is_contiguous() && out.numel() >= C, "colsum_f32 shapes");
  ok(pddl::colsum_f32_launch(f32p(g), g.numel() / ld(g), (int)C, ld(g), f32p(out), cur_stream()), "colsum_f32");
}
void softmax_xent_f32(Tensor logits, Tensor labels, int64_t ncls, double gscale, Tensor dlogits, Tensor loss_sum,
                      Tensor correct) {
  PCHECK(labels.scalar_type() == torch::kInt64 && labels.is_cuda(), "labels int64 GPU");
  ok(pddl::softmax_xent_f32_launch(f32p(logits), ld(logits), labels.data_ptr<int64_t>(), (int)logits.size(0),
                                   (int)ncls, (float)gscale, f32p(dlogits), ld(dlogits), f32p(loss_sum),
                                   f32p(correct), cur_stream()),
     "softmax_xent_f32");
}
void prep_f32(Tensor params, Tensor table, int64_t nlayers, Tensor wf32, Tensor scale, Tensor shift, double eps) {
  PCHECK(table.is_cuda() && table.scalar_type() == torch::kUInt8, "prep table");
  PCHECK(table.numel() == nlayers * (int64_t)sizeof(pddl::PrepLayer), "prep table size");
  ok(pddl::prep_f32_launch(f32p(params), reinterpret_cast<const pddl::PrepLayer*>(table.data_ptr()), (int)nlayers,
                           f32p(wf32), f32p(scale), f32p(shift), (float)eps, cur_stream()),
     "prep_f32");
}

// dw[Cout, R*S*C] += sum_m dy[m, Cout] * im2col(x)[m, :]
void wgrad_f32(Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, Tensor dy, Tensor dw) {
  pddl::ConvF32Params p{};
  PCHECK(x.is_contiguous() && x.dim() == 4 && dy.is_contiguous() && dy.dim() == 4 && dw.is_contiguous(),
         "wgrad_f32: contiguous NHWC x / dy and [Cout, K] dw");
  p.x = f32p(x); p.N = (int)x.size(0); p.H = (int)x.size(1); p.W = (int)x.size(2); p.C = (int)x.size(3);
  p.R = (int)R; p.S = (int)S; p.stride = (int)stride; p.pad = (int)pad;
  p.Ho = (int)dy.size(1); p.Wo = (int)dy.size(2); p.M = p.N * p.Ho * p.Wo;
  PCHECK(dy.size(0) == p.N && p.Ho == (p.H + 2 * p.pad - p.R) / p.stride + 1 &&
         p.Wo == (p.W + 2 * p.pad - p.S) / p.stride + 1, "wgrad_f32: gradient shape");
  p.Cout = (int)dy.size(3); p.K = p.R * p.S * p.C;
  PCHECK(dw.size(0) == p.Cout && dw.numel() == (int64_t)p.Cout * p.K, "wgrad_f32: dw shape");
  p.y = f32p(dy); p.dw = f32p(dw);
  ok(pddl::wgrad_f32_launch(p, cur_stream()), "wgrad_f32");
}

void stem_s2d(Tensor in, OptT flip, int64_t mode, int64_t Hc, int64_t Wc, int64_t oy, int64_t ox, Tensor out,
              OptT crop_dev) {
  pddl::StemParams p{};
  PCHECK(in.is_cuda() && in.is_contiguous() && in.dim() == 4 && in.size(3) == 3, "stem input must be [B,H,W,3]");
  PCHECK(in.scalar_type() == torch::kUInt8 || in.scalar_type() == torch::kFloat32, "stem input uint8 or fp32");
  p.in = in.data_ptr(); p.in_u8 = in.scalar_type() == torch::kUInt8;
  p.B = (int)in.size(0); p.Hin = (int)in.size(1); p.Win = (int)in.size(2);
  p.Hc = (int)Hc; p.Wc = (int)Wc; p.mode = (int)mode; p.oy = (int)oy; p.ox = (int)ox;
  if (mode == 2) PCHECK(oy >= 0 && ox >= 0 && oy + Hc <= p.Hin && ox + Wc <= p.Win, "crop window out of range");
  if (crop_dev.has_value()) {
    // the caller keeps the device offsets within [0, Hin - Hc] x [0, Win - Wc]
    PCHECK(crop_dev->is_cuda() && crop_dev->scalar_type() == torch::kInt32 && crop_dev->numel() >= 2,
           "crop_dev: device int32[2]");
    p.crop_dev = crop_dev->data_ptr<int32_t>();
  }
  if (flip.has_value()) {
    PCHECK(flip->scalar_type() == torch::kUInt8 && flip->numel() == p.B && flip->is_cuda(), "flip flags [B] uint8");
    p.flip = flip->data_ptr<uint8_t>();
  }
  p.scale = 1.f / 255.f;
  p.Hs = (int)((Hc + 6) / 2); p.Ws = (int)((Wc + 6) / 2);
  PCHECK(out.is_contiguous() && out.numel() >= (int64_t)p.B * p.Hs * p.Ws * 16, "stem s2d output too small");
  if (out.scalar_type() == torch::kFloat32) {   // the fp32 engine's stem image
    ok(pddl::stem_s2d_f32_launch(p, f32p(out), cur_stream()), "stem_s2d_f32");
    return;
  }
  p.out = bfpm(out);
  ok(pddl::stem_s2d_launch(p, cur_stream()), "stem_s2d");
}
void stem_wgrad_fold(Tensor g2, Tensor dw, int64_t cout) {
  PCHECK(g2.numel() >= cout * 256 && dw.numel() >= cout * 147, "stem fold sizes");
  ok(pddl::stem_wgrad_fold_launch(f32p(g2), f32p(dw), (int)cout, cur_stream()), "stem_wgrad_fold");
}
void maxpool_fwd(Tensor x, Tensor y, Tensor idx, OptT bits) {
  PCHECK(x.is_contiguous() && y.is_contiguous() && idx.is_contiguous() && idx.scalar_type() == torch::kUInt8,
         "maxpool layouts");
  if (bits.has_value())
    PCHECK(bits->scalar_type() == torch::kUInt8 && bits->is_contiguous() && bits->numel() * 8 >= y.numel(),
           "maxpool bits [B,Ho,Wo,C/8] uint8");
  ok(pddl::maxpool_fwd_launch(bfp(x), bfpm(y), idx.data_ptr<uint8_t>(),
                              bits.has_value() ? bits->data_ptr<uint8_t>() : nullptr, (int)x.size(0), (int)x.size(1),
                              (int)x.size(2), (int)x.size(3), (int)y.size(1), (int)y.size(2), cur_stream()),
     "maxpool_fwd");
}
// Fused stem: x2 [B,Hs,Ws,16] bf16, w [64,>=256] bf16 rows, scale/shift fp32 [>=64] ->
// pool [B,H2,W2,64] bf16, idx uint8 same shape, bits (optional) [B,H2,W2,8] uint8.
void stem_pool_fwd(Tensor x2, Tensor w, Tensor scale, Tensor shift, Tensor pool, Tensor idx, OptT bits,
                   int64_t pool_rows) {
  PCHECK(x2.dim() == 4 && x2.size(3) == 16 && x2.is_contiguous(), "stem_pool: x2 [B,Hs,Ws,16] contiguous");
  PCHECK(w.dim() == 2 && w.size(0) == 64 && w.size(1) == 256 && w.stride(1) == 1 && w.stride(0) == 256,
         "stem_pool: w [64,256] contiguous");
  PCHECK(scale.numel() >= 64 && shift.numel() >= 64, "stem_pool: 64 scale / shift values");
  PCHECK(pool.dim() == 4 && pool.size(3) == 64 && pool.is_contiguous() && pool.size(0) == x2.size(0),
         "stem_pool: pool [B,H2,W2,64] contiguous");
  PCHECK(idx.scalar_type() == torch::kUInt8 && idx.is_contiguous() && idx.numel() == pool.numel(),
         "stem_pool: idx uint8 like pool");
  if (bits.has_value())
    PCHECK(bits->scalar_type() == torch::kUInt8 && bits->is_contiguous() && bits->numel() * 8 == pool.numel(),
           "stem_pool: bits [B,H2,W2,8] uint8");
  PCHECK((reinterpret_cast<uintptr_t>(scale.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(shift.data_ptr()) & 15) == 0,
         "stem_pool: 16-byte aligned scale / shift");
  pddl::StemPoolParams p{};
  p.x2 = bfp(x2); p.w = bfp(w); p.scale = f32p(scale); p.shift = f32p(shift);
  p.pool = bfpm(pool); p.idx = idx.data_ptr<uint8_t>(); p.bits = bits.has_value() ? bits->data_ptr<uint8_t>() : nullptr;
  p.B = (int)x2.size(0); p.Hs = (int)x2.size(1); p.Ws = (int)x2.size(2);
  p.H1 = p.Hs - 3; p.W1 = p.Ws - 3; p.H2 = (int)pool.size(1); p.W2 = (int)pool.size(2);
  p.PB = (int)pool_rows;
  ok(pddl::stem_pool_fwd_launch(p, cur_stream()), "stem_pool_fwd");
}
// Fused stem backward: gpool / idx [B,H2,W2,64], x2 [B,Hs,Ws,16] -> dw [64,256] fp32 (added),
// colsum partial rows [stem_pool_bwd_partial_rows, 64].
void stem_pool_bwd(Tensor x2, Tensor gpool, Tensor idx, Tensor dw, Tensor colsum, int64_t pool_rows) {
  PCHECK(x2.dim() == 4 && x2.size(3) == 16 && x2.is_contiguous(), "stem_pool_bwd: x2 [B,Hs,Ws,16] contiguous");
  PCHECK(gpool.dim() == 4 && gpool.size(3) == 64 && gpool.is_contiguous() && gpool.size(0) == x2.size(0),
         "stem_pool_bwd: gpool [B,H2,W2,64] contiguous");
  PCHECK(idx.scalar_type() == torch::kUInt8 && idx.is_contiguous() && idx.numel() == gpool.numel(),
         "stem_pool_bwd: idx uint8 like gpool");
  PCHECK(dw.is_contiguous() && dw.numel() >= 64 * 256, "stem_pool_bwd: dw [64,256] fp32");
  pddl::StemPoolBwdParams p{};
  p.x2 = bfp(x2); p.gpool = bfp(gpool); p.idx = idx.data_ptr<uint8_t>(); p.dw = f32p(dw);
  p.B = (int)x2.size(0); p.Hs = (int)x2.size(1); p.Ws = (int)x2.size(2);
  p.H1 = p.Hs - 3; p.W1 = p.Ws - 3; p.H2 = (int)gpool.size(1); p.W2 = (int)gpool.size(2);
  p.PB = (int)pool_rows;
  PCHECK(colsum.numel() >= (int64_t)pddl::stem_pool_bwd_partial_rows(p.B, p.H2, p.PB) * 64,
         "stem_pool_bwd: colsum needs stem_pool_bwd_partial_rows x 64 floats");
  p.colsum = f32p(colsum);
  ok(pddl::stem_pool_bwd_launch(p, cur_stream()), "stem_pool_bwd");
}
// 3x3 / pad 1 / stride 1 convolution 64 -> 64 on the persistent row-tile kernel.
// mode 0 (forward): out = relu(conv(x, w) * scale + shift), bits = its ReLU bits (optional);
// mode 1 (data gradient): out = conv(x, w) masked by `bits` (input ReLU bits, required),
// colsum = partial rows [conv3x3c64_partial_rows(M), 64] of out's column sums (optional).
void conv3x3c64(Tensor x, Tensor w, int64_t mode, Tensor out, OptT scale, OptT shift, OptT bits, OptT colsum) {
  PCHECK(x.dim() == 4 && x.size(3) == 64 && x.is_contiguous() && x.scalar_type() == torch::kBFloat16,
         "conv3x3c64: x [N,H,W,64] bf16 contiguous");
  PCHECK(out.sizes() == x.sizes() && out.is_contiguous() && out.scalar_type() == torch::kBFloat16,
         "conv3x3c64: out like x");
  PCHECK(w.dim() == 2 && w.size(0) == 64 && w.size(1) == 576 && w.stride(1) == 1 && w.stride(0) == 576,
         "conv3x3c64: w [64,576] contiguous rows");
  pddl::C64Params p{};
  p.x = bfp(x); p.w = bfp(w); p.out = bfpm(out);
  p.N = (int)x.size(0); p.H = (int)x.size(1); p.W = (int)x.size(2);
  PCHECK((int64_t)p.N * p.H * p.W < (1LL << 30), "conv3x3c64: too many pixels");
  p.M = p.N * p.H * p.W;
  if (bits.has_value())
    PCHECK(bits->scalar_type() == torch::kUInt8 && bits->is_contiguous() && bits->numel() == (int64_t)p.M * 8,
           "conv3x3c64: bits [N,H,W,8] uint8");
  if (mode == pddl::C64_FWD) {
    PCHECK(scale.has_value() && shift.has_value() && scale->numel() >= 64 && shift->numel() >= 64,
           "conv3x3c64: forward needs 64 scale / shift values");
    PCHECK((reinterpret_cast<uintptr_t>(scale->data_ptr()) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(shift->data_ptr()) & 15) == 0, "conv3x3c64: 16-byte aligned scale / shift");
    p.scale = f32p(*scale); p.shift = f32p(*shift);
    p.bits_out = bits.has_value() ? bits->data_ptr<uint8_t>() : nullptr;
  } else {
    PCHECK(mode == pddl::C64_DGRAD && bits.has_value(), "conv3x3c64: mode 1 needs the ReLU bits");
    p.bits_mask = bits->data_ptr<uint8_t>();
    if (colsum.has_value()) {
      PCHECK(colsum->numel() >= (int64_t)pddl::conv3x3c64_partial_rows(p.M) * 64,
             "conv3x3c64: colsum needs conv3x3c64_partial_rows x 64 floats");
      p.colsum = f32p(*colsum);
    }
  }
  ok(pddl::conv3x3c64_launch(p, (int)mode, cur_stream()), "conv3x3c64");
}
// Weight gradient of the 64 -> 64 3x3 / pad 1 conv: dw [64, >=576] fp32 += (x, g) correlation.
void conv3x3c64_wgrad(Tensor x, Tensor g, Tensor dw) {
  PCHECK(x.dim() == 4 && x.size(3) == 64 && x.is_contiguous() && x.scalar_type() == torch::kBFloat16,
         "conv3x3c64_wgrad: x [N,H,W,64] bf16 contiguous");
  PCHECK(g.sizes() == x.sizes() && g.is_contiguous() && g.scalar_type() == torch::kBFloat16,
         "conv3x3c64_wgrad: g like x");
  PCHECK(dw.dim() == 2 && dw.size(0) == 64 && dw.size(1) >= 576 && dw.stride(1) == 1 &&
         dw.scalar_type() == torch::kFloat32, "conv3x3c64_wgrad: dw [64, >=576] fp32 rows");
  pddl::C64WgradParams p{};
  p.x = bfp(x); p.g = bfp(g); p.dw = f32p(dw); p.ld_dw = (int)dw.stride(0);
  p.N = (int)x.size(0); p.H = (int)x.size(1); p.W = (int)x.size(2);
  ok(pddl::conv3x3c64_wgrad_launch(p, cur_stream()), "conv3x3c64_wgrad");
}
// Fused 64-channel bottleneck boundary: out = relu(a . w3^T * scale3 + shift3 (+ res)), bits3;
// y1 = relu(out . w1^T * scale1 + shift1), bits1 (a2: second K source of the fused projection).
void c3c1(Tensor a, Tensor w3, Tensor scale3, Tensor shift3, OptT res, Tensor out, OptT bits3, Tensor w1,
          Tensor scale1, Tensor shift1, Tensor y1, OptT bits1) {
  PCHECK(a.size(-1) == 64 && a.is_contiguous() && a.scalar_type() == torch::kBFloat16, "c3c1: a [..,64] bf16");
  const int64_t M = a.numel() / 64;
  PCHECK(M < (1LL << 30), "c3c1: too many rows");
  PCHECK(w3.dim() == 2 && w3.size(0) == 256 && w3.size(1) == 64 && w3.is_contiguous(), "c3c1: w3 [256, 64]");
  PCHECK(w1.dim() == 2 && w1.size(0) == 64 && w1.size(1) == 256 && w1.is_contiguous(), "c3c1: w1 [64, 256]");
  PCHECK(scale3.numel() >= 256 && shift3.numel() >= 256 && scale1.numel() >= 64 && shift1.numel() >= 64,
         "c3c1: scale / shift sizes");
  for (const Tensor* t : {&scale3, &shift3, &scale1, &shift1})
    PCHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "c3c1: 16-byte aligned scale / shift");
  PCHECK(out.numel() == M * 256 && out.is_contiguous() && out.scalar_type() == torch::kBFloat16, "c3c1: out [M,256]");
  PCHECK(y1.numel() == M * 64 && y1.is_contiguous() && y1.scalar_type() == torch::kBFloat16, "c3c1: y1 [M,64]");
  if (res.has_value()) PCHECK(res->numel() == M * 256 && res->is_contiguous(), "c3c1: res [M,256]");
  if (bits3.has_value()) PCHECK(bits3->numel() == M * 32 && bits3->scalar_type() == torch::kUInt8, "c3c1: bits3 [M,32]");
  if (bits1.has_value()) PCHECK(bits1->numel() == M * 8 && bits1->scalar_type() == torch::kUInt8, "c3c1: bits1 [M,8]");
  pddl::C3C1Params p{};
  p.a = bfp(a); p.w3 = bfp(w3);
  p.scale3 = f32p(scale3); p.shift3 = f32p(shift3); p.res = obfp(res); p.out = bfpm(out);
  p.bits3 = bits3.has_value() ? bits3->data_ptr<uint8_t>() : nullptr;
  p.w1 = bfp(w1); p.scale1 = f32p(scale1); p.shift1 = f32p(shift1); p.y1 = bfpm(y1);
  p.bits1 = bits1.has_value() ? bits1->data_ptr<uint8_t>() : nullptr;
  p.M = (int)M;
  ok(pddl::c3c1_launch(p, cur_stream()), "c3c1");
}
void maxpool_bwd(Tensor gy, Tensor idx, OptT xmask, Tensor gx, OptT colsum) {
  ok(pddl::maxpool_bwd_launch(bfp(gy), idx.data_ptr<uint8_t>(), obfp(xmask), bfpm(gx), (int)gx.size(0),
                              (int)gx.size(1), (int)gx.size(2), (int)gx.size(3), (int)gy.size(1), (int)gy.size(2),
                              colsum.has_value() ? f32p(*colsum) : nullptr, cur_stream()),
     "maxpool_bwd");
}
void gap_fwd(Tensor x, Tensor y) {
  ok(pddl::gap_fwd_launch(bfp(x), bfpm(y), (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(3),
                          cur_stream()),
     "gap_fwd");
}
void gap_bwd(Tensor gp, Tensor ymask, Tensor g, OptT colsum) {
  ok(pddl::gap_bwd_launch(bfp(gp), ld(gp), bfp(ymask), bfpm(g), (int)g.size(0), (int)(g.size(1) * g.size(2)),
                          (int)g.size(3), colsum.has_value() ? f32p(*colsum) : nullptr, cur_stream()),
     "gap_bwd");
}
void colsum(Tensor g, int64_t C, Tensor out) {
  const int ldg = ld(g);
  const int64_t M = g.numel() / g.size(-1);
  ok(pddl::colsum_launch(bfp(g), (int)M, (int)C, ldg, f32p(out), cur_stream()), "colsum");
}
void colsum_reduce(Tensor part, Tensor table, int64_t nlayers, Tensor colsum) {
  PCHECK(table.numel() == nlayers * (int64_t)sizeof(pddl::ColRedLayer), "colsum_reduce table size");
  ok(pddl::colsum_reduce_launch(f32p(part), reinterpret_cast<const pddl::ColRedLayer*>(table.data_ptr()),
                                (int)nlayers, f32p(colsum), cur_stream()),
     "colsum_reduce");
}
void softmax_xent(Tensor logits, Tensor labels, int64_t ncls, double gscale, Tensor dlogits, Tensor loss_sum,
                  Tensor correct) {
  PCHECK(labels.scalar_type() == torch::kInt64 && labels.is_cuda(), "labels int64 GPU");
  ok(pddl::softmax_xent_launch(f32p(logits), ld(logits), labels.data_ptr<int64_t>(), (int)logits.size(0),
                               (int)ncls, (float)gscale, bfpm(dlogits), ld(dlogits), f32p(loss_sum),
                               f32p(correct), cur_stream()),
     "softmax_xent");
}
void prep(Tensor params, Tensor table, int64_t nlayers, int64_t max_elems, Tensor wbf, Tensor scale, Tensor shift,
          double eps, int64_t parts) {
  PCHECK(table.is_cuda() && table.scalar_type() == torch::kUInt8, "prep table");
  PCHECK(table.numel() == nlayers * (int64_t)sizeof(pddl::PrepLayer), "prep table size");
  PCHECK(parts >= 1 && parts <= 3, "prep: parts 1 (forward), 2 (dgrad) or 3 (both)");
  ok(pddl::prep_launch(f32p(params), reinterpret_cast<const pddl::PrepLayer*>(table.data_ptr()), (int)nlayers,
                       (int)max_elems, bfpm(wbf), f32p(scale), f32p(shift), (float)eps, cur_stream(), (int)parts),
     "prep");
}
void prep_fuse(Tensor params, Tensor table, int64_t nlayers, int64_t max_elems, Tensor wbf, Tensor scale, Tensor shift,
               double eps) {
  PCHECK(table.is_cuda() && table.scalar_type() == torch::kUInt8, "prep_fuse table");
  PCHECK(table.numel() == nlayers * (int64_t)sizeof(pddl::FuseLayer), "prep_fuse table size");
  ok(pddl::prep_fuse_launch(f32p(params), reinterpret_cast<const pddl::FuseLayer*>(table.data_ptr()), (int)nlayers,
                            (int)max_elems, bfpm(wbf), f32p(scale), f32p(shift), (float)eps, cur_stream()),
     "prep_fuse");
}
void wgrad_finalize(Tensor params, Tensor grads, Tensor table, int64_t nlayers, Tensor scale, Tensor dgamma_raw,
                    int64_t max_cout) {
  PCHECK(table.numel() == nlayers * (int64_t)sizeof(pddl::FinLayer), "finalize table size");
  ok(pddl::wgrad_finalize_launch(f32p(params), f32p(grads), reinterpret_cast<const pddl::FinLayer*>(table.data_ptr()),
                                 (int)nlayers, f32p(scale), f32p(dgamma_raw), cur_stream(), (int)max_cout),
     "wgrad_finalize");
}
void bn_grad(Tensor params, Tensor grads, Tensor table, int64_t nlayers, Tensor colsum, Tensor dgamma_raw,
             Tensor scale, double eps) {
  PCHECK(table.numel() == nlayers * (int64_t)sizeof(pddl::BnGradLayer), "bn_grad table size");
  ok(pddl::bn_grad_launch(f32p(params), f32p(grads), reinterpret_cast<const pddl::BnGradLayer*>(table.data_ptr()),
                          (int)nlayers, f32p(colsum), f32p(dgamma_raw), f32p(scale), (float)eps, cur_stream()),
     "bn_grad");
}
void synth(Tensor idx, int64_t seed, int64_t ncls, Tensor img, Tensor lab) {
  PCHECK(idx.is_cuda() && idx.scalar_type() == torch::kInt64 && img.scalar_type() == torch::kUInt8 &&
             lab.scalar_type() == torch::kInt64 && img.is_contiguous() && img.size(0) == idx.numel() &&
             lab.numel() == idx.numel(),
         "synth: idx int64 [n], img uint8 [n,...], lab int64 [n]");
  ok(pddl::synth_launch(idx.data_ptr<int64_t>(), (int)idx.numel(), (long)(img.numel() / std::max<int64_t>(1, idx.numel())),
                        seed, (int)ncls, img.data_ptr<uint8_t>(), lab.data_ptr<int64_t>(), cur_stream()),
     "synth");
}
void opt_hparams(Tensor hs, double b1, double b2, bool adam) {
  PCHECK(hs.is_cuda() && hs.scalar_type() == torch::kFloat32 && hs.numel() >= 3, "hparams: device float[>=3]");
  ok(pddl::opt_hparams_launch(f32p(hs), (float)b1, (float)b2, adam ? 1 : 0, cur_stream()), "opt_hparams");
}
void adam(Tensor p, Tensor g, Tensor m, Tensor v, double lr_t, double b1, double b2, double eps, double gscale,
          OptT hs) {
  ok(pddl::adam_launch(f32p(p), f32p(g), f32p(m), f32p(v), p.numel(), (float)lr_t, (float)b1, (float)b2, (float)eps,
                       (float)gscale, of32p(hs), cur_stream()),
     "adam");
}
void sgd(Tensor p, Tensor g, Tensor mom, double lr, double momentum, double wd, bool nesterov, double gscale,
         OptT hs) {
  ok(pddl::sgd_launch(f32p(p), f32p(g), f32p(mom), p.numel(), (float)lr, (float)momentum, (float)wd,
                      nesterov ? 1 : 0, (float)gscale, of32p(hs), cur_stream()),
     "sgd");
}
void scale_(Tensor x, double a) { ok(pddl::scale_launch(f32p(x), x.numel(), (float)a, cur_stream()), "scale"); }
void cast_bf16(Tensor x, Tensor y) { ok(pddl::cast_bf16_launch(f32p(x), bfpm(y), x.numel(), cur_stream()), "cast"); }
void cast_f32(Tensor x, Tensor y) { ok(pddl::cast_f32_launch(bfp(x), f32p(y), x.numel(), cur_stream()), "cast"); }

}  // namespace

void register_rccl(pybind11::module& m);
void register_fusion(pybind11::module& m);
void register_loader(pybind11::module& m);
void register_ps(pybind11::module& m);
void register_crash_trace(pybind11::module& m);
void register_graph_launch(pybind11::module& m);

// Kernel launches release the GIL: replica threads (Mirrored / multi-GPU workers) then enqueue
// their launch streams concurrently instead of serializing on the interpreter lock.
#define REL py::call_guard<py::gil_scoped_release>()

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "pddl MI355X (gfx950) HIP kernels + native runtime (RCCL comm, fusion engine, loader)";
  register_rccl(m);
  register_fusion(m);
  register_loader(m);
  register_ps(m);
  register_crash_trace(m);
  register_graph_launch(m);
  // rows: host int64 [n, 3] of (flat offset, packed offset, length), bounds-checked here
  m.def("range_copy", [](Tensor src, Tensor dst, Tensor rows, bool scatter) {
    PCHECK(!rows.is_cuda() && rows.scalar_type() == torch::kInt64 && rows.dim() == 2 && rows.size(1) == 3,
           "range rows: host int64 [n, 3]");
    Tensor r = rows.contiguous();
    const int64_t* q = r.data_ptr<int64_t>();
    const int64_t flat_n = scatter ? dst.numel() : src.numel(), packed_n = scatter ? src.numel() : dst.numel();
    for (int64_t i = 0; i < r.size(0); ++i) {
      PCHECK(q[3 * i] >= 0 && q[3 * i + 1] >= 0 && q[3 * i + 2] >= 0 && q[3 * i] + q[3 * i + 2] <= flat_n &&
                 q[3 * i + 1] + q[3 * i + 2] <= packed_n,
             "range out of bounds");
      PCHECK(i == 0 || q[3 * i + 1] == q[3 * (i - 1) + 1] + q[3 * (i - 1) + 2], "ranges must be laid end to end in packed order");
    }
    static_assert(sizeof(pddl::RangeRow) == 3 * sizeof(int64_t), "RangeRow layout");
    Tensor dev = r.to(src.device());
    ok(pddl::range_copy_launch(f32p(src), f32p(dst), reinterpret_cast<const pddl::RangeRow*>(dev.data_ptr()),
                               (int)r.size(0), scatter ? 1 : 0, cur_stream()),
       "range_copy");
  });
  // bf16 wire of the PS data plane (tests): gather fp32 -> packed bf16 / scatter packed bf16 -> fp32
  m.def("range_copy_cvt", [](Tensor src, Tensor dst, Tensor rows, bool scatter) {
    PCHECK(!rows.is_cuda() && rows.scalar_type() == torch::kInt64 && rows.dim() == 2 && rows.size(1) == 3,
           "range rows: host int64 [n, 3]");
    PCHECK(src.is_cuda() && dst.is_cuda() && src.is_contiguous() && dst.is_contiguous(), "range_copy_cvt: GPU tensors");
    PCHECK(scatter ? (src.scalar_type() == torch::kBFloat16 && dst.scalar_type() == torch::kFloat32)
                   : (src.scalar_type() == torch::kFloat32 && dst.scalar_type() == torch::kBFloat16),
           "range_copy_cvt: gather fp32 -> bf16, scatter bf16 -> fp32");
    Tensor r = rows.contiguous();
    const int64_t* q = r.data_ptr<int64_t>();
    const int64_t flat_n = scatter ? dst.numel() : src.numel(), packed_n = scatter ? src.numel() : dst.numel();
    for (int64_t i = 0; i < r.size(0); ++i) {
      PCHECK(q[3 * i] >= 0 && q[3 * i + 1] >= 0 && q[3 * i + 2] >= 0 && q[3 * i] + q[3 * i + 2] <= flat_n &&
                 q[3 * i + 1] + q[3 * i + 2] <= packed_n,
             "range out of bounds");
      PCHECK(i == 0 || q[3 * i + 1] == q[3 * (i - 1) + 1] + q[3 * (i - 1) + 2], "ranges must be laid end to end in packed order");
    }
    Tensor dev = r.to(src.device());
    ok(pddl::range_copy_cvt_launch(src.data_ptr(), dst.data_ptr(), reinterpret_cast<const pddl::RangeRow*>(dev.data_ptr()),
                                   (int)r.size(0), scatter ? 1 : 0, cur_stream()),
       "range_copy_cvt");
  });
  m.def("adam_bf16_wire", [](Tensor p, Tensor g, Tensor m_, Tensor v, Tensor snap, double lr_t, double b1, double b2,
                             double eps) {
    PCHECK(g.scalar_type() == torch::kBFloat16 && snap.scalar_type() == torch::kBFloat16 && g.numel() == p.numel() &&
               snap.numel() == p.numel() && m_.numel() == p.numel() && v.numel() == p.numel(),
           "adam_bf16_wire: p/m/v fp32, g/snap bf16, equal sizes");
    ok(pddl::adam_bf16_wire_launch(f32p(p), bfp(g), f32p(m_), f32p(v), bfpm(snap), p.numel(), (float)lr_t, (float)b1,
                                   (float)b2, (float)eps, cur_stream()),
       "adam_bf16_wire");
  });
  // bench.py --comm-proxy: a paced, CU-holding stand-in for one bucket's RCCL all-reduce
  m.def("comm_proxy", [](Tensor src, Tensor scratch, int passes, int64_t ticks, int nch) {
    PCHECK(src.is_cuda() && scratch.is_cuda() && src.scalar_type() == torch::kFloat32 &&
               scratch.scalar_type() == torch::kFloat32 && src.is_contiguous() && scratch.is_contiguous() &&
               scratch.numel() >= src.numel() && src.numel() % 4 == 0,
           "comm_proxy: fp32 device tensors, scratch >= src, 4-element multiple");
    ok(pddl::comm_proxy_launch(f32p(src), f32p(scratch), src.numel(), passes, ticks, nch, cur_stream()),
       "comm_proxy");
  }, REL);
  m.def("igemm", &igemm, REL);
  m.def("igemm_bn", &igemm_impl, REL);
  m.def("bn_stats", &bn_stats, REL);
  m.def("bn_apply", &bn_apply, REL);
  m.def("bn_bwd_reduce", &bn_bwd_reduce, REL);
  m.def("bn_bwd_apply", &bn_bwd_apply, REL);
  m.attr("BNSTAT_LAYER_BYTES") = (int)sizeof(pddl::BnStatLayer);
  m.def("wgrad", &wgrad, REL);
  m.def("bwd1x1", &bwd1x1, REL, py::arg("g"), py::arg("x"), py::arg("wd"), py::arg("bits"), py::arg("out"),
        py::arg("colsum"), py::arg("dw"), py::arg("out2") = py::none(), py::arg("g1") = py::none(),
        py::arg("w1d") = py::none(), py::arg("gmask") = py::none(), py::arg("gx") = py::none(),
        py::arg("colsum_gx") = py::none());
  m.def("bwd1x1_partial_rows", &bwd1x1_partial_rows);
  m.def("conv_f32", &conv_f32, REL);
  m.def("conv_f32_epi", &conv_f32_epi, REL);
  m.def("maxpool_fwd_f32", &maxpool_fwd_f32, REL);
  m.def("maxpool_bwd_f32", &maxpool_bwd_f32, REL);
  m.def("gap_fwd_f32", &gap_fwd_f32, REL);
  m.def("gap_bwd_f32", &gap_bwd_f32, REL);
  m.def("colsum_f32", &colsum_f32, REL);
  m.def("softmax_xent_f32", &softmax_xent_f32, REL);
  m.def("prep_f32", &prep_f32, REL);
  m.def("wgrad_f32", &wgrad_f32, REL);
  m.def("stem_s2d", &stem_s2d, REL);
  m.def("stem_wgrad_fold", &stem_wgrad_fold, REL);
  m.def("maxpool_fwd", &maxpool_fwd, REL);
  m.def("stem_pool_bwd", &stem_pool_bwd, REL, py::arg("x2"), py::arg("gpool"), py::arg("idx"), py::arg("dw"),
        py::arg("colsum"), py::arg("pool_rows") = 0);
  m.def("stem_pool_bwd_partial_rows", [](int B, int H2, int PB) { return pddl::stem_pool_bwd_partial_rows(B, H2, PB); },
        py::arg("B"), py::arg("H2"), py::arg("pool_rows") = 0);
  m.def("stem_pool_fwd", &stem_pool_fwd, REL, py::arg("x2"), py::arg("w"), py::arg("scale"), py::arg("shift"),
        py::arg("pool"), py::arg("idx"), py::arg("bits") = py::none(), py::arg("pool_rows") = 0);
  m.def("maxpool_bwd", &maxpool_bwd, REL);
  m.def("conv3x3c64", &conv3x3c64, REL, py::arg("x"), py::arg("w"), py::arg("mode"), py::arg("out"),
        py::arg("scale") = py::none(), py::arg("shift") = py::none(), py::arg("bits") = py::none(),
        py::arg("colsum") = py::none());
  m.def("conv3x3c64_wgrad", &conv3x3c64_wgrad, REL, py::arg("x"), py::arg("g"), py::arg("dw"));
  m.def("c3c1", &c3c1, REL, py::arg("a"), py::arg("w3"), py::arg("scale3"), py::arg("shift3"),
        py::arg("res"), py::arg("out"), py::arg("bits3"), py::arg("w1"), py::arg("scale1"), py::arg("shift1"),
        py::arg("y1"), py::arg("bits1"));
  m.def("conv3x3c64_partial_rows", [](int64_t M) { return pddl::conv3x3c64_partial_rows((int)M); });
  m.def("gap_fwd", &gap_fwd, REL);
  m.def("gap_bwd", &gap_bwd, REL);
  m.def("colsum", &colsum, REL);
  m.def("softmax_xent", &softmax_xent, REL);
  m.def("colsum_reduce", &colsum_reduce, REL);
  m.def("allow_knob_changes", [](bool on) { g_knob_tuning.store(on); }, py::arg("on") = true);
  m.def("knobs_frozen", []() { return g_launched.load() && !g_knob_tuning.load(); });
  m.def("set_variant", [](const std::string& which, int v) {
    TORCH_CHECK(!g_launched.load() || g_knob_tuning.load(), "kernel knob ", which,
                ": knobs are read-only once a kernel has launched (set them before the first launch, "
                "e.g. PDDL_KNOBS, or call allow_knob_changes(True) in tuning code)");
    if (which == "igemm") pddl::g_igemm_variant = v;
    else if (which == "igemm_deep") pddl::g_igemm_deep = v;
    else if (which == "igemm_pf") pddl::g_igemm_pf = v;
    else if (which == "igemm8") pddl::g_igemm8 = v;
    else if (which == "igemm8_min_tiles") pddl::g_igemm8_min_tiles = v;
    else if (which == "wgrad8") pddl::g_wgrad8 = v;
    else if (which == "igemm_ns1_kt") pddl::g_igemm_ns1_kt = v;
    else if (which == "igemm8_min_n") pddl::g_igemm8_min_n = v;
    else if (which == "wgrad1") pddl::g_wgrad1 = v;
    else if (which == "igemm_n64") pddl::g_igemm_n64 = v;
    else if (which == "igemm_splitk") pddl::g_igemm_splitk = v;
    else if (which == "igemm_sk_fill") { TORCH_CHECK(v >= 1 && v <= 8, "igemm_sk_fill: 1-8"); pddl::g_igemm_sk_fill = v; }
    else if (which == "igemm_sk_cap") { TORCH_CHECK(v >= 2 && v <= 16, "igemm_sk_cap: 2-16"); pddl::g_igemm_sk_cap = v; }
    else if (which == "igemm_sk_elig") { TORCH_CHECK(v >= 1 && v <= 8, "igemm_sk_elig: 1-8"); pddl::g_igemm_sk_elig = v; }
    else if (which == "igemm_pk_all") pddl::g_igemm_pk_all = v;
    else if (which == "igemm_pk_dual") pddl::g_igemm_pk_dual = v;
    else if (which == "igemm_pk") { TORCH_CHECK(v == 0 || (v >= 2 && v <= 4), "igemm_pk: 0 or ring depth 2-4"); pddl::g_igemm_pk = v; }
    else if (which == "wgrad8_min_rows") { TORCH_CHECK(v >= 64, "wgrad8_min_rows"); pddl::g_wgrad8_min_rows = v; }
    else if (which == "stem") pddl::g_stem_variant = v;
    else if (which == "conv_f32") pddl::g_conv_f32_variant = v;
    else if (which == "conv_f32_splitk") pddl::g_conv_f32_splitk = v;
    else if (which == "conv_f32_sk_elig") { TORCH_CHECK(v >= 1 && v <= 8, "conv_f32_sk_elig: 1-8"); pddl::g_conv_f32_sk_elig = v; }
    else if (which == "wgrad_f32_wpc64") { TORCH_CHECK(v >= 1 && v <= 32, "wgrad_f32_wpc64"); pddl::g_wgrad_f32_wpc[0] = v; }
    else if (which == "wgrad_f32_wpc128") { TORCH_CHECK(v >= 1 && v <= 32, "wgrad_f32_wpc128"); pddl::g_wgrad_f32_wpc[1] = v; }
    else if (which == "c64_grid") pddl::g_c64_grid = v;
    else if (which == "c64w_grid") pddl::g_c64w_grid = v;
    else if (which == "bn_red_blocks") pddl::g_bn_red_blocks = v;
    else if (which == "bn_apply_blocks") pddl::g_bn_apply_blocks = v;
    else if (which == "pool_blocks") pddl::g_pool_blocks = v;
    else if (which == "colred_chunks") { TORCH_CHECK(v >= 1 && v <= 65535, "colred_chunks"); pddl::g_colred_chunks = v; }
    else TORCH_CHECK(false, "unknown kernel knob ", which);
  });
  // (train/graph.py: is the stream's current capture still empty?) (hip error, capture status, #deps)
  m.def("stream_capture_deps", [](int64_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t n = 0;
    const hipError_t e = hipStreamGetCaptureInfo_v2(reinterpret_cast<hipStream_t>(stream), &st, &id, &g, &deps, &n);
    return std::make_tuple((int)e, (int)st, (int64_t)n);
  });
  m.def("igemm_partial_rows", [](int M, int Nn, int K, bool bnz) { return pddl::igemm_partial_rows(M, Nn, K, bnz); },
        py::arg("M"), py::arg("Nn"), py::arg("K"), py::arg("bnz") = false);
  m.def("igemm_splitk_floats", [](int M, int Nn, int K) { return (int64_t)pddl::igemm_splitk_floats(M, Nn, K); });
  m.def("splitk_use", &splitk_use, py::arg("workspace"));
  m.def("splitk_default_floats", &splitk_default_floats, py::arg("device"));
  m.def("igemm_plan", [](int M, int Nn, int K) {
    int cfg = 0, split = 0, ks = 1;
    pddl::igemm_plan_query(M, Nn, K, &cfg, &split, &ks);
    return std::make_tuple(cfg, split, ks);
  });
  m.def("maxpool_bwd_partial_rows", &pddl::maxpool_bwd_partial_rows);
  m.attr("COLRED_LAYER_BYTES") = (int)sizeof(pddl::ColRedLayer);
  m.def("prep", &prep, REL, py::arg("params"), py::arg("table"), py::arg("nlayers"), py::arg("max_elems"),
        py::arg("wbf"), py::arg("scale"), py::arg("shift"), py::arg("eps"), py::arg("parts") = 3);
  m.def("prep_fuse", &prep_fuse, REL);
  m.def("wgrad_finalize", &wgrad_finalize, REL, py::arg("params"), py::arg("grads"), py::arg("table"),
        py::arg("nlayers"), py::arg("scale"), py::arg("dgamma_raw"), py::arg("max_cout") = 2048);
  m.def("bn_grad", &bn_grad, REL);
  m.def("synth", &synth, REL);
  m.def("opt_hparams", &opt_hparams, REL);
  m.def("adam", &adam, REL);
  m.def("sgd", &sgd, REL);
  m.def("scale_", &scale_, REL);
  m.def("cast_bf16", &cast_bf16, REL);
  m.def("cast_f32", &cast_f32, REL);
  m.attr("PREP_LAYER_BYTES") = (int)sizeof(pddl::PrepLayer);
  m.attr("FUSE_LAYER_BYTES") = (int)sizeof(pddl::FuseLayer);
  m.attr("FIN_LAYER_BYTES") = (int)sizeof(pddl::FinLayer);
  m.attr("BNGRAD_LAYER_BYTES") = (int)sizeof(pddl::BnGradLayer);
  m.attr("EPI_FWD") = (int)pddl::EPI_FWD;
  m.attr("EPI_DGRAD") = (int)pddl::EPI_DGRAD;
  m.attr("EPI_F32") = (int)pddl::EPI_F32;
}
