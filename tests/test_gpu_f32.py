"""Reference-precision (fp32) path: the fp32-MFMA HIP convolutions (csrc/kernels/conv_f32.hip)
against float64 PyTorch, and the assembled fp32 engine (models/engine_f32.py) against the
PyTorch reference model (models/reference.py, the Keras graph of imagenet-resnet50.py:51-61)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def N():
    from pddl.ops.native import require_native
    return require_native()


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


CASES = [   # N, H, C, Cout, R, stride, pad
    (2, 9, 64, 96, 1, 1, 0),
    (2, 11, 32, 64, 3, 1, 1),
    (3, 8, 128, 64, 1, 2, 0),
    (2, 23, 3, 64, 7, 2, 3),       # the stem: C = 3 (scalar gather), K = 147
    (1, 5, 2048, 40, 1, 1, 0),     # dense-like: long K, Cout tail
]


@pytest.mark.parametrize("case", CASES)
def test_conv_f32_forward_and_wgrad(case):
    torch.manual_seed(0)
    n, h, c, co, r, st, pad = case
    ho = (h + 2 * pad - r) // st + 1
    x = torch.randn(n, h, h, c, device=dev)
    w = torch.randn(co, r, r, c, device=dev) * 0.1
    b = torch.randn(co, device=dev)
    y = torch.empty(n, ho, ho, co, device=dev)
    N().conv_f32(x, r, r, st, pad, w.view(co, -1), b, y)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(), stride=st,
                   padding=pad).permute(0, 2, 3, 1)
    assert rel(y, ref) < 1e-5
    g = torch.randn(n, ho, ho, co, device=dev)
    dw = torch.zeros(co, r * r * c, device=dev)
    N().wgrad_f32(x, r, r, st, pad, g, dw)
    rw = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (co, c, r, r), g.double().permute(0, 3, 1, 2),
                                     stride=st, padding=pad).permute(0, 2, 3, 1).reshape(co, -1)
    assert rel(dw, rw) < 1e-5


@pytest.mark.parametrize("case", [(2, 9, 64, 96, 1, 1, 0), (2, 11, 32, 64, 3, 1, 1), (3, 8, 128, 64, 1, 2, 0),
                                  (4, 3, 512, 2048, 1, 1, 0), (4, 3, 512, 512, 3, 1, 1), (4, 6, 1024, 512, 1, 2, 0),
                                  (4, 6, 1024, 2048, 1, 2, 0)])
def test_conv2d_f32_autograd(case):
    """conv2d_f32's three gradients (dgrad as a flipped-weight conv / strided scatter, wgrad,
    bias) against float64 autograd of F.conv2d."""
    from pddl.ops.conv_f32 import conv2d_f32
    torch.manual_seed(1)
    n, h, c, co, r, st, pad = case
    x = torch.randn(n, c, h, h, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(co, r, r, c, device=dev) * 0.1).requires_grad_(True)
    b = torch.randn(co, device=dev).requires_grad_(True)
    y = conv2d_f32(x, w, b, st, pad)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd, wd, bd = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xd, wd.permute(0, 3, 1, 2), bd, stride=st, padding=pad)
    yr.backward(gy.double())
    assert rel(y, yr) < 1e-5
    assert rel(x.grad, xd.grad) < 1e-5
    assert rel(w.grad, wd.grad) < 1e-5
    assert rel(b.grad, bd.grad) < 1e-5


class _FProxy:
    """torch.nn.functional with `relu` replaced (recording or replaying ReLU masks)."""

    def __init__(self, relu):
        self.relu = relu

    def __getattr__(self, name):
        return getattr(F, name)


def _ref_grads(L, params, img, lab, B, crop, dtype, masks=None, bn_mode="frozen"):
    """The reference step in `dtype` on the CPU; with `masks`, every ReLU applies the engine's
    recorded mask instead of its own sign test (same arithmetic, same decisions)."""
    from pddl.models import reference as R
    ref = R.TorchEngine(L, B, crop=crop, device="cpu", bn_mode=bn_mode)
    ref.params = params.detach().cpu().to(dtype)
    ref.grads = torch.zeros(L.n_trainable, dtype=dtype)
    orig_pre, orig_f = R.preprocess, R.F
    R.preprocess = lambda *a, **k: orig_pre(*a, **k).to(dtype)
    if masks is not None:
        it = iter(masks)
        R.F = _FProxy(lambda x: x * next(it).to(x.dtype))
    try:
        st = ref.forward_backward(img, lab, 1.0 / B)
    finally:
        R.preprocess, R.F = orig_pre, orig_f
    return st, ref.grads


def test_f32_autograd_engine_matches_reference():
    """One training step of the autograd fp32 HIP engine (tests/f32_autograd.py, the test oracle) vs the PyTorch reference model in float64 on
    the CPU, every gradient tensor within 1e-4 relative.  The reference replays the engine's
    ReLU masks: a pre-activation within fp32 rounding of zero (1-2 of ~10^6 per step) can take
    the other side of the ReLU in any fp32 run, which re-routes that element's gradient and
    moves a small bias / BN-beta gradient by up to ~1e-2 -- a decision, not an arithmetic error.
    Without replay, the count of such flips is reported."""
    import f32_autograd as E
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(2)
    L = ParamLayout()
    B, crop = 4, 96
    eng = E.HipF32AutogradEngine(L, B, crop=crop, device=dev)
    eng.init(seed=3)
    img = torch.randint(0, 256, (B, crop, crop, 3), dtype=torch.uint8)
    lab = torch.randint(0, 1000, (B,))
    masks = []

    def rec(x):
        y = F.relu(x)
        masks.append((x > 0).detach().cpu())
        return y
    orig_f = E.F
    E.F = _FProxy(rec)
    try:
        st = eng.forward_backward(img.to(dev), lab.to(dev), 1.0 / B)
    finally:
        E.F = orig_f
    assert len(masks) == 1 + 3 * len(L.blocks)
    s64, g64 = _ref_grads(L, eng.params, img, lab, B, crop, torch.float64, masks)
    assert abs(st[0].item() - s64[0].item()) / abs(s64[0].item()) < 1e-5
    g = eng.grads.cpu().double()
    rows = []
    for e in L.entries.values():
        if e.offset + e.size > L.n_trainable:
            continue
        sl = slice(e.offset, e.offset + e.size)
        if g64[sl].norm() < 1e-12:
            continue
        rows.append((rel(g[sl], g64[sl]), e.name))
    rows.sort(reverse=True)
    print("worst (engine vs f64 with the engine's ReLU masks):", rows[:3])
    assert rows[0][0] < 1e-4, rows[:3]


def _engine_masks(eng, B):
    """The ReLU decisions the fused engine took, in the reference's call order (stem, then per
    block y1, y2, out), as NCHW bool tensors."""
    nchw = lambda t: (t[:B] > 0).permute(0, 3, 1, 2).cpu()   # noqa: E731
    out = [nchw(eng.c1)]
    for b in eng.L.blocks:
        a = eng.acts[b.name]
        out += [nchw(a["y1"]), nchw(a["y2"]), nchw(a["out"])]
    return out


@pytest.mark.parametrize("crop,image", [(96, 96), (64, 80)])
def test_f32_fused_engine_matches_reference(crop, image):
    """One training step of the explicit fp32 engine (fused conv epilogues, fp32 pool / GAP /
    softmax kernels, no PyTorch op in the step) vs the reference model in float64 on the CPU,
    with the engine's ReLU decisions replayed: every gradient tensor within 1e-4 relative and
    the loss within 1e-5 (crop < image: the RandomCrop offset path)."""
    from pddl.models.engine_f32 import HipF32Engine
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(2)
    L = ParamLayout()
    B = 4
    eng = HipF32Engine(L, B, crop=crop, image_size=image, device=dev)
    eng.init(seed=3)
    # non-trivial frozen-BN statistics / affine so the folding is exercised
    g = torch.Generator().manual_seed(11)
    host = eng.params.cpu()
    for e in L.entries.values():
        sl = host[e.offset:e.offset + e.size]
        if e.kind == "gamma":
            sl.copy_(0.5 + torch.rand(e.size, generator=g))
        elif e.kind in ("beta", "bias", "moving_mean"):
            sl.copy_(0.1 * torch.randn(e.size, generator=g))
        elif e.kind == "moving_variance":
            sl.copy_(0.5 + torch.rand(e.size, generator=g))
    eng.params.copy_(host.to(dev))
    eng.after_update()
    img = torch.randint(0, 256, (B, image, image, 3), dtype=torch.uint8)
    lab = torch.randint(0, 1000, (B,))
    off = (5, 9) if crop < image else (0, 0)
    st = eng.forward_backward(img.to(dev), lab.to(dev), 1.0 / B, crop_offset=off).clone()
    torch.cuda.synchronize()
    masks = _engine_masks(eng, B)
    src = img[:, off[0]:off[0] + crop, off[1]:off[1] + crop] if crop < image else img
    s64, g64 = _ref_grads(L, eng.params, src.contiguous(), lab, B, crop, torch.float64, masks)
    assert abs(st[0].item() - s64[0].item()) / abs(s64[0].item()) < 1e-5
    gr = eng.grads.cpu().double()
    rows = []
    for e in L.entries.values():
        if e.offset + e.size > L.n_trainable:
            continue
        sl = slice(e.offset, e.offset + e.size)
        if g64[sl].norm() < 1e-12:
            continue
        rows.append((rel(gr[sl], g64[sl]), e.name))
    rows.sort(reverse=True)
    print("worst (fused fp32 engine vs f64 with the engine's ReLU masks):", rows[:3])
    assert rows[0][0] < 1e-4, rows[:3]


@pytest.mark.parametrize("crop", [96, 64])
def test_f32_train_bn_engine_matches_reference(crop):
    """One training step of the explicit fp32 train-BN engine (batch statistics through bn.hip's
    fp32 kernels, no PyTorch op in the step) vs the reference model with training=True BN in
    float64 on the CPU, the engine's ReLU decisions replayed: every gradient tensor within 5e-4,
    the loss within 1e-5, the moving statistics updated, evaluation on them finite."""
    from pddl.models.engine_f32 import HipF32EngineBNTrain
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(2)
    L = ParamLayout()
    B = 4
    eng = HipF32EngineBNTrain(L, B, crop=crop, device=dev)
    eng.init(seed=3)
    g = torch.Generator().manual_seed(12)
    host = eng.params.cpu()
    for e in L.entries.values():
        sl = host[e.offset:e.offset + e.size]
        if e.kind == "gamma":
            sl.copy_(0.5 + torch.rand(e.size, generator=g))
        elif e.kind in ("beta", "bias"):
            sl.copy_(0.1 * torch.randn(e.size, generator=g))
    eng.params.copy_(host.to(dev))
    eng.after_update()
    p0 = eng.params.clone()
    img = torch.randint(0, 256, (B, crop, crop, 3), dtype=torch.uint8)
    lab = torch.randint(0, 1000, (B,))
    st = eng.forward_backward(img.to(dev), lab.to(dev), 1.0 / B).clone()
    torch.cuda.synchronize()
    masks = _engine_masks(eng, B)
    s64, g64 = _ref_grads(L, p0, img, lab, B, crop, torch.float64, masks, bn_mode="train")
    lerr = abs(st[0].item() - s64[0].item()) / abs(s64[0].item())
    # (fp32 summation order moves it by ~1e-5 through the batch statistics: 2.9e-6 / 5.8e-6 at
    # crops 64 / 96 unsplit, 1.2e-5 / 2.2e-6 with the small-M layers on split-K, round 6)
    assert lerr < 3e-5, lerr
    gr = eng.grads.cpu().double()
    rows = []
    for e in L.entries.values():
        if e.offset + e.size > L.n_trainable:
            continue
        sl = slice(e.offset, e.offset + e.size)
        if g64[sl].norm() < 1e-12 or e.kind == "bias":   # (conv bias before BN: gradient 0 in exact arithmetic)
            continue
        rows.append((rel(gr[sl], g64[sl]), e.name))
    rows.sort(reverse=True)
    print("worst (fp32 train-BN engine vs f64 with the engine's ReLU masks):", rows[:3])
    # (5e-4, not the frozen engine's 1e-4: at B = 4 the stage-5 BNs normalise over 36 rows per
    # channel, and the batch-statistics backward's centred sums cancel their terms to ~1e-3,
    # so fp32 rounding reaches ~2e-4 of those layers' gamma / kernel gradients -- measured
    # 1.8e-4 worst, every other tensor below 1e-4)
    assert rows[0][0] < 5e-4, rows[:3]
    # moving statistics: momentum 0.99 toward the batch mean / Bessel-corrected variance
    ev = eng.params.cpu()
    moved = [e for e in L.entries.values() if e.kind in ("moving_mean", "moving_variance")]
    assert all(not torch.equal(ev[e.offset:e.offset + e.size], p0.cpu()[e.offset:e.offset + e.size]) for e in moved)
    # evaluation runs on the moving statistics
    out = eng.evaluate(img.to(dev), lab.to(dev))
    assert torch.isfinite(out).all()


def test_f32_fused_engine_trains_and_evaluates():
    """Adam steps of the fused fp32 engine follow the autograd fp32 engine (same model, same
    precision, PyTorch autograd over the fp32 conv op) step for step; odd class count
    (Cout % 4 != 0 through the Dense head's wgrad / dgrad / column sums)."""
    from f32_autograd import HipF32AutogradEngine
    from pddl.models.engine_f32 import HipF32Engine
    from pddl.models.resnet50 import ParamLayout
    from pddl.train.optim import make_optimizer
    torch.manual_seed(0)
    B, ncls = 8, 10
    L = ParamLayout(ncls)
    img = torch.randint(0, 256, (B, 64, 64, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, ncls, (B,), device=dev)
    traj = []
    for cls in (HipF32Engine, HipF32AutogradEngine):
        eng = cls(L, B, crop=64, device=dev, num_classes=ncls)
        eng.init(seed=1)
        opt = make_optimizer("adam", eng, lr=1e-3)
        losses = []
        for _ in range(8):
            losses.append(eng.forward_backward(img, lab, 1.0 / B)[0].item() / B)
            opt.step()
            eng.after_update()
        traj.append(losses)
        if cls is HipF32Engine:
            ev = eng.evaluate(img, lab)
            assert torch.isfinite(ev).all()
    fused, ref = traj
    print("fused / autograd fp32 losses:", [(round(a, 5), round(b, 5)) for a, b in zip(fused, ref)])
    # measured: identical to 1e-5 for 3 steps, then fp32 summation-order differences grow in
    # this lr-1e-3 / 8-image problem (loss 2.30 -> 1.42 -> 1.63: the trajectory turns chaotic)
    dev_ = [abs(a - b) / abs(b) for a, b in zip(fused, ref)]
    assert fused[-1] < fused[0]
    assert max(dev_[:5]) < 1e-3 and max(dev_) < 2e-2, (fused, ref)


@pytest.mark.parametrize("up2", [0, 1])
def test_conv_f32_fused_epilogues(up2):
    """conv_f32_epi against float64: forward (folded BN affine + residual + ReLU) and dgrad
    (residual-gradient add + ReLU mask + stride-2 grid scatter + per-m-tile column sums)."""
    torch.manual_seed(4)
    n, h, c, co = 3, 9, 64, 100            # 100 output channels: a ragged last column group
    x = torch.randn(n, h, h, c, device=dev)
    w = torch.randn(co, c, device=dev) * 0.1
    sc, sh = torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev)
    res = torch.randn(n, h, h, co, device=dev)
    y = torch.empty(n, h, h, co, device=dev)
    N().conv_f32_epi(x, 1, 1, 1, 0, h, h, w, 1, sc, sh, res, 1, None, None, 0, y, None)
    ref = (x.double() @ w.double().t() * sc.double() + sh.double() + res.double()).relu()
    assert rel(y, ref) < 1e-6
    # dgrad: GEMM rows over an h x h grid, optionally scattered to a (2h - 1) x (2h - 1) grid
    H = 2 * h - 1 if up2 else h
    add = torch.randn(n, h, h, co, device=dev) if up2 else torch.randn(n, H, H, co, device=dev)
    mask = torch.randn(n, H, H, co, device=dev)
    out = torch.zeros(n, H, H, co, device=dev)
    rows = (n * h * h + 63) // 64
    part = torch.full((rows * co,), float("nan"), device=dev)
    N().conv_f32_epi(x, 1, 1, 1, 0, h, h, w, 2, None, None, None, 0, add, mask, up2, out, part)
    acc = x.double() @ w.double().t()
    full = torch.zeros(n, H, H, co, dtype=torch.float64, device=dev)
    if up2:
        full[:, ::2, ::2] = acc + add.double()
    else:
        full = acc + add.double()
    want = full * (mask.double() > 0)
    assert rel(out, want) < 1e-6
    if up2:
        assert out[:, 1::2].abs().sum().item() == 0 and out[:, :, 1::2].abs().sum().item() == 0
    assert rel(part.view(rows, co).sum(0), want.sum((0, 1, 2))) < 1e-6


def test_f32_pool_gap_softmax_kernels():
    torch.manual_seed(6)
    B, H, C = 3, 13, 64
    x = torch.randn(B, H, H, C, device=dev).relu()
    Ho = (H + 2 - 3) // 2 + 1
    y = torch.empty(B, Ho, Ho, C, device=dev)
    idx = torch.empty(B, Ho, Ho, C, dtype=torch.uint8, device=dev)
    N().maxpool_fwd_f32(x, y, idx)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(F.pad(xr, (1, 1, 1, 1)), 3, 2)
    assert rel(y, yr.permute(0, 2, 3, 1)) == 0
    gy = torch.randn(B, Ho, Ho, C, device=dev)
    gx = torch.empty_like(x)
    N().maxpool_bwd_f32(gy, idx, x, gx)
    yr.backward(gy.double().permute(0, 3, 1, 2))
    want = xr.grad.permute(0, 2, 3, 1) * (x.double() > 0)
    assert rel(gx, want) < 1e-6          # (fp32 sums of up to 4 routed gradients)
    # GAP
    p = torch.empty(B, C, device=dev)
    N().gap_fwd_f32(x, p)
    assert rel(p, x.double().mean((1, 2))) < 1e-6
    gp = torch.randn(B, C, device=dev)
    g = torch.empty_like(x)
    rows = torch.empty(B * C, device=dev)
    N().gap_bwd_f32(gp, x, g, rows)
    wg = (gp.double()[:, None, None, :] / (H * H)) * (x.double() > 0)
    assert rel(g, wg) < 1e-6 and rel(rows.view(B, C).sum(0), wg.sum((0, 1, 2))) < 1e-6
    cs = torch.zeros(C, device=dev)
    N().colsum_f32(g.view(-1, C), C, cs)
    assert rel(cs, wg.sum((0, 1, 2))) < 1e-6
    # softmax-xent with fp32 dlogits
    logits = torch.randn(5, 10, device=dev)
    lab = torch.randint(0, 10, (5,), device=dev)
    dl = torch.empty(5, 10, device=dev)
    ls, cr = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
    N().softmax_xent_f32(logits, lab, 10, 0.5, dl, ls, cr)
    lr = logits.double().requires_grad_(True)
    loss = F.cross_entropy(lr, lab, reduction="sum")
    (loss * 0.5).backward()
    assert abs(ls.item() - loss.item()) < 1e-4 and rel(dl, lr.grad) < 1e-6
    assert cr.item() == (logits.argmax(1) == lab).sum().item()


@pytest.mark.parametrize("case", [(4, 28, 64, 128, 3, 1, 1), (2, 30, 16, 64, 4, 1, 0), (2, 14, 256, 1024, 1, 1, 0),
                                  (8, 7, 512, 512, 3, 1, 1), (3, 15, 128, 200, 1, 2, 0)])
def test_conv_f32_128_tile_kernels_match_64_and_fp64(case):
    """The LDS-DMA fp32 kernels (conv_f32_big_kernel<128> / <64> and wgrad_f32_big_kernel; knob
    conv_f32 = 1 runs 128 x 64 conv tiles for C % 16 == 0; forced here: 2 = 128 x 128 conv tiles,
    3 = 128 x 64; both force the 128 x 128 weight-gradient tiles on any shape) against float64 and against the 64 x 64 kernels (knob 0): forward with the fused
    frozen-BN epilogue, data-gradient epilogue with column sums, and the weight gradient, over
    multi-tile shapes incl. the stem's 4x4 window (C = 16) and a ragged Cout."""
    torch.manual_seed(1)
    n, h, c, co, r, st, pad = case
    ho = (h + 2 * pad - r) // st + 1
    x = torch.randn(n, h, h, c, device=dev)
    w = torch.randn(co, r, r, c, device=dev) * 0.1
    sc, sh = torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev)
    res = torch.randn(n, ho, ho, co, device=dev)
    g = torch.randn(n, ho, ho, co, device=dev)
    outs = []
    for v in (2, 3, 0):   # (the LDS-DMA kernels wherever they apply, whatever the tile count)
        N().set_variant("conv_f32", v)
        try:
            y = torch.empty(n, ho, ho, co, device=dev)
            N().conv_f32_epi(x, r, r, st, pad, ho, ho, w.view(co, -1), 1, sc, sh, res, 1, None, None, 0, y, None)
            yd = torch.empty(n, ho, ho, co, device=dev)
            cs = torch.zeros((n * ho * ho + 63) // 64, co, device=dev)
            N().conv_f32_epi(x, r, r, st, pad, ho, ho, w.view(co, -1), 2, None, None, None, 0, res, g, 0, yd, cs)
            dw = torch.zeros(co, r * r * c, device=dev)
            N().wgrad_f32(x, r, r, st, pad, g, dw)
            torch.cuda.synchronize()
            outs.append((y, yd, cs.sum(0), dw))
        finally:
            N().set_variant("conv_f32", 1)
    conv = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), stride=st,
                    padding=pad).permute(0, 2, 3, 1)
    ref_y = torch.relu(conv * sc.double() + sh.double() + res.double())
    ref_yd = torch.where(g > 0, conv + res.double(), torch.zeros_like(conv))
    ref_dw = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (co, c, r, r), g.double().permute(0, 3, 1, 2),
                                         stride=st, padding=pad).permute(0, 2, 3, 1).reshape(co, -1)
    y0, yd0, cs0, dw0 = outs[-1]
    for y1, yd1, cs1, dw1 in outs[:-1]:
        assert rel(y1, ref_y) < 1e-5 and rel(yd1, ref_yd) < 1e-5 and rel(dw1, ref_dw) < 1e-5
        assert rel(cs1, ref_yd.reshape(-1, co).sum(0)) < 1e-5
        assert rel(y1, y0) < 1e-5 and rel(dw1, dw0) < 1e-5


@pytest.mark.parametrize("case", [(2, 7, 512, 512, 3, 1, 1), (8, 14, 256, 256, 3, 1, 1), (4, 7, 2048, 512, 1, 1, 0),
                                  (3, 7, 512, 2048, 1, 1, 0)])
@pytest.mark.parametrize("v", [1, 2])
def test_conv_f32_splitk_matches_unsplit_and_fp64(case, v):
    """Split-K of the underfilled fp32 convs (conv_f32_big_kernel slices -> fp32 partial tiles in the
    engine's workspace -> conv_f32_splitk_kernel running the fused epilogue): the reference's
    per-replica batch leaves stage 5 at ~100 tiles of a 288-step K loop on 256 CUs.  Forward with
    the frozen-BN + residual + ReLU epilogue and dgrad with add / mask / column sums, against the
    unsplit kernels (knob conv_f32_splitk 0) and float64, 128 x 64 (v 1) and 128 x 128 (v 2) tiles."""
    torch.manual_seed(5)
    n, h, c, co, r, st, pad = case
    ho = (h + 2 * pad - r) // st + 1
    x = torch.randn(n, h, h, c, device=dev)
    w = torch.randn(co, r, r, c, device=dev) * 0.05
    sc, sh = torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev)
    res = torch.randn(n, ho, ho, co, device=dev)
    g = torch.randn(n, ho, ho, co, device=dev)
    ws = torch.empty(N().splitk_default_floats(0), device=dev)
    outs = []
    for sk in (4, 0):
        N().set_variant("conv_f32_splitk", sk)
        N().set_variant("conv_f32", v)
        N().splitk_use(ws)
        try:
            y = torch.empty(n, ho, ho, co, device=dev)
            N().conv_f32_epi(x, r, r, st, pad, ho, ho, w.view(co, -1), 1, sc, sh, res, 1, None, None, 0, y, None)
            yd = torch.empty(n, ho, ho, co, device=dev)
            cs = torch.full(((n * ho * ho + 63) // 64, co), float("nan"), device=dev)
            N().conv_f32_epi(x, r, r, st, pad, ho, ho, w.view(co, -1), 2, None, None, None, 0, res, g, 0, yd, cs)
            torch.cuda.synchronize()
            outs.append((y, yd, cs.sum(0)))
        finally:
            N().set_variant("conv_f32_splitk", 4)
            N().set_variant("conv_f32", 1)
            N().splitk_use(None)
    conv = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), stride=st,
                    padding=pad).permute(0, 2, 3, 1)
    ref_y = torch.relu(conv * sc.double() + sh.double() + res.double())
    ref_yd = torch.where(g > 0, conv + res.double(), torch.zeros_like(conv))
    (y1, yd1, cs1), (y0, yd0, cs0) = outs
    assert rel(y1, ref_y) < 1e-5 and rel(yd1, ref_yd) < 1e-5 and rel(cs1, ref_yd.sum((0, 1, 2))) < 1e-5
    assert rel(y1, y0) < 1e-5 and rel(yd1, yd0) < 1e-5 and rel(cs1, cs0) < 1e-5
