"""End-to-end parity: the HIP engine (bf16 MFMA kernels, fused epilogues, explicit backward)
against the fp32 PyTorch reference of the Keras graph, on identical parameters and inputs."""
import pytest

from pddl.utils.envopts import with_opt
import torch

pytestmark = pytest.mark.gpu


def _engines(B, crop, image_size, bf16_points=False):
    from pddl.models.engine import HipEngine
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    he = HipEngine(L, B, crop=crop, image_size=image_size)
    # the bf16-point reference models the engine's fused projection GEMM (BN scales folded into
    # the bf16 weights) when the engine runs it
    te = TorchEngine(L, B, crop=crop, device="cuda", bf16_points=bf16_points, fused_proj=he.fuse_proj)
    he.init(seed=3)
    # perturb BN statistics / affine so the frozen-BN folding is exercised (not identity)
    g = torch.Generator(device="cpu").manual_seed(11)
    host = he.params.cpu()
    for e in L.entries.values():
        sl = host[e.offset:e.offset + e.size]
        if e.kind == "gamma":
            sl.copy_(0.5 + torch.rand(e.size, generator=g))
        elif e.kind == "beta" or e.kind == "bias":
            sl.copy_(0.1 * torch.randn(e.size, generator=g))
        elif e.kind == "moving_mean":
            sl.copy_(0.1 * torch.randn(e.size, generator=g))
        elif e.kind == "moving_variance":
            sl.copy_(0.5 + torch.rand(e.size, generator=g))
    he.params.copy_(host.cuda())
    he.after_update()
    te.params.copy_(he.params)
    return L, he, te


@pytest.mark.parametrize("crop,image_size", [(224, 224), (160, 224), (244, 224)])   # 244: Q1 up-size, odd grids
def test_engine_matches_reference(crop, image_size):
    torch.manual_seed(0)
    B = 4
    L, he, te = _engines(B, crop, image_size)
    img = torch.randint(0, 256, (B, image_size, image_size, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 1000, (B,), device="cuda")
    flip = torch.tensor([0, 1, 1, 0], dtype=torch.uint8, device="cuda")
    off = (5, 9) if crop < image_size else (0, 0)
    s_h = he.forward_backward(img, lab, 1.0 / B, flip=flip, crop_offset=off).clone()
    s_t = te.forward_backward(img, lab, 1.0 / B, flip=flip, crop_offset=off)
    torch.cuda.synchronize()
    assert abs(s_h[0].item() - s_t[0].item()) / s_t[0].item() < 0.03
    bad = []
    for e in L.entries.values():
        if not e.trainable:
            continue
        a = he.grads[e.offset:e.offset + e.size].float()
        b = te.grads[e.offset:e.offset + e.size].float()
        r = ((a - b).norm() / (b.norm() + 1e-20)).item()
        if r > 0.15:
            bad.append((e.name, r))
    assert not bad, bad[:10]
    cos = torch.nn.functional.cosine_similarity(he.grads, te.grads, dim=0).item()
    assert cos > 0.99


def _grad_errors(L, he, te):
    out = []
    for e in L.entries.values():
        if not e.trainable:
            continue
        a = he.grads[e.offset:e.offset + e.size].float()
        b = te.grads[e.offset:e.offset + e.size].float()
        out.append((((a - b).norm() / (b.norm() + 1e-20)).item(), e.name))
    return sorted(out, reverse=True)


@pytest.mark.parametrize("crop,image_size", [(224, 224), (160, 224), (244, 224)])
def test_engine_matches_bf16_point_reference_within_its_noise_floor(crop, image_size):
    """Against the reference with the engine's bf16 storage points (models/reference.py
    bf16_points) only accumulation order differs -- and that alone moves a tensor's gradient by a
    few % through the bf16 roundings downstream (the SAME reference run on the CPU instead of
    the GPU differs from itself by 2.5 % median, 3.7 % max per tensor: scripts/parity_noise.py,
    profiles/r2_parity_noise_floor.txt).  So each tensor is bounded by that measured floor:
    engine error <= 3 x (GPU-vs-CPU reference error) + 0.5 %, which a mis-scaled bias / BN
    parameter (error ~100 %) cannot pass, unlike the fixed 15 % bound above; and across tensors
    the engine's median error is at most 1.5 x the floor's.  (The factor 3 covers the engine's
    own run-to-run spread: its weight gradients are summed with fp32 atomics in no fixed order,
    which moves a cancellation-heavy BN-gamma gradient -- a dot product of W and dW -- by ~1 %
    between runs, e.g. 3.3 % against a 1.1 % floor in one run and within 2x in the next.)
    The reference models the fused projection GEMM (BN scales folded into bf16 weights,
    models/reference.py fused_proj): without it the crop-244 median ratio sat at 1.52 and failed
    on a fresh box (GPUTEST_r03); with it the ratios are 0.94 / 0.99 / 1.21 at crops 224 / 160 /
    244 (profiles/r4_parity_ratios.txt)."""
    from pddl.models.reference import TorchEngine
    torch.manual_seed(0)
    B = 4
    L, he, te = _engines(B, crop, image_size, bf16_points=True)
    tc = TorchEngine(L, B, crop=crop, device="cpu", bf16_points=True, fused_proj=he.fuse_proj)
    tc.params.copy_(te.params.cpu())
    img = torch.randint(0, 256, (B, image_size, image_size, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 1000, (B,), device="cuda")
    flip = torch.tensor([1, 0, 0, 1], dtype=torch.uint8, device="cuda")
    off = (7, 3) if crop < image_size else (0, 0)
    s_h = he.forward_backward(img, lab, 1.0 / B, flip=flip, crop_offset=off).clone()
    s_t = te.forward_backward(img, lab, 1.0 / B, flip=flip, crop_offset=off)
    tc.forward_backward(img.cpu(), lab.cpu(), 1.0 / B, flip=flip.cpu(), crop_offset=off)
    torch.cuda.synchronize()
    assert abs(s_h[0].item() - s_t[0].item()) / s_t[0].item() < 2e-3

    class _Cpu:
        grads = tc.grads.cuda()
    floor = {n: r for r, n in _grad_errors(L, _Cpu, te)}
    errs = _grad_errors(L, he, te)
    over = [(n, round(r, 4), round(floor[n], 4)) for r, n in errs if r > 3 * floor[n] + 0.005]
    assert not over, over[:8]
    med = lambda v: sorted(v)[len(v) // 2]   # noqa: E731
    m_e, m_f = med([r for r, _ in errs]), med(list(floor.values()))
    print(f"crop {crop}: engine median {m_e:.4f}, floor median {m_f:.4f}, ratio {m_e / m_f:.3f}")
    assert m_e <= 1.5 * m_f, (m_e, m_f)


def test_engine_loss_trajectory_20_steps():
    """20 Adam steps on one fixed batch (the reference's training step, imagenet-resnet50.py:62-67):
    the HIP engine's loss trajectory tracks the bf16-point reference run on the CPU as closely as
    the SAME reference run on the GPU does.  Past the first few steps the trajectory is chaotic
    (the loss oscillates 2.1-3.0 while Adam memorises the batch), so small accumulation-order
    differences grow to a few % for any implementation -- the GPU reference (MIOpen, itself not
    run-to-run deterministic) deviates from the CPU one by up to ~4 % per step -- and the bound is
    relative to that spread: mean deviation <= 2 x the reference's own + 1 %, worst step < 10 %."""
    from pddl.models.reference import TorchEngine
    from pddl.train.optim import make_optimizer
    torch.manual_seed(0)
    B = 8
    L, he, te = _engines(B, 128, 128, bf16_points=True)
    tc = TorchEngine(L, B, crop=128, device="cpu", bf16_points=True, fused_proj=he.fuse_proj)
    tc.params.copy_(te.params.cpu())
    opts = [make_optimizer("adam", e, lr=1e-4) for e in (he, te, tc)]
    img = torch.randint(0, 256, (B, 128, 128, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 1000, (B,), device="cuda")
    traj = [[], [], []]
    for _ in range(20):
        for k, (e, o) in enumerate(zip((he, te, tc), opts)):
            dev_img, dev_lab = (img, lab) if k < 2 else (img.cpu(), lab.cpu())
            traj[k].append(e.forward_backward(dev_img, dev_lab, 1.0 / B)[0].item() / B)
            o.step()
            if k == 0:
                he.after_update()
    lh, lt, lc = traj
    assert lh[-1] < 0.5 * lh[0] and lt[-1] < 0.5 * lt[0], (lh, lt)       # both learn the batch
    dev_e = [abs(a - c) / abs(c) for a, c in zip(lh, lc)]                # engine vs CPU reference
    dev_r = [abs(b - c) / abs(c) for b, c in zip(lt, lc)]                # GPU reference vs CPU reference
    print("losses engine / reference / cpu reference:", [(round(a, 4), round(b, 4), round(c, 4))
                                                        for a, b, c in zip(lh, lt, lc)])
    # before the chaotic phase: within 3e-3, or 1.5x the GPU reference's own deviation there
    # (both references model the fused projection blocks' bf16 rounding of the BN-scaled weights)
    assert max(dev_e[:4]) < max(3e-3, 1.5 * max(dev_r[:4])), (dev_e[:4], dev_r[:4])
    # (chaotic phase: the engine's own run-to-run spread -- fp32 atomics in no fixed order --
    # reaches a 2 % mean deviation in some runs while the GPU reference may happen to sit within
    # 0.2 % of the CPU one, so the mean bound has a 3 % floor; GPUTEST r5: 2.06 % vs 0.18 %)
    mean_e, mean_r = sum(dev_e) / len(dev_e), sum(dev_r) / len(dev_r)
    assert max(dev_e) < 0.10 and mean_e <= max(2 * mean_r + 0.01, 0.03), (dev_e, dev_r)


def test_engine_trains():
    from pddl.train.optim import make_optimizer
    torch.manual_seed(0)
    B = 8
    L, he, _ = _engines(B, 96, 96)
    opt = make_optimizer("adam", he, lr=1e-3)
    img = torch.randint(0, 256, (B, 96, 96, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 10, (B,), device="cuda")
    losses = []
    for _ in range(12):
        s = he.forward_backward(img, lab, 1.0 / B)
        losses.append(s[0].item() / B)
        opt.step()
        he.after_update()
    assert losses[-1] < losses[0] * 0.5, losses
    ev = he.evaluate(img, lab)
    assert torch.isfinite(ev).all()


def test_engine_bitmask_equivalent():
    """ReLU masks carried as bitmasks give the same step as masks re-read from bf16 activations."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(0)
    B = 4
    L = ParamLayout()
    img = torch.randint(0, 256, (B, 128, 128, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 1000, (B,), device="cuda")
    out = []
    for bm in (False, True):
        he = HipEngine(L, B, crop=128, image_size=128, bitmask=bm)
        he.init(seed=5)
        s = he.forward_backward(img, lab, 1.0 / B).clone()
        out.append((s, he.grads.clone()))
    torch.cuda.synchronize()
    assert torch.allclose(out[0][0], out[1][0], rtol=1e-5)
    r = ((out[0][1] - out[1][1]).norm() / out[0][1].norm()).item()
    assert r < 1e-4, r


def test_graphed_step_matches_eager():
    """A HIP-graph replay of the full step (fwd, bwd, Adam with device-side step count,
    weight re-prep) follows the same trajectory as eager steps."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    from pddl.train.graph import GraphedTrainStep
    from pddl.train.optim import make_optimizer
    torch.manual_seed(0)
    B = 4
    L = ParamLayout()
    img = torch.randint(0, 256, (4, B, 96, 96, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 1000, (4, B), device="cuda")
    flips = torch.randint(0, 2, (4, B), dtype=torch.uint8, device="cuda")
    res = []
    for graphed in (False, True):
        he = HipEngine(L, B, crop=80, image_size=96)
        he.init(seed=7)
        opt = make_optimizer("adam", he, lr=1e-3)
        gs = GraphedTrainStep(he, opt, B, (96, 96), 1.0 / B) if graphed else None
        losses = []
        for i in range(4):
            off = (i, 2 * i)
            if graphed:
                s = gs(img[i], lab[i], flips[i], off)
            else:
                s = he.forward_backward(img[i], lab[i], 1.0 / B, flip=flips[i], crop_offset=off)
                opt.step()
                he.after_update()
            losses.append(s[0].item())
        res.append((losses, he.params.clone(), opt.iterations))
    torch.cuda.synchronize()
    (l0, p0, it0), (l1, p1, it1) = res
    assert it0 == it1 == 4
    assert all(abs(a - b) <= 1e-3 * abs(a) for a, b in zip(l0, l1)), (l0, l1)
    # (wgrad fp32 atomics make runs non-bitwise; Adam amplifies near-zero gradient noise)
    assert ((p0 - p1).norm() / p0.norm()).item() < 2e-3


def test_fused_projection_matches_unfused(monkeypatch):
    """Projection blocks run conv3 + the shortcut conv as one dual-source GEMM (second source = the
    block input at the block's stride, both frozen-BN scales folded into bf16 weights), so the
    shortcut activation is never materialised.  Same parameters and batch with the fusion off
    (PDDL_ENGINE fuse_proj=0: conv1 + shortcut launch, residual read by conv3): the losses and the
    flat gradients agree to the bf16 rounding of the scaled weights."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(5)
    L = ParamLayout()
    B = 8
    res = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "fuse_proj", fuse))
        he = HipEngine(L, B, crop=224, image_size=224)
        he.init(seed=7)
        assert he.fuse_proj == (fuse == "1")
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1)).cuda()
        lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(2)).cuda()
        st = he.forward_backward(img, lab, 1.0 / B)
        torch.cuda.synchronize()
        res.append((st[0].item() / B, he.grads.clone()))
    (l1, g1), (l0, g0) = res
    assert abs(l1 - l0) < 2e-2 * abs(l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 5e-2


def test_fused_conv3_backward_matches_unfused(monkeypatch):
    """Stage-2 conv3 backward as one launch (bwd1x1.hip: data and weight gradient from one read
    of the 256-channel output gradient) against the two-launch form (PDDL_ENGINE fuse_bwd=0: wgrad
    kernel + igemm dgrad): same parameters and batch, losses equal and flat gradients agree to
    fp32 accumulation order."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    B = 8
    res = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "fuse_bwd", fuse))
        he = HipEngine(L, B, crop=224, image_size=224)
        he.init(seed=7)
        assert he.fuse_bwd == (fuse == "1")
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1)).cuda()
        lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(2)).cuda()
        st = he.forward_backward(img, lab, 1.0 / B)
        torch.cuda.synchronize()
        res.append((st[0].item() / B, he.grads.clone()))
    (l1, g1), (l0, g0) = res
    assert abs(l1 - l0) < 1e-4 * abs(l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-2


def test_c64_kernels_in_engine_match_generic(monkeypatch):
    """The stage-2 3x3 convs on conv3x3c64.hip (forward, data gradient and weight gradient; the
    engine enables them from b >= 84 at 224, here forced on with PDDL_ENGINE c64_min_m) against the
    generic implicit GEMM / wgrad kernels: same loss, flat gradients to fp32 accumulation order."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    B = 8
    res = []
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c64_min_m", "1"))
    for on in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c64", on))
        he = HipEngine(L, B, crop=224, image_size=224)
        he.init(seed=7)
        assert he.c64 == (on == "1") and he._use_c64(64, B * 56 * 56, 56) == (on == "1")
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8,
                            generator=torch.Generator().manual_seed(1)).cuda()
        lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(2)).cuda()
        st = he.forward_backward(img, lab, 1.0 / B)
        torch.cuda.synchronize()
        res.append((st[0].item() / B, he.grads.clone()))
    (l1, g1), (l0, g0) = res
    print(f"c64: loss rel {abs(l1 - l0) / abs(l0):.2e}, grad rel {((g1 - g0).norm() / g0.norm()).item():.3e}")
    assert abs(l1 - l0) < 1e-4 * abs(l0)
    # (every c64 kernel form measured lands at 1.5e-2 -- not a kernel defect: the swapped-operand
    # MFMAs round a few bf16 activations the other way and the flat gradient, dominated by
    # cancellation-heavy BN-gamma terms, moves by that much; the numeric check of the c64 path
    # against the fp32 reference is test_c64_engine_within_noise_floor)
    assert ((g1 - g0).norm() / g0.norm()).item() < 3e-2


def test_c3c1_boundary_fusion_in_engine(monkeypatch):
    """Stage-2 block boundaries with conv3 + the next conv1 in one launch (c3c1.hip, PDDL_ENGINE c3c1=1,
    the default) against separate launches: same loss, flat gradients to fp32 order; and the
    engine with the fusion stays within the fp32 reference's bf16-point noise floor."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    B = 8
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c3c1", on))
        he = HipEngine(L, B, crop=224, image_size=224)
        assert he.c3c1 == int(on)
        he.init(seed=7)
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1)).cuda()
        lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(2)).cuda()
        st = he.forward_backward(img, lab, 1.0 / B)
        torch.cuda.synchronize()
        res.append((st[0].item() / B, he.grads.clone()))
    (l1, g1), (l0, g0) = res
    print(f"c3c1: loss rel {abs(l1 - l0) / abs(l0):.2e}, grad rel {((g1 - g0).norm() / g0.norm()).item():.3e}")
    assert abs(l1 - l0) < 1e-4 * abs(l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 3e-2
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c3c1", "1"))
    test_engine_matches_bf16_point_reference_within_its_noise_floor(224, 224)


def test_c1_dgrad_fused_into_conv3_backward(monkeypatch):
    """Stage-2 backward boundaries with the next block's conv1 data gradient computed inside the
    fused conv3 backward (bwd1x1 pre form, PDDL_ENGINE c1pre=1, the default) against separate launches:
    same loss, flat gradients to fp32 order; and within the fp32 reference's noise floor."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    B = 8
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c1pre", on))
        he = HipEngine(L, B, crop=224, image_size=224)
        assert he.c1pre == (on == "1")
        he.init(seed=7)
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1)).cuda()
        lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(2)).cuda()
        st = he.forward_backward(img, lab, 1.0 / B)
        torch.cuda.synchronize()
        res.append((st[0].item() / B, he.grads.clone()))
    (l1, g1), (l0, g0) = res
    print(f"c1pre: loss rel {abs(l1 - l0) / abs(l0):.2e}, grad rel {((g1 - g0).norm() / g0.norm()).item():.3e}")
    assert abs(l1 - l0) < 1e-4 * abs(l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 3e-2
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c1pre", "1"))
    test_engine_matches_bf16_point_reference_within_its_noise_floor(224, 224)


def test_s2_fed_blocks_store_compact_outputs(monkeypatch):
    """Blocks feeding a downsampling block store only their stride-2 grid (PDDL_ENGINE s2c=1, the
    default: conv3 on the compact quarter, the next block's conv1 / shortcut / weight gradient
    and ReLU mask read it as a stride-1 input) against full-resolution storage: same loss, flat
    gradients to fp32 order; and within the fp32 reference's noise floor."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    B = 8
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "s2c", on))
        he = HipEngine(L, B, crop=224, image_size=224)
        assert he.s2c == (on == "1")
        he.init(seed=7)
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1)).cuda()
        lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(2)).cuda()
        st = he.forward_backward(img, lab, 1.0 / B)
        torch.cuda.synchronize()
        res.append((st[0].item() / B, he.grads.clone()))
    (l1, g1), (l0, g0) = res
    print(f"s2c: loss rel {abs(l1 - l0) / abs(l0):.2e}, grad rel {((g1 - g0).norm() / g0.norm()).item():.3e}")
    assert abs(l1 - l0) < 1e-4 * abs(l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 3e-2
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "s2c", "1"))
    test_engine_matches_bf16_point_reference_within_its_noise_floor(224, 224)


def test_c64_engine_within_noise_floor(monkeypatch):
    """The engine with the stage-2 3x3 convs forced onto conv3x3c64.hip is as close to the fp32
    reference as the reference's own bf16-point floor (same criteria as the generic path:
    measured ratios 0.92-1.00 on the 8-wave row tiles vs 0.98-1.15 generic, crops 224/160/244)."""
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c64_min_m", "1"))
    test_engine_matches_bf16_point_reference_within_its_noise_floor(224, 224)


@pytest.mark.parametrize("graphed", [False, True])
def test_two_stream_backward_matches_one_stream(monkeypatch, graphed):
    """Small-batch backward with the weight gradients on a side stream (PDDL_ENGINE two_stream=1, the
    default up to 1024 images) against the single-stream schedule: same loss and gradients to
    fp32-atomic order, eager and captured in a HIP graph (the side stream forks from and joins
    the capture)."""
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    from pddl.train.graph import GraphedTrainStep
    from pddl.train.optim import make_optimizer
    L = ParamLayout()
    B = 8
    img = torch.randint(0, 256, (B, 112, 112, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(3)).cuda()
    lab = torch.randint(0, 1000, (B,), generator=torch.Generator().manual_seed(4)).cuda()
    flips = torch.zeros(B, dtype=torch.uint8, device="cuda")
    res = []
    for two in ("1", "0"):
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "two_stream", two))
        he = HipEngine(L, B, crop=112, image_size=112)
        assert he.two_stream == (two == "1")
        he.init(seed=7)
        if graphed:
            opt = make_optimizer("adam", he, lr=1e-3)
            gs = GraphedTrainStep(he, opt, B, (112, 112), 1.0 / B)
            for _ in range(3):
                st = gs(img, lab, flips, (0, 0))
            res.append((st[0].item(), he.params.clone()))
        else:
            st = he.forward_backward(img, lab, 1.0 / B)
            torch.cuda.synchronize()
            res.append((st[0].item(), he.grads.clone()))
    (l1, g1), (l0, g0) = res
    assert abs(l1 - l0) <= 1e-3 * abs(l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < (2e-3 if graphed else 1e-3)
