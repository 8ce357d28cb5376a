"""CPU tests: Keras-parity model facts, layout/buckets, reference engine, optimizers."""
import math

import numpy as np
import pytest
import torch


def test_param_counts_match_keras():
    from pddl.models.resnet50 import param_count_keras
    c = param_count_keras()
    assert c == {"total": 25636712, "trainable": 25583592, "non_trainable": 53120}


def test_layout_names_and_shapes():
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    convs = [e for e in L.entries.values() if e.kind == "kernel" and e.layer != "dense"]
    assert len(convs) == 53
    bns = {e.layer for e in L.entries.values() if e.kind == "gamma"}
    assert len(bns) == 53
    assert L.entry("conv1_conv", "kernel").keras_shape == (7, 7, 3, 64)
    assert L.entry("conv2_block1_0_conv", "kernel").keras_shape == (1, 1, 64, 256)
    assert L.entry("conv5_block3_3_conv", "kernel").keras_shape == (1, 1, 512, 2048)
    assert L.entry("dense", "kernel").keras_shape == (2048, 1000)
    # v1: stride on the first 1x1 of a block
    blk = {b.name: b for b in L.blocks}
    assert blk["conv3_block1"].convs["1"].stride == 2 and blk["conv3_block1"].convs["2"].stride == 1
    # trainable prefix, backward order: dense kernel first, stem kernel last of the kernels
    assert L.entry("dense", "kernel").offset == 0
    stem = L.entry("conv1_conv", "kernel")
    assert stem.offset + stem.size == L.kernels_end
    # projection conv1 and conv0 adjacent (one fused wgrad)
    c1, c0 = L.entry("conv4_block1_1_conv", "kernel"), L.entry("conv4_block1_0_conv", "kernel")
    assert c1.offset + c1.size == c0.offset
    for e in L.entries.values():
        assert (e.offset < L.n_trainable) == e.trainable


def test_buckets_cover_trainable_prefix():
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    for mb in (1, 8, 32, 1000):
        b = L.buckets(mb)
        assert b[0][0] == 0 and b[-1][1] == L.n_trainable
        for (s0, e0), (s1, e1) in zip(b, b[1:]):
            assert e0 == s1 and s0 < e0
        assert b[-1][0] == L.kernels_end     # per-channel tail bucket


def test_init_is_keras_default():
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    p = torch.zeros(L.total)
    L.init_params(p, seed=0)
    assert torch.all(L.view(p, "conv2_block1_1_bn", "gamma") == 1)
    assert torch.all(L.view(p, "conv2_block1_1_bn", "moving_variance") == 1)
    assert torch.all(L.view(p, "conv2_block1_1_conv", "bias") == 0)
    w = L.view(p, "conv4_block2_2_conv", "kernel")
    lim = math.sqrt(6 / (9 * 256 + 9 * 256))
    assert w.abs().max() <= lim and w.abs().max() > 0.9 * lim


def _tiny_engine(B=2, crop=64):
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    e = TorchEngine(L, B, crop=crop)
    e.init(0)
    return L, e


def test_reference_engine_grads_match_autograd_finite_difference():
    torch.manual_seed(0)
    L, e = _tiny_engine(2, 32)
    img = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    lab = torch.tensor([3, 7])
    s = e.forward_backward(img, lab, 0.5)
    assert torch.isfinite(s).all()
    # directional finite difference on the dense bias
    off = L.off("dense", "bias")
    d = torch.zeros(L.total)
    d[off:off + 1000] = torch.randn(1000)
    g = e.grads[off:off + 1000] @ d[off:off + 1000]
    base = e.params.clone()
    eps = 1e-2
    e.params.copy_(base + eps * d)
    lp = e.forward_backward(img, lab, 0.5)[0].item() * 0.5
    e.params.copy_(base - eps * d)
    lm = e.forward_backward(img, lab, 0.5)[0].item() * 0.5
    e.params.copy_(base)
    assert abs((lp - lm) / (2 * eps) - g.item()) < 2e-2 * max(1.0, abs(g.item()))


def test_fused_projection_reference_is_the_same_function():
    """The fused-projection form of the reference (BN scales folded into the conv3 / shortcut
    weights, shifts summed: what the engine's dual-source GEMM computes) is the unfused Keras
    graph in fp32 math -- loss and every gradient agree to fp32 rounding."""
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(0)
    L = ParamLayout()
    img = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    lab = torch.tensor([3, 7])
    out = []
    for fused in (False, True):
        e = TorchEngine(L, 2, crop=32, fused_proj=fused)
        e.init(seed=1)
        g = torch.Generator().manual_seed(4)
        for ent in L.entries.values():   # non-identity BN so the fold is exercised
            sl = e.params[ent.offset:ent.offset + ent.size]
            if ent.kind in ("gamma", "moving_variance"):
                sl.copy_(0.5 + torch.rand(ent.size, generator=g))
            elif ent.kind in ("beta", "bias", "moving_mean"):
                sl.copy_(0.1 * torch.randn(ent.size, generator=g))
        s = e.forward_backward(img, lab, 0.5)
        out.append((s[0].item(), e.grads.clone()))
    (l0, g0), (l1, g1) = out
    assert abs(l0 - l1) <= 1e-5 * abs(l0)
    assert ((g0 - g1).norm() / g0.norm()).item() < 1e-5


def test_frozen_bn_is_inference_mode():
    """training=False in the reference (Q3): BN uses moving stats, which never change."""
    L, e = _tiny_engine(2, 32)
    stats_before = e.params[L.n_trainable:].clone()
    img = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    e.forward_backward(img, torch.tensor([1, 2]), 0.5)
    assert torch.equal(stats_before, e.params[L.n_trainable:])


def test_train_bn_mode_updates_moving_stats():
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    L = ParamLayout()
    e = TorchEngine(L, 2, crop=32, bn_mode="train")
    e.init(0)
    before = e.params[L.n_trainable:].clone()
    img = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    e.forward_backward(img, torch.tensor([1, 2]), 0.5)
    assert not torch.equal(before, e.params[L.n_trainable:])


def test_cpu_adam_matches_keras_formula():
    from pddl.train.optim import Adam
    L, e = _tiny_engine()
    opt = Adam(e, lr=1e-3)
    e.grads.normal_()
    p0 = e.params[:L.n_trainable].clone()
    g = e.grads.clone()
    opt.step()
    lr_t = 1e-3 * math.sqrt(1 - 0.999) / (1 - 0.9)
    m = 0.1 * g
    v = 0.001 * g * g
    ref = p0 - lr_t * m / (v.sqrt() + 1e-7)
    assert torch.allclose(e.params[:L.n_trainable], ref, atol=1e-6)


def test_cpu_sgd_momentum_keras_semantics():
    from pddl.train.optim import SGD
    L, e = _tiny_engine()
    opt = SGD(e, lr=0.1, momentum=0.9)
    e.grads.fill_(1.0)
    p0 = e.params[:L.n_trainable].clone()
    opt.step()
    opt.step()
    # v1 = -0.1; v2 = 0.9*-0.1 - 0.1 = -0.19; p = p0 - 0.29
    assert torch.allclose(e.params[:L.n_trainable], p0 - 0.29, atol=1e-6)


def test_cpu_training_reduces_loss():
    from pddl.train.optim import Adam
    torch.manual_seed(0)
    L, e = _tiny_engine(4, 32)
    opt = Adam(e, lr=1e-3)
    img = torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8)
    lab = torch.tensor([1, 2, 3, 4])
    losses = []
    for _ in range(6):
        s = e.forward_backward(img, lab, 0.25)
        losses.append(s[0].item() / 4)
        opt.step()
    assert losses[-1] < losses[0]


def test_preprocess_semantics():
    from pddl.models.reference import preprocess
    img = torch.arange(2 * 4 * 4 * 3, dtype=torch.float32).view(2, 4, 4, 3) % 256
    x = preprocess(img, 4, True)
    assert torch.allclose(x, img.permute(0, 3, 1, 2) / 255)
    x = preprocess(img, 4, True, flip=torch.tensor([0, 1]))
    assert torch.allclose(x[1], img[1].permute(2, 0, 1).flip(-1) / 255)
    x = preprocess(img, 2, True, crop_offset=(1, 2))
    assert torch.allclose(x, img[:, 1:3, 2:4].permute(0, 3, 1, 2) / 255)
    x = preprocess(img, 8, True)            # RandomCrop larger than the input -> resize (Q1)
    assert x.shape == (2, 3, 8, 8)


def test_ps_bf16_wire_loss_trajectory_tracks_fp32_wire():
    """--ps-wire bf16 (opt-in; the reference's PS moves fp32): the PS keeps fp32 master weights
    and Adam state, the worker pushes bf16-rounded gradients and trains on bf16-rounded pulled
    weights (csrc/runtime/ps_service.cpp, exactly tests/test_gpu_ps.py's pack / Adam kernels).
    Emulated here on the fp32 reference engine over 12 Adam steps on a fixed batch: the bf16-wire
    loss trajectory (6.90 -> 1.38 nats) stays within 3 % / 0.08 nats of the fp32-wire one at every
    step and ends within 1 % of it (measured: at most 2.0 %, 0.047 nats, in the steepest step)."""
    from pddl.train.optim import Adam
    torch.manual_seed(5)
    img = torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8)
    lab = torch.tensor([1, 2, 3, 4])
    traj = {}
    for wire in ("fp32", "bf16"):
        L, e = _tiny_engine(4, 32)
        opt = Adam(e, lr=1e-4)
        master = e.params.clone()
        losses = []
        for _ in range(12):
            # pull: the worker's copy of the PS weights
            e.params.copy_(master.to(torch.bfloat16).float() if wire == "bf16" else master)
            losses.append(e.forward_backward(img, lab, 0.25)[0].item() / 4)
            if wire == "bf16":   # push: bf16-rounded gradient
                e.grads.copy_(e.grads.to(torch.bfloat16).float())
            e.params.copy_(master)   # the PS applies Adam to its fp32 master
            opt.step()
            master.copy_(e.params)
        traj[wire] = losses
    a, b = torch.tensor(traj["fp32"]), torch.tensor(traj["bf16"])
    assert ((a - b).abs() / a.abs()).max().item() < 0.03 and (a - b).abs().max().item() < 0.08, (traj["fp32"], traj["bf16"])
    assert abs(b[-1] - a[-1]) / a[-1] < 0.01 and b[-1] < 0.3 * b[0]
