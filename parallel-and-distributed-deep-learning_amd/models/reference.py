"""PyTorch fp32 reference of the reference model (numerics oracle + CPU execution path).

Implements exactly the Keras graph of imagenet-resnet50.py:51-61 with plain PyTorch ops
and autograd, reading parameters as views of the flat layout (models/resnet50.py):
Rescaling(1/255) -> RandomCrop (resize when the crop exceeds the input, Q1; random crop
otherwise, Q2) -> RandomFlip("horizontal") -> ResNet50 v1 with BN in inference mode (Q3,
`training=False`) or batch statistics (`bn_mode="train"`) -> GAP -> Dense -> softmax
cross-entropy.  The GPU engine's kernels are tested against this module.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .resnet50 import BN_EPS, BN_MOMENTUM, ParamLayout


def preprocess(images: torch.Tensor, crop: int, training: bool, flip: Optional[torch.Tensor] = None,
               crop_offset=(0, 0)) -> torch.Tensor:
    """[B,H,W,3] uint8/float (0..255) -> NCHW float32 in [0,1] at crop x crop."""
    x = images.float().permute(0, 3, 1, 2) * (1.0 / 255.0)
    H, W = x.shape[-2:]
    if crop > H or crop > W or (not training and crop != H):
        x = F.interpolate(x, size=(crop, crop), mode="bilinear", align_corners=False, antialias=False)
    elif crop < H:
        oy, ox = crop_offset
        x = x[:, :, oy:oy + crop, ox:ox + crop]
    if training and flip is not None:
        f = flip.to(torch.bool).to(x.device)
        x = torch.where(f.view(-1, 1, 1, 1), x.flip(-1), x)
    return x


class _RoundBF16(torch.autograd.Function):
    """bf16 storage point: the value AND the gradient flowing back through it are rounded to
    bf16 (where the HIP engine stores an activation / writes a dgrad output in bf16)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


class _RoundGradBF16(torch.autograd.Function):
    """Identity forward, bf16-rounded gradient (fp32 logits whose gradient is stored in bf16)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


class ReferenceResNet50:
    """Functional ResNet-50 over a flat parameter buffer (fp32, any device).

    bf16_points=True: the fp32 math with the HIP engine's bf16 storage points (models/engine.py)
    -- the preprocessed input, every fused conv+BN(+residual)+ReLU output, the GAP output, conv
    weights (straight-through: the weight gradient stays fp32), and the gradients stored at those
    points on the way back (dlogits, dpooled, every dgrad output) -- so an engine-vs-reference
    comparison measures accumulation order, not bf16 storage.

    fused_proj=True (frozen BN): a projection block's conv3 and shortcut conv are
    modelled as the engine's ONE dual-source GEMM (`prep_fuse_kernel`, csrc/kernels/eltwise.hip):
    both frozen-BN scales are folded into the weights BEFORE the bf16 rounding,
    `conv(y2, bf16(a3*W3)) + conv(x, bf16(a0*W0)) + (b3 + b0)`, and the shortcut activation is
    never stored (no bf16 point on it)."""

    def __init__(self, layout: ParamLayout, bn_mode: str = "frozen", bf16_points: bool = False,
                 fused_proj: bool = False):
        self.L = layout
        self.bn_mode = bn_mode
        self.bf16 = bf16_points
        self.fused_proj = fused_proj and bn_mode == "frozen"
        self.stats = None   # flat buffer holding the BN moving statistics (non-trainable)
        self._bound = None  # (flat tensor, {name: view}) of the last bind()

    def bind(self, params):
        """Per-tensor views of a flat buffer through ONE `split`: autograd then concatenates
        the per-tensor gradients once, instead of materialising a full-size zero gradient per
        slice (214 x 25.6M floats per backward)."""
        ents = sorted((e for e in self.L.entries.values() if e.offset + e.size <= params.numel()),
                      key=lambda e: e.offset)
        sizes, names, pos = [], [], 0
        for e in ents:
            if e.offset > pos:
                sizes.append(e.offset - pos)
                names.append(None)
            sizes.append(e.size)
            names.append(e)
            pos = e.offset + e.size
        if pos < params.numel():
            sizes.append(params.numel() - pos)
            names.append(None)
        views = {e.name: t.view(e.shape) for e, t in zip(names, torch.split(params, sizes)) if e is not None}
        self._bound = (params, views)

    def _w(self, params, layer, kind):
        if kind in ("moving_mean", "moving_variance") and self.stats is not None:
            return self.L.view(self.stats, layer, kind)
        if self._bound is not None and self._bound[0] is params:
            return self._bound[1][f"{layer}/{kind}:0"]
        return self.L.view(params, layer, kind)

    def _q(self, x):
        return _RoundBF16.apply(x) if self.bf16 else x

    def _conv(self, params, x, c, pad_explicit=False):
        w = self._w(params, c.name, "kernel").permute(0, 3, 1, 2)
        if self.bf16:
            w = w + (w.to(torch.bfloat16).float() - w).detach()
        b = self._w(params, c.name, "bias")
        pad = 0 if pad_explicit else c.pad
        return F.conv2d(x, w, b, stride=c.stride, padding=pad)

    def _bn(self, params, x, c, training):
        g = self._w(params, c.bn, "gamma")
        be = self._w(params, c.bn, "beta")
        mu = self._w(params, c.bn, "moving_mean")
        var = self._w(params, c.bn, "moving_variance")
        if self.bn_mode == "train" and training:
            bm = x.mean(dim=(0, 2, 3))
            bv = x.var(dim=(0, 2, 3), unbiased=False)
            with torch.no_grad():
                n = x.numel() / x.shape[1]
                mu.mul_(BN_MOMENTUM).add_((1 - BN_MOMENTUM) * bm.detach())
                var.mul_(BN_MOMENTUM).add_((1 - BN_MOMENTUM) * bv.detach() * n / max(n - 1, 1))
            mu_, var_ = bm, bv
        else:
            mu_, var_ = mu.detach(), var.detach()
        inv = torch.rsqrt(var_ + BN_EPS)
        return (x - mu_.view(1, -1, 1, 1)) * (g * inv).view(1, -1, 1, 1) + be.view(1, -1, 1, 1)

    def _folded_conv(self, params, x, c):
        """Frozen-BN conv with the BN scale folded into bf16 weights (the fused projection GEMM):
        returns (conv(x, bf16(a*W)), shift b) -- straight-through on the rounding, so W, gamma and
        the bias get the fp32 gradients of the unrounded product."""
        g = self._w(params, c.bn, "gamma")
        be = self._w(params, c.bn, "beta")
        mu = self._w(params, c.bn, "moving_mean").detach()
        var = self._w(params, c.bn, "moving_variance").detach()
        a = g * torch.rsqrt(var + BN_EPS)
        w = self._w(params, c.name, "kernel").permute(0, 3, 1, 2) * a.view(-1, 1, 1, 1)
        if self.bf16:
            w = w + (w.to(torch.bfloat16).float() - w).detach()
        b = (self._w(params, c.name, "bias") - mu) * a + be
        return F.conv2d(x, w, None, stride=c.stride, padding=c.pad), b

    def features(self, params, x, training=True):
        L = self.L
        s = L.stem
        q = self._q
        x = q(F.pad(x, (3, 3, 3, 3)))
        x = q(F.relu(self._bn(params, self._conv(params, x, s, pad_explicit=True), s, training)))
        x = F.pad(x, (1, 1, 1, 1))
        x = F.max_pool2d(x, 3, 2)
        for b in L.blocks:
            c = b.convs
            if b.proj and self.fused_proj:
                y = q(F.relu(self._bn(params, self._conv(params, x, c["1"]), c["1"], training)))
                y = q(F.relu(self._bn(params, self._conv(params, y, c["2"]), c["2"], training)))
                z3, b3 = self._folded_conv(params, y, c["3"])
                z0, b0 = self._folded_conv(params, x, c["0"])
                x = q(F.relu(z3 + z0 + (b3 + b0).view(1, -1, 1, 1)))
                continue
            if b.proj:
                sc = q(self._bn(params, self._conv(params, x, c["0"]), c["0"], training))
            else:
                sc = x
            y = q(F.relu(self._bn(params, self._conv(params, x, c["1"]), c["1"], training)))
            y = q(F.relu(self._bn(params, self._conv(params, y, c["2"]), c["2"], training)))
            y = self._bn(params, self._conv(params, y, c["3"]), c["3"], training)
            x = q(F.relu(y + sc))
        return q(x.mean(dim=(2, 3)))

    def logits(self, params, x, training=True):
        f = self.features(params, x, training)
        w = self._w(params, "dense", "kernel")
        if self.bf16:
            w = w + (w.to(torch.bfloat16).float() - w).detach()
        out = f @ w.t() + self._w(params, "dense", "bias")
        return _RoundGradBF16.apply(out) if self.bf16 else out


class TorchEngine:
    """CPU (or any-device fp32) execution engine with the same interface as the HIP engine.

    Parameters are views of one flat fp32 buffer; `.grad` of each view is a view of the
    flat gradient buffer, so autograd accumulates straight into the bucketed layout.
    """

    def __init__(self, layout: ParamLayout, batch: int, crop: int = 224, device="cpu", bn_mode="frozen",
                 num_classes: int = 1000, bf16_points: bool = False, fused_proj: bool = False):
        self.L = layout
        self.device = torch.device(device)
        self.batch = batch
        self.crop = crop
        self.params = torch.zeros(layout.total, dtype=torch.float32, device=self.device)
        self.grads = torch.zeros(layout.n_trainable, dtype=torch.float32, device=self.device)
        self.model = ReferenceResNet50(layout, bn_mode, bf16_points=bf16_points, fused_proj=fused_proj)
        self.num_classes = num_classes
        self._leaf = None

    def init(self, seed=0):
        self.L.init_params(self.params, seed)
        self.after_update()

    def after_update(self):
        pass

    def forward_backward(self, images, labels, gscale, flip=None, crop_offset=(0, 0), bucket_cb=None, buckets=None):
        # leaf over the trainable prefix; BN statistics are read (and, in train mode,
        # updated in place) straight from the flat buffer
        # (a copy: BN statistics share the flat buffer and train-mode BN updates them in place)
        p = self.params[: self.L.n_trainable].clone().requires_grad_(True)
        self.model.stats = self.params
        self.model.bind(p)
        x = preprocess(images.to(self.device), self.crop, True, flip, crop_offset)
        logits = self.model.logits(p, x, training=True)
        lab = labels.to(self.device)
        loss_sum = F.cross_entropy(logits, lab, reduction="sum")
        (loss_sum * gscale).backward()
        with torch.no_grad():
            self.grads.copy_(p.grad)
            correct = (logits.argmax(1) == lab).sum().float()
            stats = torch.stack([loss_sum.detach(), correct])
        if bucket_cb is not None:   # autograd produces every gradient at once: all buckets ready
            for i in range(len(buckets) if buckets is not None else 1):
                bucket_cb(i)
        return stats

    @torch.no_grad()
    def evaluate(self, images, labels):
        x = preprocess(images.to(self.device), self.crop, False)
        self.model.stats = self.params
        logits = self.model.logits(self.params, x, training=False)
        lab = labels.to(self.device)
        loss_sum = F.cross_entropy(logits, lab, reduction="sum")
        return torch.stack([loss_sum, (logits.argmax(1) == lab).sum().float()])
