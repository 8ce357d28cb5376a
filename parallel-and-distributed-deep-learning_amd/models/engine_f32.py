"""Reference-precision (fp32) GPU engine: every convolution and the Dense layer run on the
hand-written fp32-MFMA kernels (ops/conv_f32.py -> csrc/kernels/conv_f32.hip); the elementwise
rest of the graph (frozen / batch-statistics BN, ReLU, residual add, max-pool, GAP, softmax
cross-entropy) runs as PyTorch's native GPU kernels with MIOpen switched off, so no library
convolution is involved anywhere in the step.

The graph is models/reference.py's (the Keras model of imagenet-resnet50.py:51-61) with its
convolutions swapped for `conv2d_f32`; activations live channels_last (NHWC in memory), the
layout the kernels read.  Selected by `--precision fp32` on a GPU (parallel/strategies.py);
the bf16 engine (models/engine.py) is the throughput path.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.conv_f32 import conv2d_f32
from .reference import ReferenceResNet50, TorchEngine, preprocess
from .resnet50 import ParamLayout


class HipF32ResNet50(ReferenceResNet50):
    """ReferenceResNet50 with fp32 HIP convolutions (the explicit stem pad becomes the
    kernel's zero padding: same values, no padded copy of the input)."""

    def __init__(self, layout: ParamLayout, bn_mode: str = "frozen"):
        super().__init__(layout, bn_mode, bf16_points=False)

    def _conv(self, params, x, c, pad_explicit=False):
        w = self._w(params, c.name, "kernel")          # OHWI
        b = self._w(params, c.name, "bias")
        return conv2d_f32(x, w, b, c.stride, 0 if pad_explicit else c.pad)

    def features(self, params, x, training=True):
        # the stem's explicit (3, 3, 3, 3) pad folded into the conv's padding
        L = self.L
        s = L.stem
        x = F.relu(self._bn(params, conv2d_f32(x, self._w(params, s.name, "kernel"), self._w(params, s.name, "bias"),
                                               s.stride, 3), s, training))
        x = F.pad(x, (1, 1, 1, 1))
        x = F.max_pool2d(x, 3, 2)
        for b in L.blocks:
            c = b.convs
            sc = self._bn(params, self._conv(params, x, c["0"]), c["0"], training) if b.proj else x
            y = F.relu(self._bn(params, self._conv(params, x, c["1"]), c["1"], training))
            y = F.relu(self._bn(params, self._conv(params, y, c["2"]), c["2"], training))
            y = self._bn(params, self._conv(params, y, c["3"]), c["3"], training)
            x = F.relu(y + sc)
        return x.mean(dim=(2, 3))

    def logits(self, params, x, training=True):
        f = self.features(params, x, training)
        w = self._w(params, "dense", "kernel")        # [classes, 2048]
        out = conv2d_f32(f.view(f.shape[0], -1, 1, 1), w.view(w.shape[0], 1, 1, -1), self._w(params, "dense", "bias"))
        return out.reshape(f.shape[0], -1)


class HipF32Engine(TorchEngine):
    """TorchEngine interface (flat fp32 params / grads, forward_backward, evaluate) over
    HipF32ResNet50 on the GPU."""

    def __init__(self, layout: ParamLayout, batch: int, crop: int = 224, device="cuda", bn_mode="frozen",
                 num_classes: int = 1000):
        super().__init__(layout, batch, crop=crop, device=device, bn_mode=bn_mode, num_classes=num_classes)
        self.model = HipF32ResNet50(layout, bn_mode)

    def forward_backward(self, images, labels, gscale, flip=None, crop_offset=(0, 0), bucket_cb=None, buckets=None):
        with torch.backends.cudnn.flags(enabled=False):
            return super().forward_backward(images, labels, gscale, flip, crop_offset, bucket_cb, buckets)

    @torch.no_grad()
    def evaluate(self, images, labels):
        with torch.backends.cudnn.flags(enabled=False):
            x = preprocess(images.to(self.device), self.crop, False)
            self.model.stats = self.params
            logits = self.model.logits(self.params, x, training=False)
            lab = labels.to(self.device)
            loss_sum = F.cross_entropy(logits, lab, reduction="sum")
            return torch.stack([loss_sum, (logits.argmax(1) == lab).sum().float()])
