"""Keras-v1 ResNet-50 topology, Keras layer/weight names, and the flat parameter layout.

Reference: the model every script builds (imagenet-resnet50.py:51-61):
    Input(224,224,3) -> Rescaling(1/255) -> RandomCrop(c,c) -> RandomFlip ->
    keras.applications.ResNet50(include_top=False, weights=None|'imagenet', pooling='avg')
    called with training=False -> Dense(1000, softmax)
Topology facts: stride on the first 1x1 conv of a block (v1), conv biases on,
BN epsilon 1.001e-5, ZeroPadding2D(3) + 7x7/s2 stem, ZeroPadding2D(1) + MaxPool 3x3/s2.
Total parameters 25,636,712 (25,583,592 trainable + 53,120 BN moving statistics).

Layout (MI355X-first): all parameters live in ONE fp32 buffer.  The trainable prefix is
ordered by backward completion (dense kernel first, stem kernel last, then every
per-channel vector in a tail), so gradient buckets for the overlapped all-reduce are plain
contiguous slices of the flat gradient buffer — no pack/unpack kernels.  Conv kernels are
stored OHWI ([Cout][R][S][Cin], K-contiguous for the implicit GEMM); checkpoints transpose
to Keras HWIO.  A block's conv1 and projection conv0 are adjacent so one GEMM computes both
(forward: one read of x; backward: one wgrad and one dgrad).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

BN_EPS = 1.001e-5       # keras.applications.resnet: BatchNormalization(epsilon=1.001e-5)
BN_MOMENTUM = 0.99      # Keras default


@dataclass
class ConvSpec:
    name: str           # Keras Conv2D name, e.g. "conv2_block1_1_conv"
    cin: int
    cout: int
    k: int
    stride: int
    pad: int
    bn: Optional[str]   # Keras BatchNormalization name
    relu: bool


@dataclass
class BlockSpec:
    name: str           # "conv2_block1"
    cin: int
    filters: int
    stride: int
    proj: bool
    convs: Dict[str, ConvSpec] = field(default_factory=dict)   # keys "0" (proj), "1", "2", "3"


def resnet50_blocks() -> Tuple[ConvSpec, List[BlockSpec]]:
    stem = ConvSpec("conv1_conv", 3, 64, 7, 2, 3, "conv1_bn", True)
    blocks: List[BlockSpec] = []
    cin = 64
    for stage, (f, n, s1) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)], start=2):
        for b in range(1, n + 1):
            name = f"conv{stage}_block{b}"
            stride = s1 if b == 1 else 1
            proj = b == 1
            blk = BlockSpec(name, cin, f, stride, proj)
            if proj:
                blk.convs["0"] = ConvSpec(f"{name}_0_conv", cin, 4 * f, 1, stride, 0, f"{name}_0_bn", False)
            blk.convs["1"] = ConvSpec(f"{name}_1_conv", cin, f, 1, stride, 0, f"{name}_1_bn", True)
            blk.convs["2"] = ConvSpec(f"{name}_2_conv", f, f, 3, 1, 1, f"{name}_2_bn", True)
            blk.convs["3"] = ConvSpec(f"{name}_3_conv", f, 4 * f, 1, 1, 0, f"{name}_3_bn", False)
            blocks.append(blk)
            cin = 4 * f
    return stem, blocks


@dataclass
class Entry:
    name: str                 # Keras weight name, e.g. "conv1_conv/kernel:0"
    layer: str
    kind: str                 # kernel | bias | gamma | beta | moving_mean | moving_variance
    shape: Tuple[int, ...]    # internal shape (conv kernels OHWI, dense kernel [out][in])
    keras_shape: Tuple[int, ...]
    offset: int
    size: int
    trainable: bool


class ParamLayout:
    """Flat fp32 parameter layout with Keras names and gradient buckets."""

    def __init__(self, num_classes: int = 1000, align: int = 64):
        self.num_classes = num_classes
        self.stem, self.blocks = resnet50_blocks()
        self.entries: Dict[str, Entry] = {}
        self.order: List[str] = []
        self._off = 0
        self.align = align
        convs_fwd = [self.stem] + [c for b in self.blocks for c in self._block_conv_order(b)]
        self.convs = convs_fwd
        # --- trainable kernels in backward-completion order
        self._add("dense", "kernel", (num_classes, 2048), (2048, num_classes), True)
        for b in reversed(self.blocks):
            for key in ("3", "2", "1", "0"):
                if key in b.convs:
                    c = b.convs[key]
                    self._add(c.name, "kernel", (c.cout, c.k, c.k, c.cin), (c.k, c.k, c.cin, c.cout), True)
        c = self.stem
        self._add(c.name, "kernel", (c.cout, c.k, c.k, c.cin), (c.k, c.k, c.cin, c.cout), True)
        self.kernels_end = self._off
        # --- trainable per-channel tail (one bucket)
        self._add("dense", "bias", (num_classes,), (num_classes,), True)
        for c in convs_fwd:
            self._add(c.name, "bias", (c.cout,), (c.cout,), True)
            self._add(c.bn, "gamma", (c.cout,), (c.cout,), True)
            self._add(c.bn, "beta", (c.cout,), (c.cout,), True)
        self.n_trainable = self._pad(self._off)
        self._off = self.n_trainable
        # --- non-trainable BN statistics
        for c in convs_fwd:
            self._add(c.bn, "moving_mean", (c.cout,), (c.cout,), False)
            self._add(c.bn, "moving_variance", (c.cout,), (c.cout,), False)
        self.total = self._pad(self._off)

    @staticmethod
    def _block_conv_order(b: BlockSpec) -> List[ConvSpec]:
        keys = ["1", "0", "2", "3"] if b.proj else ["1", "2", "3"]
        return [b.convs[k] for k in keys]

    def _pad(self, n: int) -> int:
        return (n + self.align - 1) // self.align * self.align

    def _add(self, layer, kind, shape, keras_shape, trainable):
        size = int(np.prod(shape))
        name = f"{layer}/{kind}:0"
        self.entries[name] = Entry(name, layer, kind, tuple(shape), tuple(keras_shape), self._off, size, trainable)
        self.order.append(name)
        self._off += size

    # ------------------------------------------------------------------ queries
    def off(self, layer: str, kind: str) -> int:
        return self.entries[f"{layer}/{kind}:0"].offset

    def entry(self, layer: str, kind: str) -> Entry:
        return self.entries[f"{layer}/{kind}:0"]

    def count(self, trainable: Optional[bool] = None) -> int:
        return sum(e.size for e in self.entries.values() if trainable is None or e.trainable == trainable)

    def view(self, flat: torch.Tensor, layer: str, kind: str) -> torch.Tensor:
        e = self.entry(layer, kind)
        return flat[e.offset:e.offset + e.size].view(e.shape)

    def buckets(self, bucket_mb: float, elem_bytes: int = 4) -> List[Tuple[int, int]]:
        """Contiguous [start, end) ranges of the trainable prefix, in backward-completion
        order, each about `bucket_mb` MiB, split at tensor boundaries; the per-channel tail
        is always its own final bucket."""
        limit = max(1, int(bucket_mb * (1 << 20) / elem_bytes))
        out: List[Tuple[int, int]] = []
        start = 0
        kern = [e for e in self.entries.values() if e.trainable and e.kind == "kernel"]
        kern.sort(key=lambda e: e.offset)
        cur_end = 0
        for e in kern:
            end = e.offset + e.size
            if end - start > limit and cur_end > start:
                out.append((start, cur_end))
                start = cur_end
            cur_end = end
        if cur_end > start:
            out.append((start, cur_end))
        out.append((self.kernels_end, self.n_trainable))
        return out

    # ------------------------------------------------------------------ init
    def init_params(self, flat: torch.Tensor, seed: int = 0) -> None:
        """Keras defaults: glorot_uniform kernels, zero biases, BN gamma=1 beta=0 mean=0 var=1."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        host = torch.zeros(self.total, dtype=torch.float32)
        for e in self.entries.values():
            sl = host[e.offset:e.offset + e.size]
            if e.kind == "kernel":
                if len(e.keras_shape) == 4:
                    kh, kw, ci, co = e.keras_shape
                    fan_in, fan_out = kh * kw * ci, kh * kw * co
                else:
                    fan_in, fan_out = e.keras_shape
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                sl.uniform_(-lim, lim, generator=g)
            elif e.kind in ("gamma", "moving_variance"):
                sl.fill_(1.0)
        flat.copy_(host.to(flat.device))


def param_count_keras() -> Dict[str, int]:
    lay = ParamLayout()
    return {"total": lay.count(), "trainable": lay.count(True), "non_trainable": lay.count(False)}
