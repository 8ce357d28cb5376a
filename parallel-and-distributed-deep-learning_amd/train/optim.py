"""Flat-buffer optimizers: one fused HIP launch over all trainable parameters.

Adam reproduces TF/Keras `ResourceApplyAdam` (epsilon-hat form; imagenet-resnet50.py:62),
SGD reproduces `keras.optimizers.SGD(momentum, nesterov)` — the north-star optimizer
(BASELINE.json).  On CPU the same update runs as torch ops (reference semantics).
"""
from __future__ import annotations

import math

import torch


class FlatOptimizer:
    """On the GPU the step counter and learning rate live in a device buffer
    `hs = {t, lr, lr_t}` advanced by a one-thread kernel, so a captured step (HIP graph)
    replays correctly; host-side changes (LR callbacks, checkpoint restore) are written to it
    before the next step, outside any capture."""

    def __init__(self, engine, lr: float):
        self.engine = engine
        self.n = engine.L.n_trainable
        self.params = engine.params[: self.n]
        self.grads = engine.grads
        self.gscale = 1.0
        self.hs = torch.zeros(4, dtype=torch.float32, device=self.params.device) if self.params.is_cuda else None
        self._lr = float(lr)
        self._iterations = 0         # Keras `optimizer.iterations`
        self._dirty = True

    @property
    def on_gpu(self):
        return self.params.is_cuda

    @property
    def lr(self):
        return self._lr

    @lr.setter
    def lr(self, v):
        self._lr = float(v)
        self._dirty = True

    @property
    def iterations(self):
        return self._iterations

    @iterations.setter
    def iterations(self, v):
        self._iterations = int(v)
        self._dirty = True

    def sync_hparams(self):
        """Write host-side lr / step count into the device buffer (never inside a capture)."""
        if self.hs is not None and self._dirty:
            self.hs.copy_(torch.tensor([float(self._iterations), self._lr, 0.0, 0.0]), non_blocking=False)
            self._dirty = False

    def _device_step(self, adam: bool, b1=0.0, b2=0.0):
        from ..ops.native import native
        if not torch.cuda.is_current_stream_capturing():
            self.sync_hparams()
        native.opt_hparams(self.hs, b1, b2, adam)

    def state_tensors(self):
        return {}


class Adam(FlatOptimizer):
    def __init__(self, engine, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7):
        super().__init__(engine, lr)
        self.b1, self.b2, self.eps = beta1, beta2, eps
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)

    def step(self):
        if self.on_gpu:
            from ..ops.native import native
            self._device_step(True, self.b1, self.b2)
            self._iterations += 1
            native.adam(self.params, self.grads, self.m, self.v, 0.0, self.b1, self.b2, self.eps, self.gscale, self.hs)
        else:
            self._iterations += 1
            t = self._iterations
            lr_t = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
            g = self.grads * self.gscale
            self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            self.params.sub_(lr_t * self.m / (self.v.sqrt() + self.eps))

    def state_tensors(self):
        return {"m": self.m, "v": self.v}


class SGD(FlatOptimizer):
    def __init__(self, engine, lr=0.1, momentum=0.9, nesterov=False, weight_decay=0.0):
        super().__init__(engine, lr)
        self.mu, self.nesterov, self.wd = momentum, nesterov, weight_decay
        self.mom = torch.zeros_like(self.params)

    def step(self):
        if self.on_gpu:
            from ..ops.native import native
            self._device_step(False)
            self._iterations += 1
            native.sgd(self.params, self.grads, self.mom, 0.0, self.mu, self.wd, self.nesterov, self.gscale, self.hs)
        else:
            self._iterations += 1
            g = self.grads * self.gscale + self.wd * self.params
            self.mom.mul_(self.mu).sub_(self.lr * g)
            if self.nesterov:
                self.params.add_(self.mu * self.mom - self.lr * g)
            else:
                self.params.add_(self.mom)

    def state_tensors(self):
        return {"momentum": self.mom}


def make_optimizer(name: str, engine, lr: float, **kw) -> FlatOptimizer:
    if name == "adam":
        return Adam(engine, lr, kw.get("beta1", 0.9), kw.get("beta2", 0.999), kw.get("eps", 1e-7))
    if name == "sgd":
        return SGD(engine, lr, kw.get("momentum", 0.9), kw.get("nesterov", False), kw.get("weight_decay", 0.0))
    raise ValueError(f"unknown optimizer {name!r}")
