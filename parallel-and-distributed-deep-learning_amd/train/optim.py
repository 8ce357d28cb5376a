"""Flat-buffer optimizers: one fused HIP launch over all trainable parameters.

Adam reproduces TF/Keras `ResourceApplyAdam` (epsilon-hat form; imagenet-resnet50.py:62),
SGD reproduces `keras.optimizers.SGD(momentum, nesterov)` — the north-star optimizer
(BASELINE.json).  On CPU the same update runs as torch ops (reference semantics).
"""
from __future__ import annotations

import math

import torch


class FlatOptimizer:
    def __init__(self, engine, lr: float):
        self.engine = engine
        self.n = engine.L.n_trainable
        self.lr = float(lr)
        self.iterations = 0          # Keras `optimizer.iterations`
        self.params = engine.params[: self.n]
        self.grads = engine.grads
        self.gscale = 1.0

    @property
    def on_gpu(self):
        return self.params.is_cuda

    def state_tensors(self):
        return {}


class Adam(FlatOptimizer):
    def __init__(self, engine, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7):
        super().__init__(engine, lr)
        self.b1, self.b2, self.eps = beta1, beta2, eps
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)

    def step(self):
        self.iterations += 1
        t = self.iterations
        lr_t = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
        if self.on_gpu:
            from ..ops.native import native
            native.adam(self.params, self.grads, self.m, self.v, lr_t, self.b1, self.b2, self.eps, self.gscale)
        else:
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
        self.iterations += 1
        if self.on_gpu:
            from ..ops.native import native
            native.sgd(self.params, self.grads, self.mom, self.lr, self.mu, self.wd, self.nesterov, self.gscale)
        else:
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
