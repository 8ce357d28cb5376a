"""Strategy-agnostic fit loop (Keras `model.fit` semantics; reference imagenet-resnet50.py:62-67).

The loop is identical for every distribution strategy, as `strategy.scope()` + `model.fit`
is identical across the reference scripts (imagenet-resnet50-mirror.py:64-81 vs
imagenet-resnet50.py:51-67).  Per epoch: iterate the (sharded) training pipeline, one
`strategy.train_step` per batch, accumulate [loss_sum, correct] on the device (no host sync
per step), reduce metrics across replicas, validate, run callbacks, print the Keras-style
epoch line on the chief, stop on EarlyStopping.  `model.save` at the end goes through the
strategy (chief-only write, fixing the reference's every-worker-same-file race, Q8).
"""
from __future__ import annotations

import math
import sys
import time
from typing import Dict, List, Optional

import torch

from .callbacks import (Callback, EarlyStopping, JsonlLogger, ModelCheckpoint, ReduceLROnPlateau, ThroughputMeter,
                        TimeHistory)


class History:
    def __init__(self):
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []

    def append(self, epoch, logs):
        self.epoch.append(epoch)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(v)


class Trainer:
    def __init__(self, cfg, strategy):
        self.cfg = cfg
        self.strategy = strategy
        self.stop_training = False
        self.steps_per_epoch = None
        self.lr = cfg.lr * (strategy.num_replicas_in_sync if cfg.lr_scale_by_size else 1)
        strategy.setup(self)
        strategy.set_lr(self.lr)

    # -- helpers used by callbacks
    @property
    def global_batch(self) -> int:
        return self.strategy.global_batch

    def set_lr(self, lr: float):
        self.lr = float(lr)
        self.strategy.set_lr(self.lr)

    def sync(self):
        self.strategy.sync()

    def log(self, msg: str):
        if self.strategy.is_chief:
            print(msg, flush=True)

    def progress(self, epochs_done: int) -> dict:
        """What --resume needs beyond weights and optimizer slots: completed epochs, the
        current LR (ReduceLROnPlateau / warmup may have moved it) and callback state."""
        cbs = {type(cb).__name__: cb.get_state() for cb in getattr(self, "callbacks", [])
               if cb.get_state() is not None}
        return {"epoch": int(epochs_done), "lr": float(self.lr), "callbacks": cbs}

    def save(self, path: str, include_optimizer: bool = True, epoch: Optional[int] = None):
        prog = self.progress(epoch) if epoch is not None else None
        self.strategy.save(self, path, include_optimizer=include_optimizer, progress=prog)

    # -- the loop
    def fit(self, epochs: int, callbacks: Optional[List[Callback]] = None, validation: bool = True,
            steps_per_epoch: Optional[int] = None, validation_steps: Optional[int] = None,
            initial_epoch: int = 0) -> History:
        cfg = self.cfg
        st = self.strategy
        cbs = list(callbacks or [])
        self.callbacks = cbs
        for cb in cbs:
            cb.set_trainer(self)
        hist = History()
        train_pipe = st.train_pipeline()
        val_pipe = st.val_pipeline() if validation else None
        spe = steps_per_epoch or cfg.steps_per_epoch or train_pipe.num_batches()
        if cfg.max_steps:
            spe = min(spe, cfg.max_steps)
        self.steps_per_epoch = spe
        vsteps = validation_steps or cfg.validation_steps
        if val_pipe is not None:
            vsteps = min(vsteps or val_pipe.num_batches(), val_pipe.num_batches() if not val_pipe.repeat else 10 ** 12)
            if cfg.max_steps:
                vsteps = min(vsteps, cfg.max_steps)
        for cb in cbs:
            cb.on_train_begin()
        rs = getattr(self, "resume_state", None)
        if rs:                                    # --resume: continue the callbacks' bookkeeping
            for cb in cbs:
                cst = rs.get("callbacks", {}).get(type(cb).__name__)
                if cst is not None:
                    cb.set_state(cst)
        it = train_pipe.iterate(st.device, epoch=initial_epoch) if train_pipe.repeat else None
        for epoch in range(initial_epoch, epochs):
            if self.stop_training:
                break
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            self.log(f"Epoch {epoch + 1}/{epochs}")
            t0 = time.time()
            acc = torch.zeros(2, dtype=torch.float64, device=st.metrics_device)
            n_seen = 0
            batches = it if it is not None else train_pipe.iterate(st.device, epoch=epoch)
            for step in range(spe):
                try:
                    images, labels = next(batches)
                except StopIteration:
                    break
                for cb in cbs:
                    cb.on_batch_begin(step)
                s = st.train_step(images, labels)
                acc += s.to(acc.device, torch.float64)
                n_seen += images.shape[0]
                for cb in cbs:
                    cb.on_batch_end(step)
                if cfg.verbose == 1 and st.is_chief and (step + 1) % max(1, spe // 20) == 0:
                    print(f"\r{step + 1}/{spe}", end="", flush=True)
            if cfg.verbose == 1 and st.is_chief:
                print()
            for cb in cbs:
                cb.on_train_batches_end(epoch)
            # metric reduction across replicas happens BEFORE callbacks read logs (Q11)
            tot = st.reduce_metrics(torch.cat([acc, torch.tensor([float(n_seen)], dtype=torch.float64,
                                                                 device=acc.device)]))
            logs = {"loss": tot[0] / max(tot[2], 1), "accuracy": tot[1] / max(tot[2], 1)}
            if val_pipe is not None and vsteps:
                vacc = torch.zeros(3, dtype=torch.float64, device=st.metrics_device)
                vit = val_pipe.iterate(st.device, epoch=0)
                for vs in range(vsteps):
                    try:
                        vi, vl = next(vit)
                    except StopIteration:
                        break
                    s = st.eval_step(vi, vl)
                    vacc[:2] += s.to(vacc.device, torch.float64)
                    vacc[2] += vi.shape[0]
                vt = st.reduce_metrics(vacc)
                logs["val_loss"] = vt[0] / max(vt[2], 1)
                logs["val_accuracy"] = vt[1] / max(vt[2], 1)
            logs = {k: float(v) for k, v in logs.items()}
            dt = time.time() - t0
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            logs["lr"] = self.lr
            hist.append(epoch, logs)
            if cfg.verbose and st.is_chief:
                parts = [f"{k}: {v:.4f}" for k, v in logs.items() if k not in ("lr", "images_per_sec")]
                ips = logs.get("images_per_sec")
                extra = f" - {ips:.1f} img/s" if ips else ""
                print(f"{spe}/{spe} - {int(dt)}s - " + " - ".join(parts) + f" - lr: {self.lr:.4g}"
                      + f" - {dt / max(spe, 1) * 1000:.0f}ms/step{extra}", flush=True)
        for cb in cbs:
            cb.on_train_end()
        return hist


def default_callbacks(cfg, strategy, extra: Optional[List[Callback]] = None) -> List[Callback]:
    """The callback list every reference script passes to fit (imagenet-resnet50.py:64-65),
    plus the Horovod ones for the horovod preset (imagenet-resnet50-hvd.py:106-115)."""
    from .callbacks import BroadcastGlobalVariablesCallback, LearningRateWarmupCallback, MetricAverageCallback
    cbs: List[Callback] = []
    if cfg.strategy in ("horovod", "multiworker", "mirrored"):
        cbs.append(BroadcastGlobalVariablesCallback(0))
        cbs.append(MetricAverageCallback())
    cbs.append(ReduceLROnPlateau(monitor="val_loss", factor=cfg.reduce_lr_factor, patience=cfg.reduce_lr_patience,
                                 min_lr=cfg.min_lr))
    cbs.append(EarlyStopping(monitor="val_loss", min_delta=cfg.early_stop_min_delta, patience=cfg.early_stop_patience))
    if cfg.warmup_epochs:
        size = strategy.num_replicas_in_sync
        cbs.append(LearningRateWarmupCallback(cfg.lr * (size if cfg.lr_scale_by_size else 1),
                                              warmup_epochs=cfg.warmup_epochs, size=size, verbose=1))
    cbs.append(ThroughputMeter())
    cbs.append(TimeHistory())
    if cfg.metrics_jsonl:
        cbs.append(JsonlLogger(cfg.metrics_jsonl, cfg.baseline_ips))
    if cfg.checkpoint_every:
        cbs.append(ModelCheckpoint(f"{cfg.save_dir}/ckpt-{{epoch:03d}}.h5", cfg.checkpoint_every))
    cbs += list(extra or [])
    return cbs
