"""Keras / Horovod callback semantics used by the reference scripts.

* ReduceLROnPlateau(monitor='val_loss', factor=0.1, patience=5, min_lr=1e-5)   imagenet-resnet50.py:64
* EarlyStopping(monitor='val_loss', min_delta=0.001, patience=10)               imagenet-resnet50.py:65
* BroadcastGlobalVariablesCallback(0)                                            imagenet-resnet50-hvd.py:111
* MetricAverageCallback()                                                        imagenet-resnet50-hvd.py:113
* LearningRateWarmupCallback(0.1*size, warmup_epochs=3)                          imagenet-resnet50-hvd.py:115
plus additive ones: ThroughputMeter (images/sec), JsonlLogger, ModelCheckpoint (periodic),
and TimeHistory (the reference's `Total time` print, hvd.py:119-126).

Q11 fix: `fit` averages metrics across ranks BEFORE any callback reads them, so the
LR / stop decisions are identical on every rank (the reference orders MetricAverage after
ReduceLROnPlateau/EarlyStopping, which lets ranks diverge).
"""
from __future__ import annotations

import json
import math
import time
from typing import Dict, Optional

import numpy as np


class Callback:
    trainer = None

    def set_trainer(self, t):
        self.trainer = t

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_batch_begin(self, batch, logs=None): ...
    def on_batch_end(self, batch, logs=None): ...
    def on_train_batches_end(self, epoch): ...   # after the epoch's last training step, before validation
    def get_state(self): return None            # resumable state (--resume), JSON-serialisable
    def set_state(self, state): ...


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="val_loss", factor=0.1, patience=10, min_lr=0.0, min_delta=1e-4, cooldown=0,
                 verbose=0):
        if factor >= 1.0:
            raise ValueError("ReduceLROnPlateau does not support a factor >= 1.0")
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.min_lr, self.min_delta, self.cooldown, self.verbose = min_lr, min_delta, cooldown, verbose
        self.best = np.inf
        self.wait = 0
        self.cooldown_counter = 0

    def on_train_begin(self, logs=None):
        self.best, self.wait, self.cooldown_counter = np.inf, 0, 0

    def get_state(self):
        return {"best": float(self.best), "wait": self.wait, "cooldown_counter": self.cooldown_counter}

    def set_state(self, st):
        self.best, self.wait, self.cooldown_counter = float(st["best"]), int(st["wait"]), int(st["cooldown_counter"])

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        logs["lr"] = self.trainer.lr
        cur = logs.get(self.monitor)
        if cur is None:
            return
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if cur < self.best - self.min_delta:
            self.best = cur
            self.wait = 0
        elif self.cooldown_counter <= 0:
            self.wait += 1
            if self.wait >= self.patience:
                old = self.trainer.lr
                if old > np.float32(self.min_lr):
                    new = max(old * self.factor, self.min_lr)
                    self.trainer.set_lr(new)
                    if self.verbose:
                        self.trainer.log(f"\nEpoch {epoch + 1:05d}: ReduceLROnPlateau reducing learning rate to {new}.")
                    self.cooldown_counter = self.cooldown
                    self.wait = 0


class EarlyStopping(Callback):
    def __init__(self, monitor="val_loss", min_delta=0.0, patience=0, verbose=0):
        self.monitor, self.min_delta, self.patience, self.verbose = monitor, abs(min_delta), patience, verbose
        self.best = np.inf
        self.wait = 0
        self.stopped_epoch = 0

    def on_train_begin(self, logs=None):
        self.best, self.wait, self.stopped_epoch = np.inf, 0, 0

    def get_state(self):
        return {"best": float(self.best), "wait": self.wait}

    def set_state(self, st):
        self.best, self.wait = float(st["best"]), int(st["wait"])

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        self.wait += 1
        if cur + self.min_delta < self.best:     # Keras: monitor_op(current - (-min_delta), best)
            self.best = cur
            self.wait = 0
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            self.trainer.stop_training = True

    def on_train_end(self, logs=None):
        if self.stopped_epoch > 0 and self.verbose:
            self.trainer.log(f"Epoch {self.stopped_epoch + 1:05d}: early stopping")


class BroadcastGlobalVariablesCallback(Callback):
    """Rank `root`'s parameters, BN statistics and optimizer slots are broadcast to every
    rank before the first step (Horovod broadcasts after the first batch so that Keras'
    lazily created slots exist; our flat slots exist up front)."""

    def __init__(self, root_rank=0):
        self.root = root_rank

    def on_train_begin(self, logs=None):
        self.trainer.strategy.broadcast_state(self.trainer, self.root)


class MetricAverageCallback(Callback):
    """Marker: `fit` averages epoch metrics over ranks before other callbacks run (Q11)."""


class LearningRateWarmupCallback(Callback):
    """Horovod warmup: lr(e) = initial_lr / size * (e * (size - 1) / warmup_epochs + 1) for
    fractional epoch e < warmup_epochs (adjusted every batch), then initial_lr."""

    def __init__(self, initial_lr, warmup_epochs=5, size=1, steps_per_epoch=None, verbose=0):
        self.initial_lr, self.warmup_epochs, self.size = initial_lr, warmup_epochs, size
        self.steps_per_epoch, self.verbose = steps_per_epoch, verbose
        self.epoch = 0

    def multiplier(self, epoch_f: float) -> float:
        if epoch_f >= self.warmup_epochs:
            return 1.0
        return 1.0 / self.size * (epoch_f * (self.size - 1) / self.warmup_epochs + 1)

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self.epoch >= self.warmup_epochs:
            return
        spe = self.steps_per_epoch or self.trainer.steps_per_epoch or 1
        e = self.epoch + float(batch) / spe
        self.trainer.set_lr(self.initial_lr * self.multiplier(e))

    def on_epoch_end(self, epoch, logs=None):
        if epoch == self.warmup_epochs - 1 and self.verbose:
            self.trainer.log(f"\nEpoch {epoch + 1}: finished gradual learning rate warmup to {self.initial_lr:g}.")


class ThroughputMeter(Callback):
    """images/sec per epoch (global, excluding the first `skip` steps of each epoch)."""

    def __init__(self, skip=2):
        self.skip = skip
        self.history = []

    def on_epoch_begin(self, epoch, logs=None):
        self.t0 = None
        self.t1 = None
        self.n = 0

    def on_batch_end(self, batch, logs=None):
        if batch + 1 == self.skip:
            self.trainer.sync()
            self.t0 = time.perf_counter()
            self.n = 0
        elif batch + 1 > self.skip:
            self.n += self.trainer.global_batch

    def on_train_batches_end(self, epoch):
        if self.t0 is not None and self.n > 0:   # training steps only: validation is not timed
            self.trainer.sync()
            self.t1 = time.perf_counter()

    def on_epoch_end(self, epoch, logs=None):
        if self.t0 is not None and self.n > 0:
            if self.t1 is None:
                self.trainer.sync()
                self.t1 = time.perf_counter()
            ips = self.n / (self.t1 - self.t0)
            self.history.append(ips)
            if logs is not None:
                logs["images_per_sec"] = ips


class TimeHistory(Callback):
    def on_train_begin(self, logs=None):
        self.t0 = time.time()

    def on_train_end(self, logs=None):
        self.total = time.time() - self.t0
        if self.trainer.strategy.is_chief:
            self.trainer.log(f"Total time:  {round(self.total, 2)} (s)")


class JsonlLogger(Callback):
    """One JSON line per epoch (chief only): the epoch's logs -- loss / accuracy / val_*, lr,
    images_per_sec (ThroughputMeter, runs before this) -- plus the replica count and, with a
    configured 1-GPU rate (`baseline_ips`), the weak-scaling efficiency
    images_per_sec / (replicas * baseline_ips) (utils/scaling.py)."""

    def __init__(self, path, baseline_ips=None):
        self.path = path
        self.baseline_ips = baseline_ips

    def on_epoch_end(self, epoch, logs=None):
        if not self.trainer.strategy.is_chief:
            return
        from ..utils.scaling import efficiency
        rec = {"epoch": epoch + 1, **{k: float(v) for k, v in (logs or {}).items()}}
        n = self.trainer.strategy.num_replicas_in_sync
        rec["replicas"] = n
        if "images_per_sec" in rec and self.baseline_ips:
            rec["baseline_ips"] = float(self.baseline_ips)
            rec["scaling_efficiency"] = efficiency(rec["images_per_sec"], n, self.baseline_ips)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


class ModelCheckpoint(Callback):
    """Additive (not in the reference): periodic checkpoints for --resume."""

    def __init__(self, path_fmt, every=1):
        self.path_fmt, self.every = path_fmt, every

    def on_epoch_end(self, epoch, logs=None):
        if self.every and (epoch + 1) % self.every == 0:
            self.trainer.save(self.path_fmt.format(epoch=epoch + 1), include_optimizer=True, epoch=epoch + 1)
