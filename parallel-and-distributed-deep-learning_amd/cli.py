"""Shared `main` of the drop-in entry scripts.

Each reference script (8 files under /root/reference) has a same-named script at the
repository root that calls `run(<preset>)`: identical defaults (batch, crop, optimizer,
epochs, callbacks, checkpoint file name), CLI overrides on top.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import List, Optional

from .config import config_from_args


def _banner(cfg, strategy):
    import torch
    print(f"Using pddl {__import__('pddl').__version__} (torch {torch.__version__}, HIP {torch.version.hip}), "
          f"strategy={cfg.strategy}, replicas={strategy.num_replicas_in_sync}, "
          f"per-replica batch={strategy.per_replica_batch}, global batch={strategy.global_batch}, "
          f"crop={cfg.crop}, bn={cfg.bn_mode}, optimizer={cfg.optimizer}", flush=True)


def model_summary(cfg) -> str:
    from .models.resnet50 import ParamLayout
    L = ParamLayout(cfg.num_classes)
    return (f'Model: "{cfg.model_name}"\n'
            f"  input_1 (InputLayer) [(None, {cfg.image_size}, {cfg.image_size}, 3)]\n"
            f"  rescaling (Rescaling)  random_crop (RandomCrop {cfg.crop}x{cfg.crop})  random_flip (RandomFlip)\n"
            f"  resnet50 (Functional) (None, 2048)   {L.count() - 2048 * cfg.num_classes - cfg.num_classes:,}\n"
            f"  dense (Dense) (None, {cfg.num_classes})  {2048 * cfg.num_classes + cfg.num_classes:,}\n"
            f"Total params: {L.count():,}\nTrainable params: {L.count(True):,}\n"
            f"Non-trainable params: {L.count(False):,}")


def run(preset: str, argv: Optional[List[str]] = None, extra=None) -> int:
    from .parallel.strategies import make_strategy
    from .train.trainer import Trainer, default_callbacks
    cfg = config_from_args(preset, argv, extra)
    if cfg.strategy == "ps":
        if cfg.resume:
            # (the PS job's variables and Adam slots live on the PS roles; the reference has no
            # resume path at all, imagenet-resnet50-ps.py:142-148)
            sys.stderr.write("--resume is not supported for --strategy ps: the parameter-server job restarts from "
                             "--weights (the final PS checkpoint holds the trained variables, no optimizer state)\n")
            return 2
        from .parallel.parameter_server import run_ps_job
        return run_ps_job(cfg)
    if cfg.roctx:
        from .utils import profiling
        profiling.enable(True)
    strategy = make_strategy(cfg)
    trainer = Trainer(cfg, strategy)
    if strategy.is_chief:
        _banner(cfg, strategy)
        if cfg.verbose:
            print(model_summary(cfg), flush=True)
    if cfg.strategy == "multiworker":
        # the reference's informational print (imagenet-resnet50-multiworkers.py:76; 10M-image
        # epoch assumption, Q9) -- printed by every worker, as there
        print("Steps per epoch: ", int((10000000 / strategy.num_replicas_in_sync) / strategy.world), flush=True)
    cbs = default_callbacks(cfg, strategy)
    initial_epoch = 0
    rs = getattr(strategy, "resume_state", None)
    if rs:          # --resume of a periodic checkpoint: epochs, LR and callback state continue
        initial_epoch = int(rs.get("epoch", 0))
        trainer.set_lr(float(rs.get("lr", trainer.lr)))
        trainer.resume_state = rs
        if strategy.is_chief:
            print(f"Resuming after epoch {initial_epoch} at lr {trainer.lr:.4g}", flush=True)
    trainer.fit(cfg.epochs, cbs, initial_epoch=initial_epoch)
    if cfg.timeline and hasattr(strategy, "write_timeline"):
        strategy.write_timeline(cfg.timeline)
    if cfg.save:
        fname = os.path.join(cfg.save_dir, cfg.checkpoint_name(n_gpus=strategy.num_replicas_in_sync))
        if strategy.is_chief:
            print("Saving model to ", fname, flush=True)
        trainer.save(fname)
    if cfg.strategy in ("horovod", "multiworker"):
        print("All done for rank", strategy.rank, flush=True)
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
    except Exception:
        pass
    return 0
