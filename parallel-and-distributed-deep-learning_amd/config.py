"""One dataclass config with per-entrypoint presets.

The reference hard-codes every constant per script; each preset below reproduces one
script's constants (file:line cited), and every field can be overridden from the CLI
(`parse_args`).
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class TrainConfig:
    # identity
    preset: str = "single"
    model_name: str = "ResNet50_ImageNet"          # imagenet-resnet50.py:61
    # data
    data: str = "synthetic"                        # synthetic | records:<dir>
    image_size: int = 224                          # resize_with_crop target (imagenet-resnet50.py:39)
    crop: int = 244                                # RandomCrop(244,244) (imagenet-resnet50.py:54), Q1
    flip: bool = True                              # RandomFlip("horizontal") (imagenet-resnet50.py:55)
    num_classes: int = 1000
    train_images: int = 1281167                    # ImageNet-1k train split
    val_images: int = 50000
    steps_per_epoch: Optional[int] = None          # PS: 312500 (imagenet-resnet50-ps.py:143)
    validation_steps: Optional[int] = None
    seed: int = 0
    # batch
    batch_size: int = 32                           # per replica (imagenet-resnet50.py:46)
    val_batch_size: Optional[int] = None           # MWMS: 256 per replica (multiworkers.py:72)
    global_batch_mode: str = "per_replica"         # per_replica | global (pretrained MWMS: 32*n_workers global)
    # model
    weights: str = "none"                          # none | imagenet | <path.h5>
    bn_mode: str = "frozen"                        # frozen (training=False, Q3) | train
    precision: str = "bf16"                        # bf16 compute, fp32 master
    # optimizer
    optimizer: str = "adam"                        # imagenet-resnet50.py:62
    lr: float = 1e-3                               # Keras Adam default
    lr_scale_by_size: bool = False                 # hvd: lr = 0.1 * size (imagenet-resnet50-hvd.py:99)
    momentum: float = 0.9
    nesterov: bool = False
    weight_decay: float = 0.0
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-7
    # training loop
    epochs: int = 50                               # imagenet-resnet50.py:67
    verbose: int = 2
    reduce_lr_patience: int = 5                    # ReduceLROnPlateau (imagenet-resnet50.py:64)
    reduce_lr_factor: float = 0.1
    min_lr: float = 1e-5
    early_stop_patience: int = 10                  # EarlyStopping (imagenet-resnet50.py:65)
    early_stop_min_delta: float = 1e-3
    warmup_epochs: int = 0                         # hvd LearningRateWarmupCallback (hvd.py:115): 3
    # distribution
    strategy: str = "single"                       # single | mirrored | multiworker | horovod | ps
    bucket_mb: float = 32.0                        # gradient bucket size (7-link xGMI tuned); <= 0: autotune
    grad_dtype: str = "fp32"                       # all-reduce dtype
    num_ps: int = 1
    num_workers: int = 1
    port_base: int = 12345                         # SlurmClusterResolver(port_base=12345) (multiworkers.py:16)
    min_shard_bytes: int = 256 << 10               # MinSizePartitioner (ps.py:77)
    shard_by: str = "batch"                        # hvd: batch-then-shard (hvd.py:77-78); mwms: element DATA
    ps_overlap: bool = True                        # PS: a worker's push/pull round trip overlaps its next step
    ps_wire: str = "bf16"                          # PS: gradient push / parameter pull element type on GPU roles
                                                   # (bf16 halves the xGMI bytes; fp32 master + Adam on the PS; CPU: fp32)
    # device / output
    device: str = "auto"                           # auto | cpu | cuda
    save: bool = True
    save_dir: str = "."
    checkpoint_every: int = 0                      # additive: periodic checkpoints (0 = off)
    resume: Optional[str] = None
    metrics_jsonl: Optional[str] = None
    data_cache: Optional[str] = None               # tfds / folder data: decoded-image cache directory (--cache)
    baseline_ips: Optional[float] = None           # 1-GPU images/sec: the JSONL log adds scaling efficiency
    timeline: Optional[str] = None                 # chrome-trace JSON of the fusion engine
    graphs: Optional[bool] = None                  # HIP graphs: None = auto (on for Mirrored / local replicas)
    roctx: bool = False                            # roctx ranges per step phase (utils/profiling.py)
    max_steps: Optional[int] = None                # cap steps per epoch (smoke / bench)

    def replace(self, **kw) -> "TrainConfig":
        return dataclasses.replace(self, **kw)

    def checkpoint_name(self, n_gpus: Optional[int] = None) -> str:
        """'ImageNet-' + model.name + '-reuse.h5' (imagenet-resnet50.py:69-70); Horovod adds
        '-<N>GPUs' (imagenet-resnet50-hvd.py:127, with the int+str bug Q7 fixed)."""
        if self.preset == "horovod" and n_gpus is not None:
            return f"ImageNet-{self.model_name}-{n_gpus}GPUs-reuse.h5"
        return f"ImageNet-{self.model_name}-reuse.h5"


PRESETS = {
    # imagenet-resnet50.py / imagenet-pretrained-resnet50.py
    "single": dict(strategy="single", model_name="ResNet50_ImageNet", batch_size=32, crop=244),
    "single_pretrained": dict(strategy="single", model_name="ResNet50_ImageNet", batch_size=32, crop=244,
                              weights="imagenet"),
    # imagenet-resnet50-mirror.py:21,54 (global = 32 * replicas)
    "mirrored": dict(strategy="mirrored", model_name="ResNet50_ImageNet_mirror", batch_size=32, crop=244),
    "mirrored_pretrained": dict(strategy="mirrored", model_name="ResNet50_ImageNet_mirror", batch_size=32,
                                crop=244, weights="imagenet"),
    # imagenet-resnet50-multiworkers.py:70,72 (128 / 256 per replica, DATA sharding)
    "multiworker": dict(strategy="multiworker", model_name="ResNet50_ImageNet_Multiworkers", batch_size=128,
                        val_batch_size=256, crop=244, shard_by="element", verbose=1),
    # imagenet-pretrained-resnet50-multiworkers.py:63,65 (global 32 * n_workers)
    "multiworker_pretrained": dict(strategy="multiworker", model_name="ResNet50_Pretrained_ImageNet_Multiworkers",
                                   batch_size=32, crop=244, weights="imagenet", shard_by="element"),
    # imagenet-resnet50-ps.py:77,120,143
    "ps": dict(strategy="ps", model_name="ResNet50_ImageNet_PS", batch_size=32, crop=244,
               steps_per_epoch=312500, validation_steps=1562, num_ps=1, num_workers=1),
    # imagenet-resnet50-hvd.py:25,89,99,115
    "horovod": dict(strategy="horovod", model_name="ResNet50_ImageNet", batch_size=32, crop=160,
                    lr=0.1, lr_scale_by_size=True, warmup_epochs=3, shard_by="batch"),
    # the benchmark configuration (BASELINE.json: synthetic 3x224x224, random init, bf16)
    "bench": dict(strategy="horovod", model_name="ResNet50_ImageNet", batch_size=256, crop=224,
                  lr=1e-3, lr_scale_by_size=False, warmup_epochs=0, save=False, verbose=0),
}


def make_config(preset: str = "single", **overrides) -> TrainConfig:
    if preset not in PRESETS:
        raise ValueError(f"unknown preset {preset!r}; choose from {sorted(PRESETS)}")
    kw = dict(PRESETS[preset])
    kw.update({k: v for k, v in overrides.items() if v is not None})
    kw["preset"] = preset.split("_")[0] if preset.endswith("_pretrained") else preset
    return TrainConfig(**kw)


def add_cli_args(ap: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """CLI overrides shared by every entry script."""
    a = ap.add_argument
    a("--epochs", type=int)
    a("--batch-size", type=int, dest="batch_size")
    a("--val-batch-size", type=int, dest="val_batch_size")
    a("--crop", type=int)
    a("--image-size", type=int, dest="image_size")
    a("--precision", choices=["bf16", "fp32"])
    a("--bn-mode", choices=["frozen", "train"], dest="bn_mode")
    a("--optimizer", choices=["adam", "sgd"])
    a("--lr", type=float)
    a("--momentum", type=float)
    a("--data", type=str)
    a("--cache", type=str, dest="data_cache")
    a("--steps-per-epoch", type=int, dest="steps_per_epoch")
    a("--validation-steps", type=int, dest="validation_steps")
    a("--max-steps", type=int, dest="max_steps")
    a("--bucket-mb", type=float, dest="bucket_mb")
    a("--grad-dtype", choices=["fp32", "bf16"], dest="grad_dtype")
    a("--weights", type=str)
    a("--device", choices=["auto", "cpu", "cuda"])
    a("--seed", type=int)
    a("--save-dir", type=str, dest="save_dir")
    a("--no-save", action="store_false", dest="save", default=None)
    a("--resume", type=str)
    a("--checkpoint-every", type=int, dest="checkpoint_every")
    a("--metrics-jsonl", type=str, dest="metrics_jsonl")
    a("--baseline-ips", type=float, dest="baseline_ips")
    a("--timeline", type=str)
    a("--graphs", action="store_true", default=None)
    a("--no-graphs", action="store_false", dest="graphs", default=None)
    a("--roctx", action="store_true", default=None)
    a("--verbose", type=int)
    a("--ps-wire", choices=["fp32", "bf16"], dest="ps_wire",
      help="PS: element type of the gradient push and the parameter pull (GPU roles)")
    a("--ps-sync", action="store_false", dest="ps_overlap", default=None,
      help="PS: block on every push/pull round trip (no overlap with the next step)")
    return ap


def config_from_args(preset: str, argv: Optional[List[str]] = None, extra=None) -> TrainConfig:
    ap = argparse.ArgumentParser(description=f"pddl ResNet-50 training ({preset})")
    add_cli_args(ap)
    if extra is not None:
        extra(ap)
    ns, _ = ap.parse_known_args(argv)
    kw = {k: v for k, v in vars(ns).items() if v is not None and k in TrainConfig.__dataclass_fields__}
    cfg = make_config(preset, **kw)
    cfg._ns = ns  # type: ignore[attr-defined]
    return cfg
