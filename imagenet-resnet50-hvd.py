#!/usr/bin/env python3
"""ResNet-50, Horovod-style data parallelism: one process per GPU, Adam(lr=0.1*size) + 3-epoch warmup, rank-0 broadcast, metric averaging, RandomCrop(160), native gradient fusion engine over RCCL.

Drop-in MI355X-native replacement for the reference script of the same name
(/root/reference/imagenet-resnet50-hvd.py).  Defaults reproduce that script; see `--help` for overrides.
Launch: torchrun --nproc-per-node 8 --master-addr 127.0.0.1 imagenet-resnet50-hvd.py   (or mpirun / horovodrun-style OMPI env)
Checkpoint: ImageNet-ResNet50_ImageNet-<N>GPUs-reuse.h5 on rank 0 (the reference's int+str crash, Q7, fixed).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pddl  # noqa: E402
from pddl.cli import run  # noqa: E402

if __name__ == "__main__":
    sys.exit(run("horovod"))
