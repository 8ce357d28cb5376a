#!/usr/bin/env python3
"""ResNet-50, MirroredStrategy equivalent: one process drives every local GPU (global batch 32 x replicas).

Drop-in MI355X-native replacement for the reference script of the same name
(/root/reference/imagenet-resnet50-mirror.py).  Defaults reproduce that script; see `--help` for overrides.
Launch: python imagenet-resnet50-mirror.py   (native RCCL ncclCommInitAll across the local MI355Xs)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pddl  # noqa: E402
from pddl.cli import run  # noqa: E402

if __name__ == "__main__":
    sys.exit(run("mirrored"))
