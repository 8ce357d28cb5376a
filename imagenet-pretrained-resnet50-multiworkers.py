#!/usr/bin/env python3
"""ResNet-50, MultiWorkerMirroredStrategy equivalent, ImageNet-pretrained backbone (global batch 32 x workers).

Drop-in MI355X-native replacement for the reference script of the same name
(/root/reference/imagenet-pretrained-resnet50-multiworkers.py).  Defaults reproduce that script; see `--help` for overrides.
Launch: srun -n N python imagenet-pretrained-resnet50-multiworkers.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pddl  # noqa: E402
from pddl.cli import run  # noqa: E402

if __name__ == "__main__":
    sys.exit(run("multiworker_pretrained"))
