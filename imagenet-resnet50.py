#!/usr/bin/env python3
"""ResNet-50 on ImageNet, single process (random init, batch 32, RandomCrop 244, Adam, 50 epochs).

Drop-in MI355X-native replacement for the reference script of the same name
(/root/reference/imagenet-resnet50.py).  Defaults reproduce that script; see `--help` for overrides.
Launch: python imagenet-resnet50.py [--data synthetic|records:DIR] [--epochs N]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pddl  # noqa: E402
from pddl.cli import run  # noqa: E402

if __name__ == "__main__":
    sys.exit(run("single"))
