#!/usr/bin/env python3
"""ResNet-50, MultiWorkerMirroredStrategy equivalent (128 per replica, DATA sharding, SLURM resolver port_base 12345).

Drop-in MI355X-native replacement for the reference script of the same name
(/root/reference/imagenet-resnet50-multiworkers.py).  Defaults reproduce that script; see `--help` for overrides.
Launch: srun -n 2 python imagenet-resnet50-multiworkers.py   or   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 imagenet-resnet50-multiworkers.py
(PDDL_LOCAL_GPUS=4 with 2 processes = the 2 x 4 GPU layout over one 8-rank RCCL communicator)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pddl  # noqa: E402
from pddl.cli import run  # noqa: E402

if __name__ == "__main__":
    sys.exit(run("multiworker"))
