"""pddl — an MI355X-native (gfx950 / CDNA4) distributed ResNet-50 training framework.

Capabilities mirror rrrickyz/Parallel-and-Distributed-Deep-Learning (8 Keras/TF scripts:
single-process, MirroredStrategy, MultiWorkerMirroredStrategy, ParameterServerStrategy and
Horovod training of ResNet-50 on ImageNet), re-designed MI355X-first:

* every ResNet-50 op is a hand-written HIP kernel (`csrc/kernels`): MFMA implicit-GEMM conv
  forward / dgrad / wgrad with fused frozen-BN + bias + residual + ReLU epilogues, pooling,
  softmax cross-entropy, fused Adam / SGD-momentum;
* the model runs as an explicit forward/backward schedule over preallocated NHWC bf16
  buffers (no autograd tape on the GPU path), fp32 master weights in one flat buffer;
* data parallelism uses RCCL over xGMI (torch.distributed "nccl") with gradient buckets
  carved out of the flat gradient buffer and overlapped with backward.

Import as ``import pddl`` (the repository root ships a small shim, ``pddl.py``).
"""
__version__ = "0.1.0"

from . import config  # noqa: F401
