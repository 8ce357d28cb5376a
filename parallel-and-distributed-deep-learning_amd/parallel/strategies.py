"""Distribution strategies, one interface for the strategy-agnostic fit loop.

| reference                                     | here                      | transport                       |
|-----------------------------------------------|---------------------------|---------------------------------|
| no strategy (imagenet-resnet50.py)            | SingleStrategy            | —                               |
| MirroredStrategy (imagenet-resnet50-mirror.py:21)     | MirroredStrategy  | native RcclComm (ncclCommInitAll), one replica thread per GPU |
| MultiWorkerMirroredStrategy (multiworkers.py:20-26)   | MultiWorkerStrategy | 1 GPU/process: c10d "nccl" (RCCL); R GPUs/process: native RcclComm over all P*R ranks |
| Horovod (imagenet-resnet50-hvd.py:15-115)     | HorovodStrategy           | native FusionEngine over c10d (RCCL), buckets overlapped with backward |
| ParameterServerStrategy (imagenet-resnet50-ps.py:75-84) | parallel/parameter_server.py | p2p push/pull |

Interface: setup(trainer), train_pipeline()/val_pipeline() (= distribute
dataset), train_step(images, labels), eval_step, reduce_metrics(t), set_lr, broadcast_state,
is_chief, num_replicas_in_sync, save.  Gradient math: every replica scales its loss by
1 / global_batch, so a SUM all-reduce yields the global-batch mean gradient (= Horovod's
Average of per-rank means; = Mirrored's sum of per-replica grads of loss/global_batch).
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..data.datasets import Pipeline, make_source
from ..models.resnet50 import ParamLayout
from ..train.optim import make_optimizer
from ..utils import profiling as prof
from ..utils.envopts import opt
from .collectives import BucketAllReducer
from .faults import StepFaults
from .launch import ClusterInfo, export_torch_env, resolve_cluster


def rehearsing() -> bool:
    """PDDL_REHEARSE=1: several ranks / replicas may share one GPU (1-GPU rehearsals of the
    multi-GPU code).  Outside a rehearsal a rank never wraps onto another rank's device."""
    return os.environ.get("PDDL_REHEARSE", "0") == "1"


def stall_timeout() -> float:
    """Seconds a gradient collective may stay incomplete before the stall watchdogs (fusion
    engine, native RCCL communicator) report it (Horovod's HOROVOD_STALL_CHECK_TIME_SECONDS)."""
    return float(os.environ.get("PDDL_STALL_TIMEOUT", "60"))


def stall_shutdown() -> float:
    """Grace after a stall report before the process exits 124 (HOROVOD_STALL_SHUTDOWN_TIME_SECONDS);
    0 = report only (the next collective call raises)."""
    return float(os.environ.get("PDDL_STALL_SHUTDOWN", "0"))


def stall_abort() -> bool:
    """Whether the native RCCL watchdog aborts the communicators on a stall (irreversible).  Off
    by default -- like Horovod's stall check it only reports, so a slow but live peer (a cold
    input pipeline, a long validation or checkpoint) does not end the job; on with
    PDDL_STALL_ABORT=1 or a PDDL_STALL_SHUTDOWN grace (bench.py sets 30 s)."""
    return os.environ.get("PDDL_STALL_ABORT", "0") == "1" or stall_shutdown() > 0


def collective_timeout():
    """c10d process-group timeout: ProcessGroupNCCL's own watchdog tears the process down when a
    collective exceeds it, so a dead peer cannot hang a rank inside a device synchronize."""
    import datetime
    return datetime.timedelta(seconds=float(os.environ.get("PDDL_COLLECTIVE_TIMEOUT", "600")))


def gpu_available() -> bool:
    return torch.cuda.is_available() and torch.cuda.device_count() > 0


def build_engine(cfg, device: torch.device, cap: int, graphed=None):
    """On a GPU: the bf16 HIP engine (bf16 MFMA kernels; frozen or train-mode BN), or for
    precision=fp32 the reference-precision engine on the fp32-MFMA HIP convolutions
    (models/engine_f32.py).  On CPU: the fp32 PyTorch reference engine (config 1 of
    BASELINE.json: CPU plumbing).  graphed (default: cfg.graphs is True): the step will replay
    from HIP graphs, which keep the shallower gradient rings (HipEngine.GRAD_RING) and stay on
    one stream (HipEngine.TWO_STREAM_MAX_BATCH); "segmented": bucket-segmented graphs whose
    weight gradients replay as a side graph per segment (HipEngine._side_run)."""
    L = ParamLayout(cfg.num_classes)
    if device.type == "cuda" and cfg.precision == "bf16":
        from ..models.engine import HipEngine, make_hip_engine
        if graphed is None:
            graphed = cfg.graphs is True
        return make_hip_engine(L, cap, bn_mode=cfg.bn_mode, crop=cfg.crop, image_size=cfg.image_size,
                               device=device, num_classes=cfg.num_classes,
                               grad_ring=HipEngine.GRAD_RING if graphed else None, graphed=graphed)
    if device.type == "cuda":
        from ..models.engine_f32 import HipF32Engine, HipF32EngineBNTrain
        # frozen: the reference's configuration; train: batch statistics (both explicit fp32 schedules)
        cls = HipF32Engine if cfg.bn_mode == "frozen" else HipF32EngineBNTrain
        return cls(L, cap, crop=cfg.crop, image_size=cfg.image_size, device=device, num_classes=cfg.num_classes)
    from ..models.reference import TorchEngine
    return TorchEngine(L, cap, crop=cfg.crop, device=device, bn_mode=cfg.bn_mode, num_classes=cfg.num_classes)


class Augment:
    """RandomFlip (per image) and RandomCrop offset (per batch, crop < input) draws."""

    def __init__(self, cfg, device, seed):
        self.cfg = cfg
        self.device = device
        self.gen = torch.Generator(device=device).manual_seed(seed)
        self.rng = np.random.default_rng(seed)

    def __call__(self, B):
        flip = None
        if self.cfg.flip:
            flip = torch.randint(0, 2, (B,), dtype=torch.uint8, device=self.device, generator=self.gen)
        off = (0, 0)
        if self.cfg.crop < self.cfg.image_size:
            m = self.cfg.image_size - self.cfg.crop
            off = (int(self.rng.integers(0, m + 1)), int(self.rng.integers(0, m + 1)))
        return flip, off


class Strategy:
    name = "base"

    def __init__(self, cfg):
        self.cfg = cfg
        self.rank = 0
        self.world = 1
        self.local_replicas = 1
        self.device = torch.device("cpu")
        self.engine = None
        self.opt = None

    # ------------------------------------------------------------------ properties
    @property
    def num_replicas_in_sync(self) -> int:
        return self.world * self.local_replicas

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def per_replica_batch(self) -> int:
        return self.cfg.batch_size

    @property
    def global_batch(self) -> int:
        return self.per_replica_batch * self.num_replicas_in_sync

    @property
    def metrics_device(self):
        return self.device

    def _pick_device(self, local_index: int = 0) -> torch.device:
        want = self.cfg.device
        if want == "cpu" or (want == "auto" and not gpu_available()):
            return torch.device("cpu")
        have = torch.cuda.device_count()
        if local_index >= have:
            if not rehearsing():
                raise RuntimeError(f"local rank {local_index} needs GPU {local_index} but only {have} GPU(s) are "
                                   "visible: launch at most one rank per visible GPU (PDDL_REHEARSE=1 lets "
                                   "rehearsal ranks share devices)")
            local_index %= have
        torch.cuda.set_device(local_index)
        return torch.device("cuda", local_index)

    # ------------------------------------------------------------------ setup
    def setup(self, trainer):
        self._build(trainer)
        self._load_initial_weights()

    def _make_engine_and_opt(self, device, cap):
        eng = build_engine(self.cfg, device, cap)
        eng.init(seed=self.cfg.seed)
        opt = make_optimizer(self.cfg.optimizer, eng, lr=self.cfg.lr, momentum=self.cfg.momentum,
                             nesterov=self.cfg.nesterov, weight_decay=self.cfg.weight_decay, beta1=self.cfg.beta1,
                             beta2=self.cfg.beta2, eps=self.cfg.adam_eps)
        return eng, opt

    def _build(self, trainer):
        raise NotImplementedError

    def _load_initial_weights(self):
        w = self.cfg.weights
        if self.cfg.resume:
            from ..utils.checkpoint import load_checkpoint, read_resume_state
            for eng, opt in self._replicas():
                load_checkpoint(self.cfg.resume, eng, opt)
                eng.after_update()
            self.resume_state = read_resume_state(self.cfg.resume)
        elif w and w != "none":
            from ..utils.checkpoint import load_pretrained
            for eng, _ in self._replicas():
                load_pretrained(w, eng)
                eng.after_update()

    def _replicas(self):
        return [(self.engine, self.opt)]

    # ------------------------------------------------------------------ data
    def _pipe(self, split: str, batch: int, shards: int, index: int) -> Pipeline:
        cfg = self.cfg
        src = make_source(cfg.data, split, cfg)
        # Real data is read in a fresh permutation every epoch (the reference's
        # shuffle_files=True, imagenet-resnet50.py:31; folder sources list files class by
        # class).  Every rank uses the same seed, so the shards of one epoch stay disjoint.
        shuffle = split == "train" and cfg.data not in ("synthetic", "synthetic_fixed")
        return Pipeline(src, batch, num_shards=shards, shard_index=index, shard_by=cfg.shard_by,
                        repeat=cfg.strategy == "ps", shuffle=shuffle, seed=cfg.seed)

    def train_pipeline(self) -> Pipeline:
        return self._pipe("train", self.per_replica_batch * self.local_replicas, self.world, self.rank)

    def val_pipeline(self) -> Pipeline:
        vb = (self.cfg.val_batch_size or self.cfg.batch_size) * self.local_replicas
        return self._pipe("val", vb, self.world, self.rank)

    # ------------------------------------------------------------------ steps
    def _fault_tick(self):
        if not hasattr(self, "_faults"):
            self._faults = StepFaults(self.rank)
        self._faults.tick()

    def set_lr(self, lr: float):
        for _, opt in self._replicas():
            opt.lr = lr

    def eval_step(self, images, labels):
        return self.engine.evaluate(images, labels).clone()

    def reduce_metrics(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu()

    def broadcast_state(self, trainer, root: int = 0):
        pass

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def save(self, trainer, path: str, include_optimizer: bool = True, progress: Optional[dict] = None):
        if not self.is_chief:
            return
        from ..utils.checkpoint import save_keras_h5
        save_keras_h5(path, self.engine, self.opt if include_optimizer else None, self.cfg, progress=progress)


class SingleStrategy(Strategy):
    """One process, one device (imagenet-resnet50.py)."""
    name = "single"

    def _build(self, trainer):
        self.device = self._pick_device(0)
        cap = max(self.cfg.batch_size, self.cfg.val_batch_size or 0)
        self.engine, self.opt = self._make_engine_and_opt(self.device, cap)
        self.aug = Augment(self.cfg, self.device, self.cfg.seed)
        self.graphed = None
        if self.cfg.graphs and self.device.type == "cuda" and hasattr(self.engine, "wbf"):
            from ..train.graph import GraphedTrainStep   # HIP-graph replay of the whole step
            B = self.cfg.batch_size
            self.graphed = GraphedTrainStep(self.engine, self.opt, B, (self.cfg.image_size, self.cfg.image_size),
                                            1.0 / B)

    def train_step(self, images, labels):
        self._fault_tick()
        B = images.shape[0]
        flip, off = self.aug(B)
        if self.graphed is not None and B == self.graphed.B and tuple(images.shape[1:3]) == self.graphed.images.shape[1:3]:
            return self.graphed(images.to(self.device, non_blocking=True), labels.to(self.device, non_blocking=True),
                                flip, off).clone()
        eng = self.engine
        s = eng.forward_backward(images, labels, 1.0 / B, flip=flip, crop_offset=off).clone()
        self.opt.step()
        eng.after_update()
        return s


class _ProcessGroupMixin:
    def _init_process_group(self, info: ClusterInfo):
        export_torch_env(info)
        self.rank, self.world = info.rank, info.world_size
        self.info = info
        if not dist.is_initialized() and info.world_size > 1:   # (a 1-rank job needs no rendezvous)
            backend = "nccl" if self.device.type == "cuda" else "gloo"
            # PDDL_DIST_BACKEND=gloo: rehearse GPU ranks sharing one device (RCCL refuses that)
            backend = os.environ.get("PDDL_DIST_BACKEND", backend)
            kw = {"timeout": collective_timeout()}
            if backend == "nccl":
                kw["device_id"] = self.device
            dist.init_process_group(backend, init_method="env://", rank=info.rank, world_size=info.world_size, **kw)

    def reduce_metrics(self, t):
        if self.world > 1:
            x = t.to(self.device if self.device.type == "cuda" else "cpu", torch.float64)
            dist.all_reduce(x)
            return x.cpu()
        return t.cpu()

    def broadcast_state(self, trainer, root=0):
        if self.world <= 1:
            return
        dist.broadcast(self.engine.params, root)
        for t in self.opt.state_tensors().values():
            dist.broadcast(t, root)
        self.engine.after_update()


class HorovodStrategy(_ProcessGroupMixin, Strategy):
    """One process per GPU (horovodrun / mpirun / torchrun / srun), Horovod semantics:
    shard-after-batch data (hvd.py:77-78), rank-0 broadcast, metric averaging, LR scaled by
    size + warmup (callbacks), and gradient buckets all-reduced by the native fusion engine
    while backward runs (DistributedOptimizer, hvd.py:101)."""
    name = "horovod"

    def __init__(self, cfg, comm: str = "fusion"):
        super().__init__(cfg)
        self.comm = comm

    # (Round 6 removed the graphed-rank variant -- the step replayed from bucket-segmented HIP
    # graphs with each bucket all-reduced on a native RCCL communicator between the segment
    # replays: at the Horovod preset's b32 / crop 160 it ran 3.81 ms per step against 3.19 ms
    # eager with the FusionEngine (profiles/r6_mirror_host_loop.txt), and a rank issues only
    # its own ~220 launches, which the eager step hides behind the GPU.)
    def _build(self, trainer):
        info = resolve_cluster(port_base=self.cfg.port_base)
        self.device = self._pick_device(info.local_rank if gpu_available() else 0)
        self._init_process_group(info)
        cap = max(self.cfg.batch_size, self.cfg.val_batch_size or 0)
        self.engine, self.opt = self._make_engine_and_opt(self.device, cap)
        self.aug = Augment(self.cfg, self.device, self.cfg.seed + 1000 * self.rank)
        self.graphed = None
        if self.world == 1 and self.cfg.graphs and self.device.type == "cuda" and hasattr(self.engine, "wbf"):
            from ..train.graph import GraphedTrainStep   # one rank: the whole step as one HIP graph
            B = self.cfg.batch_size
            self.graphed = GraphedTrainStep(self.engine, self.opt, B, (self.cfg.image_size, self.cfg.image_size),
                                            1.0 / B)
        # bucket_mb <= 0: autotune (Horovod's HOROVOD_AUTOTUNE analogue for the fusion threshold)
        self._tune = None
        mb = self.cfg.bucket_mb
        if mb <= 0 and self.world > 1:
            self._tune = {"cands": [8.0, 16.0, 32.0, 64.0], "i": 0, "t": [], "best": []}
            mb = self._tune["cands"][0]
        self._make_reducer(mb if mb > 0 else 32.0)

    def _make_reducer(self, bucket_mb: float):
        if getattr(self, "fusion", None) is not None:
            self.fusion.shutdown()
        self.bucket_mb = bucket_mb
        self.buckets = self.engine.L.buckets(bucket_mb)
        self.fusion = None
        self.reducer = None
        if self.world > 1:
            if self.comm == "fusion":
                from ..ops.native import native_available, require_native
                if native_available():
                    self.fusion = require_native().FusionEngine(
                        dist.group.WORLD, self.engine.grads, [(s, e - s) for s, e in self.buckets],
                        stall_timeout(), False, self.rank, self.cfg.grad_dtype)
                    self.fusion.set_stall_shutdown(stall_shutdown())
                    if self.cfg.timeline:
                        self.fusion.set_timeline(True)
            if self.fusion is None:
                self.reducer = BucketAllReducer(self.engine.grads, self.buckets, comm_dtype=self.cfg.grad_dtype,
                                                stall_timeout=stall_timeout())
        elif os.environ.get("PDDL_COMM_PROXY") and self.device.type == "cuda":
            # 1 GPU: paced CU-holding stand-ins for the buckets' RCCL all-reduces (bench --comm-proxy)
            from .collectives import CommProxy
            self.reducer = CommProxy(self.engine.grads, self.buckets, os.environ["PDDL_COMM_PROXY"])

    _TUNE_STEPS = int(os.environ.get("PDDL_AUTOTUNE_STEPS", "4"))   # per candidate: 1 discarded + rest timed

    def _autotune_step(self, images, labels):
        """Time a few steps per bucket size; rank 0's pick (min median) is broadcast so every
        rank builds the same buckets (the collectives must match)."""
        import time as _t
        tu = self._tune
        self.sync()
        t0 = _t.perf_counter()
        s = self._step(images, labels)
        self.sync()
        tu["t"].append(_t.perf_counter() - t0)
        if len(tu["t"]) == self._TUNE_STEPS:
            tu["best"].append(float(np.median(tu["t"][1:] or tu["t"])))
            tu["t"] = []
            tu["i"] += 1
            if tu["i"] < len(tu["cands"]):
                self._make_reducer(tu["cands"][tu["i"]])
            else:
                pick = [tu["cands"][int(np.argmin(tu["best"]))]]
                dist.broadcast_object_list(pick, src=0)
                if self.is_chief:
                    ms = ", ".join(f"{c:g} MiB: {b * 1e3:.1f} ms" for c, b in zip(tu["cands"], tu["best"]))
                    print(f"[autotune] gradient bucket size {pick[0]:g} MiB ({ms})", flush=True)
                self._make_reducer(pick[0])
                self._tune = None
        return s

    def train_step(self, images, labels):
        self._fault_tick()
        if getattr(self, "mirror", None) is not None:
            return self.mirror.step(images, labels, self.global_batch)
        if self._tune is not None:
            return self._autotune_step(images, labels)
        return self._step(images, labels)

    def _replicas(self):
        m = getattr(self, "mirror", None)
        return m.replicas if m is not None else super()._replicas()

    def broadcast_state(self, trainer, root=0):
        if getattr(self, "mirror", None) is not None:
            self.mirror.broadcast()      # (RCCL broadcast of parameters + optimizer slots from rank 0)
        else:
            super().broadcast_state(trainer, root)

    def _step(self, images, labels):
        g = getattr(self, "graphed", None)
        if g is not None and images.shape[0] == g.B and tuple(images.shape[1:3]) == tuple(g.images.shape[1:3]):
            flip, off = self.aug(images.shape[0])
            return g(images.to(self.device, non_blocking=True), labels.to(self.device, non_blocking=True),
                     flip, off).clone()
        s = self.compute_gradients(images, labels)
        prof.push("step/optimizer")
        self.opt.step()
        self.engine.after_update()
        prof.pop()
        return s

    def compute_gradients(self, images, labels):
        """Forward + backward + the bucketed all-reduce, without applying the update
        (Optimizer.compute_gradients of the reference's DistributedOptimizer,
        imagenet-resnet50-hvd.py:101): afterwards `engine.grads` holds the global-batch mean
        gradient on every rank.  Returns the step's (loss sum, correct) stats."""
        if getattr(self, "mirror", None) is not None:
            return self.mirror.compute_gradients(images, labels, self.global_batch)
        B = images.shape[0]
        flip, off = self.aug(B)
        gscale = 1.0 / (B * self.world)
        cb = None
        bks = self.buckets
        if self.fusion is not None:
            self.fusion.begin_step()
            cb = self.fusion.bucket_ready
        elif self.reducer is not None:
            self.reducer.begin()
            cb = self.reducer.on_bucket_ready
        s = self.engine.forward_backward(images, labels, gscale, flip=flip, crop_offset=off, bucket_cb=cb,
                                         buckets=bks).clone()
        prof.push("step/allreduce")
        if self.fusion is not None:
            self.fusion.finish()
        elif self.reducer is not None:
            self.reducer.finish()
        prof.pop()
        return s

    def write_timeline(self, path: str):
        js = None
        if self.fusion is not None:
            js = self.fusion.timeline_json()
        elif getattr(self, "mirror", None) is not None:
            js = self.mirror.timeline_json(self.rank)
        if js is not None:
            with open(f"{path}.rank{self.rank}.json", "w") as f:
                f.write(js)


class MultiWorkerStrategy(HorovodStrategy):
    """MultiWorkerMirroredStrategy (imagenet-resnet50-multiworkers.py): SLURM-resolved worker
    processes (SlurmClusterResolver(port_base=12345)), element-wise DATA sharding, synchronous
    all-reduce.  With several GPUs per worker process (PDDL_LOCAL_GPUS=R, e.g. 2 procs x 4
    GPUs, multiworkers.py:20-26), each process drives R local replicas and ONE native RCCL
    communicator spans all P*R replicas (unique id exchanged through the c10d store).  On CPU
    the same layout runs R CPU replicas per process with the cross-process sum over gloo (the
    test double of that communicator)."""
    name = "multiworker"

    def __init__(self, cfg, local_gpus: Optional[int] = None):
        super().__init__(cfg, comm="bucket")
        self.req_local = int(os.environ.get("PDDL_LOCAL_GPUS", local_gpus or 1))

    def _local_devices(self, info: ClusterInfo) -> list:
        R = self.req_local
        want_gpu = self.cfg.device == "cuda" or (self.cfg.device == "auto" and gpu_available())
        if not want_gpu:
            return ["cpu"] * R
        if not gpu_available():
            raise RuntimeError(f"PDDL_LOCAL_GPUS={R} with device={self.cfg.device!r} but no GPU is visible")
        have = torch.cuda.device_count()
        devs = [info.local_rank * R + i for i in range(R)]
        if devs[-1] >= have:
            if os.environ.get("PDDL_REHEARSE", "0") != "1":
                raise RuntimeError(f"local rank {info.local_rank} needs GPUs {devs[0]}..{devs[-1]} "
                                   f"(PDDL_LOCAL_GPUS={R}) but only {have} are visible")
            devs = [d % have for d in devs]    # rehearsal: replicas share devices (no RCCL)
        return devs

    def _build(self, trainer):
        if self.req_local <= 1:
            return super()._build(trainer)
        info = resolve_cluster(port_base=self.cfg.port_base)
        R = self.req_local
        devs = self._local_devices(info)
        self.local_replicas = R
        # control plane: gloo process group over the same rendezvous
        export_torch_env(info)
        self.rank, self.world = info.rank, info.world_size
        if not dist.is_initialized() and self.world > 1:
            dist.init_process_group("gloo", init_method="env://", rank=info.rank, world_size=info.world_size,
                                    timeout=collective_timeout())
        self.mirror = _LocalReplicas(self.cfg, devs, global_rank_base=self.rank * R, world_ranks=self.world * R)
        self.engine, self.opt = self.mirror.replicas[0]
        self.device = self.mirror.devices[0]

    def _replicas(self):
        return self.mirror.replicas if hasattr(self, "mirror") else super()._replicas()

    def reduce_metrics(self, t):
        if self.req_local > 1 and hasattr(self, "mirror") and self.world > 1:
            x = t.to("cpu", torch.float64)       # (the P x R layout's control group is gloo)
            dist.all_reduce(x)
            return x
        return super().reduce_metrics(t)

    def train_step(self, images, labels):
        if not hasattr(self, "mirror"):
            return super().train_step(images, labels)
        self._fault_tick()
        return self.mirror.step(images, labels, self.global_batch)

    def broadcast_state(self, trainer, root=0):
        if hasattr(self, "mirror"):
            self.mirror.broadcast()
        else:
            super().broadcast_state(trainer, root)


class _LocalReplicas:
    """R model replicas in this process, one per device; gradients are summed across every
    replica of the job.

    GPU (distinct devices): ONE native RCCL communicator (in-process ncclCommInitAll for
    Mirrored, ncclCommInitRank over P processes for multi-worker).  By default every replica's
    step is replayed from HIP graphs segmented at the gradient-bucket boundaries
    (train/graph.py SegmentedStepGraphs): segment k on all devices, then the grouped all-reduce
    of bucket k on per-device comm streams while segment k+1 computes, then a captured
    optimizer graph per device -- so one host thread drives R GPUs with ~R*(nb+1) graph
    launches per step (no per-kernel Python launch cost).  cfg.graphs=False (--no-graphs): eager
    replica threads (launch bindings release the GIL) with the same bucket overlap.

    CPU (and rehearsals with replicas sharing a device): replicas run in turn and the
    reduction is an in-process sum, plus a gloo all-reduce across processes when replicas of
    the job live in other processes (the multi-worker test double of the RCCL communicator)."""

    def __init__(self, cfg, devices: List, global_rank_base: int = 0, world_ranks: Optional[int] = None):
        self.cfg = cfg
        self.devices = [torch.device(d) if not isinstance(d, int) else torch.device("cuda", d) for d in devices]
        self.R = len(self.devices)
        world_ranks = world_ranks or self.R
        self.world_ranks = world_ranks
        self.cross = world_ranks > self.R           # replicas of the job in other processes
        cap = max(cfg.batch_size, cfg.val_batch_size or 0)
        self.replicas = []
        self.augs = []
        # (several replicas / ranks replay graphed segments unless --no-graphs; one replica in the
        # whole job runs eager unless --graphs)
        single = self._single_replica_job()
        graphed = cfg.graphs is True or (cfg.graphs is None and not single)
        # (segmented replica graphs defer their weight gradients into side graphs; a one-replica
        # job's --graphs whole-step graph stays one stream: GraphedTrainStep captures no side graphs)
        graphed = ("segmented" if not single else True) if graphed else False
        for i, d in enumerate(self.devices):
            if d.type == "cuda":
                torch.cuda.set_device(d)
            eng = build_engine(cfg, d, cap, graphed=graphed)
            eng.init(seed=cfg.seed)
            opt = make_optimizer(cfg.optimizer, eng, lr=cfg.lr, momentum=cfg.momentum, nesterov=cfg.nesterov,
                                 weight_decay=cfg.weight_decay, beta1=cfg.beta1, beta2=cfg.beta2, eps=cfg.adam_eps)
            self.replicas.append((eng, opt))
            self.augs.append(Augment(cfg, d, cfg.seed + 7919 * (global_rank_base + i)))
        self.comm = None
        self.gpu = self.devices[0].type == "cuda"
        distinct = len({str(d) for d in self.devices}) == self.R
        if self.gpu and distinct:
            from ..ops.native import require_native
            N = require_native()
            # (PDDL_RCCL_INIT=rank forces the multi-process constructor for a single-process job:
            # the 1-GPU test of MWMS's P x R path)
            if world_ranks == self.R and os.environ.get("PDDL_RCCL_INIT", "all") != "rank":
                self.comm = N.RcclComm.init_all([d.index for d in self.devices])
            else:
                uid = N.RcclComm.unique_id() if global_rank_base == 0 else b""
                obj = [uid]
                if dist.is_initialized() and dist.get_world_size() > 1:
                    dist.broadcast_object_list(obj, src=0)
                self.comm = N.RcclComm(world_ranks, obj[0], [global_rank_base + i for i in range(self.R)],
                                       [d.index for d in self.devices])
            # stall watchdog: a bucket collective not complete within the timeout is reported;
            # with stall_abort() the communicators are aborted (blocked kernels exit), the next
            # step raises with the bucket id and the rank exits 124 after the shutdown grace
            self.comm.set_watchdog(stall_timeout(), stall_shutdown(), global_rank_base, stall_abort())
        self.graph_mode = (self.comm is not None and hasattr(self.replicas[0][0], "wbf")
                           and (cfg.graphs if cfg.graphs is not None else True))
        self.graphs = None
        self.buckets = None
        # graph launch stream per replica (None: train/graph.py replay_stream of its device; the
        # host-loop rehearsal with every replica on one device gives each its own)
        self.launch_streams = None

    # ------------------------------------------------------------------ state
    def broadcast(self):
        if self.comm is not None:
            self.comm.broadcast([e.params for e, _ in self.replicas], 0)
            for k in self.replicas[0][1].state_tensors():
                self.comm.broadcast([o.state_tensors()[k] for _, o in self.replicas], 0)
        else:
            e0, o0 = self.replicas[0]
            if self.cross:
                dist.broadcast(e0.params, 0)
                for t in o0.state_tensors().values():
                    dist.broadcast(t, 0)
            for e, o in self.replicas[1:]:
                e.params.copy_(e0.params)
                for k, t in o.state_tensors().items():
                    t.copy_(o0.state_tensors()[k])
        for e, _ in self.replicas:
            e.after_update()

    def _split(self, images, labels):
        """Per-replica (images, labels) on each replica's device: a list (one pre-placed batch
        per device) or one global batch split along dim 0."""
        if isinstance(images, (list, tuple)):
            assert len(images) == self.R and len(labels) == self.R
            return [(im.to(d, non_blocking=True), lb.to(d, non_blocking=True))
                    for im, lb, d in zip(images, labels, self.devices)]
        B = images.shape[0] // self.R
        return [(images[i * B:(i + 1) * B].to(d, non_blocking=True), labels[i * B:(i + 1) * B].to(d, non_blocking=True))
                for i, d in enumerate(self.devices)]

    def _sum_stats(self, stats):
        out = stats[0].to(self.devices[0]).clone()
        for s in stats[1:]:
            out = out + s.to(self.devices[0])
        return out

    # ------------------------------------------------------------------ graphed step
    def _bucket_mb(self) -> float:
        return self.cfg.bucket_mb if self.cfg.bucket_mb > 0 else 32.0

    def _capture(self, parts, global_batch: int):
        from ..train.graph import SegmentedStepGraphs
        eng0 = self.replicas[0][0]
        B = parts[0][0].shape[0]
        # (tail cuts: b256 segmented 19,182 -> 19,431 img/s, b32 7,622 -> 7,522: on from batch 128)
        tc = opt("PDDL_MIRROR", "tail_cuts", "auto")
        bks = eng0.L.buckets(self._bucket_mb())
        self.buckets = self._split_tail(bks, eng0.L) if (tc == "1" or (tc == "auto" and B >= 128)) else bks
        H, W = parts[0][0].shape[1:3]
        self.graphs = []
        for (eng, optim), d in zip(self.replicas, self.devices):
            with torch.cuda.device(d):
                g = SegmentedStepGraphs(eng, optim, B, (H, W), 1.0 / global_batch, self.buckets,
                                        image_dtype=parts[0][0].dtype)
                g.capture()
                self.graphs.append(g)
        self.comm_streams = [torch.cuda.Stream(device=d) for d in self.devices]
        self.evs = [[torch.cuda.Event() for _ in self.devices] for _ in self.buckets]
        # deferred replicas: segment k's side graph runs on the engine's side stream after segment
        # k; bucket k's all-reduce waits for it (sevs[k])
        self.deferred = all(g.deferred for g in self.graphs)
        self.sevs = [[torch.cuda.Event() for _ in self.devices] for _ in self.buckets] if self.deferred else None
        self._plan_cache = None   # (raw handles of the previous capture's graphs and events)
        # bf16 wire (cfg.grad_dtype, Horovod's fp16 compression analogue): each bucket is rounded
        # into a bf16 copy on the comm stream, all-reduced, and widened back into the fp32 grads
        self.lowp = None
        if self.cfg.grad_dtype == "bf16":
            self.lowp = [torch.empty(e.grads.numel(), dtype=torch.bfloat16, device=d)
                         for (e, _), d in zip(self.replicas, self.devices)]
        # timeline (cfg.timeline): READY / ALLREDUCE per bucket from GPU events of device 0
        self.tl = None
        if self.cfg.timeline:
            d0 = self.devices[0]
            mk = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
            with torch.cuda.device(d0):
                self.tl = {"t0": mk(), "b": [(mk(), mk(), mk()) for _ in self.buckets], "steps": 0}
        self._gb = global_batch

    @staticmethod
    def _split_tail(bks, L):
        """The last kernel bucket (stage 2-3 and the stem: few parameters, much of the backward's
        time) split at every block boundary inside it, so the side graphs of those blocks run
        under the next blocks' data gradients instead of after the last segment."""
        if len(bks) < 2:
            return bks
        s, e = bks[-2]
        cuts = set()
        for b in L.blocks:
            last = L.entry(b.convs["0" if b.proj else "1"].name, "kernel")
            off = last.offset + last.size
            if s < off < e:
                cuts.add(off)
        edges = [s] + sorted(cuts) + [e]
        return bks[:-2] + [(a, b) for a, b in zip(edges, edges[1:])] + bks[-1:]

    def _graphed_step(self, parts, global_batch: int):
        """Segment k on every device, then the grouped all-reduce of bucket k on per-device comm
        streams while segment k + 1 computes, then the optimizer graphs after the comm streams.
        Each phase of the R devices is ONE native call (graph_launch_group: launches, event
        records and stream waits with the GIL released), so the host loop is the runtime's graph
        submission plus nb collective calls; with one-stream graphs (small batches) a phase's R
        launches run concurrently on the native launch pool (R = 8, b32:
        profiles/r6_mirror_host_loop.txt)."""
        B = parts[0][0].shape[0]
        if self.graphs is None or self.graphs[0].B != B or self._gb != global_batch:
            out = self._eager_step(parts, global_batch)   # first step eager (lazy tables), then capture
            self._capture(parts, global_batch)
            return out
        from ..ops.native import native, require_native
        N = require_native()
        grads = [e.grads for e, _ in self.replicas]
        # Graphs are launched on a stream of their own, never on the legacy default stream: a
        # multi-branch graph (the two-stream backward) launched there segfaulted inside
        # hipGraphLaunch (its parallel-stream table read as garbage) once the process had run
        # other graphs -- train/graph.py replay_stream
        from ..train.graph import replay_stream
        amb = [torch.cuda.current_stream(d) for d in self.devices]
        cur = self.launch_streams or [replay_stream(d) for d in self.devices]
        # inputs staged on the ambient streams (where the batch was produced); the first group
        # launch makes each launch stream wait for them, the optimizer's hands the step back
        for r, (g, d) in enumerate(zip(self.graphs, self.devices)):
            with torch.cuda.device(d):
                flip, off = self.augs[r](B)
                g.load(parts[r][0], parts[r][1], flip, off)
        P = self._plan(cur, amb)
        streams = P["comm"]
        tl = self.tl
        par = P["parallel"]
        dfr = self.deferred
        for k, (s, e) in enumerate(self.buckets):
            first = k == 0
            # segment k (main graph); with deferred replicas its end forks to the side stream,
            # whose graph k then forks to the comm stream
            N.graph_launch_group(P["dev"], P["seg"][k], P["cur"], P["in_ev"] if first else [],
                                 P["amb"] if first else [], P["ev"][k], P["sides"] if dfr else P["comm"], par)
            if dfr:
                N.graph_launch_group(P["dev"], P["side"][k], P["sides"], [], [], P["sev"][k], P["comm"], par)
            if first and tl is not None:
                tl["t0"].record(cur[0])
            if tl is not None:
                tl["b"][k][0].record(self.replicas[0][0].side if dfr else cur[0])
                tl["b"][k][1].record(self.comm_streams[0])
            if self.lowp is None:
                self.comm.all_reduce_on([gr[s:e] for gr in grads], "sum", streams, f"bucket {k} all_reduce")
            else:
                for r, d in enumerate(self.devices):
                    with torch.cuda.device(d), torch.cuda.stream(self.comm_streams[r]):
                        native.cast_bf16(grads[r][s:e], self.lowp[r][s:e])
                self.comm.all_reduce_on([lp[s:e] for lp in self.lowp], "sum", streams, f"bucket {k} all_reduce (bf16)")
                for r, d in enumerate(self.devices):
                    with torch.cuda.device(d), torch.cuda.stream(self.comm_streams[r]):
                        native.cast_f32(self.lowp[r][s:e], grads[r][s:e])
            if tl is not None:
                tl["b"][k][2].record(self.comm_streams[0])
        for g in self.graphs:
            g.opt.sync_hparams()
        N.graph_launch_group(P["dev"], P["opt"], P["cur"], P["cdone"], P["comm"], P["out_ev"], P["amb"], par)
        for g in self.graphs:
            g.opt._iterations += 1
        if tl is not None:
            tl["steps"] += 1
        return self._sum_stats([g.stats for g in self.graphs])

    def _plan(self, cur, amb):
        """Raw handles of the graphed step's native group launches (per launch / ambient stream set)."""
        key = tuple(c.cuda_stream for c in cur) + tuple(a.cuda_stream for a in amb)
        if getattr(self, "_plan_cache", None) and self._plan_cache[0] == key:
            return self._plan_cache[1]
        R = self.R
        if not hasattr(self, "_cdone"):
            self._cdone = [torch.cuda.Event() for _ in range(R)]
            self._in_ev = [torch.cuda.Event() for _ in range(R)]
            self._out_ev = [torch.cuda.Event() for _ in range(R)]
        for r in range(R):      # (a torch event exists once recorded: create every handle now)
            with torch.cuda.device(self.devices[r]):
                for k in range(len(self.buckets)):
                    self.evs[k][r].record(cur[r])
                    if self.deferred:
                        self.sevs[k][r].record(self.replicas[r][0].side)
                self._cdone[r].record(self.comm_streams[r])
                self._in_ev[r].record(amb[r])
                self._out_ev[r].record(cur[r])
        ex = [g.exec_handles() for g in self.graphs]
        P = {"dev": [d.index for d in self.devices], "cur": [c.cuda_stream for c in cur],
             "amb": [a.cuda_stream for a in amb],
             "in_ev": [e.cuda_event for e in self._in_ev], "out_ev": [e.cuda_event for e in self._out_ev],
             "comm": [cs.cuda_stream for cs in self.comm_streams],
             "seg": [[ex[r][0][k] for r in range(R)] for k in range(len(self.buckets))],
             "opt": [ex[r][1] for r in range(R)],
             "ev": [[self.evs[k][r].cuda_event for r in range(R)] for k in range(len(self.buckets))],
             "cdone": [e.cuda_event for e in self._cdone],
             # (the launch pool runs one-stream graphs only: graph_launch.cpp -- deferred replicas'
             # main and side graphs are; PDDL_MIRROR pool=0 keeps every launch in this thread)
             "parallel": (opt("PDDL_MIRROR", "pool", True)
                          and (self.deferred or all(e.side is None for e, _ in self.replicas)))}
        if self.deferred:
            P["sides"] = [e.side.cuda_stream for e, _ in self.replicas]
            P["side"] = [[ex[r][2][k] for r in range(R)] for k in range(len(self.buckets))]
            P["sev"] = [[self.sevs[k][r].cuda_event for r in range(R)] for k in range(len(self.buckets))]
        self._plan_cache = (key, P)
        return P

    def timeline_json(self, rank: int = 0) -> Optional[str]:
        """Chrome-trace JSON of the last graphed step (device 0): per bucket READY (its segment
        replayed) and ALLREDUCE (the grouped RCCL call on the comm stream), microseconds from
        the step start -- the FusionEngine timeline's phases for the graphed replicas."""
        import json
        tl = getattr(self, "tl", None)
        if tl is None or not tl["steps"]:
            return None
        torch.cuda.synchronize(self.devices[0])
        ev = []
        for k, (ready, start, end) in enumerate(tl["b"]):
            s, e = self.buckets[k]
            args = {"bytes": (e - s) * (2 if self.lowp is not None else 4), "step": tl["steps"], "clock": "gpu"}
            ev.append({"name": "READY", "cat": f"bucket{k}", "ph": "i", "s": "t", "pid": rank, "tid": k,
                       "ts": round(tl["t0"].elapsed_time(ready) * 1e3, 1), "args": args})
            t0 = tl["t0"].elapsed_time(start) * 1e3
            ev.append({"name": "ALLREDUCE", "cat": f"bucket{k}", "ph": "X", "pid": rank, "tid": k, "ts": round(t0, 1),
                       "dur": round(start.elapsed_time(end) * 1e3, 1), "args": args})
        return json.dumps(ev)

    # ------------------------------------------------------------------ eager step
    def _overlap_setup(self):
        """Eager bucketed all-reduce overlapped with backward (GPU): each replica thread records
        an event when bucket i of its flat gradient is produced; once all R replicas have bucket
        i, a comm thread makes per-device comm streams wait on those events and issues ONE
        grouped RCCL all-reduce of bucket i across the devices, while the replicas keep
        computing the earlier layers' gradients.  (TF's Mirrored all-reduces one pack after
        the whole backward, imagenet-resnet50-mirror.py:21 [lib].)"""
        import queue
        eng0 = self.replicas[0][0]
        self.buckets = eng0.L.buckets(self._bucket_mb())
        self.comm_streams = [torch.cuda.Stream(device=d) for d in self.devices]
        self._q = queue.Queue()
        self._lock = threading.Lock()

    def _bucket_cb(self, r):
        def cb(i):
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.devices[r]))
            with self._lock:
                self._events[i][r] = ev
                self._count[i] += 1
                full = self._count[i] == self.R
            if full:
                self._q.put(i)
        return cb

    def _comm_loop(self):
        grads = [e.grads for e, _ in self.replicas]
        streams = [cs.cuda_stream for cs in self.comm_streams]
        for _ in range(len(self.buckets)):
            i = self._q.get()
            s, e = self.buckets[i]
            for r in range(self.R):
                self.comm_streams[r].wait_event(self._events[i][r])
            self.comm.all_reduce_on([g[s:e] for g in grads], "sum", streams, f"bucket {i} all_reduce")
        self._done = []
        for r in range(self.R):
            ev = torch.cuda.Event()
            ev.record(self.comm_streams[r])
            self._done.append(ev)

    def _eager_step(self, parts, global_batch: int, apply: bool = True):
        R = self.R
        stats = [None] * R
        overlap = self.comm is not None and opt("PDDL_MIRROR", "overlap", True)
        if overlap:
            if not hasattr(self, "_q"):
                self._overlap_setup()
            nb = len(self.buckets)
            self._events = [[None] * R for _ in range(nb)]
            self._count = [0] * nb
            comm_th = threading.Thread(target=self._comm_loop)
            comm_th.start()

        def run(i):
            eng, _ = self.replicas[i]
            d = self.devices[i]
            if d.type == "cuda":
                torch.cuda.set_device(d)
            im, lb = parts[i]
            flip, off = self.augs[i](im.shape[0])
            kw = dict(bucket_cb=self._bucket_cb(i), buckets=self.buckets) if overlap else {}
            stats[i] = eng.forward_backward(im, lb, 1.0 / global_batch, flip=flip, crop_offset=off, **kw).clone()

        if self.gpu and R > 1:
            th = [threading.Thread(target=run, args=(i,)) for i in range(R)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        else:
            for i in range(R):
                run(i)
        grads = [e.grads for e, _ in self.replicas]
        if overlap:
            comm_th.join()
            for r, d in enumerate(self.devices):
                torch.cuda.current_stream(d).wait_event(self._done[r])
        elif self.comm is not None:
            self.comm.all_reduce(grads, "sum")
        elif R > 1 or self.cross:
            if self.gpu:
                for d in {str(d) for d in self.devices}:
                    torch.cuda.synchronize(torch.device(d))   # replicas on other threads / streams
            tot = grads[0].clone() if R > 1 else grads[0]
            for g in grads[1:]:
                tot += g.to(tot.device)
            if self.cross:
                dist.all_reduce(tot)
            for g in grads:
                if g is not tot:
                    g.copy_(tot)
        if apply:
            for e, o in self.replicas:
                o.step()
                e.after_update()
        return self._sum_stats(stats)

    def compute_gradients(self, images, labels, global_batch: int):
        """Eager forward + backward + cross-replica sum without the update: afterwards every
        replica's `grads` holds the global-batch mean gradient."""
        return self._eager_step(self._split(images, labels), global_batch, apply=False)

    def step(self, images, labels, global_batch: int):
        if self.comm is not None:
            self.comm.check()      # a stall verdict of the previous step's collectives raises here
        parts = self._split(images, labels)
        if self.graph_mode and self._single_replica_job():
            if self.cfg.graphs:            # (--graphs: the whole step as one HIP graph)
                return self._whole_step(parts, global_batch)
            return self._single_step(parts, global_batch)
        if self.graph_mode:
            return self._graphed_step(parts, global_batch)
        return self._eager_step(parts, global_batch)

    def _single_replica_job(self) -> bool:
        """One replica in the whole job: the gradient needs no reduction (a 1-rank all-reduce is
        the identity), so the step runs without collectives, like TF's MirroredStrategy on one
        device (no cross-device ops): eager by default, one whole-step HIP graph with --graphs.
        PDDL_MIRROR=segmented=1 keeps the segmented multi-replica schedule and its collectives."""
        return self.world_ranks == 1 and not opt("PDDL_MIRROR", "segmented", False)

    def _single_step(self, parts, global_batch: int):
        """One replica in the whole job, default: the eager two-stream step (no collective to
        run).  Measured faster than its whole-step graph replay once the host enqueue hides
        behind the GPU step (b32: 3.77 vs 4.08 ms, profiles/r5_strategy_bench_1gpu.txt)."""
        (eng, opt), d = self.replicas[0], self.devices[0]
        im, lb = parts[0]
        with torch.cuda.device(d):
            flip, off = self.augs[0](im.shape[0])
            s = eng.forward_backward(im, lb, 1.0 / global_batch, flip=flip, crop_offset=off).clone()
            opt.step()
            eng.after_update()
        return s

    def _whole_step(self, parts, global_batch: int):
        from ..train.graph import GraphedTrainStep
        (eng, opt), d = self.replicas[0], self.devices[0]
        im, lb = parts[0]
        B = im.shape[0]
        g = getattr(self, "_whole", None)
        if g is None or g.B != B or g.gscale != 1.0 / global_batch or tuple(g.images.shape[1:3]) != tuple(im.shape[1:3]):
            g = self._whole = GraphedTrainStep(eng, opt, B, tuple(im.shape[1:3]), 1.0 / global_batch,
                                               image_dtype=im.dtype)
        with torch.cuda.device(d):
            flip, off = self.augs[0](B)
            return g(im, lb, flip, off).clone()


class MirroredStrategy(Strategy):
    """tf.distribute.MirroredStrategy (imagenet-resnet50-mirror.py:21): one process drives
    every local GPU; the global batch 32*R (mirror.py:54) is split into R replica batches."""
    name = "mirrored"

    def __init__(self, cfg, devices: Optional[List] = None):
        super().__init__(cfg)
        self._devices = devices

    def _build(self, trainer):
        if self._devices is not None:
            devs = self._devices
        elif self.cfg.device != "cpu" and gpu_available():
            devs = list(range(torch.cuda.device_count()))
        else:
            devs = ["cpu"] * int(os.environ.get("PDDL_CPU_REPLICAS", "1"))
        self.mirror = _LocalReplicas(self.cfg, devs)
        self.local_replicas = self.mirror.R
        self.engine, self.opt = self.mirror.replicas[0]
        self.device = self.mirror.devices[0]

    def _replicas(self):
        return self.mirror.replicas

    def train_step(self, images, labels):
        self._fault_tick()
        return self.mirror.step(images, labels, self.global_batch)

    def compute_gradients(self, images, labels):
        return self.mirror.compute_gradients(images, labels, self.global_batch)

    def broadcast_state(self, trainer, root=0):
        self.mirror.broadcast()

    def write_timeline(self, path: str):
        """The graphed replicas' per-bucket READY / ALLREDUCE timeline (device 0), if recorded."""
        js = self.mirror.timeline_json(0)
        if js is not None:
            with open(f"{path}.rank0.json", "w") as f:
                f.write(js)


def make_strategy(cfg) -> Strategy:
    s = cfg.strategy
    if s == "single":
        return SingleStrategy(cfg)
    if s == "horovod":
        return HorovodStrategy(cfg)
    if s == "multiworker":
        return MultiWorkerStrategy(cfg)
    if s == "mirrored":
        return MirroredStrategy(cfg)
    if s == "ps":
        from .parameter_server import ParameterServerStrategy
        return ParameterServerStrategy(cfg)
    raise ValueError(f"unknown strategy {s!r}")
