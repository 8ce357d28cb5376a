"""Bucketed gradient all-reduce over the flat gradient buffer (RCCL over xGMI on GPU,
gloo on CPU).

The reference gets its gradient all-reduce from TF's NcclAllReduce (MirroredStrategy,
imagenet-resnet50-mirror.py:21), MWMS CollectiveReduce with NCCL (multiworkers.py:20-25)
or Horovod's fused all-reduce (imagenet-resnet50-hvd.py:101).  Here every bucket is a
contiguous slice of ONE flat fp32 buffer laid out in backward-completion order, so there is
nothing to pack: `on_bucket_ready(i)` is called by the engine right after the kernels that
produce bucket i have been enqueued, and issues `all_reduce(grads[s:e], async_op=True)`.
ProcessGroupNCCL orders the collective after those kernels (stream event) and runs it on
its own stream, overlapping the rest of backward; `finish()` makes the compute stream wait.
Buckets default to 32 MiB: large enough that each of the ring channels RCCL spreads over
the 7 xGMI links of an MI355X carries multi-MiB chunks, small enough (4 kernel buckets + a
per-channel tail) to overlap with the backward of the earlier layers.

Stall detection: on a host-blocking backend (gloo) `finish()` bounds every wait by
`stall_timeout` and raises with the bucket id (the Horovod stall inspector's verdict,
imagenet-resnet50-hvd.py:101 [lib]).  On RCCL the wait is stream-ordered (the host does not
block), and ProcessGroupNCCL's own watchdog enforces the process-group timeout
(strategies.collective_timeout) by tearing the process down.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


class BucketAllReducer:
    def __init__(self, grads: torch.Tensor, buckets: List[Tuple[int, int]], average: bool = False,
                 group: Optional[dist.ProcessGroup] = None, comm_dtype: str = "fp32", timeline=None,
                 stall_timeout: float = 0.0):
        self.grads = grads
        self.buckets = list(buckets)
        self.average = average
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.comm_dtype = comm_dtype
        self.timeline = timeline
        self.stall_timeout = stall_timeout
        self.host_blocking = dist.is_initialized() and dist.get_backend(group) == "gloo"
        self.works = []
        self._lowp = None
        if comm_dtype == "bf16":
            self._lowp = torch.empty(grads.numel(), dtype=torch.bfloat16, device=grads.device)

    def begin(self):
        self.works = []

    def on_bucket_ready(self, i: int):
        s, e = self.buckets[i]
        if self.timeline is not None:
            self.timeline.instant(f"bucket{i}_ready", args={"bytes": (e - s) * 4})
        if self._lowp is not None:
            buf = self._lowp[s:e]
            buf.copy_(self.grads[s:e])
            w = dist.all_reduce(buf, group=self.group, async_op=True)
            self.works.append((w, i, buf))
        else:
            w = dist.all_reduce(self.grads[s:e], group=self.group, async_op=True)
            self.works.append((w, i, None))

    def finish(self):
        import datetime
        for w, i, buf in self.works:
            if self.host_blocking and self.stall_timeout > 0:
                try:
                    w.wait(timeout=datetime.timedelta(seconds=self.stall_timeout))
                except RuntimeError as e:
                    rank = dist.get_rank(self.group)
                    raise RuntimeError(f"pddl bucket all-reduce: rank {rank}: bucket {i} did not complete within "
                                       f"{self.stall_timeout:g} s - a peer rank is likely stuck, dead or diverged "
                                       f"({e})") from e
            else:
                w.wait()
            if buf is not None:
                s, e = self.buckets[i]
                self.grads[s:e].copy_(buf)
        self.works = []
        if self.average and self.world > 1:
            self.grads.div_(self.world)

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if self.world > 1:
            dist.broadcast(t, src, group=self.group)


class CommProxy:
    """1-GPU model of the multi-GPU gradient all-reduce's footprint (`bench.py --comm-proxy`,
    PDDL_COMM_PROXY="world=8,busbw=350,nch=32"): at the moment the fusion engine would issue
    bucket i's RCCL all-reduce (its readiness event on the compute stream), a paced copy kernel
    with RCCL's channel count of workgroups (`comm_proxy`, csrc/kernels/pack.hip) runs on a side
    stream for the collective's modelled duration -- bucket bytes x 2 (N-1)/N / bus bandwidth --
    streaming the bucket through HBM as a ring would.  It touches no gradient.  The step then
    shows what the backward kernels lose to CUs and HBM shared with the collectives
    (imagenet-resnet50-hvd.py:101's all-reduce overlapped with backward), which one GPU cannot
    otherwise measure."""

    def __init__(self, grads: torch.Tensor, buckets: List[Tuple[int, int]], spec: str):
        from ..ops.native import require_native
        self.N = require_native()
        kv = dict(p.split("=") for p in spec.split(",") if "=" in p) if spec not in ("1", "on") else {}
        self.world = int(kv.get("world", 8))
        self.busbw = float(kv.get("busbw", 350.0)) * 1e9     # bytes/s
        self.nch = int(kv.get("nch", 32))
        self.grads = grads
        self.buckets = list(buckets)
        dev = grads.device
        self.stream = torch.cuda.Stream(dev)
        self.scratch = torch.empty(max(e - s for s, e in self.buckets) + 8, dtype=torch.float32, device=dev)
        self.passes = max(1, round(2 * (self.world - 1) / self.world))
        self.modelled_s = 0.0

    def begin(self):
        self.modelled_s = 0.0

    def on_bucket_ready(self, i: int):
        s, e = self.buckets[i]
        s4 = (s + 3) // 4 * 4
        n = max(0, (e - s4) // 4 * 4)
        if n == 0:
            return
        t = (e - s) * 4 * 2 * (self.world - 1) / self.world / self.busbw
        self.modelled_s += t
        ev = torch.cuda.Event()
        ev.record()
        self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):
            self.N.comm_proxy(self.grads[s4:s4 + n], self.scratch, self.passes, int(t * 1e8), self.nch)

    def finish(self):
        torch.cuda.current_stream().wait_stream(self.stream)
