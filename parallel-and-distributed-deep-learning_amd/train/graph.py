"""HIP-graph capture of the whole training step (preprocess -> forward -> backward ->
optimizer -> bf16 weight re-prep) for one GPU.

The reference's per-step work is issued op by op by the TF runtime (imagenet-resnet50.py:67
`model.fit`); here the ~180 kernel launches of a step are recorded once into a HIP graph and
replayed with a single launch, which removes host launch cost and inter-kernel gaps (it is
what keeps small per-GPU batches, e.g. the reference's 32, from being launch-bound).

Everything that changes between steps lives in device memory the graph reads:
  * inputs are copied into static buffers (images, labels, flip flags, crop offset),
  * the optimizer's step counter and learning rate are the device buffer `opt.hs`
    (train/optim.py), advanced by a kernel inside the graph; host LR changes are written to
    it between replays.
Horovod-style multi-process steps keep eager launches: their collectives are issued from the
bucket callbacks.  The in-process Mirrored strategy replays one forward+backward graph per
device from a single thread (no per-replica Python launch cost, no GIL contention), then runs
the grouped all-reduce and the optimizer (`with_optimizer=False`).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch



# Capture in thread-local mode: under the default global mode any potentially unsafe HIP call
# from ANOTHER thread (the input pipeline's producer thread staging its next batch, a fusion
# engine worker) invalidates the capture -- seen as an intermittent
# hipErrorStreamCaptureUnsupported on the Mirrored entry script's first (captured) step.
CAPTURE_MODE = "thread_local"

_REPLAY = {}


def replay_stream(device) -> torch.cuda.Stream:
    """The stream HIP graphs of `device` are launched on (one per device, made once).

    Never the legacy default stream: launched there, a graph with parallel branches (the
    two-stream backward forks a side stream into every captured step) segfaulted inside
    hipGraphLaunch -- the runtime's per-launch stream assignment read its parallel-stream table
    as garbage (faulting address 0x1d8 = 0x30 + 0x1a8; native stack from
    csrc/runtime/crash_trace.cpp) -- once the process had created and run other graphs
    (deterministic after tests/test_gpu_{bn_train,capture,engine}.py, then the Mirrored
    graphed step; alone it passed).  The same graphs launched on a created stream ran clean in
    the same sequence (profiles/r5_graph_crash.txt).

    Owner (round 6): the runtime's multi-branch launch path, entered only by graphs with
    parallel branches.  The standalone HIP program csrc/tests/graph_replay_repro.cpp (no torch:
    fork / join captures, executables created, run, destroyed and churned, side streams
    re-created, the Mirrored replica driver's churn, thousands of replays on the legacy default
    and created streams) runs clean against both the ROCm 7.2 runtime and the runtime torch
    bundles (scripts/graph_repro.sh, profiles/r6_graph_repro.txt); in-process, three
    multi-replica graphed tests followed by a fresh two-stream capture fault at the same frames
    on a CREATED stream too, with torch's replay and with the native launch alike
    (profiles/r6_mirror_host_loop.txt).  So graphed engines run one stream (models/engine.py):
    a single-stream executable is launched from its packets and never walks the table."""
    d = torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    s = _REPLAY.get(idx)
    if s is None:
        s = _REPLAY[idx] = torch.cuda.Stream(device=idx)
    return s


def _new_graph(**kw):
    return torch.cuda.CUDAGraph(**kw)

class GraphedTrainStep:
    """with_optimizer=False records forward + backward only (optimizer may then be None: the
    parameter-server worker, whose update runs on the PS)."""

    def __init__(self, engine, optimizer, batch: int, image_hw: Tuple[int, int], gscale: float,
                 image_dtype=torch.uint8, with_optimizer: bool = True):
        if not engine.params.is_cuda:
            raise RuntimeError("GraphedTrainStep needs the GPU engine")
        self.engine, self.opt, self.B, self.gscale = engine, optimizer, batch, float(gscale)
        self.with_optimizer = with_optimizer
        dev = engine.params.device
        H, W = image_hw
        self.images = torch.zeros(batch, H, W, 3, dtype=image_dtype, device=dev)
        lab = getattr(engine, "labels_dev", None)
        if lab is not None and lab.dtype == torch.int64 and lab.device == dev and lab.shape[0] >= batch:
            self.labels = lab[:batch]   # the engine reads its labels here: no copy inside the step
        else:
            self.labels = torch.zeros(batch, dtype=torch.int64, device=dev)
        self.flip = torch.zeros(batch, dtype=torch.uint8, device=dev)
        self.crop = torch.zeros(2, dtype=torch.int32, device=dev)
        self._flip_zero = True        # (flip holds zeros: a flip-less load needs no memset)
        self._crop_host = (0, 0)      # (the tuple crop currently in `crop`: unchanged -> no copy)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.stats = None

    def _body(self):
        eng = self.engine
        stats = eng.forward_backward(self.images, self.labels, self.gscale, flip=self.flip, crop_offset=self.crop)
        if self.with_optimizer:
            self.opt.step()
            eng.after_update()
        return stats

    def _load(self, images, labels, flip, crop_offset):
        self.images.copy_(images, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)
        if flip is None:
            if not self._flip_zero:
                self.flip.zero_()
                self._flip_zero = True
        else:
            self.flip.copy_(flip, non_blocking=True)
            self._flip_zero = False
        if isinstance(crop_offset, torch.Tensor):
            self.crop.copy_(crop_offset, non_blocking=True)
            self._crop_host = None
        else:
            oy, ox = (int(v) for v in crop_offset)
            H, W = self.images.shape[1:3]
            c = self.engine.crop
            if not (0 <= oy <= H - c and 0 <= ox <= W - c) and c < H:
                raise ValueError("crop offset out of range")
            if self._crop_host != (oy, ox):
                self.crop.copy_(torch.tensor([oy, ox], dtype=torch.int32), non_blocking=True)
                self._crop_host = (oy, ox)

    def capture(self):
        """Record the step.  Call after one eager step of the engine (its lazily built tables
        exist); capture itself runs no kernels, so it does not advance training."""
        if self.with_optimizer:
            self.opt.sync_hparams()
        torch.cuda.synchronize()
        it = self.opt._iterations if self.opt is not None else 0
        g = _new_graph()
        with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
            self.stats = self._body()
        if self.opt is not None:
            self.opt._iterations = it    # the capture pass did not step (no setter: hs is current)
        self.graph = g

    def __call__(self, images, labels, flip=None, crop_offset=(0, 0)):
        self._load(images, labels, flip, crop_offset)
        if self.graph is None:
            out = self._body()        # first call: eager (builds the engine's tables), then capture
            self.capture()
            return out
        if self.with_optimizer:
            self.opt.sync_hparams()
        _launch(self.graph)
        if self.with_optimizer:
            self.opt._iterations += 1
        return self.stats


class SegmentedStepGraphs(GraphedTrainStep):
    """One replica's step as HIP graphs split at the gradient-bucket boundaries, plus an
    optimizer graph: `segments[k]` ends right after the kernels that complete bucket k, so a
    driver replaying the segments of R devices can issue the grouped all-reduce of bucket k
    (on comm streams) while segment k+1 computes -- backward/all-reduce overlap with ~(nb+1)
    host calls per device per step instead of ~180 kernel launches.

    Capture splits the stream capture from inside the engine's bucket callback (end the
    current graph, begin the next on the same capture stream and memory pool), so the
    segments replay in exactly the eager launch order.  Reference: the per-replica step of
    MirroredStrategy (imagenet-resnet50-mirror.py:21,54) with its NCCL all-reduce."""

    def __init__(self, engine, optimizer, batch: int, image_hw: Tuple[int, int], gscale: float, buckets,
                 image_dtype=torch.uint8, two_stream: Optional[bool] = None, keep_graph: bool = False,
                 probe=None):
        super().__init__(engine, optimizer, batch, image_hw, gscale, image_dtype, with_optimizer=False)
        self.buckets = list(buckets)
        self.segments = []
        self.side_segments = []          # deferred engines: segment k's weight-gradient graph (or None)
        self.opt_graph: Optional[torch.cuda.CUDAGraph] = None
        self.two_stream = two_stream
        self.keep_graph = keep_graph     # (diagnostics: keep the hipGraph_t for node queries)
        self.probe = probe               # (diagnostics: probe(segment_index, graph) after each cut)

    @property
    def captured(self) -> bool:
        return self.opt_graph is not None

    def capture(self):
        eng, opt = self.engine, self.opt
        dev = eng.params.device
        nb = len(self.buckets)
        # The engine's two-stream backward (weight gradients on its side stream) is captured as
        # is: every cut first joins the side stream into the capture stream (cut.needs_join), so
        # each segment is a closed fork/join graph.  Checked node by node on the GPU
        # (scripts/graph_diag.py, profiles/r5_graph_diag.txt): after every cut neither stream is
        # left capturing, the segments hold exactly the single-stream schedule's kernels (234 at
        # b8, 213 at b32) and one replay reproduces the eager gradient to 5e-8.
        # two_stream=False forces the single-stream schedule.
        if getattr(eng, "side", None) is not None and self.two_stream is False:
            eng.side = None
        # A deferring engine (HipEngine graphed="segmented") queues its side-stream work during the
        # capture; each cut records the queue as a single-stream side graph on the engine's side
        # stream: the replay launches segment k, then side k (after segment k, concurrently with
        # segment k + 1), and bucket k's all-reduce after side k.
        self.deferred = getattr(eng, "side", None) is not None and getattr(eng, "defer_side", False)
        opt.sync_hparams()
        torch.cuda.synchronize(dev)
        # as torch.cuda.graph does: collect garbage now, and none while capturing
        import gc
        gc.collect()
        gc_was = gc.isenabled()
        gc.disable()
        try:
            self._capture_segments(eng, opt, dev, nb)
        finally:
            if gc_was:
                gc.enable()

    def _capture_segments(self, eng, opt, dev, nb):
        it = opt._iterations
        segs = []         # segs[i]: the graph ending with bucket i, None when bucket i completed
        live = []         # at the same point as bucket i-1 (nothing captured in between)
        pool = []
        sides = []        # deferred engines: sides[i] the side graph of segment i (None: no side work)
        deferred = self.deferred
        mark = torch.zeros(1, device=dev) if deferred else None

        def begin():
            g = _new_graph(keep_graph=self.keep_graph)
            g.capture_begin(pool=pool[0] if pool else None, capture_error_mode=CAPTURE_MODE)
            live.append(g)

        def cut(i):
            q = eng.take_deferred() if deferred else []
            if _capture_is_empty():
                if not q and i < nb - 1:
                    segs.append(None)      # (an empty capture cannot end: it stays open for i+1)
                    sides.append(None)
                    return
                if not deferred:
                    raise RuntimeError("segmented capture: the last bucket captured no work")
                mark.zero_()               # (one tiny node, so the segment can end and order its side graph)
            live[-1].capture_end()
            if not pool:                   # (pool() exists once a capture has ended)
                pool.append(live[-1].pool())
            segs.append(live[-1])
            if self.probe is not None:
                self.probe(len(segs) - 1, segs[-1])
            if deferred:
                sg = None
                if q:
                    sg = _new_graph(keep_graph=self.keep_graph)
                    with torch.cuda.stream(eng.side):
                        sg.capture_begin(pool=pool[0], capture_error_mode=CAPTURE_MODE)
                        try:
                            for fn, args in q:
                                fn(*args)
                        finally:
                            sg.capture_end()
                sides.append(sg)
            if i < nb - 1:
                begin()
        cut.needs_join = True   # (a two-stream engine joins its side stream before each cut)

        with torch.cuda.device(dev):
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            if deferred:
                eng.side.wait_stream(s)
            with torch.cuda.stream(s):
                begin()
                if deferred:
                    eng.begin_defer()
                try:
                    self.stats = eng.forward_backward(self.images, self.labels, self.gscale, flip=self.flip,
                                                      crop_offset=self.crop, bucket_cb=cut, buckets=self.buckets)
                    og = _new_graph(keep_graph=self.keep_graph)
                    live.append(og)
                    og.capture_begin(pool=pool[0], capture_error_mode=CAPTURE_MODE)
                    opt.step()
                    eng.after_update()
                    og.capture_end()
                except BaseException:
                    # leave no stream capturing (a dangling capture aborts the process at exit)
                    if torch.cuda.is_current_stream_capturing():
                        try:
                            live[-1].capture_end()
                        except Exception:
                            pass
                    if deferred:
                        eng._defer = None      # (back to launching: the capture is abandoned)
                    raise
                if deferred:
                    eng.end_defer()
            torch.cuda.current_stream(dev).wait_stream(s)
        if len(segs) != nb:
            raise RuntimeError(f"segmented capture produced {len(segs)} segments for {nb} buckets")
        opt._iterations = it        # capture ran no kernels: training state did not advance
        self.segments = segs
        self.side_segments = sides if deferred else [None] * nb
        self.opt_graph = og

    def load(self, images, labels, flip=None, crop_offset=(0, 0)):
        self._load(images, labels, flip, crop_offset)

    def replay_segment(self, k: int):
        if self.segments[k] is not None:
            _launch(self.segments[k])
        if self.side_segments[k] is not None:   # (after segment k, on the engine's side stream)
            amb = torch.cuda.current_stream()
            side = self.engine.side
            side.wait_stream(amb)
            _replay(self.side_segments[k], side)
            amb.wait_stream(side)

    def exec_handles(self):
        """([segment k's raw executable, 0 if empty], the optimizer graph's, [segment k's side
        graph, 0 if none]): what the Mirrored driver's native group launches replay (sync_hparams /
        the iteration count stay with the caller, as in replay_optimizer)."""
        return ([g.raw_cuda_graph_exec() if g is not None else 0 for g in self.segments],
                self.opt_graph.raw_cuda_graph_exec(),
                [g.raw_cuda_graph_exec() if g is not None else 0 for g in self.side_segments])

    def replay_optimizer(self):
        self.opt.sync_hparams()
        _launch(self.opt_graph)
        self.opt._iterations += 1


def _capture_is_empty() -> bool:
    """True while the current stream's capture has recorded nothing since it began (no
    dependency nodes): hipStreamGetCaptureInfo_v2 through the native extension, i.e. the HIP
    runtime the kernels and torch use (no second runtime loaded by name)."""
    from ..ops.native import require_native
    rc, st, n = require_native().stream_capture_deps(torch.cuda.current_stream().cuda_stream)
    if rc != 0 or st != 1:
        raise RuntimeError(f"segmented capture: stream not capturing (hip error {rc}, status {st})")
    return n == 0


def _replay(g, stream: torch.cuda.Stream):
    """hipGraphLaunch of g's executable on `stream` through the native extension, GIL released
    (csrc/runtime/graph_launch.cpp).  The captured steps draw no torch RNG, so torch's replay
    prologue (generator offsets) has nothing to do."""
    from ..ops.native import require_native
    require_native().graph_launch(g.raw_cuda_graph_exec(), stream.cuda_stream)


def _launch(g):
    """Replay on the current stream, or through replay_stream() when that is the legacy
    default stream (ordered after and before the default stream's work)."""
    amb = torch.cuda.current_stream()
    if amb.cuda_stream != 0:
        _replay(g, amb)
        return
    rs = replay_stream(amb.device)
    rs.wait_stream(amb)
    _replay(g, rs)
    amb.wait_stream(rs)
