"""Asynchronous parameter-server training (SURVEY.md C21-C25, §2.2 "Async parameter server").

Reference (imagenet-resnet50-ps.py): create_in_process_cluster(W, P) (:31-65) starts W worker
and P PS gRPC servers; MinSizePartitioner(min_shard_bytes=256 KiB, max_shards=P) (:75-78)
shards the variables; ParameterServerStrategy + ClusterCoordinator (:80-84) schedule train
steps onto workers asynchronously; every step pulls the variables from the PS, computes
gradients on the worker and applies Adam on the PS-resident variables, with no cross-worker
synchronisation; GRPC_FAIL_FAST=use_caller (:69) surfaces failures to the coordinator;
fit(steps_per_epoch=312500) (:142-143) over repeat()-ed datasets.

MI355X-native design:
  * roles are PROCESSES, one GPU each (e.g. 2 PS + 6 workers on an 8-GPU node); a single
    launch spawns the whole "in-process cluster" (or torchrun provides WORLD_SIZE = P + W);
  * the PS holds only its shards of the flat fp32 parameter buffer plus their Adam slots and
    applies the fused HIP Adam kernel to each arriving gradient (async, staleness unbounded,
    as in the reference);
  * data plane (default, native): csrc/runtime/ps_service.cpp — a per-PS shared-memory control
    segment and HIP-IPC mailboxes: a worker's pack kernel writes its gradient ranges straight
    into its mailbox on the PS GPU over xGMI, the PS service thread applies fused Adam and
    peer-copies the fresh shard back (CPU roles: the same protocol in shared memory);
    PDDL_PS=impl=c10d selects the portable fallback: one 2-rank process group per
    (worker, PS) pair with RCCL / gloo send/recv served from Python threads;
  * a worker's push / pull round trip overlaps its next step (cfg.ps_overlap, default; the
    step then reads parameters one round trip older -- the reference's asynchronous PS has
    unbounded staleness anyway); --ps-sync restores the blocking exchange per step;
  * control plane (closure scheduling, heartbeats, LR broadcast, stop) is the c10d TCPStore:
    a worker claims step tickets; the coordinator re-queues the ticket of a worker that misses
    its heartbeats (ClusterCoordinator's closure re-queue); PDDL_FAULT=kill_worker:<i>@<step>
    injects a worker failure for tests.  A PS failure aborts the job (reference parity).
"""
from __future__ import annotations

import argparse
import datetime
import math
import os
import sys
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..models.resnet50 import ParamLayout
from ..utils.envopts import opt


P = "PDDL_PS"   # the PS runtime switches (utils/envopts.py KEYS)
_WARM_STEPS = 2   # steps of each epoch outside the throughput window (train/callbacks.py ThroughputMeter)


def add_ps_args(ap: argparse.ArgumentParser):
    """Q6: accept --ps N --worker M (the evident intent) and the positional form `N M`."""
    ap.add_argument("--ps", type=int, dest="num_ps")
    ap.add_argument("--worker", "--workers", type=int, dest="num_workers")
    ap.add_argument("positional", nargs="*", type=int)


def parse_ps_counts(ns) -> Tuple[int, int]:
    num_ps = getattr(ns, "num_ps", None)
    num_w = getattr(ns, "num_workers", None)
    pos = list(getattr(ns, "positional", []) or [])
    if num_ps is None and pos:
        num_ps = pos.pop(0)
    if num_w is None and pos:
        num_w = pos.pop(0)
    return (num_ps or 1), (num_w or 1)


# ----------------------------------------------------------------------- partitioning
def min_size_partitions(keras_shape, dtype_bytes: int, min_shard_bytes: int, max_shards: int) -> int:
    """tf.distribute.experimental.partitioners.MinSizePartitioner: number of axis-0 shards."""
    nbytes = int(np.prod(keras_shape)) * dtype_bytes
    n = max(1, min(max_shards, nbytes // max(1, min_shard_bytes)))
    return int(min(n, keras_shape[0]))


@dataclass
class Shard:
    name: str
    offset: int
    size: int
    ps: int


def partition_variables(L: ParamLayout, num_ps: int, min_shard_bytes: int = 256 << 10) -> List[Shard]:
    """Shard every trainable variable (MinSizePartitioner, split along the first axis of the
    internal layout) and place shards on PS tasks round-robin in creation order."""
    shards: List[Shard] = []
    rr = 0
    for e in sorted((e for e in L.entries.values() if e.trainable), key=lambda e: e.offset):
        n = min_size_partitions(e.keras_shape, 4, min_shard_bytes, num_ps)
        rows = e.shape[0]
        n = max(1, min(n, rows))
        per_row = e.size // rows
        bounds = [round(i * rows / n) for i in range(n + 1)]
        for i in range(n):
            r0, r1 = bounds[i], bounds[i + 1]
            shards.append(Shard(f"{e.name}/part_{i}", e.offset + r0 * per_row, (r1 - r0) * per_row, rr % num_ps))
            rr += 1
    return shards


def ps_ranges(shards: List[Shard], num_ps: int) -> List[List[Tuple[int, int]]]:
    out = [[] for _ in range(num_ps)]
    for s in shards:
        out[s.ps].append((s.offset, s.size))
    return out


def _gather(flat: torch.Tensor, ranges) -> torch.Tensor:
    return torch.cat([flat[o:o + n] for o, n in ranges])


def _scatter(flat: torch.Tensor, ranges, packed: torch.Tensor) -> None:
    p = 0
    for o, n in ranges:
        flat[o:o + n].copy_(packed[p:p + n])
        p += n


# ----------------------------------------------------------------------- roles
OP_PUSH, OP_PULL, OP_STOP = 0.0, 1.0, 2.0


def ps_impl() -> str:
    """Data plane: "native" (csrc/runtime/ps_service.cpp) unless PDDL_PS=impl=c10d."""
    if opt(P, "impl", "native") != "native":
        return "c10d"
    from ..ops.native import native_available, require_native
    return "native" if native_available() and hasattr(require_native(), "PSServer") else "c10d"


class _Cluster:
    def __init__(self, cfg, rank: int, world: int, num_ps: int, device, impl: str = "c10d"):
        self.cfg = cfg
        self.rank, self.world, self.num_ps = rank, world, num_ps
        self.num_workers = world - num_ps
        self.device = device
        self.is_ps = rank < num_ps
        self.impl = impl
        self.store = _LockedStore(dist.distributed_c10d._get_default_store())
        if rank == 0:
            self.store.set("ps_job", f"{os.getpid():x}{int(time.time() * 1e3) & 0xffffff:06x}")
        self.job = self.store.get("ps_job").decode()
        # c10d data plane: one 2-rank group per (worker, ps) pair; every rank creates every group
        self.pair: Dict[Tuple[int, int], dist.ProcessGroup] = {}
        if impl == "c10d":
            for w in range(num_ps, world):
                for p in range(num_ps):
                    self.pair[(w, p)] = dist.new_group([p, w])
        L = ParamLayout(cfg.num_classes)
        self.L = L
        self.shards = partition_variables(L, num_ps, cfg.min_shard_bytes)
        self.ranges = ps_ranges(self.shards, num_ps)
        self.sizes = [sum(n for _, n in r) for r in self.ranges]


def _hb_key(w):
    return f"hb/{w}"


class _LockedStore:
    """The c10d store shared by a role's main thread and its heartbeat thread."""

    def __init__(self, store):
        self._s = store
        self._lock = threading.Lock()

    def set(self, k, v):
        with self._lock:
            return self._s.set(k, v)

    def get(self, k):
        with self._lock:
            return self._s.get(k)

    def add(self, k, n):
        with self._lock:
            return self._s.add(k, n)

    def check(self, keys):
        with self._lock:
            return self._s.check(keys)

    def compare_set(self, k, expected, desired):
        with self._lock:
            return self._s.compare_set(k, expected, desired)

    def multi_set(self, keys, values):
        with self._lock:
            return self._s.multi_set(keys, values)


class _Heartbeat:
    """A worker's liveness beacon (the coordinator's worker-failure watch): a daemon thread
    stamps `hb/<rank>` every period while the worker is alive AND making progress.  The main
    loop marks each step with `step()` (compute + exchange) and each wait with `wait()` (epoch
    barrier, worker 0's validation, a drained ticket queue); a step that runs longer than
    `stall_s` (a GPU hang, a stuck exchange) stops the stamps, so a live but stalled worker is
    declared dead and its ticket re-queued exactly like a crashed one.  `stall_s` is its own
    threshold (PDDL_PS step_stall), separate from and larger than the coordinator's liveness
    timeout `hb_timeout`: a slow but healthy step (a cold first batch from real data, a PS slowed
    by many workers) keeps beating.  A worker still stuck `stall_s + hb_timeout / 2` into a step
    ends itself: the coordinator declares it dead (and re-queues its tickets) no earlier than
    `stall_s + hb_timeout` (the last stamp is at most one period older than `stall_s`), so a
    stalled worker is gone before its tickets can run twice -- a worker that exited only after
    the re-queue could wake up in between and push a gradient for a re-queued ticket, or count
    its steps into done/<epoch> a second time.  (The worker also checks dead/<rank> before it
    publishes a finished block of tickets.)"""

    def __init__(self, store, rank: int, period: float, stall_s: float, hb_timeout: Optional[float] = None):
        self.store, self.rank, self.period, self.stall_s = store, rank, period, stall_s
        self.hb_timeout = stall_s if hb_timeout is None else hb_timeout
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._state, self._since = "wait", time.time()
        self.beat()
        self._th = threading.Thread(target=self._run, daemon=True)
        self._th.start()

    def step(self):
        with self._lock:
            self._state, self._since = "step", time.time()

    def wait(self):
        with self._lock:
            self._state, self._since = "wait", time.time()

    def healthy(self) -> bool:
        with self._lock:
            return self._state == "wait" or time.time() - self._since < self.stall_s

    def beat(self):
        self.store.set(_hb_key(self.rank), str(time.time()))

    def _run(self):
        while not self._stop.wait(self.period):
            if not self.healthy():
                # stalled inside a step: the stamps stop; end the process before the
                # coordinator's watch expires (see the class docstring)
                with self._lock:
                    stuck = time.time() - self._since
                if stuck > self.stall_s + 0.5 * self.hb_timeout:
                    sys.stderr.write(f"[ps worker rank {self.rank}] stuck in a step for {stuck:.0f} s "
                                     f"(step stall {self.stall_s:g} s, heartbeat timeout {self.hb_timeout:g} s): "
                                     "exiting\n")
                    sys.stderr.flush()
                    os._exit(18)
                continue
            try:
                self.beat()
            except Exception:
                return

    def stop(self):
        self._stop.set()
        self._th.join(timeout=5)


def _claimed(store, epoch: int) -> int:
    key = f"claim/{epoch}"
    if not store.check([key]):
        return 0
    return int(store.get(key).decode().split("/")[0])


def _missing_tickets(store, epoch: int, lo: int, hi: int) -> List[int]:
    """Tickets in [lo, hi) of `epoch` without a completion marker (bisection over store.check,
    which is true only when every listed key exists: O(k log n) round trips for k misses)."""
    if hi <= lo:
        return []
    if store.check([f"tdone/{epoch}/{t}" for t in range(lo, hi)]):
        return []
    if hi - lo == 1:
        return [lo]
    mid = (lo + hi) // 2
    return _missing_tickets(store, epoch, lo, mid) + _missing_tickets(store, epoch, mid, hi)


def requeue_orphans_from(store, epoch: int, live_workers: List[int]) -> Dict[int, List[int]]:
    """requeue_orphans over `epoch` and every later epoch that has claims: a worker killed
    between its first claim of epoch e+1 and its `cur` write still reads e in `cur`, and its
    e+1 ticket must not be missed."""
    out = {}
    e = epoch
    while store.check([f"claim/{e}"]):
        r = requeue_orphans(store, e, live_workers)
        if r:
            out[e] = r
        e += 1
    return out


def requeue_orphans(store, epoch: int, live_workers: List[int]) -> List[int]:
    """Re-queue every claimed ticket of `epoch` that is neither done nor held by a live worker.
    Relies on nothing the dead worker may or may not have written between its claim and its
    death: a ticket is orphaned iff its `tdone` marker is missing and no live worker's `cur`
    names it.  Each orphan is counted once (atomic add on `rq/<epoch>/<ticket>`); a live
    worker caught between its claim and its `cur` write makes at most one extra step run."""
    held = set()
    for r in live_workers:
        if store.check([f"cur/{r}"]):
            f = [int(x) for x in store.get(f"cur/{r}").decode().split(":")]
            ep, lo = f[0], f[1]
            hi = f[2] if len(f) > 2 else lo + 1     # "<epoch>:<lo>:<hi>": a claimed block of tickets
            if ep == epoch and lo >= 0:
                held.update(range(lo, hi))
    out = []
    for t in _missing_tickets(store, epoch, 0, _claimed(store, epoch)):
        if t in held:
            continue
        if store.add(f"rq/{epoch}/{t}", 1) == 1:     # (atomic: exactly one scan counts it)
            store.add(f"requeue/{epoch}", 1)
            out.append(t)
    return out


class PSServer:
    """Holds shard p of the parameters + Adam slots; one service thread per worker."""

    def __init__(self, cl: _Cluster, init_params: torch.Tensor):
        self.cl = cl
        p = cl.rank
        self.n = cl.sizes[p]
        dev = cl.device
        self.params = _gather(init_params, cl.ranges[p]).to(dev).contiguous()
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.t = 0
        self.lock = threading.Lock()
        self.dead = set()
        self.updates = 0

    def _adam(self, g: torch.Tensor, lr: float):
        cfg = self.cl.cfg
        self.t += 1
        b1, b2, eps = cfg.beta1, cfg.beta2, cfg.adam_eps
        lr_t = lr * math.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t)
        if self.params.is_cuda:
            from ..ops.native import native
            native.adam(self.params, g, self.m, self.v, lr_t, b1, b2, eps, 1.0, None)
        else:
            self.m.mul_(b1).add_(g, alpha=1 - b1)
            self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
            self.params.sub_(lr_t * self.m / (self.v.sqrt() + eps))

    def serve(self, w: int):
        cl = self.cl
        grp = cl.pair[(w, cl.rank)]
        ctrl = torch.zeros(2, dtype=torch.float64, device=cl.device)
        grad = torch.empty(self.n, dtype=torch.float32, device=cl.device)
        try:
            while True:
                dist.recv(ctrl, src=w, group=grp)
                op, lr = float(ctrl[0]), float(ctrl[1])
                if op == OP_STOP:
                    return
                if op == OP_PUSH:
                    dist.recv(grad, src=w, group=grp)
                    with self.lock:
                        self._adam(grad, lr)
                        self.updates += 1
                with self.lock:
                    snap = self.params.clone()
                dist.send(snap, dst=w, group=grp)
        except Exception as e:  # worker died: its closure is re-queued by the coordinator
            self.dead.add(w)
            print(f"[ps {cl.rank}] lost worker {w}: {type(e).__name__}", flush=True)

    def run(self):
        cl = self.cl
        threads = [threading.Thread(target=self.serve, args=(w,), daemon=True) for w in range(cl.num_ps, cl.world)]
        for t in threads:
            t.start()
        if cl.rank == 0:
            self.monitor(threads)
        for t in threads:
            t.join()

    def monitor(self, threads):
        """Coordinator duty on PS 0: heartbeat watch + closure re-queue of dead workers."""
        cl = self.cl
        timeout = opt(P, "heartbeat", 30.0)
        dead = set()
        while any(t.is_alive() for t in threads):
            time.sleep(0.2)
            now = time.time()
            for w in range(cl.num_ps, cl.world):
                if w in dead:
                    continue
                try:
                    last = float(cl.store.get(_hb_key(w)).decode())
                except Exception:
                    continue
                finished = cl.store.check([f"fin/{w}"])
                if not finished and now - last > timeout:
                    dead.add(w)
                    cl.store.set(f"dead/{w}", "1")
                    cl.store.add("dead_workers", 1)
                    ep = 0
                    if cl.store.check([f"cur/{w}"]):
                        ep = int(cl.store.get(f"cur/{w}").decode().split(":")[0])
                    live = [r for r in range(cl.num_ps, cl.world) if r not in dead]
                    req = requeue_orphans_from(cl.store, ep, live)
                    print(f"[coordinator] worker {w} missed heartbeats for {now - last:.1f}s: declared dead, "
                          f"re-queued step(s) {req or 'none'} (by epoch, scanned from epoch {ep})", flush=True)


class NativePSServer(PSServer):
    """PS role on the native data plane: the C++ service thread applies every push; this
    process keeps the coordinator duties (heartbeat watch / closure re-queue on PS 0)."""

    def __init__(self, cl: _Cluster, init_params: torch.Tensor):
        from ..ops.native import require_native
        self.cl = cl
        cfg = cl.cfg
        shard = _gather(init_params, cl.ranges[cl.rank]).contiguous()
        dev = cl.device.index if cl.device.type == "cuda" else -1
        wire = 1 if getattr(cfg, "ps_wire", "fp32") == "bf16" and dev >= 0 else 0
        self.srv = require_native().PSServer(cl.job, cl.rank, shard, cl.num_workers, dev, cfg.beta1, cfg.beta2,
                                             cfg.adam_eps, wire)
        self.updates = 0
        self.dead = set()

    def run(self):
        cl = self.cl
        self.srv.start()
        mon = None
        if cl.rank == 0:
            done = threading.Event()

            class _Alive:   # monitor() polls is_alive() of the service "threads"
                def is_alive(self_inner):
                    return not done.is_set()
            mon = threading.Thread(target=self.monitor, args=([_Alive()],), daemon=True)
            mon.start()
        try:
            self.updates = self.srv.join()
        finally:
            if mon is not None:
                done.set()
                mon.join(timeout=5)
        self.dead = {w + cl.num_ps for w in self.srv.dead}
        for w in sorted(self.dead):
            print(f"[ps {cl.rank}] lost worker {w}", flush=True)


class PSWorker:
    def __init__(self, cl: _Cluster, engine, pipeline_factory):
        self.cl = cl
        self.engine = engine
        self.pipeline_factory = pipeline_factory
        self.packed = [torch.empty(n, dtype=torch.float32, device=cl.device) for n in cl.sizes]
        self.widx = cl.rank - cl.num_ps

    def _client(self):
        if not hasattr(self, "cli"):
            from ..ops.native import require_native
            cl = self.cl
            dev = cl.device.index if cl.device.type == "cuda" else -1
            self.cli = require_native().PSClient(cl.job, cl.ranges, self.widx, dev,
                                                 opt(P, "timeout", 120.0))
        return self.cli

    def exchange_begin(self, lr: float):
        """Overlapped push (native data plane): pack + publish the gradients and return; the PS
        applies them and snapshots the shard while this worker computes its next step, whose
        forward therefore reads the parameters of the previous round trip (one more step of
        staleness; the reference's async PS already has unbounded staleness, ps.py:80-84)."""
        if self.cl.impl == "native":
            self._client().begin(self.engine.grads, self.engine.params, lr, True)
        else:
            self._exchange(OP_PUSH, lr)

    def exchange_end(self):
        if self.cl.impl == "native" and self._client().in_flight:
            self.cli.end(self.engine.params)
            self.engine.after_update()

    def _exchange(self, op: float, lr: float):
        cl = self.cl
        if cl.impl == "native":
            self._client().exchange(self.engine.grads, self.engine.params, lr, op == OP_PUSH)
            self.engine.after_update()
            return
        ctrl = torch.tensor([op, lr], dtype=torch.float64, device=cl.device)
        reqs = []
        for p in range(cl.num_ps):
            grp = cl.pair[(cl.rank, p)]
            dist.send(ctrl, dst=p, group=grp)
            if op == OP_PUSH:
                dist.send(_gather(self.engine.grads, cl.ranges[p]).contiguous(), dst=p, group=grp)
        for p in range(cl.num_ps):
            dist.recv(self.packed[p], src=p, group=cl.pair[(cl.rank, p)])
            _scatter(self.engine.params, cl.ranges[p], self.packed[p])
        self.engine.after_update()

    def stop(self):
        cl = self.cl
        if cl.impl == "native":
            if hasattr(self, "cli"):
                self.cli.stop()
            self._finish()
            return
        ctrl = torch.tensor([OP_STOP, 0.0], dtype=torch.float64, device=cl.device)
        for p in range(cl.num_ps):
            dist.send(ctrl, dst=p, group=cl.pair[(cl.rank, p)])
        self._finish()

    def _finish(self):
        """Count this worker as finished BEFORE publishing its fin key: a worker that dies between
        the two is then either counted (its fin_count add landed) or, with no fin key, declared
        dead by the coordinator -- never neither, which would leave worker 0's final-save wait
        short of its target until the timeout."""
        self.cl.store.add("fin_count", 1)
        self.cl.store.set(f"fin/{self.cl.rank}", "1")


class _PSControl:
    """The slice of the trainer the LR / stop callbacks drive (worker 0 of a PS job)."""

    def __init__(self, lr: float):
        self.lr = float(lr)
        self.stop_training = False

    def set_lr(self, lr: float):
        self.lr = float(lr)

    def log(self, msg: str):
        print(msg, flush=True)


def claim_block(store, spe: int, epoch: int, rank: int, block: int, workers: int) -> Tuple[int, int]:
    """Claim up to `block` consecutive step tickets of `epoch` with one compare-and-set
    ([lo, hi), or (-1, -1) while the epoch's tickets are exhausted): a worker pays the control
    plane's round trips once per block instead of once per step.  Near the end of the epoch the
    block shrinks to an even share of what is left (no worker sits on a long tail while the
    others idle).  Same counter and re-queue budget as _claim."""
    key = f"claim/{epoch}"
    raw = store.compare_set(key, "", "0/-1").decode()
    while True:
        cur = int(raw.split("/")[0])
        budget = spe + store.add(f"requeue/{epoch}", 0)
        if cur >= budget:
            return -1, -1
        n = max(1, min(block, (budget - cur) // max(1, 2 * workers)))
        want = f"{cur + n}/{rank}"
        got = store.compare_set(key, raw, want).decode()
        if got == want:
            return cur, cur + n
        raw = got


def _claim(store, spe: int, epoch: int, rank: int) -> int:
    """Claim the next step ticket of `epoch`; -1 while the epoch's tickets are exhausted
    (re-queued tickets of dead workers extend the budget, so callers poll).  A claim is one
    compare-and-set of "<next ticket>/<claimer>" -- a poll never consumes a ticket, and the
    claimer id makes a lost race unambiguous."""
    key = f"claim/{epoch}"
    raw = store.compare_set(key, "", "0/-1").decode()       # creates the counter on first use
    while True:
        cur = int(raw.split("/")[0])
        if cur >= spe + store.add(f"requeue/{epoch}", 0):
            return -1
        want = f"{cur + 1}/{rank}"
        got = store.compare_set(key, raw, want).decode()
        if got == want:
            return cur
        raw = got


def _fault_step(rank_in_workers: int):
    from .faults import ps_fault
    return ps_fault(rank_in_workers)


def _ps_main(rank: int, world: int, num_ps: int, cfg, port: int, result_q=None):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    use_gpu = cfg.device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        n = torch.cuda.device_count()
        torch.cuda.set_device(rank % n)
        device = torch.device("cuda", rank % n)
    else:
        device = torch.device("cpu")
        # P + W role processes share the host's cores (the reference sizes the workers'
        # inter-op threads against cpu_count, imagenet-resnet50-ps.py:43-46): split the intra-op
        # pool instead of letting every role oversubscribe all cores
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // world))
    impl = ps_impl()
    # the native data plane needs c10d only for control (barriers, the TCP store): gloo
    gpu_pg = use_gpu and impl == "c10d"
    backend = "nccl" if gpu_pg else "gloo"
    dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=opt(P, "timeout", 120.0)),
                            **({"device_id": device} if gpu_pg else {}))
    cl = _Cluster(cfg, rank, world, num_ps, device, impl=impl)
    from ..parallel.strategies import build_engine
    torch.manual_seed(cfg.seed)
    if cl.is_ps:
        L = cl.L
        init = torch.zeros(L.total)
        L.init_params(init, cfg.seed)
        if cfg.weights and cfg.weights != "none":
            from .strategies import build_engine as _be
            tmp = _be(cfg.replace(device="cpu"), torch.device("cpu"), 1)
            tmp.params.copy_(init)
            from ..utils.checkpoint import load_pretrained
            load_pretrained(cfg.weights, tmp)
            init = tmp.params
        srv = NativePSServer(cl, init) if cl.impl == "native" else PSServer(cl, init)
        dist.barrier()
        srv.run()
        if result_q is not None:
            stats = srv.srv.service_stats() if impl == "native" and use_gpu else {}
            result_q.put(("ps", rank, srv.updates, sorted(srv.dead), impl, dict(stats)))
        dist.destroy_process_group()
        return
    # ---------------------------------------------------------------- worker
    st = ParameterServerStrategy(cfg, cluster=cl)
    st.setup(None)
    eng, worker, widx = st.engine, st.worker, st.widx
    from ..data.datasets import Pipeline, make_source
    src = make_source(cfg.data, "train", cfg)
    pipe = Pipeline(src, cfg.batch_size, repeat=True, shuffle=cfg.data != "synthetic", seed=cfg.seed + 17 * widx)
    dist.barrier()
    lr = cfg.lr
    worker._exchange(OP_PULL, lr)                     # initial pull (variables live on the PS)
    store = cl.store
    spe = cfg.steps_per_epoch or pipe.num_batches()
    if cfg.max_steps:
        spe = min(spe, cfg.max_steps)
    fault_at = _fault_step(widx)
    hb_timeout = opt(P, "heartbeat", 30.0)
    step_stall = opt(P, "step_stall", max(300.0, 10 * hb_timeout))
    hb = _Heartbeat(store, rank, max(0.05, hb_timeout / 6), step_stall, hb_timeout)
    epoch_timeout = opt(P, "epoch_timeout", max(600.0, 10 * hb_timeout))
    block = max(1, opt(P, "ticket_block", 16))
    it = pipe.iterate(device)
    history = []
    steps_done = 0
    ctl = _PSControl(lr)
    cbs = []
    if widx == 0:
        # the coordinator-side callbacks of the reference's fit (imagenet-resnet50-ps.py:139-140):
        # decisions taken on worker 0's validation, published on the control plane
        from ..train.callbacks import EarlyStopping, ReduceLROnPlateau
        cbs = [ReduceLROnPlateau(monitor="val_loss", factor=cfg.reduce_lr_factor, patience=cfg.reduce_lr_patience,
                                 min_lr=cfg.min_lr),
               EarlyStopping(monitor="val_loss", min_delta=cfg.early_stop_min_delta,
                             patience=cfg.early_stop_patience)]
        for cb in cbs:
            cb.set_trainer(ctl)
            cb.on_train_begin()
    for epoch in range(cfg.epochs):
        if store.check(["stop"]):
            break
        if store.check(["lr"]):
            lr = float(store.get("lr").decode())
        st.begin_epoch()
        t_epoch = time.perf_counter()
        t_drained = None
        # steady-state rate window, as the other strategies' ThroughputMeter: from this worker's
        # WARM-th step of the epoch (lazy tables, first-touch allocations and the PS's first
        # round trips before it) to its last
        ep_steps, t_warm, n_warm = 0, None, 0
        while True:
            # tickets are claimed in blocks: the control plane costs a few round trips per
            # block, none per step (no host / device synchronisation inside a block either)
            lo, hi = claim_block(store, spe, epoch, rank, block, cl.num_workers)
            if lo < 0:
                # out of tickets: the epoch ends when every ticket is DONE; until then a ticket
                # of a worker that died holding it may be re-queued by the coordinator
                hb.wait()
                if store.add(f"done/{epoch}", 0) >= spe:
                    break
                t_drained = t_drained or time.time()
                if time.time() - t_drained > epoch_timeout:
                    raise TimeoutError(
                        f"PS worker {widx}: epoch {epoch} drained its tickets {time.time() - t_drained:.0f} s ago but "
                        f"only {store.add(f'done/{epoch}', 0)}/{spe} steps are done (claimed "
                        f"{_claimed(store, epoch)}, re-queued {store.add(f'requeue/{epoch}', 0)}, dead workers "
                        f"{store.add('dead_workers', 0)}) - a worker holding a ticket is stuck and was not declared dead")
                time.sleep(0.02)
                continue
            t_drained = None
            hb.step()
            store.set(f"cur/{rank}", f"{epoch}:{lo}:{hi}")
            for t in range(lo, hi):
                hb.step()
                if fault_at is not None and steps_done == fault_at[1]:
                    print(f"[worker {widx}] injected {fault_at[0]} at step {steps_done}", flush=True)
                    if fault_at[0] == "kill_worker":
                        os._exit(17)
                    while True:                       # hang_worker: stuck inside the step
                        time.sleep(3600)
                images, labels = next(it)
                st.train_step(images, labels, lr)
                steps_done += 1
                ep_steps += 1
                if ep_steps == _WARM_STEPS:
                    if device.type == "cuda":
                        torch.cuda.synchronize(device)
                    t_warm, n_warm = time.perf_counter(), st.n_img
                # progress is published per step, not per block: a worker that dies inside a
                # block leaves only its unfinished tickets to the re-queue (each finished step
                # already pushed its gradient; re-running it would apply that update twice)
                if store.check([f"dead/{rank}"]):
                    # declared dead while running this block (its open tickets are re-queued):
                    # publishing this step now would count it twice
                    sys.stderr.write(f"[ps worker rank {rank}] declared dead by the coordinator: exiting\n")
                    sys.stderr.flush()
                    os._exit(18)
                store.multi_set([f"tdone/{epoch}/{t}", f"cur/{rank}"],
                                ["1", f"{epoch}:{t + 1}:{hi}" if t + 1 < hi else f"{epoch}:-1"])
                store.add(f"done/{epoch}", 1)
        hb.step()
        worker.exchange_end()                    # drain the last overlapped push of the epoch
        hb.wait()
        # epoch end: worker 0 (coordinator-side logic) validates and runs the callbacks
        loss_sum, correct, n_img = st.end_epoch()       # (the epoch's one device -> host read)
        if t_warm is not None and n_img > n_warm:
            store.add(f"acc/{epoch}/ips_milli", int((n_img - n_warm) / (time.perf_counter() - t_warm) * 1e3))
            store.add(f"acc/{epoch}/ips_workers", 1)
        store.add(f"acc/{epoch}/loss", int(loss_sum * 1e6))
        store.add(f"acc/{epoch}/correct", int(correct))
        store.add(f"acc/{epoch}/n", int(n_img))
        store.add(f"epoch_end/{epoch}", 1)
        if widx == 0:
            _wait_count(store, f"epoch_end/{epoch}", lambda: cl.num_workers - store.add("dead_workers", 0))
            dt = time.perf_counter() - t_epoch      # every worker's training steps, before validation
            n = max(1, store.add(f"acc/{epoch}/n", 0))
            # throughput: the sum of the workers' steady-state rates (async workers) when every
            # live worker measured one, else the whole epoch's images over its wall time
            ips = n / max(dt, 1e-9)
            live = cl.num_workers - store.add("dead_workers", 0)
            if store.add(f"acc/{epoch}/ips_workers", 0) >= live:
                ips = store.add(f"acc/{epoch}/ips_milli", 0) / 1e3
            logs = {"loss": store.add(f"acc/{epoch}/loss", 0) / 1e6 / n,
                    "accuracy": store.add(f"acc/{epoch}/correct", 0) / n, "steps": store.add(f"done/{epoch}", 0),
                    "images_per_sec": ips, "epoch_images_per_sec": n / max(dt, 1e-9)}
            if cfg.validation_steps:
                logs.update(_validate(cfg, eng, device))
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            if ctl.lr != lr:
                lr = ctl.lr
                store.set("lr", repr(lr))           # every worker picks it up at its next epoch
            if ctl.stop_training:
                store.set("stop", "1")
            logs["lr"] = lr
            history.append(logs)
            if cfg.verbose:
                print(f"Epoch {epoch + 1}/{cfg.epochs} - {logs['steps']}/{spe} steps - loss: {logs['loss']:.4f} - "
                      f"accuracy: {logs['accuracy']:.4f}" + (f" - val_loss: {logs['val_loss']:.4f}"
                                                              if 'val_loss' in logs else "")
                      + f" - {logs['images_per_sec']:.1f} img/s", flush=True)
            store.set(f"epoch_go/{epoch}", "1")
        else:
            _wait_key(store, f"epoch_go/{epoch}")
    if widx == 0 and cfg.save:
        # the reference saves the PS-held variables (imagenet-resnet50-ps.py:145-148): wait until
        # every live worker pushed its last step and stopped, then pull the final state
        others = [r for r in range(cl.num_ps, cl.world) if r != rank]
        _wait_until(lambda: all(store.check([f"fin/{r}"]) or store.check([f"dead/{r}"]) for r in others),
                    "every live worker's final push")
        worker._exchange(OP_PULL, lr)
    worker.stop()
    hb.stop()
    if widx == 0 and cfg.save:
        from ..utils.checkpoint import save_keras_h5
        path = os.path.join(cfg.save_dir, cfg.checkpoint_name())
        save_keras_h5(path, eng, None, cfg)
        print("Saving model to ", path, flush=True)
    if result_q is not None:
        result_q.put(("worker", rank, steps_done, history))
    dist.destroy_process_group()


def _wait_count(store, key, n, timeout=600):
    """Wait until counter `key` reaches n (an int, or a callable re-read every poll: the live
    worker count drops when the coordinator declares a worker dead)."""
    t0 = time.time()
    while store.add(key, 0) < (n() if callable(n) else n):
        if time.time() - t0 > timeout:
            raise TimeoutError(key)
        time.sleep(0.05)


def _wait_until(pred, what, timeout=600):
    t0 = time.time()
    while not pred():
        if time.time() - t0 > timeout:
            raise TimeoutError(what)
        time.sleep(0.05)


def _wait_key(store, key, timeout=600):
    t0 = time.time()
    while not store.check([key]):
        if time.time() - t0 > timeout:
            raise TimeoutError(key)
        time.sleep(0.05)


def _validate(cfg, eng, device):
    from ..data.datasets import Pipeline, make_source
    src = make_source(cfg.data, "val", cfg)
    pipe = Pipeline(src, cfg.val_batch_size or cfg.batch_size, repeat=True)
    tot = torch.zeros(3, dtype=torch.float64)
    it = pipe.iterate(device)
    for _ in range(cfg.validation_steps):
        im, lb = next(it)
        s = eng.evaluate(im, lb)
        tot[:2] += s.double().cpu()
        tot[2] += im.shape[0]
    return {"val_loss": float(tot[0] / tot[2]), "val_accuracy": float(tot[1] / tot[2])}


def run_ps_job(cfg, num_ps: Optional[int] = None, num_workers: Optional[int] = None, return_results=False):
    """Entry of imagenet-resnet50-ps.py.  Under torchrun (WORLD_SIZE = P + W) every process
    takes its role from RANK; otherwise spawn the whole cluster locally (the reference's
    create_in_process_cluster, imagenet-resnet50-ps.py:31-65)."""
    ns = getattr(cfg, "_ns", None)
    if ns is not None and (num_ps is None or num_workers is None):
        num_ps, num_workers = parse_ps_counts(ns)
    num_ps = num_ps or cfg.num_ps
    num_workers = num_workers or cfg.num_workers
    os.environ["GRPC_FAIL_FAST"] = "use_caller"   # reference parity flag (ps.py:69); failures surface via c10d
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        assert world == num_ps + num_workers, "WORLD_SIZE must equal --ps + --worker"
        _ps_main(int(os.environ["RANK"]), world, num_ps, cfg, int(os.environ.get("MASTER_PORT", "29500")))
        return 0
    import torch.multiprocessing as mp
    from .launch import pick_unused_port
    world = num_ps + num_workers
    port = pick_unused_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ps_main, args=(r, world, num_ps, cfg, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    deadline = time.time() + opt(P, "job_timeout", 3600.0)
    alive = set(range(world))
    while alive and time.time() < deadline:
        for i, p in enumerate(procs):
            if i in alive and not p.is_alive():
                alive.discard(i)
        while not q.empty():
            results.append(q.get())
        time.sleep(0.1)
    for p in procs:
        p.join(timeout=5)
        if p.is_alive():
            p.kill()
    while not q.empty():
        results.append(q.get())
    ps_fail = [i for i in range(num_ps) if procs[i].exitcode not in (0, None)]
    if ps_fail:
        raise RuntimeError(f"parameter server(s) {ps_fail} failed")
    return results if return_results else 0


class ParameterServerStrategy:
    """ParameterServerStrategy + ClusterCoordinator (imagenet-resnet50-ps.py:75-84) behind the
    strategy interface.  The job's roles are processes (run_job / run_ps_job spawns the
    in-process cluster); in a WORKER role this object is the worker's strategy: setup builds
    the engine, the native push/pull client and -- on the GPU -- the forward + backward as one
    HIP graph; train_step runs one step (graph replay, device-side loss / accuracy sums, the
    overlapped gradient push + parameter pull); end_epoch reads the epoch's sums once."""
    name = "ps"

    def __init__(self, cfg, cluster: Optional[_Cluster] = None):
        self.cfg = cfg
        self.cl = cluster
        self.engine = None

    @property
    def num_replicas_in_sync(self) -> int:
        return self.cfg.num_workers

    @property
    def is_chief(self) -> bool:
        return self.cl is None or self.cl.rank == self.cl.num_ps

    def run_job(self):
        return run_ps_job(self.cfg)

    # ------------------------------------------------------------------ worker role
    def setup(self, trainer=None):
        from .strategies import Augment, build_engine
        cfg, cl = self.cfg, self.cl
        if cl is None or cl.is_ps:
            raise RuntimeError("ParameterServerStrategy.setup runs in a worker role of run_ps_job")
        self.device = cl.device
        # (eager by default, like a Horovod rank: one process per GPU keeps its launches ahead of
        # the GPU, and the eager step keeps the weight-gradient side stream that graphed engines
        # give up -- models/engine.py; --graphs replays forward + backward as one HIP graph)
        eng = build_engine(cfg, cl.device, max(cfg.batch_size, cfg.val_batch_size or 0),
                           graphed=cfg.graphs is True)
        eng.init(seed=cfg.seed)
        if cfg.weights and cfg.weights != "none":
            from ..utils.checkpoint import load_pretrained
            load_pretrained(cfg.weights, eng)
            eng.after_update()
        self.engine = eng
        self.worker = PSWorker(cl, eng, None)
        self.widx = cl.rank - cl.num_ps
        self.aug = Augment(cfg, cl.device, cfg.seed + 7919 * self.widx)
        self.graphed = None
        if cl.device.type == "cuda" and hasattr(eng, "wbf") and cfg.graphs is True:
            from ..train.graph import GraphedTrainStep   # forward + backward as one HIP graph
            self.graphed = GraphedTrainStep(eng, None, cfg.batch_size, (cfg.image_size, cfg.image_size),
                                            1.0 / cfg.batch_size, with_optimizer=False)
        self.acc = torch.zeros(2, dtype=torch.float64, device=cl.device)
        self.n_img = 0

    def begin_epoch(self):
        self.acc.zero_()
        self.n_img = 0

    def train_step(self, images, labels, lr: float):
        eng, B = self.engine, images.shape[0]
        flip, off = self.aug(B)
        g = self.graphed
        if g is not None and B == g.B and tuple(images.shape[1:3]) == tuple(g.images.shape[1:3]):
            s = g(images, labels, flip, off)
        else:
            s = eng.forward_backward(images, labels, 1.0 / B, flip=flip, crop_offset=off)
        self.acc.add_(s[:2])            # (device-side: no per-step device -> host read)
        self.n_img += B
        if self.cfg.ps_overlap:
            self.worker.exchange_end()            # the previous push's fresh parameters
            self.worker.exchange_begin(lr)        # this push flies while the next step computes
        else:
            self.worker._exchange(OP_PUSH, lr)
        return s

    def end_epoch(self):
        a = self.acc.cpu()
        return float(a[0]), float(a[1]), self.n_img

    def set_lr(self, lr: float):
        self.cfg = self.cfg.replace(lr=lr)
