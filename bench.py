#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training images/sec on N MI355X GPUs (BASELINE.json).

    python bench.py                                   # 1 GPU
    python bench.py --gpus 8                          # spawns 8 rank processes (Horovod-style)
    python bench.py --gpus 8 --strategy mirrored      # ONE process drives 8 GPUs (in-process RCCL)
    python bench.py --gpus 8 --strategy multiworker --local-gpus 4   # 2 processes x 4 GPUs
    python bench.py --gpus 8 --strategy ps --ps 2      # async parameter server: 2 PS + 6 workers
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8        # what the driver runs: 1 rank per GPU

Config: Keras-v1 ResNet-50 (25,636,712 params, random init), synthetic 3x224x224 uint8
images + random labels, bf16 compute / fp32 master weights, frozen BN (the reference's
`training=False`, Q3), Adam (the reference optimizer), per-GPU batch 2560 fixed (weak
scaling).  The step is the SAME strategy code the entry scripts run (parallel/strategies.py):

  horovod      imagenet-resnet50-hvd.py: 1 process per GPU, gradient buckets all-reduced by the
               native FusionEngine (C++ background thread, RCCL on a side stream, overlapped with
               backward).  Default, and what a torchrun launch measures.
  mirrored     imagenet-resnet50-mirror.py: 1 process, R GPUs, native RcclComm (ncclCommInitAll),
               per-device HIP-graph segments with grouped bucket all-reduces between them.
  multiworker  imagenet-resnet50-multiworkers.py: P processes x R GPUs in one RCCL communicator.
  ps           imagenet-resnet50-ps.py: P parameter servers + W workers (roles are processes),
               asynchronous push/pull over the native HIP-IPC data plane.

The full training step (preprocess, forward, backward, all-reduce, optimizer, weight re-prep)
is inside the timed region: W untimed warmup steps, then K timed steps bracketed by a barrier
+ device synchronize on both sides; the MAX time over ranks is reported.  Rank 0 prints ONE
JSON line; `value` is the whole-job aggregate images/sec.

Launch checks: with --gpus N > 1 and no torchrun environment the parent spawns the rank
processes (or runs the in-process Mirrored path) before anything touches the GPU, and exits
non-zero if fewer than N GPUs are visible or the launched world does not match N.
PDDL_REHEARSE=1 lifts the device check for rehearsals of the multi-rank code on one GPU (ranks
share device 0 over gloo; the JSON then says "rehearsal": true and the number is not a
multi-GPU measurement).

Bounded by construction (a hang must never eat the driver's scaling run):
  * every rank arms a deadline (--timeout, default derived from steps + warmup): on expiry it
    dumps every thread's stack (faulthandler) and exits non-zero, which makes torchrun tear
    the other ranks down;
  * the stall watchdogs (fusion engine, native RCCL communicator, gloo bucket waits) report a
    collective that does not complete within PDDL_STALL_TIMEOUT and, under the bench,
    terminate the rank PDDL_STALL_SHUTDOWN seconds later (exit 124);
  * the spawning parent (no torchrun) enforces the same deadline over its children, stops all
    of them as soon as one fails, and names the ranks that never reported, with the last
    phase / step each one reached.
The JSON's "comm" block records what the collectives actually spanned: backend, the world
size c10d / RCCL report, an all-reduce of ones over the gradient path's communicator, and
every rank's device index + PCI bus id gathered to rank 0.
"""
import argparse
import faulthandler
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec ResNet-50/ImageNet at 1/2/4/8 MI355X + scaling efficiency"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="total GPUs (ranks x local GPUs) of the job")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--strategy", default="horovod", choices=["horovod", "mirrored", "multiworker", "ps"])
    ap.add_argument("--ps", type=int, default=None, help="ps: parameter-server roles (default gpus // 4, >= 1)")
    ap.add_argument("--local-gpus", type=int, default=1, help="multiworker: GPUs per worker process")
    # Per-GPU batch sized for 288 GB HBM3E (BASELINE north star): b2560 holds 75 GB; its stage-1
    # activations (4.1 GB) are reached through per-tile rebased buffer descriptors.  Measured on
    # 1 MI355X, round 3: b512 20.6k, b1024 23.0-23.4k, b1536 24.3k, b2048 24.6k images/s
    # (profiles/r3_batch_plateau.txt); after the fused kernels b2048 26.16-26.17k vs b2560
    # 26.57-26.58k on one box (profiles/r3_b2560_ab.txt: the ~4.4 ms per-step fixed cost
    # amortised further).  b2675+ would exceed 2^31 elements in conv1's output.
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (default 2560; train-mode BN 1024; fp32 256; CPU 32)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--crop", type=int, default=None, help="network input (default = image size)")
    ap.add_argument("--optimizer", default="adam", choices=["adam", "sgd"])
    ap.add_argument("--bn-mode", default="frozen", choices=["frozen", "train"],
                    help="frozen = the reference's training=False BN (folded); train = batch statistics")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--ps-wire", default="bf16", choices=["fp32", "bf16"],
                    help="ps: element type of the gradient push / parameter pull over xGMI (fp32 master weights and "
                         "Adam on the PS either way)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="fp32: the reference's precision on the fp32-MFMA HIP convolutions (models/engine_f32.py)")
    ap.add_argument("--graph", type=int, default=None,
                    help="HIP graphs: 1 GPU = whole step; mirrored = per-device segments (default on)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: BASELINE config 1 plumbing (fp32 PyTorch reference engine, gloo ranks)")
    ap.add_argument("--comm-proxy", default=None, metavar="SPEC",
                    help="1 GPU: run a paced, CU-holding stand-in for each bucket's RCCL all-reduce on a side "
                         "stream (e.g. 'world=8,busbw=350,nch=32'), to measure the backward under comm contention")
    ap.add_argument("--baseline-ips", type=float, default=None, metavar="IPS",
                    help="1-GPU images/sec of the same config (the reference publishes none): fills vs_baseline "
                         "(value / IPS) and scaling_efficiency (value / (n_gpus * IPS))")
    ap.add_argument("--timeout", type=float, default=None,
                    help="job deadline in seconds (default: derived from steps + warmup); on expiry every "
                         "rank dumps its stacks and the job exits non-zero")
    args = ap.parse_args(argv)
    if args.batch is None:
        # (train-mode BN keeps every pre-BN activation: at 2560 they pass the kernels' 2^31-element
        # tensor bound, so its default is the largest power-of-two batch under it)
        args.batch = 32 if args.device == "cpu" else (256 if args.precision == "fp32" else
                                                      1024 if args.bn_mode == "train" else 2560)
    if args.crop is None:
        args.crop = args.image_size
    if args.timeout is None:
        per_step = 60.0 if args.device == "cpu" else 10.0
        args.timeout = 300.0 + per_step * (args.steps + args.warmup)
    return args


def fail(msg):
    sys.stderr.write(f"bench.py: {msg}\n")
    sys.exit(2)


def rehearsing() -> bool:
    return os.environ.get("PDDL_REHEARSE", "0") == "1"


# ---------------------------------------------------------------------------- launcher
def visible_gpus() -> int:
    import torch   # device_count() does not initialise the GPU on this image
    return torch.cuda.device_count()


def launch(args, argv):
    """Parent of an N-GPU job without torchrun: spawn one child per worker process with the
    torchrun environment.  Nothing here touches the GPU.  The job is bounded: the first child
    to fail stops the rest, and at the deadline every child is stopped and the ranks that never
    reported are named with the last phase / step each reached."""
    from pddl.parallel.launch import pick_unused_port
    per = args.local_gpus if args.strategy == "multiworker" else 1
    if args.gpus % per:
        fail(f"--gpus {args.gpus} is not a multiple of --local-gpus {per}")
    nproc = args.gpus // per
    port = pick_unused_port()
    prog = tempfile.mkdtemp(prefix="pddl_bench_")
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(nproc),
                LOCAL_WORLD_SIZE=str(nproc), PDDL_BENCH_CHILD="1", PDDL_BENCH_PROGRESS=prog)
    if args.device == "cpu" or rehearsing():
        env0.setdefault("PDDL_DIST_BACKEND", "gloo")
    procs = {}
    for r in range(nproc):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs[r] = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                    stdout=None if r == 0 else subprocess.DEVNULL)
    # children arm their own deadline at args.timeout; the parent's is a little later, so a
    # child's stack dump lands first
    deadline = time.monotonic() + args.timeout + 30.0
    codes = {}
    rc = 0
    try:
        while len(codes) < nproc:
            for r, p in procs.items():
                if r in codes:
                    continue
                code = p.poll()
                if code is None:
                    continue
                codes[r] = code
                if code != 0 and rc == 0:
                    rc = code
                    sys.stderr.write(f"bench.py: rank {r} exited with status {code}; stopping the other ranks\n")
                    _report_ranks(procs, codes, prog)
                    _stop(procs, codes)
            if len(codes) < nproc and time.monotonic() > deadline:
                sys.stderr.write(f"bench.py: job deadline ({args.timeout:.0f} s) expired\n")
                _report_ranks(procs, codes, prog)
                _stop(procs, codes)
                rc = rc or 124
            time.sleep(0.2)
    finally:
        for p in procs.values():
            if p.poll() is None:
                p.kill()
    return rc


def _progress(prog, r):
    try:
        with open(os.path.join(prog, f"rank{r}")) as f:
            return f.read().strip() or "?"
    except OSError:
        return "never reported"


def _report_ranks(procs, codes, prog):
    for r, p in sorted(procs.items()):
        state = f"exited {codes[r]}" if r in codes else ("running" if p.poll() is None else f"exited {p.poll()}")
        sys.stderr.write(f"bench.py:   rank {r} (pid {p.pid}): {state}; last progress: {_progress(prog, r)}\n")
    sys.stderr.flush()


def _stop(procs, codes):
    for r, p in procs.items():
        if p.poll() is None:
            p.terminate()
    t0 = time.monotonic()
    while time.monotonic() - t0 < 10 and any(p.poll() is None for p in procs.values()):
        time.sleep(0.1)
    for r, p in procs.items():
        if p.poll() is None:
            p.kill()
        codes.setdefault(r, p.wait())


class Progress:
    """This rank's last phase / step, for the launcher's report (PDDL_BENCH_PROGRESS dir)."""

    def __init__(self, rank):
        d = os.environ.get("PDDL_BENCH_PROGRESS")
        self.path = os.path.join(d, f"rank{rank}") if d else None

    def __call__(self, phase, step=None):
        if self.path:
            with open(self.path, "w") as f:
                f.write(phase if step is None else f"{phase} step {step}")


# ---------------------------------------------------------------------------- measured job
def build_cfg(args, strategy):
    from pddl.config import make_config
    graphs = None if args.graph is None else bool(args.graph)
    return make_config("bench", strategy=strategy, batch_size=args.batch, crop=args.crop,
                       image_size=args.image_size, optimizer=args.optimizer,
                       lr=1e-3 if args.optimizer == "adam" else 0.1, bn_mode=args.bn_mode,
                       bucket_mb=args.bucket_mb, grad_dtype=args.grad_dtype, device=args.device,
                       graphs=graphs, data="synthetic_fixed", seed=0, precision=args.precision)


def arm_deadline(args):
    """Every rank: dump all stacks and exit non-zero at the deadline (faulthandler's watchdog
    thread runs without the GIL, so it fires even with the main thread stuck in native code);
    stalled collectives end the rank PDDL_STALL_SHUTDOWN seconds after their report."""
    faulthandler.dump_traceback_later(args.timeout, exit=True)
    os.environ.setdefault("PDDL_STALL_SHUTDOWN", "30")


def run(args):
    arm_deadline(args)
    import torch
    import torch.distributed as dist
    import pddl  # noqa: F401
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    progress = Progress(rank)
    progress("init")
    cpu = args.device == "cpu"
    devices = None
    if args.strategy == "mirrored":
        if world != 1:
            fail("--strategy mirrored is ONE process driving every GPU; do not launch it with torchrun")
        n_local = args.gpus
        if cpu:
            os.environ["PDDL_CPU_REPLICAS"] = str(n_local)
        if not cpu:
            have = visible_gpus()
            if have < n_local and not rehearsing():
                fail(f"--gpus {n_local} but only {have} GPU(s) are visible")
            devices = [i % max(1, have) for i in range(n_local)]
        strat_name = "mirrored"
    else:
        per = args.local_gpus if args.strategy == "multiworker" else 1
        if world * per != args.gpus:
            fail(f"--gpus {args.gpus} but the launch has {world} rank(s) x {per} GPU(s) each")
        if per > 1:
            os.environ["PDDL_LOCAL_GPUS"] = str(per)
        if not cpu:
            have = visible_gpus()
            if have < args.gpus and not rehearsing():
                fail(f"--gpus {args.gpus} but only {have} GPU(s) are visible")
        strat_name = args.strategy
    if cpu:
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, world)))
    if args.comm_proxy:
        if args.gpus != 1 or cpu or args.strategy != "horovod":
            fail("--comm-proxy models multi-GPU collectives on ONE GPU (horovod strategy)")
        os.environ["PDDL_COMM_PROXY"] = args.comm_proxy
    cfg = build_cfg(args, strat_name)
    if strat_name == "horovod" and world == 1 and args.graph and not cpu:
        cfg = cfg.replace(strategy="single", graphs=True)   # whole-step HIP graph on one GPU
    st = make_strategy(cfg)
    if devices is not None:
        st._devices = devices
    tr = Trainer(cfg, st)
    progress("broadcast")
    st.broadcast_state(tr)
    replicas = st.num_replicas_in_sync
    local_devs = [e.params.device for e, _ in st._replicas()]
    B = args.batch
    S = args.image_size
    # synthetic batch, resident on each local device (BASELINE: synthetic data)
    ims, lbs = [], []
    for i, d in enumerate(local_devs):
        # (PDDL_BENCH_SAME_DATA=1: every replica gets replica 0's batch -- a multi-rank run then
        # follows the 1-GPU loss trajectory, a check of the gradient reduction)
        rep = 0 if os.environ.get("PDDL_BENCH_SAME_DATA") == "1" else rank * len(local_devs) + i
        g = torch.Generator(device=d).manual_seed(1234 + 7919 * rep)
        ims.append(torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, device=d, generator=g))
        lbs.append(torch.randint(0, 1000, (B,), dtype=torch.int64, device=d, generator=g))
    if len(local_devs) == 1:
        images, labels = ims[0], lbs[0]
    else:
        images, labels = ims, lbs

    def sync_all():
        if not cpu:
            for d in sorted({d.index for d in local_devs}):
                torch.cuda.synchronize(d)

    def barrier():
        sync_all()
        if world > 1:
            dist.barrier()
        sync_all()

    stats = None
    for i in range(args.warmup):
        progress("warmup", i)
        stats = st.train_step(images, labels)
    progress("barrier (after warmup)")
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        progress("timed", i)
        stats = st.train_step(images, labels)
    progress("barrier (after timed steps)")
    barrier()
    dt = time.perf_counter() - t0
    progress("report")
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    loss = float(stats[0].item()) / (B * len(local_devs)) if stats is not None else float("nan")
    comm = comm_report(st, world, rank, local_devs, cpu)
    total = B * args.gpus
    ips = total * args.steps / dt
    desc = {
        "horovod": "horovod-style 1 proc/GPU, native FusionEngine: RCCL bucketed all-reduce overlapped with backward",
        "single": "single process, whole step replayed as one HIP graph",
        "mirrored": (f"mirrored: 1 process x {args.gpus} GPUs, ncclCommInitAll, grouped bucket all-reduce"
                     + (" between per-device HIP-graph segments (weight gradients as per-segment side graphs)"
                        if getattr(st, "mirror", None) is not None
                        and st.mirror.graph_mode else "")
                     if not (getattr(st, "mirror", None) is not None and st.mirror.graph_mode
                             and st.mirror._single_replica_job())
                     else ("mirrored: 1 replica, whole step as one HIP graph (no collective to run)" if cfg.graphs
                           else "mirrored: 1 replica, eager step (no collective to run)")),
        "multiworker": f"multiworker: {world} process(es) x {args.local_gpus if args.strategy == 'multiworker' else 1}"
                       " GPU(s), one RCCL communicator",
    }[cfg.strategy]
    if args.gpus == 1 and cfg.strategy == "horovod":
        desc = "single GPU (horovod strategy code path, no collectives)"
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(ips, 2), "unit": "images/sec", "n_gpus": args.gpus,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32" if cpu else args.precision,
            "data": f"synthetic (uint8 3x{S}x{S}, random labels, random-init weights)",
            "config": {"model": "ResNet-50 Keras-v1 (25,636,712 params, random init)", "global_batch": total,
                       "per_gpu_batch": B, "seq_len": None, "image_size": args.crop,
                       "parallelism": f"dp{args.gpus}", "strategy": desc, "replicas": replicas,
                       "optimizer": args.optimizer,
                       "bn": "frozen (training=False)" if args.bn_mode == "frozen" else "train (batch statistics)",
                       "hip_graph": bool(cfg.strategy == "single" or (getattr(st, "mirror", None) is not None
                                                                      and st.mirror.graph_mode)),
                       "bucket_mb": args.bucket_mb, "grad_dtype": args.grad_dtype,
                       "device": "cpu" if cpu else "MI355X"},
            "per_gpu_images_per_sec": round(ips / args.gpus, 2),
            "final_loss": round(loss, 4),
        }
        add_scaling(out, args)
        if not cpu:   # HBM footprint of the step (torch caching allocator, device of rank 0)
            out["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(local_devs[0]) / 1e9, 2)
        out["comm"] = comm
        if rehearsing():
            out["rehearsal"] = True
        if args.comm_proxy:
            px = st.reducer
            out["comm_proxy"] = {"spec": args.comm_proxy, "world": px.world, "busbw_gbs": px.busbw / 1e9,
                                 "channels": px.nch, "buckets": len(px.buckets),
                                 "modelled_ms_per_step": round(px.modelled_s * 1e3, 3),
                                 "note": "1 GPU with paced stand-ins for the bucket all-reduces: NOT a multi-GPU number"}
        print(json.dumps(out), flush=True)
    progress("done")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()
    return 0


def add_scaling(out, args):
    """--baseline-ips: vs_baseline and scaling_efficiency against a measured 1-GPU rate."""
    from pddl.utils.scaling import efficiency
    if args.baseline_ips:
        out["vs_baseline"] = round(out["value"] / args.baseline_ips, 4)
        out["scaling_efficiency"] = round(efficiency(out["value"], args.gpus, args.baseline_ips), 4)
        out["baseline_ips"] = args.baseline_ips


def comm_report(st, world, rank, local_devs, cpu):
    """What the gradient collectives actually spanned (gathered to rank 0)."""
    import socket
    import torch
    import torch.distributed as dist

    def dev_info(d):
        if cpu or d.type != "cuda":
            return {"device": str(d)}
        p = torch.cuda.get_device_properties(d)
        bus = getattr(p, "pci_bus_id", None)
        dom = getattr(p, "pci_domain_id", 0)
        devid = getattr(p, "pci_device_id", 0)
        out = {"device": d.index, "name": p.name, "gcn_arch": getattr(p, "gcnArchName", "")}
        if bus is not None:
            out["pci_bus_id"] = f"{dom:04x}:{bus:02x}:{devid:02x}.0"
        return out

    mine = {"rank": rank, "host": socket.gethostname(), "pid": os.getpid(),
            "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "devices": [dev_info(d) for d in local_devs]}
    rep = {"world_size_env": world, "local_replicas": len(local_devs)}
    mirror = getattr(st, "mirror", None)
    rccl = getattr(mirror, "comm", None) if mirror is not None else None
    if rccl is not None:            # the native RcclComm: ask RCCL what it built
        rep["native_rccl"] = {"nranks": rccl.nranks, "communicators": rccl.info(),
                              "watchdog": {k: v for k, v in rccl.watchdog_state().items() if k != "message"}}
        ones = [torch.ones(1, device=d) for d in local_devs]
        rccl.all_reduce(ones, "sum", "comm check")
        rep["allreduce_ones"] = float(ones[0].item())
    if world > 1 and dist.is_initialized():
        rep["backend"] = dist.get_backend()
        rep["c10d_world_size"] = dist.get_world_size()
        if rccl is None:            # the gradient path's process group: an all-reduce of ones
            dev = local_devs[0] if dist.get_backend() == "nccl" else "cpu"
            t = torch.ones(1, device=dev)
            dist.all_reduce(t)
            rep["allreduce_ones"] = float(t.item())
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        rep["ranks"] = gathered
    else:
        rep["backend"] = "native RCCL (in-process)" if rccl is not None else "none (1 replica)"
        rep["ranks"] = [mine]
    fusion = getattr(st, "fusion", None)
    if fusion is not None:
        rep["fusion_engine"] = {"world": fusion.world, "wire": fusion.wire, "buckets": len(st.buckets),
                                "issued": int(fusion.issued)}
    if not cpu:
        try:
            rep["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:
            pass
    return rep


def run_ps(args):
    """BASELINE config 5: asynchronous parameter server (imagenet-resnet50-ps.py) with P PS roles
    and W = gpus - P workers, one GPU each, the native HIP-IPC data plane over xGMI.  One
    untimed warmup epoch, then a timed epoch of `steps` worker steps claimed by the workers
    asynchronously; value = aggregate worker images/sec of the timed epoch (worker 0's clock
    over every worker's training steps, parameter_server.py).  The role processes are bounded
    by run_ps_job's job deadline (PDDL_PS job_timeout, set from --timeout unless given)."""
    from pddl.utils.envopts import opts, with_opt
    if "job_timeout" not in opts("PDDL_PS"):
        os.environ["PDDL_PS"] = with_opt("PDDL_PS", "job_timeout", args.timeout)
    import pddl  # noqa: F401
    from pddl.config import make_config
    from pddl.parallel.parameter_server import run_ps_job
    n_ps = args.ps if args.ps is not None else max(1, args.gpus // 4)
    n_w = args.gpus - n_ps
    if n_w < 1:
        fail(f"--gpus {args.gpus} leaves no worker next to {n_ps} parameter server(s)")
    if args.device == "cuda" and not rehearsing():
        have = visible_gpus()
        if have < args.gpus:
            fail(f"--gpus {args.gpus} but only {have} GPU(s) are visible")
    cfg = make_config("ps", batch_size=args.batch, crop=args.crop, image_size=args.image_size,
                      optimizer="adam", lr=1e-3, bn_mode=args.bn_mode, device=args.device, data="synthetic",
                      steps_per_epoch=args.steps, validation_steps=0, epochs=2, save=False, verbose=0,
                      train_images=max(1_281_167, args.steps * args.batch), num_ps=n_ps, num_workers=n_w,
                      ps_wire=args.ps_wire, graphs=None if args.graph is None else bool(args.graph))
    t0 = time.perf_counter()
    res = run_ps_job(cfg, num_ps=n_ps, num_workers=n_w, return_results=True)
    wall = time.perf_counter() - t0
    hist = [r[3] for r in res if r[0] == "worker" and r[3]]
    svc = [r[5] for r in res if r[0] == "ps" and len(r) > 5 and r[5]]
    if not hist or len(hist[0]) < 2:
        fail("parameter-server job returned no timed epoch")
    ep = hist[0][1]
    ips = ep["images_per_sec"]
    out = {
        "metric": METRIC, "value": round(ips, 2), "unit": "images/sec", "n_gpus": args.gpus, "steps": args.steps,
        "warmup": args.steps, "ms_per_step": round(args.batch * n_w / ips * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32" if args.device == "cpu" else "bf16",
        "data": f"synthetic (uint8 3x{args.image_size}x{args.image_size}, random labels, random-init weights)",
        "config": {"model": "ResNet-50 Keras-v1 (25,636,712 params, random init)", "global_batch": args.batch * n_w,
                   "per_gpu_batch": args.batch, "seq_len": None, "image_size": args.crop,
                   "parallelism": f"ps{n_ps}+w{n_w}", "strategy":
                   f"async parameter server: {n_ps} PS + {n_w} workers, native HIP-IPC push/pull, PS-side fused Adam",
                   "replicas": n_w, "optimizer": "adam", "bn": args.bn_mode, "hip_graph": args.device == "cuda" and args.graph != 0,
                   "ps_wire": args.ps_wire,
                   "device": "cpu" if args.device == "cpu" else "MI355X",
                   "note": "ms_per_step = one synchronous-equivalent step of all workers; warmup = one untimed epoch"},
        "per_gpu_images_per_sec": round(ips / n_w, 2), "steps_timed_epoch": ep.get("steps"),
        "job_wall_s": round(wall, 1), **({"rehearsal": True} if rehearsing() else {}),
        **({"ps_service": svc} if svc else {}),
    }
    add_scaling(out, args)
    print(json.dumps(out), flush=True)
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus < 1:
        fail("--gpus must be >= 1")
    if args.strategy == "ps":
        if "WORLD_SIZE" in os.environ:
            fail("--strategy ps spawns its own P + W role processes; do not launch it with torchrun")
        return run_ps(args)
    torchrun = "WORLD_SIZE" in os.environ
    if not torchrun and args.gpus > 1 and args.strategy != "mirrored":
        if args.device == "cuda" and not rehearsing():
            have = visible_gpus()
            if have < args.gpus:
                fail(f"--gpus {args.gpus} but only {have} GPU(s) are visible")
        return launch(args, argv)
    from pddl.parallel.faults import run_fail_fast
    return run_fail_fast(run, args, multi=args.gpus > 1)


if __name__ == "__main__":
    sys.exit(main())
