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
`training=False`, Q3), Adam (the reference optimizer), per-GPU batch 1024 fixed (weak
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
"""
import argparse
import json
import os
import subprocess
import sys
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
    # Per-GPU batch sized for 288 GB HBM3E (BASELINE north star): 1024 is the largest batch whose
    # biggest activation (conv1 output, 1.6 GB) stays inside the kernels' 31-bit buffer offsets.
    # Measured on 1 MI355X (round 1): b128 13.5k, b256 15.4k, b512 16.9k, b1024 18.3k images/s;
    # round 2: b256 16.8k, b1024 22.1-22.5k.
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 1024; CPU 32)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--crop", type=int, default=None, help="network input (default = image size)")
    ap.add_argument("--optimizer", default="adam", choices=["adam", "sgd"])
    ap.add_argument("--bn-mode", default="frozen", choices=["frozen", "train"],
                    help="frozen = the reference's training=False BN (folded); train = batch statistics")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="fp32: the reference's precision on the fp32-MFMA HIP convolutions (models/engine_f32.py)")
    ap.add_argument("--graph", type=int, default=None,
                    help="HIP graphs: 1 GPU = whole step; mirrored = per-device segments (default on)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: BASELINE config 1 plumbing (fp32 PyTorch reference engine, gloo ranks)")
    args = ap.parse_args(argv)
    if args.batch is None:
        args.batch = 32 if args.device == "cpu" else (256 if args.precision == "fp32" else 1024)
    if args.crop is None:
        args.crop = args.image_size
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
    torchrun environment.  Nothing here touches the GPU."""
    from pddl.parallel.launch import pick_unused_port
    per = args.local_gpus if args.strategy == "multiworker" else 1
    if args.gpus % per:
        fail(f"--gpus {args.gpus} is not a multiple of --local-gpus {per}")
    nproc = args.gpus // per
    port = pick_unused_port()
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(nproc),
                LOCAL_WORLD_SIZE=str(nproc), PDDL_BENCH_CHILD="1")
    if args.device == "cpu" or rehearsing():
        env0.setdefault("PDDL_DIST_BACKEND", "gloo")
    procs = []
    for r in range(nproc):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:      # a dead rank would leave its peers inside a collective
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
    return rc


# ---------------------------------------------------------------------------- measured job
def build_cfg(args, strategy):
    from pddl.config import make_config
    graphs = None if args.graph is None else bool(args.graph)
    return make_config("bench", strategy=strategy, batch_size=args.batch, crop=args.crop,
                       image_size=args.image_size, optimizer=args.optimizer,
                       lr=1e-3 if args.optimizer == "adam" else 0.1, bn_mode=args.bn_mode,
                       bucket_mb=args.bucket_mb, grad_dtype=args.grad_dtype, device=args.device,
                       graphs=graphs, data="synthetic_fixed", seed=0, precision=args.precision)


def run(args):
    import torch
    import torch.distributed as dist
    import pddl  # noqa: F401
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
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
    cfg = build_cfg(args, strat_name)
    if strat_name == "horovod" and world == 1 and args.graph and not cpu:
        cfg = cfg.replace(strategy="single", graphs=True)   # whole-step HIP graph on one GPU
    st = make_strategy(cfg)
    if devices is not None:
        st._devices = devices
    tr = Trainer(cfg, st)
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
    for _ in range(args.warmup):
        stats = st.train_step(images, labels)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stats = st.train_step(images, labels)
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    loss = float(stats[0].item()) / (B * len(local_devs)) if stats is not None else float("nan")
    total = B * args.gpus
    ips = total * args.steps / dt
    desc = {
        "horovod": "horovod-style 1 proc/GPU, native FusionEngine: RCCL bucketed all-reduce overlapped with backward",
        "single": "single process, whole step replayed as one HIP graph",
        "mirrored": f"mirrored: 1 process x {args.gpus} GPUs, ncclCommInitAll, grouped bucket all-reduce"
                    + (" between per-device HIP-graph segments" if getattr(st, "mirror", None) is not None
                       and st.mirror.graph_mode else ""),
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
        if not cpu:   # HBM footprint of the step (torch caching allocator, device of rank 0)
            out["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(local_devs[0]) / 1e9, 2)
        if rehearsing():
            out["rehearsal"] = True
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def run_ps(args):
    """BASELINE config 5: asynchronous parameter server (imagenet-resnet50-ps.py) with P PS roles
    and W = gpus - P workers, one GPU each, the native HIP-IPC data plane over xGMI.  One
    untimed warmup epoch, then a timed epoch of `steps` worker steps claimed by the workers
    asynchronously; value = aggregate worker images/sec of the timed epoch (worker 0's clock
    over every worker's training steps, parameter_server.py)."""
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
                      train_images=max(1_281_167, args.steps * args.batch), num_ps=n_ps, num_workers=n_w)
    t0 = time.perf_counter()
    res = run_ps_job(cfg, num_ps=n_ps, num_workers=n_w, return_results=True)
    wall = time.perf_counter() - t0
    hist = [r[3] for r in res if r[0] == "worker" and r[3]]
    if not hist or len(hist[0]) < 2:
        fail("parameter-server job returned no timed epoch")
    ep = hist[0][1]
    ips = ep["images_per_sec"]
    print(json.dumps({
        "metric": METRIC, "value": round(ips, 2), "unit": "images/sec", "n_gpus": args.gpus, "steps": args.steps,
        "warmup": args.steps, "ms_per_step": round(args.batch * n_w / ips * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32" if args.device == "cpu" else "bf16",
        "data": f"synthetic (uint8 3x{args.image_size}x{args.image_size}, random labels, random-init weights)",
        "config": {"model": "ResNet-50 Keras-v1 (25,636,712 params, random init)", "global_batch": args.batch * n_w,
                   "per_gpu_batch": args.batch, "seq_len": None, "image_size": args.crop,
                   "parallelism": f"ps{n_ps}+w{n_w}", "strategy":
                   f"async parameter server: {n_ps} PS + {n_w} workers, native HIP-IPC push/pull, PS-side fused Adam",
                   "replicas": n_w, "optimizer": "adam", "bn": args.bn_mode, "hip_graph": False,
                   "device": "cpu" if args.device == "cpu" else "MI355X",
                   "note": "ms_per_step = one synchronous-equivalent step of all workers; warmup = one untimed epoch"},
        "per_gpu_images_per_sec": round(ips / n_w, 2), "steps_timed_epoch": ep.get("steps"),
        "job_wall_s": round(wall, 1), **({"rehearsal": True} if rehearsing() else {}),
    }), flush=True)
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
    return run(args)


if __name__ == "__main__":
    sys.exit(main())
