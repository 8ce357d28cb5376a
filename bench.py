#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training images/sec on N MI355X GPUs (BASELINE.json).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Config: Keras-v1 ResNet-50 (25,636,712 params, random init), synthetic 3x224x224 uint8
images + random labels, bf16 compute / fp32 master weights, frozen BN (the reference's
`training=False`, Q3), Adam (the reference optimizer), per-GPU batch 1024 fixed (weak scaling),
Horovod-style data parallelism: one process per GPU, fp32 gradient buckets all-reduced over
RCCL/xGMI on a side stream while backward continues.  The full training step (preprocess,
forward, backward, all-reduce, optimizer, weight re-prep) is inside the timed region.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # Per-GPU batch sized for 288 GB HBM3E (BASELINE north star): 1024 is the largest batch whose
    # biggest activation (conv1 output, 1.6 GB) stays inside the kernels' 31-bit buffer offsets.
    # Measured on 1 MI355X: b128 13.5k, b256 15.4k, b512 16.9k, b1024 18.3k images/s.
    ap.add_argument("--batch", type=int, default=1024, help="per-GPU batch")
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--optimizer", default="adam", choices=["adam", "sgd"])
    ap.add_argument("--bn-mode", default="frozen", choices=["frozen", "train"],
                    help="frozen = the reference's training=False BN (folded); train = batch statistics")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--graph", type=int, default=0, help="1: replay the whole step as a HIP graph (1 GPU)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: BASELINE config 1 (CPU plumbing, fp32 PyTorch reference engine, batch 32)")
    args = ap.parse_args()
    if args.device == "cpu":
        return cpu_bench(args)

    import torch
    import torch.distributed as dist
    import pddl  # noqa: F401
    from pddl.models.engine import make_hip_engine
    from pddl.models.resnet50 import ParamLayout
    from pddl.train.optim import make_optimizer
    from pddl.parallel.collectives import BucketAllReducer
    from pddl.utils import profiling as prof

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # (modulo: lets a rehearsal put several ranks on one GPU; one rank per GPU on a real node)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        # PDDL_DIST_BACKEND=gloo only for rehearsing the multi-rank path on one GPU (RCCL refuses
        # two ranks on the same device); the measured configuration is RCCL ("nccl")
        backend = os.environ.get("PDDL_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": torch.device("cuda", local)} if backend == "nccl" else {}))
    B = args.batch
    L = ParamLayout()
    eng = make_hip_engine(L, B, bn_mode=args.bn_mode, crop=args.crop, image_size=224)
    eng.init(seed=0)
    reducer = None
    if world > 1:
        reducer = BucketAllReducer(eng.grads, L.buckets(args.bucket_mb), average=False)
        reducer.broadcast_(eng.params, src=0)
        eng.after_update()
    opt = make_optimizer(args.optimizer, eng, lr=1e-3 if args.optimizer == "adam" else 0.1)
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    images = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda", generator=gen)
    labels = torch.randint(0, 1000, (B,), dtype=torch.int64, device="cuda", generator=gen)
    flips = torch.randint(0, 2, (64, B), dtype=torch.uint8, device="cuda", generator=gen)
    gscale = 1.0 / (B * world)

    graphed = None
    if args.graph and world == 1:
        from pddl.train.graph import GraphedTrainStep
        graphed = GraphedTrainStep(eng, opt, B, (224, 224), gscale)

    def step(i):
        if graphed is not None:
            return graphed(images, labels, flips[i % 64])
        cb = None
        if reducer is not None:
            reducer.begin()
            cb = None if args.no_overlap else reducer.on_bucket_ready
        stats = eng.forward_backward(images, labels, gscale, flip=flips[i % 64], bucket_cb=cb,
                                     buckets=reducer.buckets if reducer is not None else None)
        if reducer is not None:
            prof.push("step/allreduce")
            if args.no_overlap:
                for j in range(len(reducer.buckets)):
                    reducer.on_bucket_ready(j)
            reducer.finish()
            prof.pop()
        prof.push("step/optimizer")
        opt.step()
        eng.after_update()
        prof.pop()
        return stats

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        stats = step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss = stats[0].item() / B
    ms = dt / args.steps * 1e3
    ips = B * world * args.steps / dt
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec ResNet-50/ImageNet at 1/2/4/8 MI355X + scaling efficiency",
            "value": round(ips, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (uint8 3x224x224, random labels)",
            "config": {"model": "ResNet-50 Keras-v1 (25,636,712 params, random init)", "global_batch": B * world,
                       "per_gpu_batch": B, "seq_len": None, "image_size": args.crop,
                       "parallelism": f"dp{world}", "optimizer": args.optimizer, "bn": "frozen (training=False)" if args.bn_mode == "frozen" else "train (batch statistics)",
                       "hip_graph": bool(graphed is not None),
                       "strategy": "horovod-style 1 proc/GPU, RCCL bucketed all-reduce overlapped with backward"
                       if world > 1 else "single-process"},
            "final_loss": round(loss, 4),
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_bench(args):
    """BASELINE.json config 1: the imagenet-resnet50.py plumbing on CPU (no GPU), fp32."""
    import torch
    import pddl  # noqa: F401
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    from pddl.train.optim import make_optimizer
    B = args.batch if args.batch != 1024 else 32
    eng = TorchEngine(ParamLayout(), B, crop=args.crop, device="cpu", bn_mode=args.bn_mode)
    eng.init(seed=0)
    opt = make_optimizer(args.optimizer, eng, lr=1e-3 if args.optimizer == "adam" else 0.1)
    g = torch.Generator().manual_seed(1234)
    images = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 1000, (B,), dtype=torch.int64, generator=g)
    for _ in range(args.warmup):
        eng.forward_backward(images, labels, 1.0 / B)
        opt.step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stats = eng.forward_backward(images, labels, 1.0 / B)
        opt.step()
    dt = time.perf_counter() - t0
    print(json.dumps({
        "metric": "images/sec ResNet-50/ImageNet at 1/2/4/8 MI355X + scaling efficiency",
        "value": round(B * args.steps / dt, 3), "unit": "images/sec", "n_gpus": 0, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 1), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (uint8 3x224x224, random labels)",
        "config": {"model": "ResNet-50 Keras-v1 (25,636,712 params, random init)", "global_batch": B,
                   "image_size": args.crop, "parallelism": "cpu", "optimizer": args.optimizer,
                   "bn": args.bn_mode, "threads": torch.get_num_threads(),
                   "strategy": "single-process CPU (BASELINE config 1)"},
        "final_loss": round(stats[0].item() / B, 4)}), flush=True)


if __name__ == "__main__":
    main()
