"""All-reduce bus-bandwidth sweep over RCCL (xGMI), the comm layer's tuning bench.

    python bench/allreduce.py                                   # 1 rank (RCCL runs; busbw is 0 by definition)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/allreduce.py \
        --json gpurun_out/allreduce.json
    NCCL_MIN_NCHANNELS=16 NCCL_ALGO=Ring NCCL_PROTO=Simple python -m torch.distributed.run ...   # RCCL knobs

Two measurements, rank 0 prints one JSON line each:
  * `sweep`: one all_reduce of S bytes (1 KiB .. 256 MiB) -> algbw = S / t and
    busbw = algbw * 2 (n - 1) / n (the nccl-tests convention: the per-link rate a ring needs);
  * `buckets`: the ResNet-50 step's gradient (25,583,592 fp32 = 97.6 MiB, or its bf16 half)
    cut into B-MiB buckets and reduced through the native FusionEngine exactly as the Horovod
    strategy issues them (side stream, in bucket order) -> ms per step per bucket size, the
    measurement behind the --bucket-mb default.  An MI355X has 7 xGMI links per GPU at about
    153 GB/s each; one ring uses one outbound link, so RCCL needs several channels (rings over
    disjoint link permutations) to approach 7x that: the sweep reports which message size
    first reaches the plateau, and the bucket run whether 32 MiB buckets keep every channel
    busy.
The RCCL environment (NCCL_* variables) in effect is echoed in every line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GRAD_ELEMS = 25_583_592   # trainable parameters of the Keras ResNet-50


def init():
    if "WORLD_SIZE" not in os.environ:
        from pddl.parallel.launch import pick_unused_port
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(pick_unused_port()))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dist.get_rank(), dist.get_world_size()


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-kib", type=int, default=1)
    ap.add_argument("--max-mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--buckets", default="4,8,16,32,64,128", help="bucket sizes (MiB) for the gradient run")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rank, world = init()
    env = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))}
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    esz = 4 if a.dtype == "fp32" else 2
    out = []

    def emit(row):
        row.update(world=world, dtype=a.dtype, rccl_env=env)
        out.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)

    nbytes = a.min_kib << 10
    while nbytes <= a.max_mib << 20:
        x = torch.ones(nbytes // esz, device="cuda", dtype=dt)
        t = timed(lambda: dist.all_reduce(x), a.iters)
        algbw = nbytes / t / 1e9
        emit({"kind": "sweep", "bytes": nbytes, "us": round(t * 1e6, 1), "algbw_GBs": round(algbw, 1),
              "busbw_GBs": round(algbw * 2 * (world - 1) / world, 1)})
        nbytes *= 4
    # the gradient of one training step through the FusionEngine, per bucket size
    from pddl.ops.native import require_native
    g = torch.ones(GRAD_ELEMS, device="cuda", dtype=torch.float32)
    for mb in [float(b) for b in a.buckets.split(",")]:
        per = max(1, int(mb * (1 << 20) / 4))
        buckets = [(s, min(per, GRAD_ELEMS - s)) for s in range(0, GRAD_ELEMS, per)]
        fe = require_native().FusionEngine(dist.group.WORLD, g, buckets, 60.0, False, rank, a.dtype)

        def step():
            fe.begin_step()
            for i in range(len(buckets)):
                fe.bucket_ready(i)
            fe.finish()
        t = timed(step, a.iters)
        wire = GRAD_ELEMS * esz
        algbw = wire / t / 1e9
        emit({"kind": "buckets", "bucket_mb": mb, "n_buckets": len(buckets), "wire_bytes": wire,
              "ms": round(t * 1e3, 3), "algbw_GBs": round(algbw, 1),
              "busbw_GBs": round(algbw * 2 * (world - 1) / world, 1)})
        fe.shutdown()
    if a.json and rank == 0:
        json.dump(out, open(a.json, "w"), indent=1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
