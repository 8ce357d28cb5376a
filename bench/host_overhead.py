"""Host enqueue cost of one replica step vs its GPU time (the Mirrored driver's budget).

    python bench/host_overhead.py [--batch 32] [--steps 30]

MirroredStrategy (imagenet-resnet50-mirror.py:21,54) drives every local GPU from ONE process:
per step the host enqueues R replica steps, so the driver keeps up with the GPUs only while
R x (host enqueue per replica step) < GPU step time.  At the reference's 32 images per replica
the GPU step is a few ms, so an eager step (~180 kernel launches through Python) is the risk.
Measured here on one GPU through the real strategy code (MirroredStrategy over RCCL with one
device), eager (--no-graphs: replica threads, per-kernel launches) and graphed (default:
segmented HIP graphs, grouped bucket all-reduces between segments):
  host_ms : wall time of train_step() returning (the enqueue; the GPU runs asynchronously)
  gpu_ms  : steady-state time per step with the queue kept full (synchronised at the end)
and the largest R whose enqueue still hides behind the GPU, R_max = gpu_ms / host_ms.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import pddl  # noqa: E402,F401


def measure(graphs: bool, B: int, steps: int):
    from pddl.config import make_config
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    cfg = make_config("mirrored", device="cuda", batch_size=B, crop=224, image_size=224, graphs=graphs,
                      save=False, verbose=0, data="synthetic_fixed")
    st = make_strategy(cfg)
    st._devices = [0]
    Trainer(cfg, st)
    st.broadcast_state(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    images = [torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda", generator=g)]
    labels = [torch.randint(0, 1000, (B,), dtype=torch.int64, device="cuda", generator=g)]
    for _ in range(5):
        st.train_step(images, labels)
    torch.cuda.synchronize()
    host = []
    for _ in range(steps):          # enqueue cost: the call returns before the GPU finishes
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.train_step(images, labels)
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):          # GPU time with the queue kept full
        st.train_step(images, labels)
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / steps
    host.sort()
    h = host[len(host) // 2]
    return {"mode": "graphed" if graphs else "eager", "batch_per_replica": B, "host_ms": round(h * 1e3, 3),
            "gpu_ms": round(gpu * 1e3, 3), "replicas_hidden": round(gpu / h, 1),
            "hip_graph": st.mirror.graph_mode}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = [measure(False, a.batch, a.steps), measure(True, a.batch, a.steps)]
    for r in rows:
        print(json.dumps(r), flush=True)
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
