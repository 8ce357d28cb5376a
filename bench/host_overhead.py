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


class _StubComm:
    """Stand-in for the native RCCL communicator of a Mirrored job: the host issues exactly the
    calls of the graphed step (one grouped all-reduce per bucket over the R comm streams), which
    return at once -- so what is timed is the driver's own host loop, not RCCL."""
    calls = 0

    def all_reduce_on(self, bufs, op, streams, tag):
        assert len(bufs) == len(streams)
        _StubComm.calls += 1

    def check(self):
        pass


def measure_replicas(R: int, B: int, steps: int):
    """R segmented replicas of the in-process Mirrored design, all on device 0 (the host loop of
    _LocalReplicas._graphed_step for an R-GPU node: per replica the input load, nb segment
    replays, nb event records + comm-stream waits, nb grouped collective calls, the optimizer
    graph), with the stub communicator.  host_ms: wall time of one step() call (the enqueue)."""
    from pddl.config import make_config
    from pddl.parallel.strategies import _LocalReplicas
    cfg = make_config("mirrored", device="cuda", batch_size=B, crop=224, image_size=224, save=False, verbose=0,
                      data="synthetic_fixed")
    lr = _LocalReplicas(cfg, [0] * R)
    lr.comm = _StubComm()
    lr.graph_mode = True
    lr.launch_streams = [torch.cuda.Stream() for _ in range(R)]   # one per replica, as on R devices
    eng = os.environ.get("PDDL_ENGINE", "")
    g = torch.Generator(device="cuda").manual_seed(0)
    images = [torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(R)]
    labels = [torch.randint(0, 1000, (B,), dtype=torch.int64, device="cuda", generator=g) for _ in range(R)]
    for _ in range(3):
        lr.step(images, labels, B * R)
    torch.cuda.synchronize()
    host = []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lr.step(images, labels, B * R)
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    if os.environ.get("HOST_PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        for _ in range(10):
            torch.cuda.synchronize()
            pr.enable()
            lr.step(images, labels, B * R)
            pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    host.sort()
    nb = len(lr.buckets)
    return {"mode": "graphed, stub communicator", "PDDL_ENGINE": eng,
            "two_stream": lr.replicas[0][0].side is not None, "replicas": R, "batch_per_replica": B, "buckets": nb,
            "host_ms": round(host[len(host) // 2] * 1e3, 3), "host_ms_min": round(host[0] * 1e3, 3),
            "graph_launches_per_step": R * (nb + 1), "collective_calls_per_step": nb}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--replicas", type=int, default=0,
                    help="> 0: only the R-replica host-loop rehearsal on device 0 (stub communicator)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    if a.replicas > 0:
        rows = [measure_replicas(a.replicas, a.batch, a.steps)]
    else:
        rows = [measure(False, a.batch, a.steps), measure(True, a.batch, a.steps)]
    for r in rows:
        print(json.dumps(r), flush=True)
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
