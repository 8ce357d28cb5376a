#!/usr/bin/env python3
"""Scaling curve of one strategy: bench.py at --gpus 1, 2, 4, 8 (those the node has), each a
fresh child process launched before this process touches any GPU, then per-N images/sec and
the weak-scaling efficiency ips(N) / (N * ips(1)) (the
reference's only timing is imagenet-resnet50-hvd.py:119-126).

    python bench/scaling.py                              # horovod-style, N = 1,2,4,8 <= visible
    python bench/scaling.py --strategy mirrored --gpus 1 2 4 8 --steps 20 --warmup 5
    python bench/scaling.py --strategy multiworker --local-gpus 4 --gpus 4 8
    python bench/scaling.py --strategy ps --gpus 2 4 8 --baseline-ips 30000
    python bench/scaling.py --out gpurun_out/scaling.json -- --batch 256 --crop 244

Launch per N: horovod / multiworker with N > 1 under torch.distributed.run (one rank per GPU,
or per --local-gpus GPUs), mirrored as ONE process driving N GPUs, ps as bench.py's own P + W
role processes; N = 1 is plain `bench.py`.  Arguments after `--` go to every bench.py run.
Without an N = 1 row (and no --baseline-ips) efficiencies are left empty.  Prints the table and
one JSON summary line; --out also writes the summary (with every run's bench JSON).
"""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pddl.utils.scaling import format_table, scaling_table  # noqa: E402


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def command(strategy, n, steps, warmup, local_gpus, extra):
    """argv of the bench.py run for N GPUs."""
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup),
             "--strategy", strategy] + list(extra)
    if strategy in ("horovod", "multiworker") and n > 1:
        per = local_gpus if strategy == "multiworker" else 1
        if n % per:
            raise ValueError(f"--gpus {n} is not a multiple of --local-gpus {per}")
        if strategy == "multiworker":
            bench += ["--local-gpus", str(per)]
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n // per}",
                "--master-addr", "127.0.0.1", f"--master-port={free_port()}"] + bench
    return [sys.executable] + bench


def parse_bench_json(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    if len(lines) != 1:
        raise ValueError(f"expected one bench JSON line, got {len(lines)}")
    return json.loads(lines[0])


def visible_gpus() -> int:
    import torch   # (device_count() does not initialise the GPU on this image)
    return torch.cuda.device_count()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", default="horovod", choices=["horovod", "mirrored", "multiworker", "ps"])
    ap.add_argument("--gpus", type=int, nargs="+", default=None, help="GPU counts (default 1 2 4 8 <= visible)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--local-gpus", type=int, default=1)
    ap.add_argument("--baseline-ips", type=float, default=None, help="1-GPU rate (default: the N = 1 run)")
    ap.add_argument("--timeout", type=float, default=1200.0, help="per-run limit in seconds")
    ap.add_argument("--out", default=None)
    ap.add_argument("--dry-run", action="store_true", help="print the commands only")
    a = ap.parse_args(argv)
    ns = a.gpus
    if ns is None:
        have = visible_gpus()
        ns = [n for n in (1, 2, 4, 8) if n <= have] or [1]
    runs, rows = {}, {}
    for n in ns:
        cmd = command(a.strategy, n, a.steps, a.warmup, a.local_gpus, extra)
        print("$ " + " ".join(cmd), flush=True)
        if a.dry_run:
            continue
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout)
        if r.returncode != 0:
            sys.stderr.write(r.stderr[-4000:])
            print(f"N={n}: bench.py exited {r.returncode}; stopping", flush=True)
            break
        out = parse_bench_json(r.stdout)
        runs[n] = out
        rows[n] = float(out["value"])
        print(f"N={n}: {rows[n]:.1f} images/sec ({out['ms_per_step']} ms/step)", flush=True)
    if a.dry_run:
        return 0
    table = scaling_table(rows, a.baseline_ips)
    print(format_table(table))
    summary = {"metric": "images/sec ResNet-50/ImageNet at 1/2/4/8 MI355X + scaling efficiency",
               "strategy": a.strategy, "scaling": "weak", "baseline_ips": a.baseline_ips or rows.get(1),
               "rows": table, "bench_args": extra}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({**summary, "runs": {str(k): v for k, v in runs.items()}}, f, indent=1)
    return 0 if len(rows) == len(ns) else 1


if __name__ == "__main__":
    sys.exit(main())
