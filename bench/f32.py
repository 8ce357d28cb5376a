"""fp32 convolution kernel micro-benchmark over every ResNet-50 conv shape (batch 256 @224).

Times conv_f32 (forward, and the data gradient as the forward conv the fp32 engine issues) and
wgrad_f32 for each layer shape under the conv_f32 kernel variants, weighting each shape by the
number of layers that have it, so the totals are one training step's fp32 conv time.

    python bench/f32.py [--batch 256] [--variants 0,2]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import pddl  # noqa: E402,F401
from pddl.ops.native import require_native  # noqa: E402

# name, H_in, C, Cout, R, stride, pad, count (Keras ResNet50 v1: the stride sits on conv1 / the shortcut)
LAYERS = [
    ("s2.c1a 64>64", 56, 64, 64, 1, 1, 0, 1), ("s2.c1 256>64", 56, 256, 64, 1, 1, 0, 2),
    ("s2.c2 3x3 64", 56, 64, 64, 3, 1, 1, 3), ("s2.c3 64>256", 56, 64, 256, 1, 1, 0, 4),
    ("s3.c1a 256>128 s2", 56, 256, 128, 1, 2, 0, 1), ("s3.c1 512>128", 28, 512, 128, 1, 1, 0, 3),
    ("s3.c2 3x3 128", 28, 128, 128, 3, 1, 1, 4), ("s3.c3 128>512", 28, 128, 512, 1, 1, 0, 4),
    ("s3.c0 256>512 s2", 56, 256, 512, 1, 2, 0, 1),
    ("s4.c1a 512>256 s2", 28, 512, 256, 1, 2, 0, 1), ("s4.c1 1024>256", 14, 1024, 256, 1, 1, 0, 5),
    ("s4.c2 3x3 256", 14, 256, 256, 3, 1, 1, 6), ("s4.c3 256>1024", 14, 256, 1024, 1, 1, 0, 6),
    ("s4.c0 512>1024 s2", 28, 512, 1024, 1, 2, 0, 1),
    ("s5.c1a 1024>512 s2", 14, 1024, 512, 1, 2, 0, 1), ("s5.c1 2048>512", 7, 2048, 512, 1, 1, 0, 2),
    ("s5.c2 3x3 512", 7, 512, 512, 3, 1, 1, 3), ("s5.c3 512>2048", 7, 512, 2048, 1, 1, 0, 3),
    ("s5.c0 1024>2048 s2", 14, 1024, 2048, 1, 2, 0, 1),
]


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--knob", default="conv_f32")
    ap.add_argument("--only", default="", help="comma-separated layer-name prefixes (e.g. for a counter pass)")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    N = require_native()
    N.allow_knob_changes(True)   # (A/B of tile knobs between launches)
    B, dev = a.batch, "cuda"
    variants = [int(v) for v in a.variants.split(",")]
    tot = {(v, k): 0.0 for v in variants for k in ("fwd", "dgrad", "wgrad")}
    best = {k: 0.0 for k in ("fwd", "dgrad", "wgrad")}
    print(f"{'layer':22s} {'op':6s} " + " ".join(f"{'v' + str(v) + ' us':>10s} {'TF/s':>6s}" for v in variants))
    only = [o for o in a.only.split(",") if o]
    for name, H, C, Co, R, st, pad, cnt in LAYERS:
        if only and not any(name.startswith(o) for o in only):
            continue
        Ho = (H + 2 * pad - R) // st + 1
        x = torch.randn(B, H, H, C, device=dev)
        w = torch.randn(Co, R * R * C, device=dev) * 0.05
        y = torch.empty(B, Ho, Ho, Co, device=dev)
        gy = torch.randn(B, Ho, Ho, Co, device=dev)
        wt = torch.randn(C, R * R * Co, device=dev) * 0.05
        dx = torch.empty(B, Ho, Ho, C, device=dev)   # (stride 2: the compact dgrad grid, scattered after)
        dw = torch.zeros(Co, R * R * C, device=dev)
        fl = 2.0 * B * Ho * Ho * Co * R * R * C
        ops = {
            "fwd": lambda: N.conv_f32(x, R, R, st, pad, w, None, y),
            "dgrad": (lambda: N.conv_f32(gy, R, R, 1, R - 1 - pad, wt, None, dx)) if st == 1 else
                     (lambda: N.conv_f32(gy, 1, 1, 1, 0, wt, None, dx)),
            "wgrad": lambda: N.wgrad_f32(x, R, R, st, pad, gy, dw),
        }
        for op, fn in ops.items():
            if op not in a.ops.split(","):
                continue
            row = []
            for v in variants:
                N.set_variant(a.knob, v)
                t = timeit(fn, a.iters)
                tot[(v, op)] += t * cnt
                row.append(t)
            best[op] += min(row) * cnt
            print(f"{name:22s} {op:6s} " + " ".join(f"{t:10.1f} {fl / t / 1e6:6.1f}" for t in row), flush=True)
        del x, w, y, gy, wt, dx, dw
    N.set_variant(a.knob, 1)
    for op in ("fwd", "dgrad", "wgrad"):
        print(f"total {op:6s} " + " ".join(f"v{v} {tot[(v, op)] / 1e3:7.2f} ms" for v in variants)
              + f"   best-of {best[op] / 1e3:7.2f} ms")
    print("total all    " + " ".join(f"v{v} {sum(tot[(v, k)] for k in ('fwd', 'dgrad', 'wgrad')) / 1e3:7.2f} ms"
                                     for v in variants) + f"   best-of {sum(best.values()) / 1e3:7.2f} ms")


if __name__ == "__main__":
    main()
