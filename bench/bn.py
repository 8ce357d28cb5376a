"""Train-mode BN streaming kernels on the ResNet-50 shapes at batch 256: bn_apply,
bn_bwd_reduce, sweeping the grid caps (knobs bn_apply_blocks, bn_red_blocks; 0 = heuristic);
achieved GB/s.

    python bench/bn.py [--batch 256] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import pddl  # noqa: E402,F401
from pddl.ops.native import require_native  # noqa: E402

SHAPES = [("56x56x64", 56, 64), ("56x56x256", 56, 256), ("28x28x128", 28, 128), ("14x14x256", 14, 256),
          ("14x14x1024", 14, 1024), ("7x7x512", 7, 512), ("7x7x2048", 7, 2048)]


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--caps", default="0,128,256,512,1024,2048")
    ap.add_argument("--apply-caps", default="0,256,512,1024,2048")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    N = require_native()
    N.allow_knob_changes(True)   # (A/B of tile knobs between launches)
    dev = "cuda"
    res = []
    for name, h, c in SHAPES:
        M = a.batch * h * h
        z = torch.randn(M, c, device=dev).to(torch.bfloat16)
        g = torch.randn(M, c, device=dev).to(torch.bfloat16)
        y = torch.empty_like(z)
        bits = torch.empty(M, c // 8, dtype=torch.uint8, device=dev)
        sc, sh = torch.rand(c, device=dev), torch.randn(c, device=dev)
        mean = torch.zeros(c, device=dev)
        sg, sgx = torch.zeros(c, device=dev), torch.zeros(c, device=dev)
        nbytes = z.numel() * 2
        row = {"shape": name, "M": M, "C": c}
        for cap in [int(x) for x in a.apply_caps.split(",")]:
            N.set_variant("bn_apply_blocks", cap)
            us = statistics.median(timeit(lambda: N.bn_apply(z, sc, sh, None, None, None, 1, y, bits))
                                   for _ in range(3))
            row[f"apply_cap{cap}_us"] = round(us, 1)
            row[f"apply_cap{cap}_GBps"] = round((2 * nbytes + bits.numel()) / us / 1e3)
        N.set_variant("bn_apply_blocks", 0)
        for cap in [int(x) for x in a.caps.split(",")]:
            N.set_variant("bn_red_blocks", cap)
            us = statistics.median(timeit(lambda: N.bn_bwd_reduce(g, z, None, mean, None, sg, sgx, None, None))
                                   for _ in range(3))
            row[f"reduce_cap{cap}_us"] = round(us, 1)
            row[f"reduce_cap{cap}_GBps"] = round(2 * nbytes / us / 1e3)
        N.set_variant("bn_red_blocks", 0)
        res.append(row)
        print(json.dumps(row), flush=True)
        del z, g, y
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
