"""A/B of the stem max-pool kernels (knob `pool`, csrc/kernels/eltwise.hip g_pool_variant) on the ResNet-50 shape, batch 1024 @ 112x112x64.

    python bench/pool.py [--batch 1024] [--json out.json]
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


def timeit(fn, iters=10):
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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    N = require_native()
    dev = "cuda"
    B, H, C = a.batch, 112, 64
    Ho = (H - 1) // 2 + 1
    x = torch.relu(torch.randn(B, H, H, C, device=dev)).to(torch.bfloat16)
    y = torch.empty(B, Ho, Ho, C, dtype=torch.bfloat16, device=dev)
    idx = torch.empty(B, Ho, Ho, C, dtype=torch.uint8, device=dev)
    bits = torch.empty(B, Ho, Ho, C // 8, dtype=torch.uint8, device=dev)
    gy = torch.randn(B, Ho, Ho, C, device=dev).to(torch.bfloat16)
    gx = torch.empty_like(x)
    res = {}
    outs = {}
    for v in (1, 0, 2, 3, 4):
        N.set_variant("pool", v)
        rows = N.maxpool_bwd_partial_rows(B, H, H, C)
        part = torch.empty(rows * C, device=dev)
        tf, tb = [], []
        for _ in range(a.rounds):
            tf.append(timeit(lambda: N.maxpool_fwd(x, y, idx, bits)))
            tb.append(timeit(lambda: N.maxpool_bwd(gy, idx, None, gx, part)))
        outs[v] = (y.clone(), idx.clone(), gx.clone())
        fb = x.numel() * 2 + y.numel() * 2 + idx.numel() + bits.numel()
        bb = gy.numel() * 2 + idx.numel() + gx.numel() * 2
        f, b = statistics.median(tf), statistics.median(tb)
        res[f"v{v}"] = {"fwd_us": round(f, 1), "fwd_GBps": round(fb / f / 1e3), "bwd_us": round(b, 1),
                        "bwd_GBps": round(bb / b / 1e3)}
        print(json.dumps({"variant": v, **res[f"v{v}"]}), flush=True)
    N.set_variant("pool", 0)
    for cap in (1024, 2048, 4096, 8192, 16384):   # grid cap sweep of the default kernels
        N.set_variant("pool_blocks", cap)
        rows = N.maxpool_bwd_partial_rows(B, H, H, C)
        part = torch.empty(rows * C, device=dev)
        f = statistics.median(timeit(lambda: N.maxpool_fwd(x, y, idx, bits)) for _ in range(a.rounds))
        b = statistics.median(timeit(lambda: N.maxpool_bwd(gy, idx, None, gx, part)) for _ in range(a.rounds))
        res[f"blocks{cap}"] = {"fwd_us": round(f, 1), "bwd_us": round(b, 1)}
        print(json.dumps({"blocks": cap, **res[f"blocks{cap}"]}), flush=True)
    N.set_variant("pool_blocks", 8192)
    N.set_variant("pool", 4)
    same = all(torch.equal(p, q) for v in (0, 2, 3, 4) for p, q in zip(outs[v], outs[1]))
    res["bitwise_equal"] = same
    print(json.dumps({"bitwise_equal": same}), flush=True)
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
