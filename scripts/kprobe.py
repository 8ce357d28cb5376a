"""Run one hand-written kernel on one shape in a loop, for rocprofv3 counter passes and
quick A/B timing (bench/kernels.py sweeps the ResNet-50 layers; this isolates one).

    python scripts/kprobe.py --op wgrad --shape 1024,14,256,256,3,1,1 --set wgrad8=1 --iters 50
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pddl.ops.native import require_native   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", choices=["wgrad", "fwd"], default="wgrad")
    ap.add_argument("--shape", default="1024,14,256,256,3,1,1", help="N,H,Cin,Cout,R,stride,pad")
    ap.add_argument("--set", default="", help="knobs, e.g. wgrad8=1,igemm8=2")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    N = require_native()
    for kv in filter(None, a.set.split(",")):
        k, v = kv.split("=")
        N.set_variant(k, int(v))
    n, h, c, co, r, st, pad = (int(v) for v in a.shape.split(","))
    ho = (h + 2 * pad - r) // st + 1
    dev = "cuda"
    x = torch.randn(n, h, h, c, device=dev).to(torch.bfloat16)
    g = torch.randn(n, ho, ho, co, device=dev).to(torch.bfloat16)
    w = (torch.randn(co, r * r * c, device=dev) * 0.05).to(torch.bfloat16)
    dw = torch.zeros(co, r * r * c, device=dev)
    y = torch.empty(n, ho, ho, co, dtype=torch.bfloat16, device=dev)
    sc, sh = torch.ones(co, device=dev), torch.zeros(co, device=dev)

    def step():
        if a.op == "wgrad":
            N.wgrad(x, h, h, r, r, st, pad, ho, ho, g, None, 0, dw, r * r * c, 0)
        else:
            N.igemm(x, None, h, h, r, r, st, pad, ho, ho, w, 0, sc, sh, None, None, None, y, 1, None, 0, 0, 0, 0, 0,
                    None, None)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        step()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    flops = 2.0 * n * ho * ho * co * r * r * c
    print(json.dumps({"op": a.op, "shape": a.shape, "set": a.set, "us": round(us, 1),
                      "tflops": round(flops / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
