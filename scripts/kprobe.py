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
    ap.add_argument("--op", choices=["wgrad", "fwd", "fwdres", "dgrad_add", "bwd1x1"], default="wgrad")
    ap.add_argument("--shape", default="1024,14,256,256,3,1,1", help="N,H,Cin,Cout,R,stride,pad")
    ap.add_argument("--set", default="", help="knobs, e.g. wgrad8=1,igemm8=2")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--drop", default="", help="dgrad_add: comma list of fused operands to leave out "
                    "(bits, add, colsum) to price each one")
    a = ap.parse_args()
    N = require_native()
    N.allow_knob_changes(True)   # (A/B of tile knobs between launches)
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
    res = torch.randn(n, ho, ho, co, device=dev).to(torch.bfloat16)
    # dgrad of a 1x1 conv c -> co as the engine runs it (c1 of a bottleneck): g [n,ho,ho,co] ->
    # dx [n,h,h,c] with the residual-gradient add, ReLU bitmask and fused column sums
    gd = torch.randn(n, ho, ho, co, device=dev).to(torch.bfloat16)
    wdt = (torch.randn(c, co, device=dev) * 0.05).to(torch.bfloat16)
    add = torch.randn(n, h, h, c, device=dev).to(torch.bfloat16)
    bits = torch.randint(0, 255, (n, h, h, c // 8), dtype=torch.uint8, device=dev)
    dx = torch.empty(n, h, h, c, dtype=torch.bfloat16, device=dev)
    part = torch.empty(N.igemm_partial_rows(n * h * h, c, co) * c, device=dev) if a.op == "dgrad_add" else None

    if a.op == "bwd1x1":   # fused conv3 backward (bwd1x1.hip): shape N,H,CI,CO (1x1, stride 1)
        gb = torch.randn(n, h, h, co, device=dev).to(torch.bfloat16)
        wdb = (torch.randn(c, co, device=dev) * 0.05).to(torch.bfloat16)
        outb = torch.empty(n, h, h, c, dtype=torch.bfloat16, device=dev)
        partb = torch.empty(N.bwd1x1_partial_rows(n * h * h, co, c) * c, device=dev)
        dwb = torch.zeros(co, c, device=dev)

    def step():
        if a.op == "bwd1x1":
            N.bwd1x1(gb, x, wdb, bits, outb, partb, dwb)
        elif a.op == "wgrad":
            N.wgrad(x, h, h, r, r, st, pad, ho, ho, g, None, 0, dw, r * r * c, 0)
        elif a.op == "fwd":
            N.igemm(x, None, h, h, r, r, st, pad, ho, ho, w, 0, sc, sh, None, None, None, y, 1, None, 0, 0, 0, 0, 0,
                    None, None)
        elif a.op == "fwdres":
            N.igemm(x, None, h, h, r, r, st, pad, ho, ho, w, 0, sc, sh, res, None, None, y, 1, None, 0, 0, 0, 0, 0,
                    None, None)
        else:
            drop = a.drop.split(",")
            N.igemm(gd, None, h, h, 1, 1, 1, 0, h, h, wdt, 1, None, None, None, None if "bits" in drop else bits,
                    None if "add" in drop else add, dx, 0, None, 0, 0, 0, 0, 0, None if "colsum" in drop else part,
                    None)
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
    flops = 2.0 * n * ho * ho * co * r * r * c * (2 if a.op == "bwd1x1" else 1)
    print(json.dumps({"op": a.op, "shape": a.shape, "set": a.set, "drop": a.drop, "us": round(us, 1),
                      "tflops": round(flops / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
