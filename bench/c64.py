"""A/B of the stage-2 3x3 conv kernels (conv3x3c64.hip row tiles vs the generic implicit
GEMM / wgrad) on the ResNet-50 conv2_block*_2 shape: N x 56 x 56 x 64 -> 64.

    python bench/c64.py [--batch 2560] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pddl.ops.native import require_native  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2560)
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N = require_native()
    n, h = a.batch, a.hw
    M = n * h * h
    x = torch.randn(n, h, h, 64, device="cuda").to(torch.bfloat16)
    g = torch.randn(n, h, h, 64, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 576, device="cuda") * 0.05).to(torch.bfloat16)
    sc, sh = torch.ones(64, device="cuda"), torch.zeros(64, device="cuda")
    out = torch.empty_like(x)
    bits = torch.zeros(n, h, h, 8, dtype=torch.uint8, device="cuda")
    mb = torch.randint(0, 255, (n, h, h, 8), dtype=torch.uint8, device="cuda")
    part = torch.empty(max(N.conv3x3c64_partial_rows(M), N.igemm_partial_rows(M, 64, 576)) * 64, device="cuda")
    dw = torch.zeros(64, 576, device="cuda")
    flop = 2.0 * M * 576 * 64
    res = {}
    res["fwd_row"] = timeit(lambda: N.conv3x3c64(x, w, 0, out, scale=sc, shift=sh, bits=bits), a.iters)
    res["fwd_igemm"] = timeit(lambda: N.igemm(x, None, h, h, 3, 3, 1, 1, h, h, w, 0, sc, sh, None, None, None, out, 1,
                                              None, 0, 0, 0, 0, 0, None, bits), a.iters)
    res["dgrad_row"] = timeit(lambda: N.conv3x3c64(g, w, 1, out, bits=mb, colsum=part), a.iters)
    res["dgrad_igemm"] = timeit(lambda: N.igemm(g, None, h, h, 3, 3, 1, 1, h, h, w, 1, None, None, None, mb, None, out,
                                                0, None, 0, 0, 0, 0, 0, part, None), a.iters)
    res["wgrad_row"] = timeit(lambda: N.conv3x3c64_wgrad(x, g, dw), a.iters)
    res["wgrad_generic"] = timeit(lambda: N.wgrad(x, h, h, 3, 3, 1, 1, h, h, g, None, 0, dw, 576, 0), a.iters)
    for k, v in res.items():
        print(f"{k:14s} {v:8.1f} us  {flop / v / 1e6:7.1f} TF/s  {2 * M * 128 / v / 1e3:6.0f} GB/s (2 tensors)")
    print(json.dumps({"batch": n, "hw": h, "us": res}))


if __name__ == "__main__":
    main()
