"""A/B of the igemm epilogue-operand prefetch (knob igemm_pf) on the epilogue-bound ResNet-50
layers: conv*_3 forward (+ residual) and identity-block conv*_1 dgrad (+ residual gradient,
ReLU bitmask).  Interleaved in one process; also checks both variants give identical bits.

    python bench/epilogue.py [--batch 1024] [--json out.json]
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

STAGES = [("conv2", 56, 64), ("conv3", 28, 128), ("conv4", 14, 256), ("conv5", 7, 512)]


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    N = require_native()
    N.allow_knob_changes(True)   # (A/B of tile knobs between launches)
    B, dev = a.batch, "cuda"
    out = []
    for name, H, f in STAGES:
        M = B * H * H
        y2 = torch.randn(B, H, H, f, device=dev).to(torch.bfloat16)
        w3 = (torch.randn(4 * f, f, device=dev) * 0.05).to(torch.bfloat16)
        res = torch.randn(B, H, H, 4 * f, device=dev).to(torch.bfloat16)
        o = torch.empty(B, H, H, 4 * f, dtype=torch.bfloat16, device=dev)
        bits = torch.empty(B, H, H, f // 2, dtype=torch.uint8, device=dev)
        sc, sh = torch.ones(4 * f, device=dev), torch.zeros(4 * f, device=dev)
        g1 = torch.randn(B, H, H, f, device=dev).to(torch.bfloat16)
        wd = (torch.randn(4 * f, f, device=dev) * 0.05).to(torch.bfloat16)   # dgrad weights [cin = 4f][f]
        gout = torch.randn(B, H, H, 4 * f, device=dev).to(torch.bfloat16)
        gx = torch.empty(B, H, H, 4 * f, dtype=torch.bfloat16, device=dev)
        mbits = torch.randint(0, 256, (B, H, H, f // 2), dtype=torch.uint8, device=dev)

        def c3_fwd():
            N.igemm(y2, None, H, H, 1, 1, 1, 0, H, H, w3, 0, sc, sh, res, None, None, o, 1, None, 0, 0, 0, 0, 0,
                    None, bits)

        def c1_dgrad():
            N.igemm(g1, None, H, H, 1, 1, 1, 0, H, H, wd, 1, None, None, None, mbits, gout, gx, 0, None, 0, 0, 0, 0,
                    0, None, None)
        nbytes = (M * f + 2 * M * 4 * f) * 2 + M * f // 2
        for kind, fn in (("c3 fwd +res", c3_fwd), ("c1 dgrad +add", c1_dgrad)):
            t = {0: [], 1: []}
            for _ in range(a.rounds):
                for v in (0, 1):
                    N.set_variant("igemm_pf", v)
                    t[v].append(timeit(fn))
            row = {"layer": f"{name} {kind}", "M": M, "N": 4 * f, "K": f}
            for v in (0, 1):
                us = statistics.median(t[v])
                row[f"pf{v}_us"] = round(us, 1)
                row[f"pf{v}_TBps"] = round(nbytes / us / 1e6, 2)
            print(json.dumps(row), flush=True)
            out.append(row)
        N.set_variant("igemm_pf", 0)
        c3_fwd(); c1_dgrad()
        r0 = (o.clone(), gx.clone(), bits.clone())
        N.set_variant("igemm_pf", 1)
        c3_fwd(); c1_dgrad()
        assert torch.equal(r0[0], o) and torch.equal(r0[1], gx) and torch.equal(r0[2], bits), "prefetch changed results"
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
