"""Fused stem forward (stem.hip: conv1 + BN + ReLU + max-pool in one launch) against the unfused
igemm conv1 + max-pool pair on the ResNet-50 stem shape: time and bitwise equality."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pddl.ops.native import require_native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2560)
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--fwd-only", action="store_true")
    a = ap.parse_args()
    N = require_native()
    B, H1 = a.batch, a.crop // 2
    Hs, H2 = H1 + 3, H1 // 2
    x2 = torch.randn(B, Hs, Hs, 16, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 256, device="cuda") * 0.05).to(torch.bfloat16)
    sc, sh = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.1
    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3
    flop = 2.0 * B * H1 * H1 * 64 * 256
    pool = torch.empty(B, H2, H2, 64, dtype=torch.bfloat16, device="cuda")
    idx = torch.empty(B, H2, H2, 64, dtype=torch.uint8, device="cuda")
    bits = torch.empty(B, H2, H2, 8, dtype=torch.uint8, device="cuda")
    us = timed(lambda: N.stem_pool_fwd(x2, w, sc, sh, pool, idx, bits))
    print(f"fused stem conv + pool: {us:8.1f} us  {flop / us / 1e6:6.1f} TF/s")
    # the unfused pair: conv1 (igemm, 4x4 window over the s2d input) + max-pool
    c1 = torch.empty(B, H1, H1, 64, dtype=torch.bfloat16, device="cuda")
    pool2, idx2, bits2 = torch.empty_like(pool), torch.empty_like(idx), torch.empty_like(bits)

    def unfused():
        N.igemm(x2, None, Hs, Hs, 4, 4, 1, 0, H1, H1, w, 0, sc, sh, None, None, None, c1, 1, None, 0, 0, 0, 0, 0,
                None, None)
        N.maxpool_fwd(c1, pool2, idx2, bits2)
    us2 = timed(unfused)
    print(f"igemm conv1 + maxpool:  {us2:8.1f} us  {flop / us2 / 1e6:6.1f} TF/s")
    print("outputs equal:", torch.equal(pool, pool2) and torch.equal(idx, idx2) and torch.equal(bits, bits2))
    # fused backward: max-pool routing + conv1 weight gradient (+ per-channel sums)
    gpool = torch.randn(B, H2, H2, 64, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(64, 256, device="cuda")
    rows = N.stem_pool_bwd_partial_rows(B, H2)
    cs = torch.empty(rows * 64, device="cuda")
    us3 = timed(lambda: N.stem_pool_bwd(x2, gpool, idx, dw, cs))
    print(f"fused stem pool bwd + conv1 wgrad: {us3:8.1f} us  {flop / us3 / 1e6:6.1f} TF/s")

if __name__ == "__main__":
    main()
