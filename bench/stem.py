"""A/B of the fused stem forward (stem.hip, knob `stem_pool`) on the ResNet-50 stem shape."""
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
    a = ap.parse_args()
    N = require_native()
    B, H1 = a.batch, a.crop // 2
    Hs, H2 = H1 + 3, H1 // 2
    x2 = torch.randn(B, Hs, Hs, 16, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 256, device="cuda") * 0.05).to(torch.bfloat16)
    sc, sh = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.1
    outs = {}
    for v in (0, 1):
        N.set_variant("stem_pool", v)
        pool = torch.empty(B, H2, H2, 64, dtype=torch.bfloat16, device="cuda")
        idx = torch.empty(B, H2, H2, 64, dtype=torch.uint8, device="cuda")
        bits = torch.empty(B, H2, H2, 8, dtype=torch.uint8, device="cuda")
        fn = lambda: N.stem_pool_fwd(x2, w, sc, sh, pool, idx, bits)  # noqa: E731
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        flop = 2.0 * B * H1 * H1 * 64 * 256
        print(f"stem_pool variant {v}: {us:8.1f} us  {flop / us / 1e6:6.1f} TF/s")
        outs[v] = (pool.clone(), idx.clone(), bits.clone())
    N.set_variant("stem_pool", 1)
    print("variant outputs equal:", all(torch.equal(a_, b_) for a_, b_ in zip(outs[0], outs[1])))


if __name__ == "__main__":
    main()
