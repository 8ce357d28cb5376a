"""Kernel micro-benchmark: A/B pipeline variants of the implicit-GEMM kernels on the
ResNet-50 shapes (batch 256 @224), interleaved in one process (cdna_hip_programming §5.4 r24).

    python bench/kernels.py [--batch 256] [--json out.json]
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

FWD = [  # name, H, C, Cout, R, stride, pad
    ("s2.c2 3x3 64", 56, 64, 64, 3, 1, 1), ("s3.c2 3x3 128", 28, 128, 128, 3, 1, 1),
    ("s4.c2 3x3 256", 14, 256, 256, 3, 1, 1), ("s5.c2 3x3 512", 7, 512, 512, 3, 1, 1),
    ("s4.c1 1x1 1024>256", 14, 1024, 256, 1, 1, 0), ("s5.c1 1x1 2048>512", 7, 2048, 512, 1, 1, 0),
    ("s3.c1 1x1 512>128", 28, 512, 128, 1, 1, 0), ("s4.c3 1x1 256>1024", 14, 256, 1024, 1, 1, 0),
]


def timeit(fn, iters=10):
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--knob", default="igemm8", help="igemm knob to A/B (igemm8, igemm, igemm_pf, igemm_pk, ...)")
    ap.add_argument("--variants", default="0,2", help="comma-separated knob values")
    ap.add_argument("--wgrad-knob", default="wgrad8", help="wgrad knob to A/B")
    ap.add_argument("--wgrad-variants", default="0,2", help="comma-separated wgrad knob values")
    ap.add_argument("--skip-lib", action="store_true", help="skip the MIOpen / hipBLASLt yardsticks")
    ap.add_argument("--set", default="", help="extra knobs for every variant, e.g. igemm8_min_tiles=1")
    a = ap.parse_args()
    N = require_native()
    N.allow_knob_changes(True)   # (A/B of tile knobs between launches)
    for kv in filter(None, a.set.split(",")):
        k, v = kv.split("=")
        N.set_variant(k, int(v))
    B = a.batch
    dev = "cuda"
    res = []
    for name, H, C, Co, R, st, pad in FWD:
        Ho = (H + 2 * pad - R) // st + 1
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, R * R * C, device=dev) * 0.05).to(torch.bfloat16)
        sc, sh = torch.ones(Co, device=dev), torch.zeros(Co, device=dev)
        y = torch.empty(B, Ho, Ho, Co, dtype=torch.bfloat16, device=dev)
        g = torch.randn(B, Ho, Ho, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, R * R * C, device=dev)
        flops = 2.0 * B * Ho * Ho * Co * R * R * C

        def fwd():
            N.igemm(x, None, H, H, R, R, st, pad, Ho, Ho, w, 0, sc, sh, None, None, None, y, 1, None, 0, 0, 0, 0, 0,
                    None, None)

        def wg():
            N.wgrad(x, H, H, R, R, st, pad, Ho, Ho, g, None, 0, dw, R * R * C, 0)
        # MIOpen (PyTorch conv, bf16 channels_last) on the same shapes: a same-device yardstick
        xt = x.permute(0, 3, 1, 2)
        wt = w.view(Co, R, R, C).permute(0, 3, 1, 2)
        gt = g.permute(0, 3, 1, 2)

        def mi_fwd():
            torch.nn.functional.conv2d(xt, wt, stride=st, padding=pad)

        def mi_wg():
            torch.ops.aten.convolution_backward(gt, xt, wt, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                                [False, True, False])
        if not a.skip_lib:
            mrow = {"layer": name, "kernel": "miopen", "fwd_us": round(timeit(mi_fwd), 1),
                    "wgrad_us": round(timeit(mi_wg), 1)}
            print(json.dumps(mrow), flush=True)
            res.append(mrow)
        # hipBLASLt on the same-FLOP plain GEMMs (im2col'd A already in memory, no epilogue):
        # the library ceiling for these M / N / K
        M, K = B * Ho * Ho, R * R * C
        if a.skip_lib:
            M = 0
        am = torch.randn(M, K, device=dev).to(torch.bfloat16)
        bm = (torch.randn(K, Co, device=dev) * 0.05).to(torch.bfloat16)
        gm = torch.randn(M, Co, device=dev).to(torch.bfloat16)
        if not a.skip_lib:
            f_us, w_us = timeit(lambda: torch.mm(am, bm)), timeit(lambda: torch.mm(gm.t(), am))
            brow = {"layer": name, "kernel": "hipblaslt", "fwd_us": round(f_us, 1),
                    "fwd_tflops": round(flops / f_us / 1e6, 1), "wgrad_us": round(w_us, 1),
                    "wgrad_tflops": round(flops / w_us / 1e6, 1)}
            print(json.dumps(brow), flush=True)
            res.append(brow)
        del am, bm, gm
        for kind, fn, knob, variants in (("igemm", fwd, a.knob, [int(v) for v in a.variants.split(",")]),
                                          ("wgrad", wg, a.wgrad_knob,
                                           [int(v) for v in a.wgrad_variants.split(",")])):
            t = {v: [] for v in variants}
            for _ in range(a.rounds):
                for v in variants:
                    N.set_variant(knob, v)
                    t[v].append(timeit(fn))
            N.set_variant(knob, 0)
            row = {"layer": name, "kernel": kind}
            for v in variants:
                us = statistics.median(t[v])
                row[f"v{v}_us"] = round(us, 1)
                row[f"v{v}_tflops"] = round(flops / us / 1e6, 1)
            res.append(row)
            print(json.dumps(row), flush=True)
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
