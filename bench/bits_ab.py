"""Does the ReLU-bit side output cost the write-heavy forward layers?  Times the stage-2 fused
projection forward (conv3 + shortcut, K = 64 + 64 -> 256 channels, M = B x 56 x 56) and the
stage-3 residual conv3 forward (K = 128 -> 512, M = B x 28 x 28) with and without `bits_out`,
on the per-tile kernel and (stage 3) the ring kernel, interleaved in one process
(profiles/r4_bits_pkdual.txt).

    python bench/bits_ab.py [--batch 2560]
"""
import argparse
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
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2560)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    N = require_native()
    N.allow_knob_changes(True)   # (A/B of tile knobs between launches)
    dev = "cuda"
    B = a.batch
    bf = dict(dtype=torch.bfloat16, device=dev)
    # stage-2 fused projection: y2 [B,56,56,64] + x [B,56,56,64] -> out [B,56,56,256]
    y2 = torch.randn(B, 56, 56, 64, **bf)
    x = torch.randn(B, 56, 56, 64, **bf)
    w2 = torch.randn(256, 128, **bf) * 0.05
    sc2, sh2 = torch.ones(256, device=dev), torch.randn(256, device=dev)
    out2 = torch.empty(B, 56, 56, 256, **bf)
    bits2 = torch.empty(B, 56, 56, 32, dtype=torch.uint8, device=dev)
    # (an odd-offset view: the rejected packed-store variant fell back to one-byte stores there)
    bits2u = torch.empty(B * 56 * 56 * 32 + 1, dtype=torch.uint8, device=dev)[1:].view(B, 56, 56, 32)
    # stage-3 residual conv3: y2 [B,28,28,128] -> out [B,28,28,512] + residual
    y3 = torch.randn(B, 28, 28, 128, **bf)
    w3 = torch.randn(512, 128, **bf) * 0.05
    sc3, sh3 = torch.ones(512, device=dev), torch.randn(512, device=dev)
    res3 = torch.randn(B, 28, 28, 512, **bf)
    out3 = torch.empty(B, 28, 28, 512, **bf)
    bits3 = torch.empty(B, 28, 28, 64, dtype=torch.uint8, device=dev)
    bits3u = torch.empty(B * 28 * 28 * 64 + 1, dtype=torch.uint8, device=dev)[1:].view(B, 28, 28, 64)

    def proj(bits):
        return lambda: N.igemm(y2, x, 56, 56, 1, 1, 1, 0, 56, 56, w2, 0, sc2, sh2, None, None, None, out2, 1, None,
                               0, 0, 0, 0, 0, None, bits)

    def s3c3(bits):
        return lambda: N.igemm(y3, None, 28, 28, 1, 1, 1, 0, 28, 28, w3, 0, sc3, sh3, res3, None, None, out3, 1,
                               None, 0, 0, 0, 0, 0, None, bits)

    gb2 = B * 56 * 56 * (128 + 256) * 2 / 1e9
    gb3 = B * 28 * 28 * (128 + 512 + 512) * 2 / 1e9
    cases = [("proj s2 bits (4-byte)", proj(bits2), 2, gb2), ("proj s2 bits (1-byte)", proj(bits2u), 2, gb2),
             ("proj s2 nobits", proj(None), 2, gb2),
             ("s3 c3 bits (4-byte) pk=2", s3c3(bits3), 2, gb3), ("s3 c3 bits (1-byte) pk=2", s3c3(bits3u), 2, gb3),
             ("s3 c3 nobits pk=2", s3c3(None), 2, gb3),
             ("s3 c3 bits (4-byte) pk=0", s3c3(bits3), 0, gb3), ("s3 c3 bits (1-byte) pk=0", s3c3(bits3u), 0, gb3),
             ("s3 c3 nobits pk=0", s3c3(None), 0, gb3)]
    res = {c[0]: [] for c in cases}
    for _ in range(a.rounds):
        for name, fn, kv, _gb in cases:
            N.set_variant("igemm_pk", kv)
            try:
                res[name].append(timeit(fn))
            finally:
                N.set_variant("igemm_pk", 2)
    for name, _fn, _kv, gb in cases:
        t = statistics.median(res[name])
        print(f"{name:28s} {t:8.1f} us  {gb / t * 1e6 / 1e3:6.2f} TB/s (activations only)", flush=True)


if __name__ == "__main__":
    main()
