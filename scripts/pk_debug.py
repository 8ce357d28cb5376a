"""Diagnose the persistent ring kernel (igemm_pk) against a torch reference: per case, the
relative error and where the mismatching elements sit (tile rows / columns, tiles)."""
import sys

import torch

sys.path.insert(0, ".")
import pddl  # noqa: F401,E402
from pddl.ops.native import require_native  # noqa: E402

N = require_native()
dev = "cuda"


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(torch.bfloat16)


def run(n, h, K, Nn, nb, res_on, relu=1, bits=False):
    torch.manual_seed(0)
    x = rnd(n, h, h, K)
    w = rnd(Nn, K, scale=0.05)
    sc, sh = torch.rand(Nn, device=dev) + 0.5, torch.randn(Nn, device=dev)
    res = rnd(n, h, h, Nn) if res_on else None
    outs = []
    for kv in (0, nb):
        N.set_variant("igemm_pk", kv)
        y = torch.full((n, h, h, Nn), float("nan"), dtype=torch.bfloat16, device=dev)
        bo = torch.zeros(n, h, h, Nn // 8, dtype=torch.uint8, device=dev) if bits else None
        N.igemm(x, None, h, h, 1, 1, 1, 0, h, h, w, 0, sc, sh, res, None, None, y, relu, None, 0, 0, 0, 0, 0, None, bo)
        torch.cuda.synchronize()
        outs.append(y.float().reshape(-1, Nn))
    N.set_variant("igemm_pk", 0)
    ref = (x.float().reshape(-1, K) @ w.float().t()) * sc + sh
    if res_on:
        ref = ref + res.float().reshape(-1, Nn)
    if relu:
        ref = ref.clamp_min(0)
    a, b = outs[1], outs[0]
    err = (a - b).abs()
    bad = err > 0.05 * (b.abs() + 0.1)
    bad = bad | torch.isnan(a)
    M = a.shape[0]
    print(f"case n={n} h={h} K={K} Nn={Nn} nb={nb} res={res_on} bits={bits}: M={M} rel(base,ref)="
          f"{((b - ref).norm() / ref.norm()).item():.2e} rel(pk,base)={((a - b).nan_to_num(1e9).norm() / b.norm()).item():.3e} "
          f"bad={bad.float().mean().item():.4f} nan={torch.isnan(a).float().mean().item():.4f}", flush=True)
    if bad.any():
        idx = bad.nonzero()
        rows, cols = idx[:, 0], idx[:, 1]
        print("  bad rows%128 hist:", torch.bincount(rows % 128, minlength=128).tolist()[:128:8])
        print("  bad cols%128 hist:", torch.bincount(cols % 128, minlength=128).tolist()[:128:8])
        print("  bad row tiles (first 20):", torch.unique(rows // 128).tolist()[:20], "of", (M + 127) // 128)
        print("  bad col tiles:", torch.unique(cols // 128).tolist())
        # does the pk output equal the reference somewhere else (row / column permutation)?
        t0 = a[:128, :128]
        for name, cand in (("no-res", ((x.float().reshape(-1, K) @ w.float().t()) * sc + sh).clamp_min(0)[:128, :128]),
                           ("no-scale", ((x.float().reshape(-1, K) @ w.float().t()) + sh + (res.float().reshape(-1, Nn) if res_on else 0)).clamp_min(0)[:128, :128]),
                           ("no-shift", ((x.float().reshape(-1, K) @ w.float().t()) * sc + (res.float().reshape(-1, Nn) if res_on else 0)).clamp_min(0)[:128, :128]),
                           ("raw-acc", (x.float().reshape(-1, K) @ w.float().t())[:128, :128])):
            print(f"  tile0 vs {name}: {((t0 - cand).norm() / (cand.norm() + 1e-9)).item():.3e}")
        print("  pk tile0 row0 cols0-15:", [round(v, 3) for v in t0[0, :16].tolist()])
        print("  ref tile0 row0 cols0-15:", [round(v, 3) for v in b[0, :16].tolist()])
        print("  pk tile0 col0 rows0-15:", [round(v, 3) for v in t0[:16, 0].tolist()])
        print("  ref tile0 col0 rows0-15:", [round(v, 3) for v in b[:16, 0].tolist()])


if __name__ == "__main__":
    for nb in (2, 4):
        run(1, 8, 64, 128, nb, True, bits=True)
        run(2, 32, 64, 128, nb, True, bits=True)
        run(32, 55, 64, 256, nb, True, bits=True)
        run(32, 55, 64, 256, nb, False, bits=True)
