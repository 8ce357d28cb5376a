"""Captured step with the overlapped optimizer vs the same step eager: where do params differ?"""
import os
import sys
import torch
sys.path.insert(0, ".")
from pddl.models.engine import HipEngine  # noqa: E402
from pddl.models.resnet50 import ParamLayout  # noqa: E402
from pddl.train.graph import GraphedTrainStep  # noqa: E402
from pddl.train.optim import make_optimizer  # noqa: E402
from pddl.parallel.strategies import overlap_buckets, overlap_stream  # noqa: E402

torch.manual_seed(0)
B = 4
L = ParamLayout()
img = torch.randint(0, 256, (3, B, 96, 96, 3), dtype=torch.uint8, device="cuda")
lab = torch.randint(0, 1000, (3, B), device="cuda")
res = {}
for mode in ("eager_ov", "graph_ov"):
    he = HipEngine(L, B, crop=96, image_size=96)
    he.init(seed=7)
    opt = make_optimizer("adam", he, lr=1e-3)
    gs = GraphedTrainStep(he, opt, B, (96, 96), 1.0 / B) if mode == "graph_ov" else None
    snaps = []
    for i in range(3):
        if gs is not None:
            s = gs(img[i], lab[i], None, (0, 0))
        else:
            bks = overlap_buckets(he)
            opt.overlap_begin(bks, overlap_stream(he))
            s = he.forward_backward(img[i], lab[i], 1.0 / B, bucket_cb=opt.overlap_bucket, buckets=bks)
            opt.overlap_finish()
            he.after_update()
        torch.cuda.synchronize()
        snaps.append((s[0].item(), he.params.clone(), opt.hs.clone() if opt.hs is not None else None))
    res[mode] = (snaps, overlap_buckets(he), opt.n)
(e, bks, n), (g, _, _) = res["eager_ov"], res["graph_ov"]
print("n", n, "total", L.total, "buckets", len(bks), bks[:3], bks[-3:])
for i in range(3):
    pe, pg = e[i][1], g[i][1]
    print(f"step {i}: loss eager {e[i][0]:.4f} graph {g[i][0]:.4f}; hs eager {e[i][2].tolist()} graph {g[i][2].tolist()}")
    d = (pe - pg).abs()
    for k, (s0, e0) in enumerate(bks):
        dd = d[s0:e0].max().item()
        if dd > 1e-6:
            print(f"   bucket {k} [{s0},{e0}) max diff {dd:.3e}")
    if n < pe.numel():
        print(f"   beyond n: {d[n:].max().item():.3e}")
