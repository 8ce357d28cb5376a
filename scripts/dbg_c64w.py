"""Locate wrong / non-finite entries of the conv3x3c64 weight gradient on one small problem."""
import sys
import torch
sys.path.insert(0, ".")
from pddl.ops.native import require_native  # noqa: E402

N = require_native()
for n, h in ((1, 4), (1, 8), (2, 56)):
    torch.manual_seed(1)
    x = torch.randn(n, h, h, 64, device="cuda").to(torch.bfloat16)
    g = torch.randn(n, h, h, 64, device="cuda").to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), g.float().permute(0, 3, 1, 2),
                                      padding=1).permute(0, 2, 3, 1).reshape(64, 9, 64)
    dw = torch.zeros(64, 576, device="cuda")
    N.conv3x3c64_wgrad(x, g, dw)
    torch.cuda.synchronize()
    d = dw.view(64, 9, 64)
    bad = ~torch.isfinite(d)
    print(f"n={n} h={h}: nonfinite {bad.sum().item()} / {d.numel()}")
    if bad.any():
        print("  nonfinite per tap:", bad.sum((0, 2)).tolist())
        print("  nonfinite per co block:", bad.view(4, 16, 9, 64).sum((1, 2, 3)).tolist())
        print("  nonfinite per ci block:", bad.view(64, 9, 4, 16).sum((0, 1, 3)).tolist())
    err = (d - ref).abs()
    err[bad] = 0
    print("  rel err per tap:", [round(((d[:, t] - ref[:, t]).nan_to_num().norm() / ref[:, t].norm()).item(), 4)
                                 for t in range(9)])
    print("  rel err per ci block:", [round(((d[..., 16*j:16*j+16] - ref[..., 16*j:16*j+16]).nan_to_num().norm()
                                             / ref[..., 16*j:16*j+16].norm()).item(), 4) for j in range(4)])
    print("  sample d[0,4,:4]", d[0, 4, :4].tolist(), "ref", ref[0, 4, :4].tolist())
