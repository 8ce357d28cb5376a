"""Engine-vs-reference gradient error per tensor, next to the reference's own accumulation-order
noise floor (the same bf16-point reference on the GPU vs on the CPU)."""
import json
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import pddl  # noqa
from pddl.models.reference import TorchEngine
from test_gpu_engine import _engines, _grad_errors

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.manual_seed(0)
L, he, te = _engines(B, 224, 224, bf16_points=True)
tc = TorchEngine(L, B, crop=224, device="cpu", bf16_points=True)
tc.params.copy_(te.params.cpu())
img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
lab = torch.randint(0, 1000, (B,), device="cuda")
flip = torch.tensor([1, 0, 0, 1] * (B // 4), dtype=torch.uint8, device="cuda")
he.forward_backward(img, lab, 1.0 / B, flip=flip)
te.forward_backward(img, lab, 1.0 / B, flip=flip)
tc.forward_backward(img.cpu(), lab.cpu(), 1.0 / B, flip=flip.cpu())
torch.cuda.synchronize()
eng = dict((n, r) for r, n in _grad_errors(L, he, te))


class _T:
    pass


t2 = _T()
t2.grads = tc.grads.cuda()
floor = dict((n, r) for r, n in _grad_errors(L, t2, te))
rows = sorted(((eng[n], floor[n], n) for n in eng), reverse=True)
for e, f, n in rows[:15]:
    print(f"{e:8.4f} {f:8.4f}  {n}")
import statistics
print("median engine", statistics.median(eng.values()), "median floor", statistics.median(floor.values()))
print("max ratio", max(e / max(f, 1e-6) for e, f, _ in rows))
