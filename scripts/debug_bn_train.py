"""Layer-by-layer comparison of HipEngineBNTrain's forward against the fp32 reference."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
import pddl  # noqa
from pddl.models.engine import make_hip_engine
from pddl.models.reference import ReferenceResNet50, preprocess
from pddl.models.resnet50 import ParamLayout

torch.manual_seed(0)
B, crop = 8, 128
L = ParamLayout()
he = make_hip_engine(L, B, bn_mode="train", crop=crop, image_size=crop)
he.init(seed=3)
if os.environ.get("SMALL_G3"):
    for e in L.entries.values():
        if e.kind == "gamma" and e.layer.endswith("_3_bn"):
            he.params[e.offset:e.offset + e.size] = 0.1 + 0.2 * torch.rand(e.size, device="cuda")
    he.after_update()
img = torch.randint(0, 256, (B, crop, crop, 3), dtype=torch.uint8, device="cuda")
lab = torch.randint(0, 1000, (B,), device="cuda")
p0 = he.params.clone()
he.forward_backward(img, lab, 1.0 / B)
torch.cuda.synchronize()
m = ReferenceResNet50(L, "train")
m.stats = p0.clone()
p = p0[:L.n_trainable]
x = preprocess(img, crop, True, None)


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def nhwc(t):
    return t.permute(0, 2, 3, 1)


s = L.stem
x = F.pad(x, (3, 3, 3, 3))
z = m._conv(p, x, s, pad_explicit=True)
print("stem z", rel(he.zs, nhwc(z)))
x = F.relu(m._bn(p, z, s, True))
print("stem c1", rel(he.c1, nhwc(x)))
x = F.max_pool2d(F.pad(x, (1, 1, 1, 1)), 3, 2)
print("pool", rel(he.pool, nhwc(x)))
for b in L.blocks:
    c = b.convs
    zz = he.z[b.name]
    if b.proj:
        z0 = m._conv(p, x, c["0"])
        print(b.name, "z0", rel(zz["0"], nhwc(z0)))
        sc = m._bn(p, z0, c["0"], True)
    else:
        sc = x
    z1 = m._conv(p, x, c["1"])
    print(b.name, "z1", rel(zz["1"], nhwc(z1)))
    y = F.relu(m._bn(p, z1, c["1"], True))
    print(b.name, "y1", rel(he.acts[b.name]["y1"], nhwc(y)))
    z2 = m._conv(p, y, c["2"])
    print(b.name, "z2", rel(zz["2"], nhwc(z2)))
    y = F.relu(m._bn(p, z2, c["2"], True))
    z3 = m._conv(p, y, c["3"])
    print(b.name, "z3", rel(zz["3"], nhwc(z3)))
    y = m._bn(p, z3, c["3"], True)
    x = F.relu(y + sc)
    print(b.name, "out", rel(he.acts[b.name]["out"], nhwc(x)))
print("pooled", rel(he.pooled, x.mean(dim=(2, 3))))
print("moving", rel(he.params[L.n_trainable:], m.stats[L.n_trainable:]))
