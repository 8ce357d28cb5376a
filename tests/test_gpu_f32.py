"""Reference-precision (fp32) path: the fp32-MFMA HIP convolutions (csrc/kernels/conv_f32.hip)
against float64 PyTorch, and the assembled fp32 engine (models/engine_f32.py) against the
PyTorch reference model (models/reference.py, the Keras graph of imagenet-resnet50.py:51-61)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def N():
    from pddl.ops.native import require_native
    return require_native()


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


CASES = [   # N, H, C, Cout, R, stride, pad
    (2, 9, 64, 96, 1, 1, 0),
    (2, 11, 32, 64, 3, 1, 1),
    (3, 8, 128, 64, 1, 2, 0),
    (2, 23, 3, 64, 7, 2, 3),       # the stem: C = 3 (scalar gather), K = 147
    (1, 5, 2048, 40, 1, 1, 0),     # dense-like: long K, Cout tail
]


@pytest.mark.parametrize("case", CASES)
def test_conv_f32_forward_and_wgrad(case):
    torch.manual_seed(0)
    n, h, c, co, r, st, pad = case
    ho = (h + 2 * pad - r) // st + 1
    x = torch.randn(n, h, h, c, device=dev)
    w = torch.randn(co, r, r, c, device=dev) * 0.1
    b = torch.randn(co, device=dev)
    y = torch.empty(n, ho, ho, co, device=dev)
    N().conv_f32(x, r, r, st, pad, w.view(co, -1), b, y)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(), stride=st,
                   padding=pad).permute(0, 2, 3, 1)
    assert rel(y, ref) < 1e-5
    g = torch.randn(n, ho, ho, co, device=dev)
    dw = torch.zeros(co, r * r * c, device=dev)
    N().wgrad_f32(x, r, r, st, pad, g, dw)
    rw = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (co, c, r, r), g.double().permute(0, 3, 1, 2),
                                     stride=st, padding=pad).permute(0, 2, 3, 1).reshape(co, -1)
    assert rel(dw, rw) < 1e-5


@pytest.mark.parametrize("case", [(2, 9, 64, 96, 1, 1, 0), (2, 11, 32, 64, 3, 1, 1), (3, 8, 128, 64, 1, 2, 0),
                                  (4, 3, 512, 2048, 1, 1, 0), (4, 3, 512, 512, 3, 1, 1), (4, 6, 1024, 512, 1, 2, 0),
                                  (4, 6, 1024, 2048, 1, 2, 0)])
def test_conv2d_f32_autograd(case):
    """conv2d_f32's three gradients (dgrad as a flipped-weight conv / strided scatter, wgrad,
    bias) against float64 autograd of F.conv2d."""
    from pddl.ops.conv_f32 import conv2d_f32
    torch.manual_seed(1)
    n, h, c, co, r, st, pad = case
    x = torch.randn(n, c, h, h, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(co, r, r, c, device=dev) * 0.1).requires_grad_(True)
    b = torch.randn(co, device=dev).requires_grad_(True)
    y = conv2d_f32(x, w, b, st, pad)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd, wd, bd = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xd, wd.permute(0, 3, 1, 2), bd, stride=st, padding=pad)
    yr.backward(gy.double())
    assert rel(y, yr) < 1e-5
    assert rel(x.grad, xd.grad) < 1e-5
    assert rel(w.grad, wd.grad) < 1e-5
    assert rel(b.grad, bd.grad) < 1e-5


class _FProxy:
    """torch.nn.functional with `relu` replaced (recording or replaying ReLU masks)."""

    def __init__(self, relu):
        self.relu = relu

    def __getattr__(self, name):
        return getattr(F, name)


def _ref_grads(L, params, img, lab, B, crop, dtype, masks=None):
    """The reference step in `dtype` on the CPU; with `masks`, every ReLU applies the engine's
    recorded mask instead of its own sign test (same arithmetic, same decisions)."""
    from pddl.models import reference as R
    ref = R.TorchEngine(L, B, crop=crop, device="cpu")
    ref.params = params.detach().cpu().to(dtype)
    ref.grads = torch.zeros(L.n_trainable, dtype=dtype)
    orig_pre, orig_f = R.preprocess, R.F
    R.preprocess = lambda *a, **k: orig_pre(*a, **k).to(dtype)
    if masks is not None:
        it = iter(masks)
        R.F = _FProxy(lambda x: x * next(it).to(x.dtype))
    try:
        st = ref.forward_backward(img, lab, 1.0 / B)
    finally:
        R.preprocess, R.F = orig_pre, orig_f
    return st, ref.grads


def test_f32_engine_matches_reference():
    """One training step of the fp32 HIP engine vs the PyTorch reference model in float64 on
    the CPU, every gradient tensor within 1e-4 relative.  The reference replays the engine's
    ReLU masks: a pre-activation within fp32 rounding of zero (1-2 of ~10^6 per step) can take
    the other side of the ReLU in any fp32 run, which re-routes that element's gradient and
    moves a small bias / BN-beta gradient by up to ~1e-2 -- a decision, not an arithmetic error.
    Without replay, the count of such flips is reported."""
    import pddl.models.engine_f32 as E
    from pddl.models.resnet50 import ParamLayout
    torch.manual_seed(2)
    L = ParamLayout()
    B, crop = 4, 96
    eng = E.HipF32Engine(L, B, crop=crop, device=dev)
    eng.init(seed=3)
    img = torch.randint(0, 256, (B, crop, crop, 3), dtype=torch.uint8)
    lab = torch.randint(0, 1000, (B,))
    masks = []

    def rec(x):
        y = F.relu(x)
        masks.append((x > 0).detach().cpu())
        return y
    orig_f = E.F
    E.F = _FProxy(rec)
    try:
        st = eng.forward_backward(img.to(dev), lab.to(dev), 1.0 / B)
    finally:
        E.F = orig_f
    assert len(masks) == 1 + 3 * len(L.blocks)
    s64, g64 = _ref_grads(L, eng.params, img, lab, B, crop, torch.float64, masks)
    assert abs(st[0].item() - s64[0].item()) / abs(s64[0].item()) < 1e-5
    g = eng.grads.cpu().double()
    rows = []
    for e in L.entries.values():
        if e.offset + e.size > L.n_trainable:
            continue
        sl = slice(e.offset, e.offset + e.size)
        if g64[sl].norm() < 1e-12:
            continue
        rows.append((rel(g[sl], g64[sl]), e.name))
    rows.sort(reverse=True)
    print("worst (engine vs f64 with the engine's ReLU masks):", rows[:3])
    assert rows[0][0] < 1e-4, rows[:3]
