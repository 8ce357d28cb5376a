"""Shape fuzzing of the implicit-GEMM kernels (SURVEY.md §4 "kernel unit ... shape sweeps"):
hypothesis draws batch / spatial / channel / kernel / stride combinations (channels multiples
of 64 as the kernels require, odd spatial sizes like the 244 / 160 crops produce) and every
draw is compared with an fp32 PyTorch reference of the same op.  Includes the residual and
residual-gradient epilogues, so both prefetch variants are exercised (knob igemm_pf), and the
8-phase 256x256 kernel is forced onto tiny problems (igemm8_min_tiles=1) on half the draws."""
import pytest
import torch

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu
dev = "cuda"


def N():
    from pddl.ops.native import require_native
    return require_native()


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


conv = st.tuples(
    st.integers(1, 3),                       # batch
    st.integers(3, 19),                      # input H = W
    st.sampled_from([64, 128, 192, 256]),    # Cin
    st.sampled_from([64, 128, 136, 256, 320]),   # Cout (multiple of 8)
    st.sampled_from([(1, 1, 0), (1, 2, 0), (3, 1, 1)]),   # (R, stride, pad)
)


def _k8(on):
    N().set_variant("igemm8", 2 if on else 0)
    N().set_variant("igemm8_min_tiles", 1 if on else 128)
    N().set_variant("igemm8_min_n", 256 if on else 512)


@settings(max_examples=25, deadline=None, derandomize=True)
@given(conv, st.booleans(), st.integers(0, 1), st.booleans())
def test_igemm_forward_fuzz(case, with_res, pf, k8):
    n, h, c, co, (r, s, pad) = case
    ho = (h + 2 * pad - r) // s + 1
    if ho < 1:
        return
    torch.manual_seed(n * 1000 + h * 10 + r)
    x = rnd(n, h, h, c)
    w = rnd(co, r, r, c, scale=0.05)
    sc = torch.rand(co, device=dev) + 0.5
    sh = torch.randn(co, device=dev)
    res = rnd(n, ho, ho, co) if with_res else None
    out = torch.empty(n, ho, ho, co, dtype=torch.bfloat16, device=dev)
    N().set_variant("igemm_pf", pf)
    _k8(k8)
    try:
        N().igemm(x, None, h, h, r, r, s, pad, ho, ho, w.view(co, -1), 0, sc, sh, res, None, None, out, 1, None, 0,
                  0, 0, 0, 0, None, None)
    finally:
        N().set_variant("igemm_pf", 1)
        _k8(True)
        N().set_variant("igemm8_min_tiles", 128)
    N().set_variant("igemm8_min_n", 512)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=s,
                                     padding=pad).permute(0, 2, 3, 1) * sc + sh
    if with_res:
        ref = ref + res.float()
    ref = torch.relu(ref)
    assert rel(out, ref) < 1e-2


@settings(max_examples=25, deadline=None, derandomize=True)
@given(conv, st.integers(0, 1), st.booleans())
def test_igemm_dgrad_and_wgrad_fuzz(case, pf, k8):
    n, cin_h, cin, co, (r, s, pad) = case
    h = cin_h
    ho = (h + 2 * pad - r) // s + 1
    if ho < 1 or co % 64:
        return
    torch.manual_seed(n * 7 + h + r)
    g = rnd(n, ho, ho, co)
    w = rnd(co, r, r, cin, scale=0.05)
    add = rnd(n, h, h, cin)
    mask = rnd(n, h, h, cin)
    wt = w.float().flip(1).flip(2).permute(3, 1, 2, 0).contiguous().to(torch.bfloat16)   # [cin][R][S][co]
    out = torch.empty(n, h, h, cin, dtype=torch.bfloat16, device=dev)
    N().set_variant("igemm_pf", pf)
    _k8(k8)
    try:
        N().igemm(g, None, ho, ho, r, r, 1, r - 1 - pad, ho, ho, wt.view(cin, -1), 1, None, None, None, mask, add,
                  out, 0, None, 0, 0, 1 if s == 2 else 0, h, h, None, None)
    finally:
        N().set_variant("igemm_pf", 1)
        _k8(True)
        N().set_variant("igemm8_min_tiles", 128)
    N().set_variant("igemm8_min_n", 512)
    ref = torch.nn.grad.conv2d_input((n, cin, h, h), w.float().permute(0, 3, 1, 2), g.float().permute(0, 3, 1, 2),
                                     stride=s, padding=pad)
    ref = (ref.permute(0, 2, 3, 1) + add.float()) * (mask.float() > 0)
    assert rel(out, ref) < 1e-2
    x = rnd(n, h, h, cin)
    dw = torch.zeros(co, r * r * cin, device=dev)
    N().wgrad(x, h, h, r, r, s, pad, ho, ho, g, None, 0, dw, r * r * cin, 0)
    wref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (co, cin, r, r), g.float().permute(0, 3, 1, 2),
                                       stride=s, padding=pad).permute(0, 2, 3, 1).reshape(co, -1)
    assert rel(dw, wref) < 5e-3


@pytest.mark.parametrize("n,h,c,r,s,pad", [(2, 13, 64, 3, 1, 1), (3, 19, 128, 1, 1, 0), (1, 9, 256, 1, 2, 0),
                                           (4, 17, 64, 3, 1, 1), (2, 28, 64, 1, 1, 0)])
def test_igemm_n64_tiles(n, h, c, r, s, pad):
    """GEMM width 64 (the 256x64 tile): forward with residual and dgrad with add + mask, M tails
    included.  (A 512x64 tile of 128x64 wave tiles was measured 4x slower -- register spills.)"""
    co = 64
    ho = (h + 2 * pad - r) // s + 1
    torch.manual_seed(n * 100 + h + c)
    x = rnd(n, h, h, c)
    w = rnd(co, r, r, c, scale=0.05)
    sc = torch.rand(co, device=dev) + 0.5
    sh = torch.randn(co, device=dev)
    res = rnd(n, ho, ho, co)
    out = torch.empty(n, ho, ho, co, dtype=torch.bfloat16, device=dev)
    N().igemm(x, None, h, h, r, r, s, pad, ho, ho, w.view(co, -1), 0, sc, sh, res, None, None, out, 1, None, 0,
              0, 0, 0, 0, None, None)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=s,
                                     padding=pad).permute(0, 2, 3, 1) * sc + sh
    assert rel(out, torch.relu(ref + res.float())) < 1e-2
    # dgrad of a conv with Cin = 64 (GEMM width 64): g [n, ho, ho, c'] -> [n, h, h, 64]
    if s == 1:
        cp = c
        g = rnd(n, ho, ho, cp)
        w2 = rnd(cp, r, r, co, scale=0.05)
        add = rnd(n, h, h, co)
        mask = rnd(n, h, h, co)
        wt = w2.float().flip(1).flip(2).permute(3, 1, 2, 0).contiguous().to(torch.bfloat16)
        gx = torch.empty(n, h, h, co, dtype=torch.bfloat16, device=dev)
        N().igemm(g, None, ho, ho, r, r, 1, r - 1 - pad, ho, ho, wt.view(co, -1), 1, None, None, None, mask, add,
                  gx, 0, None, 0, 0, 0, h, h, None, None)
        ref = torch.nn.grad.conv2d_input((n, co, h, h), w2.float().permute(0, 3, 1, 2),
                                         g.float().permute(0, 3, 1, 2), stride=1, padding=pad)
        ref = (ref.permute(0, 2, 3, 1) + add.float()) * (mask.float() > 0)
        assert rel(gx, ref) < 1e-2
