"""Pack / unpack kernel of the native parameter-server data plane on the MI355X.

The multi-process PS job itself (1 PS + 2 workers on one GPU over HIP IPC) runs from
scripts/gpu_ps_check.py: spawning role processes from a pytest process that has already
initialised the GPU is not allowed on the GPU pool."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_range_copy_gather_scatter():
    from pddl.ops.native import require_native
    N = require_native()
    flat = torch.randn(1000, device="cuda")
    rows = torch.tensor([[10, 0, 100], [500, 100, 37], [990, 137, 10]], dtype=torch.int64)
    packed = torch.zeros(147, device="cuda")
    N.range_copy(flat, packed, rows, False)
    want = torch.cat([flat[10:110], flat[500:537], flat[990:1000]])
    assert torch.equal(packed, want)
    back = torch.zeros_like(flat)
    N.range_copy(packed, back, rows, True)
    assert torch.equal(back[500:537], flat[500:537]) and back[200:300].abs().sum().item() == 0
    with pytest.raises(RuntimeError):
        N.range_copy(flat, packed, torch.tensor([[995, 0, 10]], dtype=torch.int64), False)


def test_bf16_wire_pack_unpack_and_adam():
    """--ps-wire bf16 data plane: the push gathers fp32 gradient ranges rounded to bf16, the
    pull scatters the bf16 snapshot into fp32 parameters, and the PS's Adam reads bf16 gradients
    and writes the bf16 snapshot -- the fp32 Adam's arithmetic on the bf16-rounded gradient."""
    from pddl.ops.native import require_native
    N = require_native()
    flat = torch.randn(1000, device="cuda")
    rows = torch.tensor([[10, 0, 100], [500, 100, 37], [990, 137, 10]], dtype=torch.int64)
    packed = torch.zeros(147, dtype=torch.bfloat16, device="cuda")
    N.range_copy_cvt(flat, packed, rows, False)
    want = torch.cat([flat[10:110], flat[500:537], flat[990:1000]]).to(torch.bfloat16)
    assert torch.equal(packed, want)
    back = torch.zeros_like(flat)
    N.range_copy_cvt(packed, back, rows, True)
    assert torch.equal(back[500:537], flat[500:537].to(torch.bfloat16).float())
    n = 4096
    p = torch.randn(n, device="cuda")
    g = (torch.randn(n, device="cuda") * 1e-2).to(torch.bfloat16)
    m, v = torch.rand(n, device="cuda") * 1e-3, torch.rand(n, device="cuda") * 1e-5
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    snap = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    N.adam_bf16_wire(p, g, m, v, snap, 1e-3, 0.9, 0.999, 1e-7)
    N.adam(p2, g.float(), m2, v2, 1e-3, 0.9, 0.999, 1e-7, 1.0, None)
    torch.cuda.synchronize()
    assert torch.equal(p, p2) and torch.equal(m, m2) and torch.equal(v, v2)
    assert torch.equal(snap, p.to(torch.bfloat16))
