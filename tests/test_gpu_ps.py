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
