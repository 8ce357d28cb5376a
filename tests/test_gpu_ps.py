"""Pack / unpack kernel of the native parameter-server data plane on the MI355X.

The multi-process PS job itself (1 or 2 PS + 2 workers on one GPU over HIP IPC) runs in
scripts/gpu_ps_check.py, started as a child process: spawning role processes from a pytest
process that has already initialised the GPU is not allowed on the GPU pool."""
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


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_range_copy_many_ranges_matches_reference(wire):
    """A shard of 300 ranges (lengths 0-70,000: BN vectors next to conv kernels, one empty),
    scattered over a flat buffer in shuffled order and laid end to end in the packed buffer, is
    gathered and scattered exactly as index copies do (bf16: rounded / widened)."""
    from pddl.ops.native import require_native
    N = require_native()
    g = torch.Generator().manual_seed(7)
    lens = torch.randint(1, 70000, (300,), generator=g)
    lens[::7] = torch.randint(1, 64, (len(lens[::7]),), generator=g)
    lens[13] = 0
    gaps = torch.randint(0, 50, (300,), generator=g)
    starts = torch.cumsum(lens + gaps, 0) - lens
    order = torch.randperm(300, generator=g)
    flat_n = int((starts + lens).max()) + 5
    rows, packed = [], 0
    for i in order.tolist():
        rows.append([int(starts[i]), packed, int(lens[i])])
        packed += int(lens[i])
    rows = torch.tensor(rows, dtype=torch.int64)
    flat = torch.randn(flat_n, device="cuda")
    idx = torch.cat([torch.arange(f, f + n) for f, _, n in rows.tolist()]).cuda()
    pdt = torch.float32 if wire == "fp32" else torch.bfloat16
    buf = torch.zeros(packed, dtype=pdt, device="cuda")
    (N.range_copy if wire == "fp32" else N.range_copy_cvt)(flat, buf, rows, False)
    assert torch.equal(buf, flat[idx].to(pdt))
    back = torch.zeros_like(flat)
    (N.range_copy if wire == "fp32" else N.range_copy_cvt)(buf, back, rows, True)
    want = torch.zeros_like(flat)
    want[idx] = flat[idx].to(pdt).float()
    assert torch.equal(back, want)
    with pytest.raises(RuntimeError):   # (not end to end in packed order)
        N.range_copy(flat, buf.float(), torch.tensor([[0, 10, 5], [100, 0, 5]], dtype=torch.int64), False)


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


def test_two_ps_job_applies_every_push_on_every_shard():
    """The reference's multi-PS shape on one card (imagenet-resnet50-ps.py:75-84): 2 PS roles +
    2 workers as four processes over the native HIP-IPC data plane, the variables split over two
    shards.  scripts/gpu_ps_check.py (a child process: roles are never spawned from this
    GPU-initialised process) asserts that each PS applied every pushed step."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NUM_PS="2", STEPS="8")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "gpu_ps_check.py")], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "native PS job ok: 8 async steps" in r.stdout and "on 2 PS" in r.stdout, r.stdout[-2000:]
    assert "updates per PS [8, 8]" in r.stdout, r.stdout[-2000:]
