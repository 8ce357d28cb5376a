"""Stall inspector of the native fusion engine (Horovod's stall check): a rank
that never joins a bucket's all-reduce turns into a diagnostic error on its peer within the
stall timeout instead of a silent hang.  CPU, gloo, 2 spawned ranks."""
import os
import time

import pytest
import torch
import torch.multiprocessing as mp


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import pddl  # noqa: F401
    import torch.distributed as dist
    from pddl.ops.native import require_native
    dist.init_process_group("gloo", rank=rank, world_size=2)
    flat = torch.ones(1024)
    eng = require_native().FusionEngine(dist.group.WORLD, flat, [(0, 512), (512, 512)], 2.0, False, rank)
    if rank == 1:          # the stuck peer: never produces its gradients
        time.sleep(8)
        q.put((rank, "idle"))
        q.close()
        q.join_thread()   # flush before the hard exit
        os._exit(0)
    eng.begin_step()
    eng.bucket_ready(0)
    eng.bucket_ready(1)
    t0 = time.time()
    try:
        eng.finish()
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, f"{time.time() - t0:.1f}s {e}"))
    q.close()
    q.join_thread()       # flush before the hard exit (the stuck collective would hang a clean one)
    os._exit(0)


def test_stuck_peer_raises_stall_error():
    from pddl.ops.native import native_available
    if not native_available():
        pytest.skip("native extension not built")
    from pddl.parallel.launch import pick_unused_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = pick_unused_port()
    ps = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    msg = out[0]
    assert "stall detected" in msg and "bucket 0" in msg, msg
    assert float(msg.split("s ", 1)[0]) < 7.0, msg      # raised at the 2 s timeout, not at the peer's exit
