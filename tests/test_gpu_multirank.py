"""Multi-rank gradient correctness of the HIP engine on the GPU (VERDICT r2 "Next round" #2).

Two data-parallel replicas, each with a DIFFERENT batch of 8, must produce -- after the gradient
reduction and before the optimizer -- the same flat gradient as one replica on the concatenated
batch of 16 (the reference's contract: Horovod averages per-rank gradients,
imagenet-resnet50-hvd.py:99-101; Mirrored sums per-replica gradients of loss/global_batch,
imagenet-resnet50-mirror.py:21,54).  Unlike the same-data rehearsal this catches a wrong
averaging factor, a bucket that is never reduced, or a reduction over the wrong slice: each
shows up as a ~50-100 % error on the affected tensors.

The ranks are rehearsal processes sharing the one GPU (PDDL_REHEARSE=1, gloo transport: RCCL
refuses two ranks on one device), running the real HorovodStrategy path (fusion engine bucket
callbacks during backward, gscale = 1/(B*world)).  The bound per tensor is the engine's own
run-to-run noise floor on the 16-batch (wgrad fp32 atomics in no fixed order): error <=
3 x floor + 2e-3 (measured on an MI355X: 0 -- the two-rank reduced gradient is bitwise the
one-rank gradient, and the engine is run-to-run deterministic at this size).  A 6-step Adam
trajectory of the global loss is compared as well, at lr 1e-4: at 1e-3 this 16-image problem
overshoots to a loss of ~107 at step 3, where a 1e-6 difference grows to ~1 %.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, S, STEPS = 8, 64, 6


def _cfg(strategy, batch):
    from pddl.config import make_config
    return make_config("bench", strategy=strategy, batch_size=batch, crop=S, image_size=S, optimizer="adam", lr=1e-4,
                       device="cuda", graphs=False, flip=False, data="synthetic_fixed", seed=0, bucket_mb=4.0,
                       num_classes=1000)


def _data():
    g = torch.Generator().manual_seed(1234)
    img = torch.randint(0, 256, (2 * B, S, S, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, 1000, (2 * B,), generator=g)
    return img, lab


def _rank_main(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE="2", PDDL_REHEARSE="1", PDDL_DIST_BACKEND="gloo")
    sys.path.insert(0, ROOT)
    import pddl  # noqa: F401
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    cfg = _cfg("horovod", B)
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    st.broadcast_state(tr)
    img, lab = _data()
    im, lb = img[rank * B:(rank + 1) * B].cuda(), lab[rank * B:(rank + 1) * B].cuda()
    assert st.fusion is not None and st.world == 2
    s = st.compute_gradients(im, lb)
    torch.cuda.synchronize()
    grads = st.engine.grads.cpu().clone()
    loss0 = float(st.reduce_metrics(s.double())[0]) / (2 * B)
    st.opt.step()
    st.engine.after_update()
    losses = [loss0]
    for _ in range(STEPS - 1):
        s = st.train_step(im, lb)
        losses.append(float(st.reduce_metrics(s.double())[0]) / (2 * B))
    torch.save({"grads": grads, "losses": losses, "params": st.engine.params.cpu()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _single_reference():
    """One replica on the concatenated batch of 16: gradients twice (noise floor), then STEPS."""
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    cfg = _cfg("single", 2 * B)
    st = make_strategy(cfg)
    Trainer(cfg, st)
    img, lab = _data()
    img, lab = img.cuda(), lab.cuda()
    runs = []
    for _ in range(2):
        st.engine.forward_backward(img, lab, 1.0 / (2 * B))
        torch.cuda.synchronize()
        runs.append(st.engine.grads.cpu().clone())
    losses = []
    for _ in range(STEPS):
        losses.append(float(st.train_step(img, lab)[0]) / (2 * B))
    return st.engine.L, runs, losses, st.engine.params.cpu()


def _per_tensor(L, a, b):
    out = {}
    for e in L.entries.values():
        if e.trainable:
            x, y = a[e.offset:e.offset + e.size].double(), b[e.offset:e.offset + e.size].double()
            out[e.name] = ((x - y).norm() / (y.norm() + 1e-30)).item()
    return out


def _check(L, got, ref_runs, tag):
    floor = _per_tensor(L, ref_runs[1], ref_runs[0])
    err = _per_tensor(L, got, ref_runs[0])
    worst = sorted(err.items(), key=lambda kv: -kv[1])[:5]
    print(f"{tag}: worst per-tensor errors {[(n, round(r, 5), round(floor[n], 5)) for n, r in worst]}")
    over = [(n, r, floor[n]) for n, r in err.items() if r > 3 * floor[n] + 2e-3]
    assert not over, (tag, over[:8])
    ratio = (got.double().norm() / ref_runs[0].double().norm()).item()
    assert abs(ratio - 1) < 1e-3, (tag, ratio)      # a wrong averaging factor moves this by 50-100 %


def test_two_horovod_ranks_match_one_rank_on_concatenated_batch(tmp_path):
    import torch.multiprocessing as mp
    from pddl.parallel.launch import pick_unused_port
    ctx = mp.get_context("spawn")
    port = pick_unused_port()
    procs = [ctx.Process(target=_rank_main, args=(r, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert torch.equal(r0["grads"], r1["grads"])          # the reduction leaves every rank identical
    assert torch.equal(r0["params"], r1["params"])        # ... and so do the updates
    L, ref_runs, ref_losses, _ = _single_reference()
    _check(L, r0["grads"], ref_runs, "horovod 2x8 vs 1x16")
    dev = [abs(a - b) / abs(b) for a, b in zip(r0["losses"], ref_losses)]
    print("global loss 2 ranks / 1 rank:", [(round(a, 4), round(b, 4)) for a, b in zip(r0["losses"], ref_losses)])
    assert max(dev) < 5e-3, dev


def test_two_mirrored_replicas_match_one_replica_on_concatenated_batch():
    """Mirrored (one process, 2 replicas sharing the GPU in a rehearsal: the in-process sum)."""
    from pddl.parallel.strategies import MirroredStrategy
    from pddl.train.trainer import Trainer
    os.environ["PDDL_REHEARSE"] = "1"
    try:
        cfg = _cfg("mirrored", B)
        st = MirroredStrategy(cfg, devices=[0, 0])
        Trainer(cfg, st)
        st.broadcast_state(None)
        img, lab = _data()
        img, lab = img.cuda(), lab.cuda()
        st.compute_gradients(img, lab)
        torch.cuda.synchronize()
        g = [e.grads.cpu().clone() for e, _ in st.mirror.replicas]
        assert torch.equal(g[0], g[1])
        L, ref_runs, ref_losses, _ = _single_reference()
        _check(L, g[0], ref_runs, "mirrored 2x8 vs 1x16")
        for e, o in st.mirror.replicas:
            o.step()
            e.after_update()
        losses = [None]
        for _ in range(STEPS - 1):
            losses.append(float(st.train_step(img, lab)[0]) / (2 * B))
        dev = [abs(a - b) / abs(b) for a, b in zip(losses[1:], ref_losses[1:])]
        print("mirrored loss 2 replicas / 1:", [(round(a, 4), round(b, 4)) for a, b in zip(losses[1:], ref_losses[1:])])
        assert max(dev) < 5e-3, dev
    finally:
        os.environ.pop("PDDL_REHEARSE", None)
