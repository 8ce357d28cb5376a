"""Strategy equivalence on CPU (gloo, spawned processes; SURVEY.md §4 "strategy equivalence"):
N-rank synchronous data parallelism with global batch B must produce the same weights after
k steps as one process with batch B.  Exercises the native FusionEngine (C++ background
thread over the c10d gloo group), bucketed all-reduce, sharding policies and Mirrored
in-process replicas."""
import os

import pytest
import torch
import torch.multiprocessing as mp

STEPS = 2


def _cfg(preset, **kw):
    from pddl.config import make_config
    base = dict(device="cpu", data="synthetic", image_size=32, crop=32, flip=False, epochs=1, max_steps=STEPS,
                verbose=0, save=False, train_images=64, val_images=8, seed=5, lr=1e-2)
    base.update(kw)
    return make_config(preset, **base)


def _train(preset, **kw):
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    cfg = _cfg(preset, **kw)
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    hist = tr.fit(1, [], validation=False)
    return st, hist


def _rank_main(rank, world, port, preset, kw, q, env=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    os.environ.update(env or {})
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import pddl  # noqa
    st, hist = _train(preset, **kw)
    n = st.engine.L.n_trainable
    reps = [e.params[:n].numpy().copy() for e, _ in st._replicas()]
    q.put((rank, reps[0], hist.history["loss"][0], type(getattr(st, "fusion", None)).__name__,
           getattr(st, "bucket_mb", None), reps, st.num_replicas_in_sync))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _spawn(world, preset, kw, env=None, full=False):
    from pddl.parallel.launch import pick_unused_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = pick_unused_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, preset, kw, q, env)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=600) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = sorted(out, key=lambda t: t[0])
    if full:
        return out
    return [(r, torch.from_numpy(p), l, f, mb) for r, p, l, f, mb, _, _ in out]


@pytest.fixture(scope="module")
def single_b4():
    st, hist = _train("single", batch_size=4)
    return st.engine.params[:st.engine.L.n_trainable].clone(), hist.history["loss"][0]


def _close(a, b, tol=1e-5):
    return ((a - b).norm() / b.norm()).item() < tol


def test_horovod_2_ranks_equals_single_global_batch(single_b4):
    ref, ref_loss = single_b4
    out = _spawn(2, "horovod", dict(batch_size=2, lr=1e-2, lr_scale_by_size=False, warmup_epochs=0,
                                    shard_by="batch"))
    assert out[0][3] == "FusionEngine"          # the native C++ fusion engine was used
    for _, p, loss, _, _ in out:
        assert _close(p, ref)
    assert abs(out[0][2] - ref_loss) <= 1e-5 * abs(ref_loss)


def test_multiworker_element_sharding_equals_single(single_b4):
    ref, _ = single_b4
    out = _spawn(2, "multiworker", dict(batch_size=2, val_batch_size=2))
    for _, p, _, _, _ in out:
        assert _close(p, ref)


def test_multiworker_2_procs_x_2_replicas_equals_single(single_b4):
    """The MWMS 2 workers x R GPUs layout (imagenet-resnet50-multiworkers.py:20-26) as its CPU
    double: 2 processes x 2 local replicas (PDDL_LOCAL_GPUS=2), in-process sum + gloo sum across
    processes standing in for the one RCCL communicator; global batch 4 = single b4."""
    ref, ref_loss = single_b4
    out = _spawn(2, "multiworker", dict(batch_size=1, val_batch_size=1), env={"PDDL_LOCAL_GPUS": "2"}, full=True)
    for rank, _, loss, _, _, reps, nrep in out:
        assert nrep == 4 and len(reps) == 2
        for p in reps:   # batch-1 replicas sum in another order than one b4 conv: Adam amplifies
            assert _close(torch.from_numpy(p), ref, 2e-4)   # the reassociation of tiny grads (~7e-5)
    assert abs(out[0][2] - ref_loss) <= 1e-5 * abs(ref_loss)
    for p in out[1][5]:          # every replica of every process holds the same weights
        assert (torch.from_numpy(p) == torch.from_numpy(out[0][5][0])).all()


def test_multiworker_local_gpus_refuses_missing_devices(monkeypatch):
    """PDDL_LOCAL_GPUS>1 on a GPU request that cannot be honoured errors out (no silent fallback
    to one replica)."""
    from pddl.parallel.strategies import MultiWorkerStrategy
    from pddl.parallel.launch import ClusterInfo
    monkeypatch.setenv("PDDL_LOCAL_GPUS", "4")
    st = MultiWorkerStrategy(_cfg("multiworker", device="cuda"))
    with pytest.raises(RuntimeError, match="no GPU is visible|GPUs"):
        st._local_devices(ClusterInfo())


def test_mirrored_two_cpu_replicas_equals_single(single_b4, monkeypatch):
    ref, _ = single_b4
    monkeypatch.setenv("PDDL_CPU_REPLICAS", "2")
    st, _ = _train("mirrored", batch_size=2)
    assert st.num_replicas_in_sync == 2 and st.global_batch == 4
    for eng, _ in st.mirror.replicas:
        assert _close(eng.params[:eng.L.n_trainable], ref)


def test_horovod_bucket_autotune_picks_one_size_and_matches_fixed(monkeypatch):
    """--bucket-mb 0: 4 candidate bucket sizes timed in turn (fusion engine rebuilt between
    them), rank 0's pick broadcast; the trajectory equals a fixed-bucket run."""
    monkeypatch.setenv("PDDL_AUTOTUNE_STEPS", "2")
    kw = dict(batch_size=2, lr=1e-2, lr_scale_by_size=False, warmup_epochs=0, shard_by="batch", max_steps=9,
              train_images=64)
    tuned = _spawn(2, "horovod", dict(kw, bucket_mb=0))
    fixed = _spawn(2, "horovod", dict(kw, bucket_mb=32))
    assert tuned[0][4] in (8.0, 16.0, 32.0, 64.0) and tuned[0][4] == tuned[1][4]
    for (_, p, _, _, _), (_, q, _, _, _) in zip(tuned, fixed):
        assert _close(p, q)


def test_horovod_bf16_wire_close_to_fp32():
    """--grad-dtype bf16: the FusionEngine reduces bf16 buckets (half the bytes on the wire)
    and widens the sum back; the trajectory stays within bf16 rounding of the fp32 run."""
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    kw = dict(batch_size=2, lr=1e-3, lr_scale_by_size=False, warmup_epochs=0, shard_by="batch")
    fp32 = _spawn(2, "horovod", dict(kw, grad_dtype="fp32"))
    bf16 = _spawn(2, "horovod", dict(kw, grad_dtype="bf16"))
    e0 = TorchEngine(ParamLayout(), 1, crop=32)
    e0.init(seed=5)
    p0 = e0.params[:e0.L.n_trainable]
    assert bf16[0][3] == "FusionEngine"
    upd = (fp32[0][1] - p0).norm()
    assert upd > 0
    assert ((bf16[0][1] - fp32[0][1]).norm() / upd).item() < 0.05
    assert torch.equal(bf16[0][1], bf16[1][1])        # both ranks applied the same reduced gradient


def test_segmented_tail_cuts_split_the_last_kernel_bucket_at_block_boundaries():
    """Graphed replicas' tail cuts (strategies._LocalReplicas._split_tail): the last kernel bucket is
    split at every block boundary inside it, the ranges stay contiguous and cover the same span,
    and the per-channel tail bucket stays last."""
    from pddl.models.resnet50 import ParamLayout
    from pddl.parallel.strategies import _LocalReplicas
    L = ParamLayout()
    bks = L.buckets(32.0)
    out = _LocalReplicas._split_tail(bks, L)
    assert out[:len(bks) - 2] == bks[:-2] and out[-1] == bks[-1]
    assert len(out) > len(bks)
    assert all(a[1] == b[0] for a, b in zip(out, out[1:-1]))
    assert out[len(bks) - 2][0] == bks[-2][0] and out[-2][1] == bks[-2][1]
    ends = {L.entry(b.convs["0" if b.proj else "1"].name, "kernel").offset
            + L.entry(b.convs["0" if b.proj else "1"].name, "kernel").size for b in L.blocks}
    assert all(e in ends for _, e in out[len(bks) - 2:-2])
