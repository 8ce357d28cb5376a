"""Parameter-server job (async, sharded, fault-injected), Keras-layout .h5 checkpoints and the
drop-in entry scripts — all on CPU."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from pddl.utils.envopts import with_opt
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(preset, **kw):
    from pddl.config import make_config
    base = dict(device="cpu", data="synthetic", image_size=32, crop=32, flip=False, epochs=1, verbose=0, save=False,
                train_images=64, val_images=8, seed=1)
    base.update(kw)
    return make_config(preset, **base)


# ------------------------------------------------------------------ parameter server
@pytest.mark.parametrize("impl", ["native", "c10d"])
def test_ps_async_job_runs_and_applies_every_step(impl, monkeypatch):
    from pddl.parallel.parameter_server import run_ps_job
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "impl", impl))
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "heartbeat", "600"))   # a loaded CI box must not look like a dead worker
    cfg = _cfg("ps", steps_per_epoch=6, validation_steps=1, batch_size=2, epochs=2)
    res = run_ps_job(cfg, num_ps=2, num_workers=2, return_results=True)
    ps = [r for r in res if r[0] == "ps"]
    wk = [r for r in res if r[0] == "worker"]
    assert len(ps) == 2 and len(wk) == 2
    assert sum(r[2] for r in wk) == 12                       # 2 epochs x 6 steps, split asynchronously
    assert all(r[2] == 12 for r in ps)                       # every PS applied every push
    assert all(r[4] == impl for r in ps)
    hist = [r for r in wk if r[3]][0][3]
    assert len(hist) == 2 and "val_loss" in hist[0]


@pytest.mark.parametrize("impl", ["native", "c10d"])
def test_ps_worker_failure_requeues_closure(impl, monkeypatch):
    from pddl.parallel.parameter_server import run_ps_job
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "impl", impl))
    monkeypatch.setenv("PDDL_FAULT", "kill_worker:1@1")
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "heartbeat", "3"))
    cfg = _cfg("ps", steps_per_epoch=6, batch_size=2, epochs=1)
    res = run_ps_job(cfg, num_ps=1, num_workers=2, return_results=True)
    wk = [r for r in res if r[0] == "worker"]
    ps = [r for r in res if r[0] == "ps"]
    assert len(wk) == 1                                      # the killed worker reported nothing
    assert ps[0][3] == [2]                                   # PS saw worker rank 2 die
    assert ps[0][2] >= 6                                     # all 6 closures done despite the failure


def test_ps_worker_death_inside_a_ticket_block_is_not_replayed(monkeypatch):
    """A worker killed at its 4th step, in the middle of a claimed block of >= 4 tickets: the
    three steps it finished were pushed and published, so only the unfinished tickets are
    re-queued and the PS applies spe updates (spe + 1 if the last push was in flight), not
    spe + 3 as with per-block publishing."""
    from pddl.parallel.parameter_server import run_ps_job
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "impl", "c10d"))
    monkeypatch.setenv("PDDL_FAULT", "kill_worker:1@3")
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "heartbeat", "3"))
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "ticket_block", "16"))
    spe = 40
    cfg = _cfg("ps", steps_per_epoch=spe, batch_size=2, epochs=1, train_images=2 * spe)
    res = run_ps_job(cfg, num_ps=1, num_workers=2, return_results=True)
    ps = [r for r in res if r[0] == "ps"]
    assert ps[0][3] == [2]
    assert spe <= ps[0][2] <= spe + 1, ps[0][2]


def test_ps_plateau_lowers_lr_and_early_stop_ends_job(monkeypatch):
    """The coordinator runs ReduceLROnPlateau / EarlyStopping (imagenet-resnet50-ps.py:139-140)
    on worker 0's val_loss and publishes the LR and the stop flag to every worker: a flat
    val_loss (lr ~ 0) lowers the LR after `patience` epochs and stops the job early."""
    from pddl.parallel.parameter_server import run_ps_job
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "heartbeat", "600"))
    cfg = _cfg("ps", steps_per_epoch=2, validation_steps=1, batch_size=2, epochs=6, lr=1e-12, min_lr=1e-14,
               reduce_lr_patience=1, early_stop_patience=3)
    res = run_ps_job(cfg, num_ps=1, num_workers=2, return_results=True)
    wk = [r for r in res if r[0] == "worker"]
    hist = [r for r in wk if r[3]][0][3]
    assert len(hist) == 4                                    # EarlyStopping(patience=3) ended epoch 4 of 6
    assert sum(r[2] for r in wk) == 4 * 2                    # no worker ran past the stop
    lrs = [h["lr"] for h in hist]
    assert lrs[0] == 1e-12 and lrs[1] < lrs[0] and lrs[-1] < lrs[1]


def test_ps_final_checkpoint_holds_the_ps_state(tmp_path, monkeypatch):
    """The saved file is the PS-resident state after every worker's last push (the reference
    saves the PS variables, imagenet-resnet50-ps.py:145-148), not worker 0's last snapshot."""
    from pddl.parallel.parameter_server import run_ps_job
    from pddl.utils.checkpoint import read_keras_weights
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "heartbeat", "600"))
    cfg = _cfg("ps", steps_per_epoch=4, batch_size=2, epochs=1, save=True, save_dir=str(tmp_path))
    res = run_ps_job(cfg, num_ps=1, num_workers=2, return_results=True)
    ps = [r for r in res if r[0] == "ps"]
    assert ps[0][2] == 4
    w = read_keras_weights(str(tmp_path / cfg.checkpoint_name()))
    assert "dense/kernel:0" in w and np.isfinite(w["dense/kernel:0"]).all()


# ------------------------------------------------------------------ checkpoint
def _engine():
    from pddl.models.reference import TorchEngine
    from pddl.models.resnet50 import ParamLayout
    e = TorchEngine(ParamLayout(), 1, crop=32)
    e.init(seed=3)
    return e


def test_keras_h5_roundtrip_and_layout(tmp_path):
    from pddl.train.optim import Adam
    from pddl.utils.checkpoint import h5, load_checkpoint, save_keras_h5
    e = _engine()
    opt = Adam(e, lr=1e-3)
    e.grads.normal_()
    opt.step()
    path = str(tmp_path / "ImageNet-ResNet50_ImageNet-reuse.h5")
    save_keras_h5(path, e, opt, _cfg("single"))
    m = h5()
    assert m.read_attr(path, "", "backend") == "tensorflow"
    mc = json.loads(m.read_attr(path, "", "model_config"))
    assert mc["config"]["layers"][4]["name"] == "resnet50"
    assert len([l for l in mc["config"]["layers"][4]["config"]["layers"] if l["class_name"] == "Conv2D"]) == 53
    assert m.read_attr(path, "model_weights", "layer_names") == ["input_1", "rescaling", "random_crop",
                                                                  "random_flip", "resnet50", "dense"]
    wn = m.read_attr(path, "model_weights/resnet50", "weight_names")
    assert len(wn) == 53 * 2 + 53 * 4 and wn[0] == "conv1_conv/kernel:0"
    k = m.read_dataset(path, "model_weights/resnet50/conv1_conv/kernel:0")
    assert k.shape == (7, 7, 3, 64)                                       # Keras HWIO
    assert m.read_dataset(path, "model_weights/dense/dense/kernel:0").shape == (2048, 1000)
    on = m.read_attr(path, "optimizer_weights", "weight_names")
    assert on[0] == "Adam/iter:0" and "Adam/conv1_conv/kernel/m:0" in on and len(on) == 1 + 2 * 214
    # round trip
    e2 = _engine()
    e2.params.zero_()
    opt2 = Adam(e2, lr=1e-3)
    load_checkpoint(path, e2, opt2)
    for ent in e.L.entries.values():      # (alignment padding between tensors is not saved)
        sl = slice(ent.offset, ent.offset + ent.size)
        assert torch.equal(e2.params[sl], e.params[sl]), ent.name
        if ent.trainable:
            assert torch.equal(opt2.m[sl], opt.m[sl]) and torch.equal(opt2.v[sl], opt.v[sl]), ent.name
    assert opt2.iterations == 1
    # h5dump sees the Keras group layout
    r = subprocess.run(["/opt/conda/bin/h5dump", "-n", path], capture_output=True, text=True)
    if r.returncode == 0:
        assert "/model_weights/resnet50/conv5_block3_3_bn/moving_variance:0" in r.stdout


def test_pretrained_weights_only_file(tmp_path):
    """The Keras applications `_notop.h5` layout (root layer_names, <layer>/<layer>/kernel:0)."""
    from pddl.utils.checkpoint import h5, load_pretrained
    e = _engine()
    L = e.L
    rng = np.random.default_rng(0)
    k = rng.standard_normal((7, 7, 3, 64)).astype(np.float32)
    g = rng.standard_normal(64).astype(np.float32)
    path = str(tmp_path / "notop.h5")
    h5().write(path, [("conv1_conv/conv1_conv/kernel:0", k), ("conv1_bn/conv1_bn/gamma:0", g)],
               [("", "layer_names", ["conv1_conv", "conv1_bn"]), ("conv1_conv", "weight_names",
                                                                  ["conv1_conv/kernel:0"]),
                ("conv1_bn", "weight_names", ["conv1_bn/gamma:0"])])
    n = load_pretrained(path, e)
    assert n == 2
    w = L.view(e.params, "conv1_conv", "kernel")        # OHWI
    assert np.allclose(w.permute(1, 2, 3, 0).numpy(), k)
    assert np.allclose(L.view(e.params, "conv1_bn", "gamma").numpy(), g)


# ------------------------------------------------------------------ entry scripts
@pytest.mark.parametrize("script,extra", [
    ("imagenet-resnet50.py", []),
    ("imagenet-resnet50-mirror.py", []),
])
def test_entry_script_trains_and_saves(tmp_path, script, extra):
    args = [sys.executable, os.path.join(ROOT, script), "--device", "cpu", "--epochs", "1", "--max-steps", "2",
            "--batch-size", "2", "--crop", "32", "--image-size", "32", "--save-dir", str(tmp_path),
            "--validation-steps", "1", "--verbose", "2"] + extra
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1/1" in r.stdout and "val_loss" in r.stdout
    assert any(f.endswith("-reuse.h5") for f in os.listdir(tmp_path)), os.listdir(tmp_path)


def test_ps_script_cli(tmp_path):
    args = [sys.executable, os.path.join(ROOT, "imagenet-resnet50-ps.py"), "--ps", "1", "--worker", "1",
            "--device", "cpu", "--epochs", "1", "--steps-per-epoch", "2", "--validation-steps", "1",
            "--batch-size", "2", "--crop", "32", "--image-size", "32", "--save-dir", str(tmp_path)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ImageNet-ResNet50_ImageNet_PS-reuse.h5" in os.listdir(tmp_path)


def test_resume_continues_epochs_lr_and_callbacks(tmp_path):
    """--resume of a periodic checkpoint restores weights + slots AND the progress (completed
    epochs, current LR, ReduceLROnPlateau / EarlyStopping bookkeeping): the resumed run starts
    at the next epoch with the LR the first run had reached."""
    base = [sys.executable, os.path.join(ROOT, "imagenet-resnet50.py"), "--device", "cpu", "--max-steps", "1",
            "--batch-size", "2", "--crop", "32", "--image-size", "32", "--save-dir", str(tmp_path),
            "--validation-steps", "1", "--verbose", "2", "--checkpoint-every", "1", "--no-save"]
    r = subprocess.run(base + ["--epochs", "2", "--lr", "0.0005"], capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    ck = tmp_path / "ckpt-002.h5"
    from pddl.utils.checkpoint import read_resume_state
    st = read_resume_state(str(ck))
    assert st["epoch"] == 2 and st["lr"] == 0.0005
    assert set(st["callbacks"]) >= {"ReduceLROnPlateau", "EarlyStopping"}
    r = subprocess.run(base + ["--epochs", "3", "--resume", str(ck)], capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Resuming after epoch 2 at lr 0.0005" in r.stdout
    assert "Epoch 3/3" in r.stdout and "Epoch 1/3" not in r.stdout and "lr: 0.0005" in r.stdout


def test_ps_stalled_worker_declared_dead_and_requeued(monkeypatch):
    """A LIVE worker stuck inside a step (hang_worker) stops heartbeating (the beacon stamps
    only while the main loop makes progress), is declared dead, its ticket is re-queued and
    the epoch completes; the stuck process ends itself after the step-stall threshold plus half
    the heartbeat timeout (before the coordinator can declare it dead)."""
    from pddl.parallel.parameter_server import run_ps_job
    monkeypatch.setenv("PDDL_FAULT", "hang_worker:1@1")
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "heartbeat", "3"))
    monkeypatch.setenv("PDDL_PS", with_opt("PDDL_PS", "step_stall", "3"))
    cfg = _cfg("ps", steps_per_epoch=6, batch_size=2, epochs=1)
    res = run_ps_job(cfg, num_ps=1, num_workers=2, return_results=True)
    wk = [r for r in res if r[0] == "worker"]
    ps = [r for r in res if r[0] == "ps"]
    assert len(wk) == 1 and wk[0][2] >= 5                    # worker 0 ran the re-queued ticket too
    assert ps[0][2] >= 6


def test_requeue_orphans_counts_each_lost_ticket_once():
    """Orphaned tickets are found from completion markers, not from what the dead worker wrote:
    a worker that died between its claim and its `cur` write still gets its ticket re-queued."""
    import torch.distributed as dist
    from pddl.parallel.parameter_server import requeue_orphans
    st = dist.HashStore()
    st.set("claim/0", "6/3")                 # tickets 0..5 claimed
    for t in (0, 1, 3, 5):
        st.set(f"tdone/0/{t}", "1")
    st.set("cur/4", "0:4")                   # live worker 4 holds ticket 4; ticket 2 is orphaned
    assert requeue_orphans(st, 0, [4]) == [2]
    assert st.add("requeue/0", 0) == 1
    assert requeue_orphans(st, 0, [4]) == []  # a second scan does not count it again
    assert st.add("requeue/0", 0) == 1


def test_requeue_orphans_scans_the_next_epoch():
    """A worker killed between its first claim of epoch e+1 and its `cur` write still shows
    `cur = e:-1`: the coordinator's scan starting at e must reach e+1's claims."""
    import torch.distributed as dist
    from pddl.parallel.parameter_server import requeue_orphans_from
    st = dist.HashStore()
    st.set("claim/0", "4/2")
    for t in range(4):
        st.set(f"tdone/0/{t}", "1")           # epoch 0 complete
    st.set("claim/1", "1/3")                  # the dead worker claimed ticket 0 of epoch 1 ...
    st.set("cur/3", "0:-1")                   # ... but its cur still names epoch 0
    assert requeue_orphans_from(st, 0, [4]) == {1: [0]}
    assert requeue_orphans_from(st, 0, [4]) == {}


def test_heartbeat_keeps_beating_through_a_slow_step():
    """The in-step stall threshold (PDDL_PS step_stall) is separate from the liveness timeout:
    a step longer than the heartbeat timeout but shorter than the stall threshold keeps the
    beacon stamping (a slow but healthy worker is not declared dead)."""
    import torch.distributed as dist
    from pddl.parallel.parameter_server import _Heartbeat
    st = dist.HashStore()
    hb = _Heartbeat(st, 5, 0.05, stall_s=5.0, hb_timeout=0.3)
    try:
        hb.step()
        t0 = float(st.get("hb/5").decode())
        time.sleep(0.8)                        # > hb_timeout, < stall_s
        assert hb.healthy() and float(st.get("hb/5").decode()) > t0 + 0.5
    finally:
        hb.stop()


def test_ps_resume_rejected(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "imagenet-resnet50-ps.py"), "--ps", "1", "--worker", "1",
                        "--resume", str(tmp_path / "x.h5"), "--device", "cpu"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2 and "--resume is not supported for --strategy ps" in r.stderr, r.stderr[-2000:]


def test_claim_block_shares_the_tail_and_requeue_sees_held_blocks():
    """Step tickets are claimed in blocks (one compare-and-set per block); near the end of the
    epoch the block shrinks to an even share of what is left; a live worker's claimed block
    (cur = <epoch>:<lo>:<hi>) is never re-queued, an unpublished block of a dead worker is."""
    import torch.distributed as dist
    from pddl.parallel.parameter_server import claim_block, requeue_orphans
    st = dist.HashStore()
    assert claim_block(st, 100, 0, 3, 16, 2) == (0, 16)
    assert claim_block(st, 100, 0, 4, 16, 2) == (16, 32)
    lo, hi = 32, 32
    while True:                                   # drain: blocks shrink to (left) // (2 * workers)
        a, b = claim_block(st, 100, 0, 3, 16, 2)
        if a < 0:
            break
        assert a == hi and b - a == max(1, min(16, (100 - a) // 4))
        lo, hi = a, b
    assert hi == 100
    for t in range(0, 16):
        st.set(f"tdone/0/{t}", "1")               # worker 3's first block published
    st.set("cur/4", "0:16:32")                    # live worker 4 still holds [16, 32)
    for t in range(32, 100):
        st.set(f"tdone/0/{t}", "1")
    assert requeue_orphans(st, 0, [4]) == []      # nothing orphaned while worker 4 lives
    assert requeue_orphans(st, 0, []) == list(range(16, 32))   # worker 4 died: its block comes back
    assert claim_block(st, 100, 0, 3, 16, 2)[0] == 100          # the re-queue extends the budget
