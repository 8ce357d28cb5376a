"""Native runtime on the GPU: RCCL communicator, fusion engine over c10d/RCCL, strategies
driving the HIP engine end to end (1 GPU box: single-rank communicators)."""
import os

import pytest

from pddl.utils.envopts import with_opt
import torch

pytestmark = pytest.mark.gpu


def test_rccl_comm_single_device():
    from pddl.ops.native import require_native
    N = require_native()
    comm = N.RcclComm.init_all([0])
    t = torch.arange(1024, dtype=torch.float32, device="cuda")
    comm.all_reduce([t], "sum")
    comm.broadcast([t], 0)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(1024, dtype=torch.float32, device="cuda"))
    assert comm.nranks == 1 and comm.async_error() == ""
    uid = N.RcclComm.unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128


def test_fusion_engine_over_rccl_process_group():
    import torch.distributed as dist
    from pddl.ops.native import require_native
    from pddl.parallel.launch import pick_unused_port
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(pick_unused_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import json
        for wire in ("fp32", "bf16"):
            g = torch.randn(10000, device="cuda")
            ref = g.clone()
            fe = require_native().FusionEngine(dist.group.WORLD, g, [(0, 4000), (4000, 6000)], 10.0, False, 0, wire)
            fe.set_timeline(True)
            for _ in range(3):
                fe.begin_step()
                g.mul_(1.0)              # kernel on the compute stream the buckets depend on
                fe.bucket_ready(0)
                g[4000:].mul_(1.0)       # bucket 1 completes later
                fe.bucket_ready(1)
                fe.finish()
            torch.cuda.synchronize()
            assert fe.issued == 6 and fe.wire == wire
            if wire == "fp32":
                assert torch.equal(g, ref)
            else:   # one rank: the bf16 round trip is the only change
                assert torch.equal(g, ref.to(torch.bfloat16).float())
            # GPU-stamped timeline: every ALLREDUCE span starts after its bucket's READY event
            ev = json.loads(fe.timeline_json())
            ready = {(e["args"]["step"], e["tid"]): e["ts"] for e in ev if e["name"] == "READY"}
            spans = [e for e in ev if e["name"] == "ALLREDUCE"]
            assert len(spans) == 6 and len(ready) == 6
            for e in spans:
                assert e["args"]["clock"] == "gpu" and e["dur"] >= 0
                assert e["ts"] >= ready[(e["args"]["step"], e["tid"])] - 1.0   # (us rounding)
            fe.shutdown()
    finally:
        dist.destroy_process_group()


def _cfg(preset, **kw):
    from pddl.config import make_config
    base = dict(device="cuda", data="synthetic", image_size=224, crop=224, epochs=1, max_steps=3, verbose=0,
                save=False, train_images=256, val_images=64, batch_size=16, validation_steps=1)
    base.update(kw)
    return make_config(preset, **base)


def test_single_strategy_fit_and_checkpoint_on_gpu(tmp_path):
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    from pddl.utils.checkpoint import load_checkpoint, save_keras_h5
    cfg = _cfg("single")
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    h = tr.fit(1, [])
    assert type(st.engine).__name__ == "HipEngine"
    assert all(map(lambda v: v == v, h.history["loss"]))
    path = str(tmp_path / "ckpt.h5")
    save_keras_h5(path, st.engine, st.opt, cfg)
    st2 = make_strategy(cfg)
    Trainer(cfg, st2)
    load_checkpoint(path, st2.engine, st2.opt)
    for e in st.engine.L.entries.values():
        sl = slice(e.offset, e.offset + e.size)
        assert torch.equal(st.engine.params[sl].cpu(), st2.engine.params[sl].cpu()), e.name


def test_single_strategy_fit_with_hip_graph():
    """--graphs: the Keras fit loop replays the captured step (random crop offsets and flips
    flow through device buffers); the run trains and the step count stays Keras-exact."""
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    cfg = _cfg("single", graphs=True, crop=192, max_steps=5)
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    h = tr.fit(1, [])
    assert st.graphed is not None and st.graphed.graph is not None
    assert st.opt.iterations == 5
    assert all(map(lambda v: v == v, h.history["loss"]))


def test_mirrored_strategy_one_gpu_uses_rccl(monkeypatch):
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    monkeypatch.setenv("PDDL_MIRROR", with_opt("PDDL_MIRROR", "segmented", "1"))   # (the multi-replica schedule on 1 GPU)
    cfg = _cfg("mirrored")
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    h = tr.fit(1, [])
    assert st.mirror.comm is not None and st.num_replicas_in_sync == torch.cuda.device_count()
    assert h.history["loss"][0] == h.history["loss"][0]
    assert len(st.mirror.buckets) >= 2          # bucketed all-reduce overlapped with backward ran


def test_single_strategy_train_mode_bn_on_hip():
    from pddl.models.engine_bn import HipEngineBNTrain
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    cfg = _cfg("single", bn_mode="train")
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    h = tr.fit(1, [])
    assert isinstance(st.engine, HipEngineBNTrain)
    assert h.history["loss"][0] == h.history["loss"][0]


@pytest.mark.parametrize("segmented", [True, False])
def test_mirrored_graphed_step_matches_eager(monkeypatch, segmented):
    """Mirrored with HIP graphs follows the eager Mirrored trajectory.  segmented: the
    multi-replica schedule (per-device step segments split at the gradient buckets, with the
    two-stream backward, grouped all-reduce of bucket k between segment k and k+1, captured
    optimizer), forced on this 1-replica job with PDDL_MIRROR segmented=1; otherwise the
    1-replica job's whole-step graph (no collective to run)."""
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    if segmented:
        monkeypatch.setenv("PDDL_MIRROR", with_opt("PDDL_MIRROR", "segmented", "1"))
    res = []
    for graphs in (False, True):
        cfg = _cfg("mirrored", graphs=graphs, flip=False, max_steps=3, batch_size=8)
        st = make_strategy(cfg)
        tr = Trainer(cfg, st)
        h = tr.fit(1, [], validation=False)
        res.append((h.history["loss"][0], st.engine.params.clone(), st.opt.iterations))
        assert st.mirror.graph_mode == graphs
        if graphs and segmented:
            g = st.mirror.graphs[0]
            assert g.captured and len(g.segments) == len(st.mirror.buckets) >= 2
            # (the weight gradients replay as a side graph per segment: HipEngine._side_run)
            assert g.deferred and any(x is not None for x in g.side_segments)
            assert st.mirror.comm.watchdog_state()["issued"] >= 2 * len(st.mirror.buckets)
        elif graphs:
            assert st.mirror.graphs is None and st.mirror._whole.graph is not None
    (l0, p0, i0), (l1, p1, i1) = res
    assert i0 == i1 == 3
    assert abs(l0 - l1) <= 1e-3 * abs(l0)
    assert ((p0 - p1).norm() / p0.norm()).item() < 2e-3


class _SumComm:
    """In-process sum of the replicas' buckets (all on device 0) on the comm streams: the
    stand-in for the grouped RCCL all-reduce when R replicas share one GPU."""
    nranks = 2

    def all_reduce_on(self, ts, op, streams, what):
        ss = [torch.cuda.ExternalStream(s) for s in streams]
        for s in ss[1:]:
            ss[0].wait_stream(s)
        with torch.cuda.stream(ss[0]):
            tot = ts[0].clone()
            for t in ts[1:]:
                tot += t
            for t in ts:
                t.copy_(tot)
        for s in ss[1:]:
            s.wait_stream(ss[0])

    def check(self):
        pass


@pytest.mark.parametrize("R,side", [(2, "1"), (3, "1"), (2, "0")])
def test_graphed_replicas_match_eager_replicas(monkeypatch, R, side):
    """R graphed replicas (segments, events and comm-stream waits issued by one native group
    launch per phase) train like R eager replicas: R replicas on device 0, each with its own
    launch stream, gradients summed per bucket on the comm streams.  side "1" (default): each
    segment's weight gradients replay as a single-stream side graph after it, concurrently with
    the next segment (HipEngine._side_run deferred); "0": one stream."""
    from pddl.parallel.strategies import _LocalReplicas
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "seg_side", side))
    B = 8
    g = torch.Generator(device="cuda").manual_seed(3)
    images = [torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(R)]
    labels = [torch.randint(0, 1000, (B,), dtype=torch.int64, device="cuda", generator=g) for _ in range(R)]
    out = []
    for graphed in (False, True):
        lr = _LocalReplicas(_cfg("mirrored", flip=False, batch_size=B, graphs=graphed, lr=1e-4), [0] * R)
        lr.broadcast()                              # (no communicator yet: in-process copies)
        lr.comm = _SumComm()
        lr.graph_mode = graphed
        lr.launch_streams = [torch.cuda.Stream() for _ in range(R)]
        losses = [lr.step(images, labels, B * R)[0].item() for _ in range(4)]
        torch.cuda.synchronize()
        if graphed:
            assert len(lr.graphs) == R and len(lr.buckets) >= 2
            assert lr.deferred == (side == "1")
            assert all(any(x is not None for x in g.side_segments) == (side == "1") for g in lr.graphs)
        assert all(o.iterations == 4 for _, o in lr.replicas)
        ps = [e.params.clone() for e, _ in lr.replicas]
        for p in ps[1:]:
            assert ((p - ps[0]).norm() / ps[0].norm()).item() < 1e-6   # replicas stay in sync
        out.append((losses, ps[0]))
        if graphed:
            # a batch-size change (the epoch's last partial batch) re-captures: the group launches
            # must replay the new graphs, never the freed ones (the launch plan is rebuilt).
            # (every graph is single-stream: re-capturing multi-branch ones is the runtime-fault trigger)
            half = [im[: B // 2] for im in images], [lb[: B // 2] for lb in labels]
            for _ in range(2):
                assert torch.isfinite(lr.step(half[0], half[1], B // 2 * R)).all()
            assert lr.graphs[0].B == B // 2
            for _ in range(2):
                assert torch.isfinite(lr.step(images, labels, B * R)).all()
            torch.cuda.synchronize()
            assert lr.graphs[0].B == B and all(o.iterations == 8 for _, o in lr.replicas)
    # (the weight-gradient atomics make runs differ in the last bits)
    for a, b in zip(out[0][0], out[1][0]):
        assert abs(a - b) <= 1e-3 * abs(a), (out[0][0], out[1][0])
    assert ((out[0][1] - out[1][1]).norm() / out[0][1].norm()).item() < 2e-3


def _bench_json(args, env):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, **env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], cwd=root, env=e,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("strategy", ["horovod", "mirrored"])
def test_bench_two_rank_rehearsal_on_one_gpu(strategy):
    """bench.py --gpus 2 on one GPU (PDDL_REHEARSE=1: ranks share device 0, gloo instead of
    RCCL): the multi-rank launch path runs end to end and reports n_gpus 2."""
    out = _bench_json(["--gpus", "2", "--strategy", strategy, "--batch", "32", "--steps", "2", "--warmup", "1"],
                      {"PDDL_REHEARSE": "1"})
    assert out["n_gpus"] == 2 and out["config"]["replicas"] == 2 and out["rehearsal"] is True
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"]


def test_bench_mirrored_one_gpu_graphed():
    """The in-process Mirrored bench on 1 GPU runs RCCL + segmented HIP graphs."""
    out = _bench_json(["--gpus", "1", "--strategy", "mirrored", "--batch", "64", "--steps", "3", "--warmup", "2"], {})
    assert out["n_gpus"] == 1 and out["config"]["hip_graph"] is True and "rehearsal" not in out


def test_rccl_comm_init_rank_constructor_and_watchdog():
    """The multi-process constructor (ncclCommInitRank for every local rank inside one group --
    MWMS's P x R layout, imagenet-resnet50-multiworkers.py:20-26) with nranks=1: collectives on
    explicit streams, what RCCL reports it built, and the stall watchdog retiring every
    collective without a false alarm."""
    import time
    from pddl.ops.native import require_native
    N = require_native()
    comm = N.RcclComm(1, N.RcclComm.unique_id(), [0], [0])
    info = comm.info()
    assert len(info) == 1 and info[0]["nranks"] == 1 and info[0]["rank"] == 0 and info[0]["device"] == 0
    assert info[0]["pci_bus_id"]
    comm.set_watchdog(20.0, 0.0, 0)
    side = torch.cuda.Stream()
    t = torch.arange(4096, dtype=torch.float32, device="cuda")
    ref = t.clone()
    side.wait_stream(torch.cuda.current_stream())
    for k in range(8):
        comm.all_reduce_on([t], "sum", [side.cuda_stream], f"bucket {k} all_reduce")
    torch.cuda.current_stream().wait_stream(side)
    comm.broadcast([t], 0)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    t0 = time.time()
    while comm.watchdog_state()["retired"] < 9 and time.time() - t0 < 10:
        time.sleep(0.05)
    st = comm.watchdog_state()
    assert st["armed"] and st["issued"] == 9 and st["retired"] == 9 and not st["stalled"], st
    comm.check()
    comm.abort()
    with pytest.raises(RuntimeError, match="aborted"):
        comm.all_reduce([t], "sum")


def test_mirrored_on_init_rank_communicator(monkeypatch):
    """The whole graphed Mirrored / MWMS replica driver on the ncclCommInitRank communicator
    (PDDL_RCCL_INIT=rank), with its bucket collectives under the watchdog."""
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    monkeypatch.setenv("PDDL_RCCL_INIT", "rank")
    monkeypatch.setenv("PDDL_MIRROR", with_opt("PDDL_MIRROR", "segmented", "1"))
    cfg = _cfg("mirrored", max_steps=4, batch_size=8)
    st = make_strategy(cfg)
    tr = Trainer(cfg, st)
    h = tr.fit(1, [], validation=False)
    comm = st.mirror.comm
    assert comm is not None and comm.info()[0]["nranks"] == 1
    assert h.history["loss"][0] == h.history["loss"][0]
    torch.cuda.synchronize()
    ws = comm.watchdog_state()
    # (step 1 runs eager, then 3 graphed steps: one collective per segment bucket each)
    assert ws["armed"] and ws["issued"] >= 3 * len(st.mirror.buckets) and not ws["stalled"], ws


def test_bench_parameter_server_rehearsal_on_one_gpu():
    """BASELINE config 5's code path on the GPU: bench.py --strategy ps with 1 PS + 2 workers as
    three processes sharing the card (PDDL_REHEARSE=1) over the native HIP-IPC data plane --
    event-chained PS service (Adam + snapshot copy per request, `done` published on event
    completion) and the workers' poster threads (no host sync on push)."""
    out = _bench_json(["--gpus", "3", "--strategy", "ps", "--ps", "1", "--batch", "32", "--steps", "8"],
                      {"PDDL_REHEARSE": "1", "PDDL_PS": "impl=native"})
    assert out["n_gpus"] == 3 and out["config"]["parallelism"] == "ps1+w2" and out["rehearsal"] is True
    assert out["steps_timed_epoch"] == 8 and out["value"] > 0


_HUNG_RCCL = r"""
import sys, time, torch
sys.path.insert(0, sys.argv[1])
import pddl
from pddl.ops.native import require_native
N = require_native()
comm = N.RcclComm(1, N.RcclComm.unique_id(), [0], [0])
comm.set_watchdog(0.5, 4.0, 0, True)      # abort on stall, exit 124 four seconds after the verdict
t = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
torch.cuda._sleep(4_000_000_000)          # a bounded spin (~2 s) holds the stream: the collective
comm.all_reduce([t], "sum", "bucket 7 all_reduce")   # queued behind it cannot complete in time
t0 = time.time()
while True:
    try:
        comm.check()
    except RuntimeError as e:
        print(f"verdict after {time.time() - t0:.2f} s: {e}", flush=True)
        break
    if time.time() - t0 > 10:
        print("no verdict", flush=True)
        sys.exit(3)
    time.sleep(0.05)
st = comm.watchdog_state()
print("state", st, flush=True)
time.sleep(30)                            # the watchdog's shutdown deadline ends the process
sys.exit(4)
"""


def test_rccl_watchdog_aborts_a_hung_collective_and_exits_124(tmp_path):
    """The native communicator's stall path on the GPU: a collective queued behind a
    bounded spin kernel misses the 0.5 s stall timeout -> the verdict names its bucket, the
    abort action (on its own thread, lock-bounded) aborts the communicator, and the watchdog's
    shutdown deadline ends the rank with exit 124 in bounded time, whatever the main thread
    is doing.  (Two RCCL ranks cannot share one GPU, so a hung PEER is modelled by the spin.)"""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "hung_rccl.py"
    script.write_text(_HUNG_RCCL)
    t0 = time.time()
    r = subprocess.run([sys.executable, str(script), root], cwd=root, capture_output=True, text=True, timeout=90)
    dt = time.time() - t0
    assert r.returncode == 124, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "verdict after" in r.stdout and "bucket 7 all_reduce" in r.stdout, r.stdout
    assert "aborting 1 local RCCL communicator" in r.stderr, r.stderr[-2000:]
    assert dt < 60, dt


def test_comm_proxy_holds_its_duration_and_leaves_the_gradient():
    """bench --comm-proxy's stand-in collective: the paced kernel runs for its modelled duration
    (within launch overhead), streams the bucket into scratch, and never writes the gradient."""
    import time
    from pddl.ops.native import require_native
    N = require_native()
    g = torch.randn(1 << 22, device="cuda")
    ref = g.clone()
    scratch = torch.zeros_like(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    N.comm_proxy(g, scratch, 2, 2_000_000, 32)      # 20 ms at 100 MHz
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert 0.019 < dt < 0.2, dt
    assert torch.equal(g, ref) and torch.equal(scratch, g)


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_mirrored_segmented_wire_and_timeline_over_one_rank_communicator(monkeypatch, tmp_path, wire):
    """The multi-replica schedule (PDDL_MIRROR segmented=1: bucket-segmented graphs, each
    bucket all-reduced on the native RCCL communicator between the segment replays, fp32 or bf16
    wire) at the reference's batch 32 (crop 160) follows the eager one-replica step, and its
    timeline has a READY and an ALLREDUCE per bucket (imagenet-resnet50-mirror.py:21,54)."""
    import json
    from pddl.parallel.strategies import make_strategy
    from pddl.train.trainer import Trainer
    res = []
    for seg in ("1", "0"):
        monkeypatch.setenv("PDDL_MIRROR", with_opt("PDDL_MIRROR", "segmented", seg))
        tl = str(tmp_path / "tl")
        cfg = _cfg("mirrored", flip=False, max_steps=4, batch_size=32, crop=160, lr=1e-3, grad_dtype=wire,
                   timeline=tl if seg == "1" else None)
        st = make_strategy(cfg)
        tr = Trainer(cfg, st)
        h = tr.fit(1, [], validation=False)
        res.append((h.history["loss"][0], st.engine.params.clone(), st.opt.iterations))
        m = st.mirror
        if seg == "1":
            assert m.graph_mode and m.graphs is not None and m.comm.nranks == 1
            assert (m.lowp is not None) == (wire == "bf16")
            st.write_timeline(tl)
            ev = json.loads(open(f"{tl}.rank0.json").read())
            nb = len(m.buckets)
            assert sum(e["name"] == "READY" for e in ev) == nb and sum(e["name"] == "ALLREDUCE" for e in ev) == nb
            assert all(e["dur"] >= 0 for e in ev if e["name"] == "ALLREDUCE")
        else:
            assert m.graphs is None
    (l0, p0, i0), (l1, p1, i1) = res
    assert i0 == i1 == 4
    if wire == "fp32":
        assert abs(l0 - l1) <= 1e-3 * abs(l1)
        assert ((p0 - p1).norm() / p1.norm()).item() < 2e-3
    else:   # (the bf16 round trip of the gradient is the one difference on one rank)
        assert l0 == l0 and abs(l0 - l1) <= 2e-2 * abs(l1)
