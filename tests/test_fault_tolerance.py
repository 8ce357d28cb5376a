"""Failure detection on the synchronous multi-rank paths (the reference's
fail-fast intent, imagenet-resnet50-ps.py:67-69, and Horovod's stall inspector behind
hvd.DistributedOptimizer, imagenet-resnet50-hvd.py:101): a stuck or dead rank must turn
`bench.py --gpus N` into a bounded, non-zero exit that names what happened -- never a job that
hangs until an outside limit kills it.  CPU, gloo rank processes (tiny images)."""
import os
import shutil
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--steps", "3", "--warmup", "1", "--batch", "2", "--image-size", "32"]


def _bench(*args, env=None, timeout=300):
    e = dict(os.environ, **(env or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PDDL_FAULT", "PDDL_STALL_TIMEOUT", "PDDL_STALL_SHUTDOWN"):
        e.pop(k, None)
    e.update(env or {})
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=timeout)
    return r, time.time() - t0


def test_hung_rank_caught_by_stall_watchdog():
    """hang_rank:1@3 -> rank 0's bucket all-reduce stalls; the fusion engine's stall inspector
    raises within PDDL_STALL_TIMEOUT, the rank fails fast, the launcher stops rank 1."""
    r, dt = _bench("--gpus", "2", *SMALL, env={"PDDL_FAULT": "hang_rank:1@3", "PDDL_STALL_TIMEOUT": "5"})
    assert r.returncode != 0
    assert "stall detected" in r.stderr and "bucket 0" in r.stderr, r.stderr[-3000:]
    assert "rank 1" in r.stderr and "last progress" in r.stderr
    assert dt < 120, dt


def test_hung_rank_caught_by_job_deadline():
    """Same hang with the stall watchdog disabled: the job deadline (--timeout) ends every rank
    with a stack dump, and the launcher reports each rank's last phase."""
    r, dt = _bench("--gpus", "2", *SMALL, "--timeout", "40",
                   env={"PDDL_FAULT": "hang_rank:1@3", "PDDL_STALL_TIMEOUT": "0"})
    assert r.returncode != 0
    assert "Timeout" in r.stderr and "faults.py" in r.stderr, r.stderr[-3000:]   # the hung rank's stack
    assert "last progress: timed step" in r.stderr, r.stderr[-3000:]
    assert dt < 40 + 60, dt


def test_dead_rank_stops_the_job():
    """kill_rank:1@2 -> rank 1 exits 17; the launcher stops rank 0 (stuck in the collective) at
    once and exits non-zero."""
    r, dt = _bench("--gpus", "2", *SMALL, env={"PDDL_FAULT": "kill_rank:1@2", "PDDL_STALL_TIMEOUT": "120"})
    assert r.returncode != 0
    assert "rank 1 exited with status 17" in r.stderr, r.stderr[-3000:]
    assert dt < 120, dt


def test_mirrored_replica_hang_bounded_by_deadline():
    """The in-process Mirrored job (one process, R replicas) is bounded by the same deadline."""
    r, dt = _bench("--gpus", "2", "--strategy", "mirrored", *SMALL, "--timeout", "30",
                   env={"PDDL_FAULT": "hang_rank:0@2"})
    assert r.returncode != 0 and "Timeout" in r.stderr, r.stderr[-2000:]
    assert dt < 30 + 60, dt


def test_fault_spec_parsing():
    from pddl.parallel import faults
    assert faults.parse("kill_worker:1@3, hang_rank:0@2") == [("kill_worker", 1, 3), ("hang_rank", 0, 2)]
    with pytest.raises(ValueError):
        faults.parse("explode:1@2")


def test_no_silent_device_wraparound(monkeypatch):
    """A rank whose local index exceeds the visible GPUs fails with a clear message instead of
    sharing another rank's device (rehearsals opt in with PDDL_REHEARSE=1)."""
    import torch
    from pddl.config import make_config
    from pddl.parallel.strategies import SingleStrategy
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    picked = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda i: picked.append(i))
    st = SingleStrategy(make_config("single", device="cuda"))
    assert st._pick_device(1).index == 1
    monkeypatch.delenv("PDDL_REHEARSE", raising=False)
    with pytest.raises(RuntimeError, match="only 2 GPU"):
        st._pick_device(3)
    monkeypatch.setenv("PDDL_REHEARSE", "1")
    assert st._pick_device(3).index == 1


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_native_comm_watchdog_core(tmp_path):
    """runtime/comm_watch.h (the RCCL communicator's stall watchdog) natively: collectives retired
    in order without false alarms, a hung one reported once with its tag, abort run once."""
    exe = tmp_path / "cw"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "csrc"),
                    os.path.join(ROOT, "csrc", "tests", "comm_watch_test.cpp"), "-lpthread", "-o", str(exe)],
                   check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "comm_watch_test: ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.exists("/opt/rocm/llvm/bin/clang++"), reason="no clang (TSan runtime)")
def test_native_launch_pool_under_tsan(tmp_path):
    """runtime/launch_pool.h (the Mirrored graphed step's per-device launch threads) under
    ThreadSanitizer: runs of changing width (late-joining workers never replay a finished run),
    plain per-task writes read by the caller after run(), concurrent callers."""
    exe = tmp_path / "lp"
    subprocess.run(["/opt/rocm/llvm/bin/clang++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I",
                    os.path.join(ROOT, "csrc"), os.path.join(ROOT, "csrc", "tests", "launch_pool_test.cpp"),
                    "-lpthread", "-o", str(exe)], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "launch_pool_test: ok" in r.stdout, r.stdout + r.stderr[-3000:]

