"""bench.py launch contract (the driver's N-GPU scaling run, BASELINE.json): --gpus N really
runs N ranks / replicas, refuses to mis-measure, and prints one JSON line with n_gpus == N.
CPU: the ranks are gloo processes running the fp32 reference engine (tiny images)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--steps", "1", "--warmup", "1", "--batch", "2", "--image-size", "32"]


def _bench(*args, env=None, timeout=600):
    e = dict(os.environ, **(env or {}))
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=timeout)
    return r


def _json(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    return json.loads(lines[0])


def test_cpu_two_ranks_spawned():
    r = _bench("--gpus", "2", *SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r)
    assert out["n_gpus"] == 2 and out["config"]["replicas"] == 2 and out["config"]["global_batch"] == 4
    assert out["config"]["parallelism"] == "dp2" and "FusionEngine" in out["config"]["strategy"]
    assert out["value"] > 0 and out["steps"] == 1


def test_cpu_mirrored_two_replicas_in_process():
    r = _bench("--gpus", "2", "--strategy", "mirrored", *SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r)
    assert out["n_gpus"] == 2 and out["config"]["replicas"] == 2 and "mirrored" in out["config"]["strategy"]


def test_cpu_multiworker_two_procs_two_local():
    r = _bench("--gpus", "4", "--strategy", "multiworker", "--local-gpus", "2", *SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r)
    assert out["n_gpus"] == 4 and out["config"]["replicas"] == 4


def test_refuses_more_gpus_than_visible():
    r = _bench("--gpus", "8", "--steps", "1", timeout=120)
    assert r.returncode != 0 and "GPU(s) are visible" in r.stderr


def test_refuses_world_mismatch():
    e = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "rank(s)" in r.stderr


def test_cpu_parameter_server_bench():
    """--strategy ps: P PS + W worker role processes (BASELINE config 5's layout, here 1 + 2 on CPU),
    one JSON line with the aggregate worker images/sec of the timed epoch."""
    r = _bench("--gpus", "3", "--strategy", "ps", "--ps", "1", "--device", "cpu", "--steps", "4", "--batch", "2",
               "--image-size", "32")
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r)
    assert out["n_gpus"] == 3 and out["config"]["parallelism"] == "ps1+w2" and out["steps_timed_epoch"] == 4
    assert out["value"] > 0
