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


def test_scaling_efficiency_arithmetic():
    """utils/scaling.py: efficiency = ips(N) / (N * ips(1)), speedup = ips(N) / ips(1)."""
    sys.path.insert(0, ROOT)
    from pddl.utils.scaling import efficiency, format_table, scaling_table
    assert efficiency(7600.0, 8, 1000.0) == pytest.approx(0.95)
    assert efficiency(100.0, 2, None) is None and efficiency(100.0, 2, 0.0) is None
    t = scaling_table({1: 1000.0, 2: 1900.0, 4: 3600.0, 8: 7200.0})
    assert [r["n_gpus"] for r in t] == [1, 2, 4, 8]
    assert [r["efficiency"] for r in t] == [1.0, 0.95, 0.9, 0.9]
    assert [r["speedup"] for r in t] == [1.0, 1.9, 3.6, 7.2] and t[3]["per_gpu_images_per_sec"] == 900.0
    t2 = scaling_table({2: 1900.0}, ips_1=1000.0)
    assert t2[0]["efficiency"] == 0.95
    assert scaling_table({2: 1900.0})[0]["efficiency"] is None
    assert "efficiency" in format_table(t)


def test_bench_baseline_ips_fills_efficiency():
    r = _bench("--gpus", "2", *SMALL, "--baseline-ips", "10")
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r)
    assert out["baseline_ips"] == 10.0
    assert out["vs_baseline"] == pytest.approx(out["value"] / 10.0, rel=1e-3)
    assert out["scaling_efficiency"] == pytest.approx(out["value"] / 20.0, rel=1e-3)
    assert "scaling_efficiency" not in _json(_bench(*SMALL))


def test_bench_scaling_script_cpu():
    """bench/scaling.py: fresh bench.py children at N = 1 and 2 (gloo CPU ranks under
    torch.distributed.run), per-N rows, efficiency 1.0 at N = 1, JSON summary schema."""
    out_path = os.path.join(ROOT, "gpurun_out", "test_scaling_cpu.json")
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "scaling.py"), "--gpus", "1", "2",
                        "--steps", "1", "--warmup", "1", "--out", out_path, "--",
                        "--device", "cpu", "--batch", "2", "--image-size", "32"],
                       cwd=ROOT, env=e, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    summary = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
    rows = {row["n_gpus"]: row for row in summary["rows"]}
    assert set(rows) == {1, 2} and rows[1]["efficiency"] == 1.0 and rows[1]["speedup"] == 1.0
    assert summary["baseline_ips"] == rows[1]["images_per_sec"]
    assert rows[2]["efficiency"] == pytest.approx(rows[2]["images_per_sec"] / (2 * rows[1]["images_per_sec"]),
                                                  abs=1e-3)
    saved = json.load(open(out_path))
    assert saved["runs"]["2"]["n_gpus"] == 2 and saved["runs"]["1"]["n_gpus"] == 1
