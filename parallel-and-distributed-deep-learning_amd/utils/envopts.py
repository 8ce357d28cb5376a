"""Grouped environment switches: one variable per subsystem holding "key=value" pairs.

    PDDL_ENGINE="fuse_bwd=0,c64=0"      engine fusion / schedule switches (models/engine.py)
    PDDL_PS="impl=c10d,heartbeat=5"     parameter-server runtime (parallel/parameter_server.py)
    PDDL_MIRROR="segmented=1"           in-process Mirrored schedule (parallel/strategies.py)

The keys each variable accepts, their defaults and meaning are listed in KEYS (and in the
README knob list); an unknown key raises, so a typo never silently runs the default.  Values
are read at use (tests set them per case); kernel tile knobs stay in PDDL_KNOBS
(ops/native.py)."""
from __future__ import annotations

import os
from typing import Dict

KEYS: Dict[str, Dict[str, str]] = {
    "PDDL_ENGINE": {
        "fuse_proj": "1: projection blocks' conv3 + shortcut as one dual-source GEMM",
        "fuse_bwd": "1: conv3 backward (dgrad + wgrad) in one launch at stages 2-3; 2: stage 2 only; 0: off",
        "fuse_bwd_s2": "1: ... also on the stride-2-grid blocks",
        "fuse_stem": "1: stem conv + BN + ReLU + max-pool in one launch (forward and backward)",
        "c64": "1: stage-2 3x3 convs on the row-tile kernels (conv3x3c64.hip)",
        "c64w": "1: ... and their weight gradient",
        "c64_min_m": "GEMM rows from which the row-tile kernels run (default 262144)",
        "c3c1": "1: stage-2 block boundaries as conv3 + next conv1 in one launch",
        "c1pre": "1: next block's conv1 dgrad inside the fused conv3 backward (stage 2)",
        "s2c": "1: blocks feeding a downsampling block store only their stride-2 grid",
        "bitmask": "1: ReLU masks as 1-bit masks (0: re-read the bf16 activation)",
        "grad_ring": "gradient buffers per kind of the two-stream backward (default 16 at b <= 64, else 5)",
        "two_stream": "auto: weight gradients on a side stream up to batch 1024; 1 / 0 force",
        "seg_side": "segmented graphs (Mirrored replicas): weight gradients in a side graph per segment (1, default) or one stream (0)",
    },
    "PDDL_PS": {
        "impl": "native: shm + HIP-IPC data plane (csrc/runtime/ps_service.cpp); c10d: process-group fallback",
        "heartbeat": "worker liveness timeout, s (default 30)",
        "step_stall": "in-step stall threshold, s (default max(300, 10 x heartbeat))",
        "epoch_timeout": "epoch drain deadline, s (default max(600, 10 x heartbeat))",
        "ticket_block": "step tickets claimed per control-plane round trip (default 16)",
        "timeout": "PS data-plane / process-group timeout, s (default 120)",
        "job_timeout": "whole-job deadline of run_ps_job, s (default 3600)",
    },
    "PDDL_MIRROR": {
        "segmented": "1: a one-replica job runs the multi-replica schedule (segmented graphs + all-reduce)",
        "overlap": "1: eager replicas all-reduce each bucket while backward continues (0: after it)",
        "pool": "1: graphed one-stream replicas launch each phase on the native launch pool (0: one thread)",
        "tail_cuts": "auto (batch >= 128) / 1 / 0: graphed replicas also cut a segment at every block of the last kernel bucket",
    },
}


def opts(var: str) -> Dict[str, str]:
    """The key=value pairs of `var` (validated against KEYS)."""
    out: Dict[str, str] = {}
    for item in os.environ.get(var, "").split(","):
        item = item.strip()
        if not item:
            continue
        k, sep, v = item.partition("=")
        k = k.strip()
        if not sep or k not in KEYS.get(var, {}):
            raise ValueError(f"{var}: unknown or malformed entry {item!r} (keys: {', '.join(KEYS.get(var, {}))})")
        out[k] = v.strip()
    return out


def opt(var: str, key: str, default=None):
    """Value of `key` in `var`, cast to the type of `default` (bool: "0" / "false" are False);
    `default` when unset."""
    assert key in KEYS[var], (var, key)
    v = opts(var).get(key)
    if v is None:
        return default
    if isinstance(default, bool):
        return v.lower() not in ("0", "false", "no", "off", "")
    if isinstance(default, int):
        return int(v)
    if isinstance(default, float):
        return float(v)
    return v


def with_opt(var: str, key: str, value) -> str:
    """The spec of `var` with `key` set to `value` (tests: monkeypatch.setenv(var, with_opt(...)))."""
    cur = opts(var)
    cur[key] = str(value)
    return ",".join(f"{k}={v}" for k, v in cur.items())
