"""Trace ranges for rocprofv3 (roctx ranges around forward / backward /
communication / optimizer; the reference has no tracing beyond `time.time()` around fit,
imagenet-resnet50-hvd.py:119-126).

Enabled with `PDDL_ROCTX=1` (or `--roctx`); otherwise every call is a cheap no-op.  The
ranges come from the ROCm profiler SDK's roctx library, so

    PDDL_ROCTX=1 rocprofv3 --marker-trace --kernel-trace -d gpurun_out/m -- python bench.py

records one `step/forward`, `step/backward`, `step/allreduce`, `step/optimizer` span per step
next to the kernel dispatches.  The fusion engine's own chrome-trace timeline (`--timeline`)
covers the per-bucket communication phases.
"""
from __future__ import annotations

import ctypes
import os
from contextlib import contextmanager

_lib = None
_enabled = os.environ.get("PDDL_ROCTX", "0") not in ("", "0")


def _load():
    global _lib
    if _lib is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                     "libroctx64.so"):
            try:
                lib = ctypes.CDLL(os.path.join("/opt/rocm/lib", name))
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
        if _lib is None:
            _lib = False
    return _lib or None


def enable(on: bool = True) -> bool:
    """Turn ranges on (returns False when no roctx library is present)."""
    global _enabled
    _enabled = bool(on) and _load() is not None
    return _enabled


def enabled() -> bool:
    return _enabled


def push(name: str) -> None:
    if _enabled and _load() is not None:
        _lib.roctxRangePushA(name.encode())


def pop() -> None:
    if _enabled and _load() is not None:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled and _load() is not None:
        _lib.roctxMarkA(name.encode())


@contextmanager
def trace_range(name: str):
    push(name)
    try:
        yield
    finally:
        pop()
