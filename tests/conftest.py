import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")

import pddl  # noqa: E402,F401  (registers the package alias)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    has_gpu = torch.cuda.is_available()
    for it in items:
        if "gpu" in it.keywords and not has_gpu:
            it.add_marker(pytest.mark.skip(reason="no GPU"))


def pytest_sessionstart(session):
    # GPU runs: a fatal signal writes the native stack (HIP runtime / RCCL / extension frames) to
    # $PDDL_CRASH_TRACE (a file: pytest captures fd 2) before pytest's faulthandler prints the
    # Python ones (csrc/runtime/crash_trace.cpp)
    import torch
    if torch.cuda.is_available():
        from pddl.ops.native import native_available, require_native
        if native_available():
            require_native().install_crash_trace(os.environ.get("PDDL_CRASH_TRACE", ""))
            # kernel-equivalence tests switch tile knobs between launches (tuning mode; a training
            # process may not: knobs freeze at its first launch, tests/test_gpu_kernels.py)
            require_native().allow_knob_changes(True)
