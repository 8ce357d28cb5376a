"""Fault injection for the failure-detection tests.

The reference has no fault injection; its failure handling is GRPC_FAIL_FAST=use_caller for
the PS (imagenet-resnet50-ps.py:67-69) and Horovod's stall inspector behind
hvd.DistributedOptimizer (imagenet-resnet50-hvd.py:101) [lib].  These hooks let the tests
prove that every strategy turns a dead or stuck rank into a bounded, non-zero exit:

  PDDL_FAULT=kill_worker:<i>@<step>   PS worker i exits (status 17) at its step-th step
  PDDL_FAULT=hang_worker:<i>@<step>   PS worker i stops forever inside its step-th step (its
                                      heartbeat stops; the coordinator re-queues its ticket)
  PDDL_FAULT=kill_rank:<r>@<step>     sync-strategy rank r exits (status 17) before step `step`
  PDDL_FAULT=hang_rank:<r>@<step>     sync-strategy rank r stops forever before step `step`
                                      (its peers block in the next collective)

Several specs may be joined with commas.
"""
from __future__ import annotations

import os
import sys
import time
from typing import List, Optional, Tuple


def parse(spec: Optional[str] = None) -> List[Tuple[str, int, int]]:
    spec = os.environ.get("PDDL_FAULT", "") if spec is None else spec
    out = []
    for part in filter(None, (p.strip() for p in spec.split(","))):
        kind, _, rest = part.partition(":")
        who, _, at = rest.partition("@")
        if kind not in ("kill_worker", "hang_worker", "kill_rank", "hang_rank") or not who or not at:
            raise ValueError(f"PDDL_FAULT: cannot parse {part!r} (kind:<rank>@<step>)")
        out.append((kind, int(who), int(at)))
    return out


def ps_fault(worker_index: int) -> Optional[Tuple[str, int]]:
    for kind, who, at in parse():
        if kind in ("kill_worker", "hang_worker") and who == worker_index:
            return kind, at
    return None


class StepFaults:
    """Per-rank step counter of a synchronous strategy; `tick()` runs before every train step."""

    def __init__(self, rank: int):
        self.rank = rank
        self.step = 0
        self.plan = [(k, at) for k, who, at in parse() if who == rank and k in ("kill_rank", "hang_rank")]

    def tick(self):
        if self.plan:
            for kind, at in self.plan:
                if self.step == at:
                    sys.stderr.write(f"[pddl fault] rank {self.rank}: injected {kind} at step {self.step}\n")
                    sys.stderr.flush()
                    if kind == "kill_rank":
                        os._exit(17)
                    while True:        # hang_rank: never returns (the watchdogs must end the job)
                        time.sleep(3600)
        self.step += 1


def run_fail_fast(fn, *a, multi=None, **kw):
    """Run `fn`; if it raises inside a multi-rank job, print the traceback and end the process at
    once (os._exit(1)) instead of unwinding: the destructors of a process group / fusion engine
    with a collective still outstanding would block interpreter shutdown on the dead peer, and
    the launcher (torchrun, bench.py) stops the other ranks as soon as this one exits non-zero
    (the reference's fail-fast intent, imagenet-resnet50-ps.py:67-69)."""
    try:
        return fn(*a, **kw)
    except BaseException as e:     # noqa: BLE001  (SystemExit of a clean refusal passes through)
        if multi is None:
            multi = int(os.environ.get("WORLD_SIZE", "1")) > 1
        if isinstance(e, SystemExit) or not multi:
            raise
        import traceback
        traceback.print_exc()
        sys.stderr.write(f"[pddl] fatal error in a multi-rank job ({type(e).__name__}); exiting without cleanup\n")
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)

