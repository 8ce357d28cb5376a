"""Deterministic checks of the two-stream backward under segmented HIP-graph capture
(train/graph.py SegmentedStepGraphs), instead of re-running a crash:

  1. after every segment cut, the capture status of the engine's side stream (it must be
     back to "not capturing": a side stream left joined to a finished capture would record
     the next segment's weight-gradient kernels into a destroyed graph);
  2. kernel nodes per segment and in total, two-stream vs single-stream (same kernels);
  3. after one replay of all segments, gradient elements the replay left at zero where the
     eager step wrote a value, and the difference from the eager step.

    python scripts/graph_diag.py [--batch 8 32] [--out FILE]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import pddl  # noqa: E402,F401
from pddl.models.engine import HipEngine  # noqa: E402
from pddl.models.resnet50 import ParamLayout  # noqa: E402
from pddl.train.graph import SegmentedStepGraphs  # noqa: E402
from pddl.train.optim import make_optimizer  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
KERNEL, EMPTY, WAIT_EV, REC_EV = 0, 5, 6, 7


def exec_layout(g):
    """The HIP runtime's private view of a graph executable (parallel branch count and its
    parallel-stream table) at the struct offsets of THIS image's libamdhip64 -- a diagnostic of
    the round-5 hipGraphLaunch fault only; nothing in the package reads runtime internals."""
    ex = g.raw_cuda_graph_exec()
    if not ex:
        return None
    n = ctypes.c_int.from_address(ex + 0x48).value
    b0 = ctypes.c_uint64.from_address(ex + 0x1b8).value
    b1 = ctypes.c_uint64.from_address(ex + 0x1c0).value
    ents = [hex(ctypes.c_uint64.from_address(b0 + 8 * i).value) for i in range((b1 - b0) // 8)] if b0 else []
    return n, (b1 - b0) // 8, hex(b0), ents


def stream_status(s):
    st = ctypes.c_int(-1)
    rc = hip.hipStreamIsCapturing(ctypes.c_void_p(s.cuda_stream), ctypes.byref(st))
    return rc, st.value


def node_types(graph):
    g = ctypes.c_void_p(graph.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    arr = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, arr, ctypes.byref(n)) == 0
    out = {}
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(arr[i]), ctypes.byref(t))
        out[t.value] = out.get(t.value, 0) + 1
    return out


def run(B, two_stream, report):
    L = ParamLayout()
    eng = HipEngine(L, B, crop=224, image_size=224)
    eng.init(seed=3)
    opt = make_optimizer("adam", eng, lr=1e-3)
    g0 = torch.Generator().manual_seed(5)
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=g0).cuda()
    lab = torch.randint(0, 1000, (B,), generator=g0).cuda()
    buckets = L.buckets(25.0)
    side0 = eng.side
    report(f"B={B} two_stream={two_stream} side={'yes' if side0 is not None else 'no'} buckets={len(buckets)}")
    # eager reference (also builds the engine's lazy tables)
    eng.forward_backward(img, lab, 1.0 / B, buckets=buckets)
    torch.cuda.synchronize()
    ref = eng.grads.clone()
    probes = []

    def probe(k, g):
        st = stream_status(side0) if side0 is not None else (0, 0)
        cur = stream_status(torch.cuda.current_stream())
        probes.append((k, st, cur))

    sg = SegmentedStepGraphs(eng, opt, B, (224, 224), 1.0 / B, buckets, two_stream=two_stream, keep_graph=True,
                             probe=probe)
    sg.capture()
    bad = [p for p in probes if p[1] != (0, 0)]
    report(f"  side-stream status after each cut (rc, status): {[p[1] for p in probes]}")
    report(f"  capture stream status after each cut: {[p[2] for p in probes]}")
    tot = {}
    per = []
    for k, g in enumerate(sg.segments):
        if g is None:      # (bucket k completed with bucket k-1: no segment of its own)
            per.append(0)
            continue
        t = node_types(g)
        per.append(t.get(KERNEL, 0))
        for a, b in t.items():
            tot[a] = tot.get(a, 0) + b
    report(f"  kernel nodes per segment: {per} total {sum(per)}; all node types {tot}")
    for g in sg.segments:
        if g is not None:
            g.instantiate()
    sg.opt_graph.instantiate()
    sg.load(img, lab, None, (0, 0))
    eng.grads.fill_(12345.0)     # (segment 0 zeroes the workspace: the sentinel only checks that)
    torch.cuda.synchronize()
    for k in range(len(sg.segments)):
        sg.replay_segment(k)
    torch.cuda.synchronize()
    unwritten = int(((eng.grads == 12345.0) | ((eng.grads == 0) & (ref != 0))).sum().item())
    rel = ((eng.grads - ref).norm() / ref.norm()).item()
    report(f"  replay: unwritten gradient elements {unwritten} of {eng.grads.numel()}, rel diff vs eager {rel:.3e}")
    return {"bad_side_status": bad, "kernels": sum(per), "per": per, "unwritten": unwritten, "rel": rel}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[8, 32])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = []

    def report(s):
        print(s, flush=True)
        lines.append(s)
    ok = True
    for B in a.batch:
        r1 = run(B, False, report)
        r2 = run(B, True, report)
        same = r1["kernels"] == r2["kernels"]
        report(f"  B={B}: kernel count single {r1['kernels']} two-stream {r2['kernels']} -> {'same' if same else 'DIFFERENT'}")
        ok &= same and not r2["bad_side_status"] and r2["unwritten"] == 0 and r1["unwritten"] == 0
    report("RESULT " + ("ok" if ok else "DEFECT"))
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
