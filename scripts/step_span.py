"""Per-step GPU timeline summary from a rocprofv3 kernel trace: step span (first kernel of a
step to the first kernel of the next), busy time (union of kernel intervals, all streams),
idle gaps, kernel count, and the kernels with the largest per-step total.

    python scripts/step_span.py run_kernel_trace.csv [marker=softmax_xent] [top=12]

A step starts at each dispatch whose kernel name contains `marker` (default the loss
kernel, launched once per training step).  The first and last steps are dropped (warmup / partial).
"""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Stream_Id") or r.get("Queue_Id") or "?"))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "softmax_xent"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = load(path)
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        steps.append(rows[a:b])
    steps = steps[1:-1] if len(steps) > 3 else steps
    if not steps:
        print("no complete steps")
        return
    out = []
    per = defaultdict(float)
    for i, s in enumerate(steps):
        t0 = s[0][0]
        t1 = steps[i + 1][0][0] if i + 1 < len(steps) else max(r[1] for r in s)
        busy = union([(r[0], r[1]) for r in s])
        out.append(((t1 - t0) / 1e6, busy / 1e6, len(s)))
        for r in s:
            per[r[2]] += (r[1] - r[0]) / 1e3 / len(steps)   # us per step
    n = len(out)
    span = sum(o[0] for o in out) / n
    busy = sum(o[1] for o in out) / n
    print(f"steps {n}: span {span:.3f} ms, busy {busy:.3f} ms, idle {span - busy:.3f} ms, "
          f"kernels/step {sum(o[2] for o in out) / n:.1f}")
    # per stream (rocprofv3 Stream_Id, else Queue_Id): busy time of each stream's own kernels
    per_s = defaultdict(float)
    for s in steps:
        by = defaultdict(list)
        for r in s:
            by[r[3]].append((r[0], r[1]))
        for k, iv in by.items():
            per_s[k] += union(iv) / 1e6 / len(steps)
    print("  per stream busy: " + ", ".join(f"{k}: {v:.3f} ms" for k, v in sorted(per_s.items(), key=lambda kv: -kv[1])))
    for name, t in sorted(per.items(), key=lambda kv: -kv[1])[:top]:
        print(f"  {t:9.1f} us  {name[:110]}")


if __name__ == "__main__":
    main()
