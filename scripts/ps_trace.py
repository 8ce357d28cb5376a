"""Per-step split of a PS job's kernel traces (one CSV per process, rocprofv3 --kernel-trace):
the worker process is the one that launches the loss kernel; each worker step span (loss kernel
to loss kernel) is divided into worker-busy, PS-only-busy and idle time, with the top kernels of
each process per step.   python scripts/ps_trace.py a_kernel_trace.csv b_kernel_trace.csv ..."""
import csv
import sys
from collections import defaultdict


def load(path):
    with open(path) as f:
        return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(f))


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def clip(iv, a, b):
    return sum(max(0, min(e, b) - max(s, a)) for s, e in iv)


def per_step(rows, marks):
    n = len(marks) - 1
    tot, cnt = defaultdict(float), defaultdict(int)
    for s, e, k in rows:
        if marks[0] <= s < marks[-1]:
            tot[k[:90]] += (e - s) / 1e3 / n
            cnt[k[:90]] += 1
    return tot, {k: v / n for k, v in cnt.items()}


def main():
    args = sys.argv[1:]
    ref = None
    if "--ref" in args:               # a single-strategy trace of the same config: per-kernel diff
        i = args.index("--ref")
        ref = load(args[i + 1])
        del args[i:i + 2]
    procs = [(p, load(p)) for p in args]
    procs = [(p, r) for p, r in procs if r]
    worker = [r for p, r in procs if any("softmax_xent" in k for _, _, k in r)]
    others = [r for p, r in procs if not any("softmax_xent" in k for _, _, k in r)]
    if not worker:
        sys.exit("no process launched the loss kernel")
    w = worker[0]
    marks = [s for s, _, k in w if "softmax_xent" in k][2:-1]
    wi = merge([(s, e) for s, e, _ in w])
    pi = merge([(s, e) for r in others for s, e, _ in r])
    both = merge(wi + pi)
    n = len(marks) - 1
    span = (marks[-1] - marks[0]) / n / 1e3
    wb = sum(clip(wi, marks[i], marks[i + 1]) for i in range(n)) / n / 1e3
    pb = sum(clip(pi, marks[i], marks[i + 1]) for i in range(n)) / n / 1e3
    ub = sum(clip(both, marks[i], marks[i + 1]) for i in range(n)) / n / 1e3
    print(f"steps {n}: span {span:.1f} us | worker busy {wb:.1f} | PS-process busy {pb:.1f} | "
          f"union {ub:.1f} | PS-only {ub - wb:.1f} | idle {span - ub:.1f}")
    # where the worker's GPU idles: the gaps between consecutive worker kernels inside the
    # steps, by the kernel the gap follows / precedes (summed per step)
    gaps = defaultdict(float)
    ws = [x for x in w if marks[0] <= x[0] < marks[-1]]
    end = ws[0][1]
    for i in range(1, len(ws)):
        s0, e0, k0 = ws[i]
        if s0 > end:
            gaps[(ws[i - 1][2][:45], k0[:45])] += (s0 - end) / 1e3
        end = max(end, e0)
    print("-- worker idle gaps, us per step (after -> before)")
    for (a, b), v in sorted(gaps.items(), key=lambda x: -x[1])[:8]:
        print(f"  {v / n:9.1f}  {a}  ->  {b}")
    for tag, rows in (("worker", w), ("ps", [x for r in others for x in r])):
        tot = defaultdict(float)
        for s, e, k in rows:
            if marks[0] <= s < marks[-1]:
                tot[k[:90]] += (e - s) / 1e3
        print(f"-- {tag}: top kernels, us per step")
        for k, v in sorted(tot.items(), key=lambda x: -x[1])[:10]:
            print(f"  {v / n:9.1f}  {k}")


    if ref is not None:
        rm = [s for s, _, k in ref if k.startswith("pddl::adam_kernel")][2:-1]   # (once per single step)
        rn = len(rm) - 1
        rspan = (rm[-1] - rm[0]) / rn / 1e3
        rb = sum(clip(merge([(s, e) for s, e, _ in ref]), rm[i], rm[i + 1]) for i in range(rn)) / rn / 1e3
        print(f"-- reference (single) steps {rn}: span {rspan:.1f} us, busy {rb:.1f}; worker - single per kernel, us per step:")
        a, ac = per_step(w, marks)
        b, bc = per_step(ref, rm)
        d = {k: a.get(k, 0.0) - b.get(k, 0.0) for k in set(a) | set(b)}
        for k, v in sorted(d.items(), key=lambda x: -abs(x[1]))[:12]:
            print(f"  {v:+9.1f}  ({ac.get(k, 0):.0f} vs {bc.get(k, 0):.0f} launches)  {k}")


if __name__ == "__main__":
    main()
