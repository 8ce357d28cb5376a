"""One training step's kernel sequence from a rocprofv3 kernel trace: every dispatch of the
median-length step in launch order with its grid, workgroup size and duration, optionally
filtered by kernel-name substrings; plus per-filter totals over all steps.

    python scripts/kernel_seq.py run_kernel_trace.csv [--marker softmax_xent] [--match splitk,igemm_kernel]

Used for the b32 split-K study (profiles/r6_b32_splitk.txt): which layers split, how long each
slice launch and its combine take.
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="softmax_xent")
    ap.add_argument("--match", default="", help="comma-separated substrings (empty: every kernel)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
            wg = r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid, wg))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.marker in r[2]]
    steps = [rows[x:y] for x, y in zip(starts, starts[1:])][1:-1]
    if not steps:
        print("no complete steps")
        return
    pats = [m for m in a.match.split(",") if m]
    keep = (lambda n: any(m in n for m in pats)) if pats else (lambda n: True)
    tot = defaultdict(float)
    for s in steps:
        for r in s:
            if keep(r[2]):
                tot[r[2]] += (r[1] - r[0]) / 1e3 / len(steps)
    mid = sorted(steps, key=lambda s: s[-1][1] - s[0][0])[len(steps) // 2]
    t0 = mid[0][0]
    print(f"{len(steps)} steps; median step {(mid[-1][1] - t0) / 1e3:.1f} us, {len(mid)} kernels")
    for r in mid:
        if keep(r[2]):
            print(f"  t={(r[0] - t0) / 1e3:8.1f}  {(r[1] - r[0]) / 1e3:7.1f} us  grid {r[3]:>8} wg {r[4]:>4}  {r[2][:90]}")
    print("per-step totals:")
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {t:8.1f} us  {n[:100]}")


if __name__ == "__main__":
    main()
