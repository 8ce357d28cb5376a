"""Per-kernel totals from a rocprofv3 SQLite database (the default output format of this
rocprofv3; `--output-format csv` writes the CSVs instead).

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db [--steps N] [--top 25]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name} "
                     f"order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"total kernel time {total / 1e6 / a.steps:.3f} ms/step over {a.steps:g} steps")
    for n, k, t in rows[:a.top]:
        print(f"{t / 1e6 / a.steps:8.3f} ms/step {k / a.steps:6.1f} calls/step {100 * t / total:5.1f}%  {n[:110]}")


if __name__ == "__main__":
    main()
