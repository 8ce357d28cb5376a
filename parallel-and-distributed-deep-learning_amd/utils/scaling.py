"""Scaling efficiency (BASELINE.json's metric "images/sec at 1/2/4/8 + scaling
efficiency").  The reference's only timing is the Horovod script's wall clock around `fit`
(imagenet-resnet50-hvd.py:119-126); here throughput and efficiency are computed outputs of the
bench, the fit loop's JSONL log and bench/scaling.py.

Weak scaling (per-GPU batch fixed): efficiency(N) = ips(N) / (N * ips(1)).
"""
from __future__ import annotations

from typing import Dict, List, Optional


def efficiency(ips_n: float, n: int, ips_1: Optional[float]) -> Optional[float]:
    """ips(N) / (N * ips(1)); None without a positive 1-GPU rate."""
    if ips_1 is None or ips_1 <= 0 or n < 1:
        return None
    return ips_n / (n * ips_1)


def scaling_table(rows: Dict[int, float], ips_1: Optional[float] = None) -> List[dict]:
    """Rows {n_gpus: images/sec} -> [{n_gpus, images_per_sec, per_gpu, speedup, efficiency}], with
    the 1-GPU rate taken from rows[1] unless given."""
    if ips_1 is None:
        ips_1 = rows.get(1)
    out = []
    for n in sorted(rows):
        v = rows[n]
        e = efficiency(v, n, ips_1)
        out.append({"n_gpus": n, "images_per_sec": round(v, 2), "per_gpu_images_per_sec": round(v / n, 2),
                    "speedup": None if not ips_1 else round(v / ips_1, 4),
                    "efficiency": None if e is None else round(e, 4)})
    return out


def format_table(table: List[dict]) -> str:
    lines = [f"{'GPUs':>5} {'images/sec':>12} {'per GPU':>10} {'speedup':>8} {'efficiency':>10}"]
    for r in table:
        sp = "-" if r["speedup"] is None else f"{r['speedup']:.2f}"
        ef = "-" if r["efficiency"] is None else f"{r['efficiency']:.3f}"
        lines.append(f"{r['n_gpus']:>5} {r['images_per_sec']:>12.1f} {r['per_gpu_images_per_sec']:>10.1f} "
                     f"{sp:>8} {ef:>10}")
    return "\n".join(lines)
