"""Host-blocking HIP calls per process from a rocprofv3 --hip-trace directory: synchronizes,
device -> host copies and event waits, next to the number of kernel launches (a PS worker step
launches ~180 kernels eagerly, 1 graph when captured).

    python scripts/hip_sync_count.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import sys
from collections import Counter, defaultdict

BLOCKING = ("hipStreamSynchronize", "hipDeviceSynchronize", "hipEventSynchronize", "hipMemcpy", "hipMemcpyDtoH",
            "hipMemcpyWithStream")


def main():
    root = sys.argv[1]
    files = glob.glob(os.path.join(root, "**", "*hip_api_trace.csv"), recursive=True)
    per = defaultdict(Counter)
    for f in files:
        for r in csv.DictReader(open(f)):
            pid = r.get("Process_Id") or os.path.basename(os.path.dirname(f))
            name = r.get("Function") or r.get("Operation") or ""
            per[pid][name] += 1
    for pid, c in sorted(per.items()):
        launches = c["hipLaunchKernel"] + c["hipExtLaunchKernel"] + c["hipModuleLaunchKernel"]
        graphs = c["hipGraphLaunch"]
        blocking = {k: v for k, v in c.items() if k in BLOCKING or (k.startswith("hipMemcpy") and "Async" not in k)}
        print(f"pid {pid}: kernel launches {launches}, graph launches {graphs}, blocking calls {blocking}")


if __name__ == "__main__":
    main()
