#!/usr/bin/env python3
"""Shrink a rocprofv3 pass's output on the GPU box before gpurun copies gpurun_out/ back (64 MiB
cap): the kernel trace keeps one row per kernel name (the register / LDS columns
tools/profile_summary.py reads) and the stats file as is; a PMC pass's counter_collection.csv
becomes one row per (kernel, counter) with the summed value and the dispatch count, in the same
columns (Kernel_Name, Counter_Name, Counter_Value, Dispatches).

    python tools/prof_reduce.py <rocprof output dir> [...]
"""
import collections
import csv
import os
import sys


def reduce_dir(d):
    for f in sorted(os.listdir(d)):
        p = os.path.join(d, f)
        if f.endswith("kernel_trace.csv"):
            rows, seen = [], set()
            with open(p) as fh:
                r = csv.DictReader(fh)
                fields = r.fieldnames
                for row in r:
                    if row["Kernel_Name"] not in seen:
                        seen.add(row["Kernel_Name"])
                        rows.append(row)
            with open(p, "w", newline="") as fh:
                w = csv.DictWriter(fh, fieldnames=fields)
                w.writeheader()
                w.writerows(rows)
        elif f.endswith("counter_collection.csv"):
            agg = collections.defaultdict(lambda: [0.0, 0])
            with open(p) as fh:
                for row in csv.DictReader(fh):
                    a = agg[(row["Kernel_Name"], row["Counter_Name"])]
                    a[0] += float(row["Counter_Value"])
                    a[1] += 1
            with open(p, "w", newline="") as fh:
                w = csv.writer(fh)
                w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "Dispatches"])
                for (k, c), (v, n) in sorted(agg.items()):
                    w.writerow([k, c, repr(v), n])
        elif f.endswith((".csv", ".json", ".txt")) and not f.endswith(("kernel_stats.csv", "agent_info.csv")):
            os.remove(p)  # other trace domains / per-dispatch files the summaries do not read


if __name__ == "__main__":
    for d in sys.argv[1:]:
        for root, _, _ in os.walk(d):
            reduce_dir(root)
