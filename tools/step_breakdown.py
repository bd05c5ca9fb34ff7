#!/usr/bin/env python3
"""Per-kernel breakdown of the LAST search step in a rocprofv3 kernel trace.

    python tools/step_breakdown.py <trace_kernel_trace.csv> [--marker k_deep_fast]

The last step is the span from the last dispatch of the marker kernel's predecessor
group: we take the time window between the end of the second-to-last k_locate (or marker)
and the end of the trace, which is one full bench step.
"""
import csv
import sys
import collections

def short(n):
    n = n.split("(")[0].replace("void ", "").replace("edsbwt::", "")
    if "rocprim" in n:
        for k in ("scan", "onesweep_iteration", "onesweep_global_offsets", "histogram", "block_sort", "merge", "lookback"):
            if k in n:
                return "rocprim:" + k
        return "rocprim"
    return n

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[3] if len(sys.argv) > 3 else "k_locate"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == marker]
lo = ends[-2] + 1
step = rows[lo:ends[-1] + 1]
t0 = int(step[0]["Start_Timestamp"]); t1 = int(step[-1]["End_Timestamp"])
agg = collections.OrderedDict()
for r in step:
    k = short(r["Kernel_Name"])
    a = agg.setdefault(k, [0, 0.0])
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"step window {(t1 - t0) / 1e3:.1f} us, kernels busy {busy:.1f} us, {len(step)} dispatches")
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:40s} {n:4d} {us:9.1f} us")
