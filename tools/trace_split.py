#!/usr/bin/env python3
"""Per-kernel time of the last search in a rocprofv3 kernel trace (from its last k_zero_multi,
k_keys, or the last k_lmax when the batch built a trie) — the device-resident leg of bench.py.
    python tools/trace_split.py <trace_dir> [--all-searches]"""
import collections
import csv
import glob
import sys


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("edsbwt::", "")
    if n.startswith("rocprim"):
        return "rocprim:" + ("scan" if "scan" in n else "sort" if "sort" in n else "other")
    return n


def main():
    d = sys.argv[1]
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # a search starts with its zeroing launch (k_zero_multi, deferred checks), k_keys (packed
    # start) or k_lmax (trie)
    starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith(("k_keys", "k_lmax", "k_zero_multi"))]
    last = starts[-1]
    agg = collections.OrderedDict()
    t0 = int(rows[last]["Start_Timestamp"])
    t1 = t0
    for r in rows[last:]:
        n = short(r["Kernel_Name"])
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg.setdefault(n, [0, 0, r.get("VGPR_Count", ""), r.get("Scratch_Size", ""), r.get("LDS_Block_Size", "")])
        a[0] += 1
        a[1] += dur
        t1 = max(t1, int(r["End_Timestamp"]))
    print(f"{'kernel':36s} {'calls':>5s} {'ms':>8s}  vgpr scratch lds")
    for n, (c, dur, v, sc, l) in agg.items():
        print(f"{n:36s} {c:5d} {dur / 1e6:8.3f}  {v:>4s} {sc:>7s} {l:>5s}")
    busy = sum(a[1] for a in agg.values())
    print(f"span {((t1 - t0) / 1e6):.3f} ms, kernels busy {busy / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
