#!/usr/bin/env python3
"""Timeline of the last end-to-end call in a rocprofv3 kernel + memory-copy trace
(a kernel + copy trace: rocprofv3 --kernel-trace --memory-copy-trace of bench.py): every kernel and copy with start/end relative to the call's first
upload, its stream, and the idle gap of the engine stream before it.
    python tools/timeline.py <trace_dir> [min_ms]"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    mn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    kf = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    mf = sorted(glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True))
    ev = []
    for r in csv.DictReader(open(kf)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("edsbwt::", "")
        if n.startswith("rocprim"):
            n = "rocprim"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n[:26], "s" + r.get("Stream_Id", "?")))
    if mf:
        for r in csv.DictReader(open(mf[0])):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", "")[:26],
                       "s" + r.get("Stream_Id", "?")))
    ev.sort()
    # the last call: from the last H2D that follows a gap of > 3 ms without H2D
    h = [e for e in ev if e[2].startswith("HOST_TO_DEVICE")]
    t0 = h[0][0]
    for a, b in zip(h, h[1:]):
        if b[0] - a[1] > 3e6:
            t0 = b[0]
    last_end = {}
    busy = {}
    for e in ev:
        if e[0] < t0 - 1000:
            continue
        gap = (e[0] - last_end.get(e[3], e[0])) / 1e6
        last_end[e[3]] = max(last_end.get(e[3], 0), e[1])
        busy[e[3]] = busy.get(e[3], 0) + (e[1] - e[0])
        dur = (e[1] - e[0]) / 1e6
        if dur >= mn or gap > 0.05:
            print(f"{(e[0] - t0) / 1e6:8.3f} {(e[1] - t0) / 1e6:8.3f} {dur:7.3f} gap {gap:6.3f} {e[3]:>4s} {e[2]}")
    end = max(last_end.values())
    print(f"span {(end - t0) / 1e6:.3f} ms; busy per stream: " + ", ".join(f"{k} {v / 1e6:.3f}" for k, v in sorted(busy.items())))


if __name__ == "__main__":
    main()
