"""Host packer rate (format.cpp edsbwt_pack_lines) on C2's pattern shape: 1M lines of 20 A/C/G/T
bases, packed by T threads each taking a contiguous range (as the engine's pool does).  One JSON
line: median / min milliseconds per whole-batch pack over the repetitions, per thread count.
EDSBWT_PACK_BULK=0 selects the per-line path (read once per process).

    python tools/pack_bench.py [--lines N] [--len L] [--reps R] [--threads 1,12]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=1_000_000)
    ap.add_argument("--len", type=int, default=20)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--threads", default="1,12")
    a = ap.parse_args()
    lib = ctypes.CDLL(os.environ.get("EDSBWT_LIB") or os.path.join(ROOT, "eds-bwt_amd", "_build", "libedsbwt.so"))
    f = lib.edsbwt_pack_lines
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    P, L = a.lines, a.len
    rng = np.random.default_rng(1)
    src = np.concatenate([np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, (P, L))], np.full((P, 1), 10, np.uint8)], 1).ravel().copy()
    S = (L + 3) // 4
    out = np.zeros(P * S + 16, np.uint8)
    nb, base, end, o = src.size, src.ctypes.data, src.ctypes.data + src.size, out.ctypes.data
    res = {"lines": P, "len": L, "bulk_env": os.environ.get("EDSBWT_PACK_BULK", "1")}
    for T in (int(t) for t in a.threads.split(",")):
        ts = []
        for _ in range(a.reps):
            ok = []
            th = [threading.Thread(target=lambda t=t: ok.append(f(base, nb, L, P * t // T, P * (t + 1) // T, end, o))) for t in range(T)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            ts.append((time.perf_counter() - t0) * 1e3)
            assert all(ok) and len(ok) == T
        res[f"T{T}_ms_median"] = round(statistics.median(ts), 4)
        res[f"T{T}_ms_min"] = round(min(ts), 4)
        res[f"T{T}_ns_per_line_thread"] = round(min(ts) * 1e6 * T / P, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
