#!/usr/bin/env python3
"""Host packing rate of the 2-bit line packer (csrc/format.cpp edsbwt_pack_lines) on a chunk of
fixed-length DNA lines, on 1..N threads (ctypes releases the GIL).

    python tools/pack_bw.py [MB] [threads,...]"""
import ctypes
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "eds-bwt_amd", "_build", "libedsbwt.so"))
L.edsbwt_lines_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]
L.edsbwt_lines_fixed.restype = ctypes.c_uint64
L.edsbwt_pack_lines.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_void_p, ctypes.c_void_p]
L.edsbwt_pack_lines.restype = ctypes.c_int


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 40
    ths = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,4,8,12,16").split(",")]
    n = int(mb * 2**20) // 32
    rng = np.random.default_rng(1)
    a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=(n, 32))]
    a[:, 31] = ord("\n")
    text = np.ascontiguousarray(a).reshape(-1)
    Lo = ctypes.c_uint32(0)
    P = L.edsbwt_lines_fixed(text.ctypes.data, text.size, ctypes.byref(Lo))
    out = np.zeros(P * 8 + 16, np.uint8)
    for T in ths:
        best = 1e9
        for _ in range(5):
            def run(t):
                L.edsbwt_pack_lines(text.ctypes.data, text.size, Lo.value, P * t // T, P * (t + 1) // T,
                                    text.ctypes.data + text.size, out.ctypes.data)
            th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            best = min(best, time.perf_counter() - t0)
        print(f'{{"threads": {T}, "MB": {mb}, "ms": {best * 1e3:.3f}, "GB_s": {text.size / best / 1e9:.1f}}}', flush=True)


if __name__ == "__main__":
    main()
