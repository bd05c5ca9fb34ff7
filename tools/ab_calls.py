#!/usr/bin/env python3
"""Interleaved A/B of per-call settings of the host pipeline in ONE process (the box-to-box
and process-to-process spread of bench.py runs is larger than most effects measured here).

    python tools/ab_calls.py [--config c3] [--rounds 6] [--calls 5] VAR=a,b,c [VAR2=x,y ...]

Each VAR must be read by the engine at call time (EDSBWT_CHUNK_MB, EDSBWT_CHUNK_RAMP,
EDSBWT_AHEAD).  Prints the median and min ms_wall per variant (the cross product)."""
import argparse
import importlib
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--workdir", default=workloads.default_workdir())
    ap.add_argument("vars", nargs="+")
    a = ap.parse_args()
    axes = [(v.split("=")[0], v.split("=")[1].split(",")) for v in a.vars]
    variants = list(itertools.product(*[[(k, x) for x in xs] for k, xs in axes]))
    import torch
    from bench import pin_to_gpu_numa
    pin_to_gpu_numa(torch, 0)  # as bench.py runs
    workloads.ensure_built()
    pkg = importlib.import_module("eds-bwt_amd")
    w = workloads.CONFIGS[a.config]
    eds, base = workloads.build_index(w, a.workdir, 0)
    lo, hi = workloads.shard(w, 0, 1, 0)
    path = workloads.pattern_file(w, eds, a.workdir, lo, hi)
    npat = hi - lo
    idx = pkg.Index(base)
    text = pkg.read_pattern_file_pinned(path)
    cb = pkg.HostBuffer(4 * (npat + 1))
    res = {v: [] for v in variants}
    for r in range(a.rounds + 1):
        for v in variants:
            for k, x in v:
                os.environ[k] = x
            for _ in range(a.calls):
                n, _, _ = idx.search_lines(text.ptr, text.nbytes, cb.ptr, npat + 1, locate=w.locate)
                assert n == npat
                if r:  # round 0 warms up
                    res[v].append(idx.stats()["ms_wall"])
    for v in variants:
        x = np.array(res[v])
        print(" ".join(f"{k}={val}" for k, val in v), f"median {np.median(x):.3f} ms  min {x.min():.3f}  mean {x.mean():.3f}  "
              f"({npat * 1e3 / np.median(x):.3e} patterns/s)", flush=True)


if __name__ == "__main__":
    main()
