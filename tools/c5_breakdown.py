#!/usr/bin/env python3
"""C5 step breakdown: where the count-only search of the 1 Gchar EDS goes.

    python tools/c5_breakdown.py [--steps 2] > out.json      (EDSBWT_TRACE=1 adds per-depth lines on stderr)

* the whole 200K mixed batch (bench.py's C5 step), timed per kernel class (EDSBWT_PROFILE);
* each pattern-length class (8, 16, 32, 64) searched alone, same timing: which lengths carry
  the interval steps (the classes share trie suffixes, so their sum exceeds the whole batch);
* the engine's own counters: interval steps, trie depths and groups, link rows.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--config", default="c5")
    a = ap.parse_args()
    pkg = importlib.import_module("eds-bwt_amd")
    w = workloads.CONFIGS[a.config]
    wd = workloads.default_workdir()
    workloads.ensure_built()
    eds, base = workloads.build_index(w, wd, 0, lambda *x: print(*x, file=sys.stderr))
    lo, hi = workloads.shard(w, 0, 1)
    pats = workloads.pattern_file(w, eds, wd, lo, hi)
    planted = workloads.planted_mask(pats)
    buf, offs = pkg.read_pattern_file(pats)
    lens = (offs[1:] - offs[:-1]).astype(np.int64)
    out = {"config": a.config, "patterns": int(lens.size)}
    with pkg.Index(base) as idx:
        out["index"] = {"rows": idx.n_rows, "words": idx.n_words, "segments": idx.n_segments, "ktab_depth": idx.ktab_depth,
                        "ktab_items": idx.ktab_items, "device_bytes": idx.device_bytes}

        def run(sel, tag, steps):
            sb = np.concatenate([buf[int(offs[i]):int(offs[i + 1])] for i in sel]) if sel.size else np.zeros(0, np.uint8)
            so = np.zeros(sel.size + 1, np.uint64)
            so[1:] = np.cumsum(lens[sel])
            idx.search((sb, so), locate=False)  # warm (grouping decided, buffers sized)
            best = None
            for _ in range(steps):
                t = time.perf_counter()
                c, _ = idx.search((sb, so), locate=False, profile=True)
                dt = time.perf_counter() - t
                st = idx.stats()
                if best is None or dt < best[0]:
                    best = (dt, st, c)
            dt, st, c = best
            rec = {"patterns": int(sel.size), "s_per_call": round(dt, 4), "device_ms": round(st["ms_total"], 2),
                   "kernel_ms": {k: round(v["ms"], 2) for k, v in st["kernels"].items() if v["ms"] > 0.05},
                   "kernel_launches": {k: v["launches"] for k, v in st["kernels"].items() if v["launches"]},
                   "step_lines": st["kernels"]["step"]["lines"],
                   "intervals_stepped": st["intervals_stepped"], "depths": st["depths"], "search_groups": st["search_groups"],
                   "trie_nodes": st["trie_nodes"], "link_hash_rows": st["link_hash_rows"], "link_ranges": st["link_ranges"],
                   "occurrences_counted": int(c.astype(np.uint64).sum()), "found": int((c > 0).sum()),
                   "found_planted": int((c[planted[sel]] > 0).sum()) if sel.size else 0}
            print(f"[c5_breakdown] {tag}: {json.dumps(rec)}", file=sys.stderr, flush=True)
            return rec

        out["whole_batch"] = run(np.arange(lens.size), "whole", a.steps)
        out["by_length"] = {}
        for L in sorted(set(lens.tolist())):
            out["by_length"][str(L)] = run(np.flatnonzero(lens == L), f"len {L}", 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
