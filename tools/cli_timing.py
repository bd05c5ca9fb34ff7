#!/usr/bin/env python3
"""Time the drop-in CLI at production size.

    python tools/cli_timing.py [--config c3] [--runs 2] [--check 512]

Runs `EDSBWTsearch <base> <patterns> --quiet` (eds-bwt_amd/tools/edsbwtsearch_cli.cpp, the
MOVE_EDSBWTSearch argv / files / console contract) on the config's index and pattern file, as
a user would: index open, the pattern file read, the search through edsbwt_search_lines, the
multi-threaded CSV formatting and the write of <patterns>output_M_LF.csv.  Reports the process
wall time, the reference's own clock `bs took:` (MOVE_EDSBWTSearch.cpp:109,145: the pattern loop
including the CSV rows, index load excluded), the CSV size, and checks that the CSV rows of the
first and last `--check` patterns are byte-identical to the oracle's rows for them
(MOVE_EDSBWTSearch.cpp:55-64,365: "pat\\tword\\tseg\\tword_in_seg\\toffset\\n", rows in the
reference's order).  The oracle is the checker only.  Prints one JSON object.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import workloads  # noqa: E402


def rows_bytes(occ) -> bytes:
    return b"".join(b"%d\t%d\t%d\t%d\t%d\n" % (int(r["pat"]), int(r["word"]), int(r["seg"]), int(r["word_in_seg"]), int(r["offset"]))
                    for r in occ)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--check", type=int, default=512)
    ap.add_argument("--log", default=None, help="write the last run's stderr here (EDSBWT_TRACE=2 host marks)")
    ap.add_argument("--cli-args", default="", help="extra EDSBWTsearch arguments (e.g. '--gpus 2')")
    args = ap.parse_args()
    w = workloads.CONFIGS[args.config]
    wd = workloads.default_workdir()
    workloads.ensure_built()
    eds, base = workloads.build_index(w, wd)
    lo, hi = workloads.shard(w, 0, 1)
    pats = workloads.pattern_file(w, eds, wd, lo, hi)
    cli = os.path.join(workloads.BUILD, "EDSBWTsearch")
    csv_path = pats + "output_M_LF.csv"
    runs = []
    for _ in range(args.runs):
        if os.path.exists(csv_path):
            os.remove(csv_path)
        t = time.perf_counter()
        r = subprocess.run([cli, base, pats, "--quiet"] + args.cli_args.split(), capture_output=True, env=dict(os.environ, EDSBWT_CLI_TIMES="1"))
        wall = time.perf_counter() - t
        if args.log:
            open(args.log, "wb").write(r.stderr[-2_000_000:])
        if r.returncode != 1:  # the reference exits 1 on success (mainMove_EDSBWT.cpp:61)
            sys.exit(f"EDSBWTsearch exited {r.returncode}: {r.stderr[-400:]!r}")
        m = re.search(rb"bs took:([0-9.e+-]+)$", r.stdout)
        found = re.search(rb"count_found = (\d+)", r.stderr)
        phases = {m_.group(1).decode(): float(m_.group(2)) for m_ in re.finditer(rb"\[cli\] ([a-z ]+?) ([0-9.]+) s", r.stderr)}
        runs.append({"wall_s": round(wall, 3), "bs_took_s": float(m.group(1)) if m else None,
                     "count_found": int(found.group(1)) if found else None, "phases_s": phases})
        print(f"[cli] run: wall {wall:.3f}s, bs took {runs[-1]['bs_took_s']}", file=sys.stderr, flush=True)
    csv = open(csv_path, "rb").read()
    header = b"#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n"
    assert csv.startswith(header)
    body = memoryview(csv)[len(header):]
    nrows = csv.count(b"\n") - 1
    # the oracle's rows for the first and last `check` patterns
    import oracle as orc  # checker only
    import importlib
    pkg = importlib.import_module("eds-bwt_amd")
    buf, offs = pkg.read_pattern_file(pats)
    npat = offs.size - 1
    k = min(args.check, npat)
    eng = orc.Engine(base, 8)
    t = time.time()
    ho = offs[: k + 1]
    hc, hocc, _ = eng.search(buf[: int(ho[-1])], ho, first_pattern_id=1, threads=16)
    to = offs[npat - k:] - offs[npat - k]
    tc, tocc, _ = eng.search(buf[int(offs[npat - k]):], to, first_pattern_id=npat - k + 1, threads=16)
    t_orc = time.time() - t
    eng.close()
    hb, tb = rows_bytes(hocc), rows_bytes(tocc)
    head_ok = bytes(body[: len(hb)]) == hb and (len(body) == len(hb) or int(bytes(body[len(hb):len(hb) + 12]).split(b"\t")[0]) > k)
    tail_ok = bytes(body[len(body) - len(tb):]) == tb
    best = min(runs, key=lambda x: x["wall_s"])
    print(json.dumps({
        "what": "EDSBWTsearch <base> <patterns> --quiet (the drop-in CLI) on the config's index and pattern file",
        "config": w.text, "patterns": int(npat), "runs": runs, "wall_s": best["wall_s"], "bs_took_s": best["bs_took_s"],
        "patterns_per_sec_bs_took": round(npat / best["bs_took_s"], 1) if best["bs_took_s"] else None,
        "patterns_per_sec_wall": round(npat / best["wall_s"], 1),
        "csv_bytes": len(csv), "csv_rows": nrows,
        "check": {"patterns_head": k, "patterns_tail": k, "rows_head": int(hocc.size), "rows_tail": int(tocc.size),
                  "head_match": bool(head_ok), "tail_match": bool(tail_ok), "oracle_s": round(t_orc, 1),
                  "what": "CSV rows of the first and last patterns byte-equal to the oracle's rows (oracle/edsbwt_oracle.c, "
                          "literal MOVE_EDSBWTSearch restatement)"},
        "match": bool(head_ok and tail_ok)}), flush=True)
    os.remove(csv_path)


if __name__ == "__main__":
    main()
