"""Every k_deep build against the oracle, many times over (diagnosis of build- or box-dependent
results; test infrastructure: imports the oracle as the checker).

For each build selected by the engine's knobs (EDSBWT_DEEPQ_WAVES 1 = unbounded / 5 / 6,
EDSBWT_EOF_ROWS, EDSBWT_DEEP_K 2 / 3 / 4 / 8) an index is opened on the README KAT EDS and on
small random / COVID-shaped EDSs, and each search variant of tests/test_gpu_parity.py::_compare
runs `--reps` times; every result is compared with the oracle's.  A mismatch prints the build,
the variant, the repetition, the counts and the search's statistics.  Run it with EDSBWT_POISON
set to fill every fresh device allocation with a marker word (reads of memory no kernel wrote
then show up as mismatches), and with EDSBWT_LIB pointing at libedsbwt_dbg.so for the device
invariant checks.

    python tools/kdeep_stress.py --reps 20 --out gpurun_out/kdeep_stress.json
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import random
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import edsgen  # noqa: E402
import oracle as orc  # noqa: E402  (the checker)

BUILDS = [
    {"EDSBWT_DEEPQ_WAVES": "1"},
    {"EDSBWT_DEEPQ_WAVES": "5"},
    {"EDSBWT_DEEPQ_WAVES": "6"},
    {"EDSBWT_EOF_ROWS": "1", "EDSBWT_DEEPQ_WAVES": "1"},
    {"EDSBWT_EOF_ROWS": "1", "EDSBWT_DEEPQ_WAVES": "5"},
    {"EDSBWT_DEEP_K": "2"},
    {"EDSBWT_DEEP_K": "3"},
    {"EDSBWT_DEEP_K": "8"},
]
VARIANTS = [{}, {"locate": False}, {"walk": True}, {"deep": False}, {"ktab": False}, {"direct": False}, {"pairs": False},
            {"text": False}, {"ordered": True}, {"locate": False, "ktab": False}]


def covid_like(rng, nseg):
    segs = []
    for t in range(nseg):
        if t % 2 == 0:
            segs.append(["".join(rng.choice("ACGT") for _ in range(rng.randint(40, 120)))])
        else:
            segs.append(["" if rng.random() < 0.1 else "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 3)))
                         for _ in range(rng.randint(2, 4))])
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    return segs


def pack(pats):
    bs = [p.encode() for p in pats]
    buf = np.frombuffer(b"".join(bs), np.uint8) if bs else np.zeros(0, np.uint8)
    return buf, np.concatenate(([0], np.cumsum([len(p) for p in bs]))).astype(np.uint64)


def cases(tmp):
    out = []
    kat = os.path.join(tmp, "kat")
    orc.transform(os.path.join(ROOT, "tests", "golden", "test.eds"), kat)
    out.append(("kat", kat, ["TATT", "ACT", "TTAT"], {}))
    out.append(("kat6", kat, ["TATT", "ACT", "TTAT", "TTA", "GTT", "T"], {}))
    for seed in (0, 3, 7):
        rng = random.Random(100 + seed)
        segs = edsgen.random_eds(rng, rng.randint(20, 400), alphabet="ACGT" if seed % 3 else "ACGTN", lmax=3 + seed,
                                 p_empty=0.0 if seed % 4 == 0 else 0.25)
        base = os.path.join(tmp, f"r{seed}")
        open(base + ".eds", "w").write(edsgen.eds_text(segs))
        orc.transform(base + ".eds", base)
        pats = []
        for _ in range(400):
            m = rng.randint(1, 24)
            p = edsgen.planted(rng, segs, m) if rng.random() < 0.6 else None
            pats.append(p or "".join(rng.choice("ACGT") for _ in range(m)))
        out.append((f"random{seed}", base, pats, {}))
    # the direct start with short lists queued for k_deep (the wide entries' inline lists)
    rng = random.Random(3232)
    segs = covid_like(rng, 700)
    base = os.path.join(tmp, "covid")
    open(base + ".eds", "w").write(edsgen.eds_text(segs))
    orc.transform(base + ".eds", base)
    pats = [edsgen.planted(rng, segs, rng.randint(16, 31)) or "ACGT" * 8 for _ in range(3000)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(16, 31))) for _ in range(500)]
    out.append(("covid_direct", base, pats, {"EDSBWT_DIRECT_ITEMS": "1e9"}))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--builds", default=None, help="comma-separated indexes into BUILDS")
    a = ap.parse_args()
    eb = importlib.import_module("eds-bwt_amd")
    orc.build()
    report = {"lib": eb.LIB_PATH, "poison": os.environ.get("EDSBWT_POISON"), "reps": a.reps, "runs": 0, "mismatches": [],
              "errors": []}
    t0 = time.time()
    builds = BUILDS if a.builds is None else [BUILDS[int(i)] for i in a.builds.split(",")]
    with tempfile.TemporaryDirectory() as tmp:
        cs = cases(tmp)
        ref = {}
        for name, base, pats, _ in cs:
            buf, offs = pack(pats)
            oc, oo, _ = orc.Engine(base, 8).search(buf, offs)
            ref[name] = (buf, offs, oc, oo)
        for b in builds:
            for name, base, pats, env in cs:
                envs = dict(b, **env)
                old = {k: os.environ.get(k) for k in envs}
                os.environ.update(envs)
                buf, offs, oc, oo = ref[name]
                print(f"[kdeep_stress] build {b} case {name}", flush=True)
                try:
                    with eb.Index(base) as idx:
                        for kw in VARIANTS:
                            for r in range(a.reps):
                                try:
                                    gc, go = idx.search((buf, offs), **kw)
                                except eb.EdsBwtError as e:
                                    report["errors"].append({"build": b, "case": name, "kw": kw, "rep": r, "error": str(e)})
                                    print("ERROR", b, name, kw, r, e, flush=True)
                                    if e.code == -4:  # a device fault: nothing more runs on this GPU
                                        if a.out:
                                            open(a.out, "w").write(json.dumps(report, indent=1))
                                        os._exit(3)
                                    continue
                                report["runs"] += 1
                                okc = np.array_equal(gc, oc)
                                oko = not kw.get("locate", True) or np.array_equal(go, oo)
                                if not (okc and oko):
                                    st = idx.stats()
                                    st.pop("kernels", None)
                                    bad = np.flatnonzero(gc != oc)[:16]
                                    m = {"build": b, "case": name, "kw": kw, "rep": r, "counts_ok": okc, "records_ok": oko,
                                         "bad_patterns": bad.tolist(), "got": gc[bad].tolist(), "want": oc[bad].tolist(),
                                         "stats": st}
                                    report["mismatches"].append(m)
                                    print("MISMATCH", json.dumps(m), flush=True)
                except eb.EdsBwtError as e:
                    report["errors"].append({"build": b, "case": name, "error": str(e)})
                    print("ERROR", b, name, e, flush=True)
                finally:
                    for k, v in old.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
            print(f"[kdeep_stress] build {b} done: runs {report['runs']}, mismatches {len(report['mismatches'])}, "
                  f"errors {len(report['errors'])} ({time.time() - t0:.0f} s)", flush=True)
    report["seconds"] = round(time.time() - t0, 1)
    js = json.dumps(report, indent=1)
    if a.out:
        open(a.out, "w").write(js)
    print(json.dumps({k: (len(v) if isinstance(v, list) else v) for k, v in report.items()}))
    return 1 if report["mismatches"] or report["errors"] else 0


if __name__ == "__main__":
    sys.exit(main())
