#!/usr/bin/env python3
"""k_deep's three-way list start (test-only libedsbwt_3way*.so): the README KAT search
that the unbounded build gets wrong, run in this process against the library EDSBWT_LIB names, with
EDSBWT_TRACE=1 and path tags, printing counts, records, the search's statistics and every pattern's
path — one JSON line.  Run once per library (tools/gpu.sh task `probe3`)."""
import importlib
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import oracle as orc  # noqa: E402  (the checker)

pkg = importlib.import_module("eds-bwt_amd")
out = {"lib": os.environ.get("EDSBWT_LIB", "default"), "env": {k: v for k, v in os.environ.items() if k.startswith("EDSBWT_")}}
with tempfile.TemporaryDirectory() as d:
    base = os.path.join(d, "test")
    orc.transform(os.path.join(ROOT, "tests", "golden", "test.eds"), base)
    pats = [b"TATT", b"ACT", b"TTAT"]
    buf, offs = pkg.pack_patterns(pats)
    oc, oo, _ = orc.Engine(base, 8).search(buf, offs)
    out["oracle_counts"] = oc.tolist()
    with pkg.Index(base) as idx:
        out["index"] = {"rows": idx.n_rows, "ktab_depth": idx.ktab_depth, "pair_blocks": idx.pair_blocks}
        runs = []
        for kw in ({}, {"locate": False}, {"ktab": False}, {"direct": False}, {"pairs": False}, {"text": False}, {"deep": False}):
            try:
                c, o = idx.search((buf, offs), **kw)
            except pkg.EdsBwtError as e:  # (a debug build's failed check) reported, the probe goes on
                runs.append({"kw": kw, "error": str(e)})
                continue
            st = idx.stats()
            runs.append({"kw": kw, "counts": c.tolist(), "match": bool(np.array_equal(c, oc)),
                         "stats": {k: st[k] for k in ("start_depth", "depths", "trie_nodes", "deep_from_depth", "deep_overflow",
                                                      "deep_level_rerun", "redo_searches", "intervals_stepped", "link_hash_rows")}})
        out["runs"] = runs
        L = pkg.lib()
        if hasattr(L, "edsbwt_debug_kdeep_dump"):
            # the first search again, then k_deep's dumped list starts (diagnostic builds)
            import ctypes
            idx.search((buf, offs))
            d = np.zeros(64 * 16, np.uint32)
            L.edsbwt_debug_kdeep_dump.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
            assert L.edsbwt_debug_kdeep_dump(d.ctypes.data, d.size) == 0
            rows = d.reshape(64, 16)
            out["kdeep_dump"] = [{"w": r[0:4].tolist(), "cn": int(r[4]), "u": int(r[5]), "cb": r[6:10].tolist(), "ce": r[10:14].tolist(),
                                  "pi": int(r[14])} for r in rows if r[15] == 0xD0D0D0D0]
print(json.dumps(out))
