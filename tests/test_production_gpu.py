"""Parity at the production configurations (BASELINE.json configs[1], [2]: C2 and C3 of
SURVEY.md §8(d)), with the engine's default knobs: the D0 = 15 k-mer start table, the
packed direct start, two-step rank entries (rent2), per-row locate samples.

* A deterministic sample — the first 1024 patterns plus 1024 strided ones — is compared
  with the oracle (the literal MOVE_EDSBWTSearch restatement, MOVE_EDSBWTSearch.cpp:228-374)
  on the same index: counts and records, in order (:328-369).
* The whole batch is checked through size-independent properties: Σ counts == records,
  every planted pattern found, records pattern-major and counted per pattern, and every
  record spells its pattern in the .eds text (orc_check_records, no BWT involved).
"""
import os

import numpy as np
import pytest

import workloads

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


def _sample(npat, head=1024, strided=1024):
    idx = np.arange(min(head, npat))
    if npat > head:
        idx = np.union1d(idx, np.linspace(head, npat - 1, strided).astype(np.int64))
    return idx


def _subset(buf, offs, idx):
    lens = (offs[idx + 1] - offs[idx]).astype(np.uint64)
    parts = [buf[int(offs[i]):int(offs[i + 1])] for i in idx]
    sb = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    so = np.zeros(idx.size + 1, np.uint64)
    so[1:] = np.cumsum(lens)
    return sb, so


def _records_of(occ, counts, idx):
    """Records of patterns idx (0-based batch positions) from pattern-major records."""
    start = np.zeros(counts.size + 1, np.int64)
    start[1:] = np.cumsum(counts.astype(np.int64))
    return [occ[start[i]:start[i + 1]] for i in idx]


def _check_production(oracle, edsbwt, name, expect_direct):
    w = workloads.CONFIGS[name]
    wd = workloads.default_workdir()
    workloads.ensure_built()
    eds, base = workloads.build_index(w, wd)
    lo, hi = workloads.shard(w, 0, 1)
    pats = workloads.pattern_file(w, eds, wd, lo, hi)
    buf, offs = edsbwt.read_pattern_file(pats)
    npat = offs.size - 1
    assert npat == w.patterns
    with edsbwt.Index(base) as idx:
        if expect_direct:
            assert idx.ktab_depth == 15 and idx.pair_blocks
        counts, occ = idx.search((buf, offs), first_pattern_id=lo + 1, locate=True)
        st = idx.stats()
        if expect_direct:
            assert st["start_depth"] == 15 and st["trie_nodes"] == 0, st  # packed direct start
        c2, o2 = idx.search((buf, offs), first_pattern_id=lo + 1, locate=False)
        assert np.array_equal(c2, counts) and o2.size == 0
    # whole-batch properties
    assert int(counts.astype(np.uint64).sum()) == occ.size
    if w.mode == "planted":
        assert (counts > 0).all()
    pat0 = occ["pat"].astype(np.int64) - (lo + 1)
    assert (np.diff(pat0) >= 0).all()
    assert np.array_equal(np.bincount(pat0, minlength=npat), counts.astype(np.int64))
    bad, first = oracle.check_records(eds, buf, offs, occ, lo + 1, threads=THREADS)
    assert bad == 0, (bad, occ[first])
    # sample vs the oracle, in order
    idx_s = _sample(npat)
    sb, so = _subset(buf, offs, idx_s)
    eng = oracle.Engine(base, 8)
    oc, oo, _ = eng.search(sb, so, first_pattern_id=1, threads=THREADS)
    eng.close()
    assert np.array_equal(counts[idx_s], oc)
    ostart = np.zeros(oc.size + 1, np.int64)
    ostart[1:] = np.cumsum(oc.astype(np.int64))
    for j, recs in enumerate(_records_of(occ, counts, idx_s)):
        ref = oo[ostart[j]:ostart[j + 1]]
        for f in ("word", "seg", "word_in_seg", "offset"):
            assert np.array_equal(recs[f], ref[f]), (name, int(idx_s[j]), f)
        assert (recs["pat"] == lo + 1 + idx_s[j]).all()
    return counts, occ


def test_c3_production_parity(oracle, edsbwt):
    """C3: ~100 Mchar COVID-like EDS, 10M planted 31-mers, full locate, default knobs."""
    _check_production(oracle, edsbwt, "c3", expect_direct=True)


def test_c2_production_parity(oracle, edsbwt):
    """C2: 10 Mchar EDS, 1M random 20-mers; counts (the configuration is count-only) and,
    for the sample, records too."""
    _check_production(oracle, edsbwt, "c2", expect_direct=False)
