"""Parity at the production configurations of BASELINE.json (C2, C3, C4, C5 of SURVEY.md
§8(d)), with the engine's default knobs: the D0 = 15 k-mer start table, the packed direct
start, two-step rank entries (rent2), per-row locate samples, the host pipeline.

* Oracle samples, compared in order (counts and records, MOVE_EDSBWTSearch.cpp:228-374,
  328-369):
  - the literal MOVE_EDSBWTSearch restatement on the first 1024 patterns plus 1024 strided ones;
  - the trie-sharing restatement (orc_search_batch_trie, pinned to the literal loop by
    tests/test_oracle.py) on 16384 strided patterns plus EVERY pattern that took a rare path
    of the device search — the wide lists, the level re-run, a searched-again batch — and up
    to 8192 of those that took the register-list walk k_deep (EDSBWT_PATH_TAGS).
* The whole batch through size-independent properties: Σ counts == records, every planted
  pattern found, records pattern-major and counted per pattern, and every record spells its
  pattern in the .eds text (orc_check_records, no BWT involved).
* C4: the last of 8 ranks' shards of the 100M batch (first_pattern_id = lo + 1) through
  edsbwt_search_lines, as bench.py's rank runs it.  C5: the 1 Gchar index, the 200K mixed
  batch (count-only, as bench.py's C5 line), the >= 32-mers located, an oracle sample of
  every length class.

Each test writes its sample sizes to gpurun_out/parity_<config>.json when that directory
exists (evidence kept under profiles/).
"""
import ctypes
import json
import os
import time

import numpy as np
import pytest

import workloads

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)))


def _report(name, rec):
    if os.path.isdir("gpurun_out"):
        with open(os.path.join("gpurun_out", f"parity_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)


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


def _compare_sample(oracle, base, buf, offs, counts, occ, idx_s, first_id, name, trie=False, records=True):
    """The oracle on patterns idx_s (batch positions) vs the device's counts and records."""
    sb, so = _subset(buf, offs, idx_s)
    eng = oracle.Engine(base, 8)
    t = time.time()
    oc, oo, _ = eng.search(sb, so, first_pattern_id=1, threads=THREADS, trie=trie)
    dt = time.time() - t
    eng.close()
    bad = np.nonzero(counts[idx_s] != oc)[0]
    assert bad.size == 0, (name, "counts differ at", idx_s[bad[:8]].tolist(), counts[idx_s][bad[:8]].tolist(), oc[bad[:8]].tolist())
    if records:
        ostart = np.zeros(oc.size + 1, np.int64)
        ostart[1:] = np.cumsum(oc.astype(np.int64))
        for j, recs in enumerate(_records_of(occ, counts, idx_s)):
            ref = oo[ostart[j]:ostart[j + 1]]
            for f in ("word", "seg", "word_in_seg", "offset"):
                assert np.array_equal(recs[f], ref[f]), (name, int(idx_s[j]), f)
            assert (recs["pat"] == first_id + idx_s[j]).all()
    return dt, int(oc.astype(np.int64).sum())


def _d2h(ptr, nbytes):
    out = np.zeros(max(1, nbytes), np.uint8)
    if nbytes:
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0
    return out[:nbytes]


def _device_search(edsbwt, idx, buf, offs, first_id, locate, counters=True, repeat=1):
    """search_device over the whole batch (no chunking) on torch's current stream, as bench.py's
    device-resident leg calls it; repeat > 1 calls it again on the same buffers (the timed steps'
    reuse) and returns the last call's counts and records."""
    torch = pytest.importorskip("torch")
    npat = offs.size - 1
    d_bytes = torch.from_numpy(buf.copy()).cuda()
    d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_counts = torch.zeros(npat, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(repeat):
        d_counts.fill_(-1)
        ptr, n = idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), npat, d_counts.data_ptr(), first_pattern_id=first_id,
                                   locate=locate, stream=stream, counters=counters)
    torch.cuda.synchronize()
    counts = d_counts.cpu().numpy().view(np.uint32).copy()
    occ = _d2h(ptr, n * 20).view(edsbwt.OCC_DTYPE) if locate else np.zeros(0, edsbwt.OCC_DTYPE)
    return counts, occ


def _device_tags(edsbwt, idx, buf, offs, first_id, locate):
    """search_device over the whole batch (no chunking): counts, records, path tags."""
    counts, occ = _device_search(edsbwt, idx, buf, offs, first_id, locate)
    tags = idx.path_tags(offs.size - 1)
    return counts, occ, tags, idx.stats()


def _rare_sample(edsbwt, tags, npat, strided=16384, deep_max=8192):
    """16384 strided patterns + every wide / level re-run / redo pattern + up to deep_max of
    the k_deep ones (evenly spaced)."""
    rare = np.flatnonzero(tags & (edsbwt.PATH_WIDE | edsbwt.PATH_LEVELS | edsbwt.PATH_REDO))
    deep = np.flatnonzero(tags & edsbwt.PATH_DEEP)
    if deep.size > deep_max:
        deep = deep[np.linspace(0, deep.size - 1, deep_max).astype(np.int64)]
    s = np.linspace(0, npat - 1, min(strided, npat)).astype(np.int64)
    return np.union1d(np.union1d(s, rare), deep), rare, deep


def _check_production(oracle, edsbwt, monkeypatch, name, expect_direct):
    monkeypatch.setenv("EDSBWT_PATH_TAGS", "1")
    w = workloads.CONFIGS[name]
    wd = workloads.default_workdir()
    workloads.ensure_built()
    eds, base = workloads.build_index(w, wd)
    lo, hi = workloads.shard(w, 0, 1)
    pats = workloads.pattern_file(w, eds, wd, lo, hi)
    planted = workloads.planted_mask(pats)
    buf, offs = edsbwt.read_pattern_file(pats)
    npat = offs.size - 1
    assert npat == w.patterns and planted.size == npat
    with edsbwt.Index(base) as idx:
        if expect_direct:
            assert idx.ktab_depth == 15 and idx.pair_blocks
        counts, occ = idx.search((buf, offs), first_pattern_id=lo + 1, locate=True)
        st = idx.stats()
        if expect_direct:
            assert st["start_depth"] == 15 and st["trie_nodes"] == 0, st  # packed direct start
        c2, o2 = idx.search((buf, offs), first_pattern_id=lo + 1, locate=False)
        assert np.array_equal(c2, counts) and o2.size == 0
        dc, do, tags, dst = _device_tags(edsbwt, idx, buf, offs, lo + 1, locate=True)
        assert np.array_equal(dc, counts) and np.array_equal(do, occ)
    # the exact build bench.py times: a fresh index without path tags, the
    # device-resident call with EDSBWT_NO_COUNTERS (the counter-free k_deep_direct / k_deep
    # instantiations), three calls on the same buffers as the timed steps make them; its counts and
    # every record equal the counted device run and the host path above
    monkeypatch.delenv("EDSBWT_PATH_TAGS")
    with edsbwt.Index(base) as idx:
        fc, fo = _device_search(edsbwt, idx, buf, offs, lo + 1, locate=True, counters=False, repeat=3)
        fst = idx.stats()
        assert fst["redo_searches"] == 0 and (not expect_direct or fst["start_depth"] == 15)
        assert np.array_equal(fc, counts) and np.array_equal(fo, occ)
        if name == "c2":  # C2's timed step is count-only
            fc2, fo2 = _device_search(edsbwt, idx, buf, offs, lo + 1, locate=False, counters=False, repeat=2)
            assert np.array_equal(fc2, counts) and fo2.size == 0
    # whole-batch properties
    assert int(counts.astype(np.uint64).sum()) == occ.size
    assert (counts[planted] > 0).all()
    pat0 = occ["pat"].astype(np.int64) - (lo + 1)
    assert (np.diff(pat0) >= 0).all()
    assert np.array_equal(np.bincount(pat0, minlength=npat), counts.astype(np.int64))
    bad, first = oracle.check_records(eds, buf, offs, occ, lo + 1, threads=THREADS)
    assert bad == 0, (bad, occ[first])
    # literal oracle: head + strided
    idx_s = _sample(npat)
    t_lit, _ = _compare_sample(oracle, base, buf, offs, counts, occ, idx_s, lo + 1, name)
    # trie-sharing oracle: strided + every rare-path pattern + k_deep ones
    idx_r, rare, deep = _rare_sample(edsbwt, tags, npat)
    t_trie, k = _compare_sample(oracle, base, buf, offs, counts, occ, idx_r, lo + 1, name, trie=True)
    _report(name, {"config": name, "patterns": int(npat), "records": int(occ.size), "planted": int(planted.sum()),
                   "check_records_bad": bad, "literal_sample": int(idx_s.size), "literal_s": round(t_lit, 1),
                   "trie_sample": int(idx_r.size), "trie_s": round(t_trie, 1), "trie_sample_records": k,
                   "tagged_deep": int((tags & edsbwt.PATH_DEEP).astype(bool).sum()), "deep_in_sample": int(deep.size),
                   "tagged_wide": int((tags & edsbwt.PATH_WIDE).astype(bool).sum()),
                   "tagged_levels": int((tags & edsbwt.PATH_LEVELS).astype(bool).sum()),
                   "tagged_redo": int((tags & edsbwt.PATH_REDO).astype(bool).sum()), "rare_in_sample": int(rare.size),
                   "device_stats": {k2: dst[k2] for k2 in ("deep_overflow", "deep_level_rerun", "redo_searches", "start_depth")},
                   "timed_build_checked": "search_device with EDSBWT_NO_COUNTERS (bench.py's timed build), 3 calls, no path "
                                          "tags: counts and every record equal to the counted device run and the host path",
                   "match": True})
    return counts, occ


def test_c3_production_parity(oracle, edsbwt, monkeypatch):
    """C3: ~100 Mchar COVID-like EDS, 10M planted 31-mers, full locate, default knobs."""
    _check_production(oracle, edsbwt, monkeypatch, "c3", expect_direct=True)


def test_c2_production_parity(oracle, edsbwt, monkeypatch):
    """C2: 10 Mchar EDS, 1M random 20-mers; counts (the configuration is count-only) and,
    for the samples, records too."""
    _check_production(oracle, edsbwt, monkeypatch, "c2", expect_direct=False)


def test_c4_rank_shard_parity(oracle, edsbwt):
    """C4 (BASELINE configs[3]): the C3 index, 100M planted 31-mers (seed 5) sharded over 8
    ranks.  The last rank's contiguous shard — stream ids [87.5M, 100M), #Pat = lo + 1 —
    through edsbwt_search_lines from page-locked memory as bench.py's rank searches it: every
    pattern found, records pattern-major, every record spells its pattern in the .eds, and
    the oracle's counts and records for its first and last 512 patterns."""
    w = workloads.CONFIGS["c4"]
    wd = workloads.default_workdir()
    workloads.ensure_built()
    eds, base = workloads.build_index(w, wd)
    lo, hi = workloads.shard(w, 7, 8)
    assert (lo, hi) == (87_500_000, 100_000_000)
    pats = workloads.pattern_file(w, eds, wd, lo, hi)
    planted = workloads.planted_mask(pats)
    npat = hi - lo
    text = edsbwt.read_pattern_file_pinned(pats)
    cb = edsbwt.HostBuffer(4 * (npat + 1))
    counts = cb.array(np.uint32, npat + 1)
    with edsbwt.Index(base) as idx:
        n, ptr, nocc = idx.search_lines(text.ptr, text.nbytes, cb.ptr, npat + 1, first_pattern_id=lo + 1, locate=True, keep=True)
        st = idx.stats()
        assert n == npat and st["chunks"] > 5
        occ = idx.occ_view(ptr, nocc).copy()
        idx.occ_free(ptr)
    counts = counts[:npat].copy()
    text.free()
    cb.free()
    buf, offs = edsbwt.read_pattern_file(pats)
    assert planted.all() and (counts > 0).all()
    assert int(counts.astype(np.uint64).sum()) == occ.size
    pat0 = occ["pat"].astype(np.int64) - (lo + 1)
    assert pat0.min() >= 0 and (np.diff(pat0) >= 0).all()
    assert np.array_equal(np.bincount(pat0, minlength=npat), counts.astype(np.int64))
    bad, first = oracle.check_records(eds, buf, offs, occ, lo + 1, threads=THREADS)
    assert bad == 0, (bad, occ[first])
    idx_s = np.union1d(np.arange(512), np.arange(npat - 512, npat))
    t_lit, k = _compare_sample(oracle, base, buf, offs, counts, occ, idx_s, lo + 1, "c4")
    _report("c4", {"config": "c4", "rank": 7, "world": 8, "first_pattern_id": lo + 1, "patterns": npat, "records": int(occ.size),
                   "chunks": st["chunks"], "redo_searches": st["redo_searches"], "check_records_bad": bad,
                   "literal_sample": int(idx_s.size), "literal_s": round(t_lit, 1), "sample_records": k, "match": True})


def _group_ends(buf, offs, alphabet, G):
    """First and last batch position of every trie-subtree search group (engine.hip run_grouped,
    kernels.hip k_pattern_group: patterns grouped by their last k characters' codes, G =
    (sigma + 2)^k groups; alphabet = the index's symbols, '#' first: code_of[byte] = its position)."""
    sigma = len(alphabet)
    if G <= 1:
        return np.zeros(0, np.int64)
    k = int(round(np.log(G) / np.log(sigma + 2)))
    assert (sigma + 2) ** k == G, (G, sigma)
    code = np.full(256, sigma + 1, np.int64)
    for j, ch in enumerate(alphabet):
        code[ch] = j + 1  # k_pattern_group: v = code_of + 1, sigma + 1 outside the alphabet
    ends = offs[1:].astype(np.int64)
    lens = np.diff(offs.astype(np.int64))
    gid = np.zeros(lens.size, np.int64)
    for t in range(k):
        v = np.where(t < lens, code[buf[np.maximum(ends - 1 - t, 0)]], 0)
        gid = gid * (sigma + 2) + v
    out = []
    for g in np.unique(gid):
        m = np.flatnonzero(gid == g)
        out += [m[0], m[-1]]
    return np.unique(np.array(out, np.int64))


def _progress(msg: str) -> None:
    """A stage line appended to $EDSBWT_TEST_PROGRESS (tools/gpu.sh points it into gpurun_out/),
    so a long production test shows progress while pytest captures its output."""
    path = os.environ.get("EDSBWT_TEST_PROGRESS")
    if path:
        with open(path, "a") as f:
            f.write(f"[c5 parity] {msg} ({time.strftime('%H:%M:%S')})\n")


def test_c5_production_parity(oracle, edsbwt, monkeypatch):
    """C5 (BASELINE configs[4]): the 1 Gchar EDS with 20% empty-word segments and the 200K
    mixed 8/16/32/64-mer batch of bench.py's C5 line.
    * Counts of the whole batch (count-only, bench.py's timed C5 leg), from the host path and
      the device-resident path with path tags (EDSBWT_PATH_TAGS): equal, every planted pattern found.
    * Located (the reference always locates, MOVE_EDSBWTSearch.cpp:328-369): every >= 32-mer, and
      512 8-mers + 512 16-mers (tens of millions of records): Σ records == counts, records
      pattern-major, every record spells its pattern in the .eds (orc_check_records).
    * The oracle's counts and records, in order, for: 8 patterns per length x planted class;
      up to 64 of the patterns the device walk sent to the wide lists / level re-run
      (deep_overflow) and up to 64 of those its register-list walk k_deep finished; the first
      and last pattern of every trie-subtree search group."""
    monkeypatch.setenv("EDSBWT_PATH_TAGS", "1")
    w = workloads.CONFIGS["c5"]
    wd = workloads.default_workdir()
    workloads.ensure_built()
    t0 = time.time()
    _progress("index")
    eds, base = workloads.build_index(w, wd)
    t_index = time.time() - t0
    _progress(f"index ready in {t_index:.0f} s")
    lo, hi = workloads.shard(w, 0, 1)
    pats = workloads.pattern_file(w, eds, wd, lo, hi)
    planted = workloads.planted_mask(pats)
    buf, offs = edsbwt.read_pattern_file(pats)
    npat = offs.size - 1
    lens = (offs[1:] - offs[:-1]).astype(np.int64)
    assert npat == w.patterns and set(np.unique(lens).tolist()) == {8, 16, 32, 64}
    rng = np.random.default_rng(5)
    samp = []
    for L in (8, 16, 32, 64):
        for pl in (True, False):
            cand = np.flatnonzero((lens == L) & (planted == pl))
            samp.append(rng.choice(cand, size=min(8, cand.size), replace=False))
    short_loc = np.sort(np.concatenate([rng.choice(np.flatnonzero(lens == L), size=512, replace=False) for L in (8, 16)]))
    loc = np.union1d(np.flatnonzero(lens >= 32), short_loc)
    with edsbwt.Index(base) as idx:
        t = time.time()
        counts, _ = idx.search((buf, offs), first_pattern_id=lo + 1, locate=False)
        t_count = time.time() - t
        _progress(f"count-only batch in {t_count:.1f} s")
        st = idx.stats()
        dc, _, tags, dst = _device_tags(edsbwt, idx, buf, offs, lo + 1, locate=False)
        assert np.array_equal(dc, counts)
        sb, so = _subset(buf, offs, loc)
        t = time.time()
        cl, ol = idx.search((sb, so), first_pattern_id=1, locate=True)
        t_loc = time.time() - t
        _progress(f"located {loc.size} patterns in {t_loc:.1f} s")
        alphabet = idx.alphabet
    assert (counts[planted] > 0).all()
    assert np.array_equal(cl, counts[loc]) and int(cl.astype(np.uint64).sum()) == ol.size
    pat0 = ol["pat"].astype(np.int64) - 1
    assert (np.diff(pat0) >= 0).all() and np.array_equal(np.bincount(pat0, minlength=loc.size), cl.astype(np.int64))
    bad, first = oracle.check_records(eds, sb, so, ol, 1, threads=THREADS)
    assert bad == 0, (bad, ol[first])
    _progress("records spelled")
    # the targeted oracle sample: the rare paths of this walk (wide lists / level re-run: round 3
    # had 433 such patterns at C5, none since the level start table; k_deep's register lists)
    def spread(a, n):
        return a[np.linspace(0, a.size - 1, min(n, a.size)).astype(np.int64)] if a.size else a
    ovf = np.flatnonzero(tags & (edsbwt.PATH_WIDE | edsbwt.PATH_LEVELS | edsbwt.PATH_REDO))
    assert np.flatnonzero(tags & (edsbwt.PATH_WIDE | edsbwt.PATH_LEVELS)).size == dst["deep_overflow"]
    ovf_s = spread(ovf, 64)
    deep_s = spread(np.flatnonzero(tags & edsbwt.PATH_DEEP), 64)
    gends = _group_ends(buf, offs, alphabet, st["search_groups"])
    idx_s = np.unique(np.concatenate(samp + [ovf_s, deep_s, gends]))
    with edsbwt.Index(base) as idx:
        ss, soo = _subset(buf, offs, idx_s)
        cs, os_ = idx.search((ss, soo), first_pattern_id=1, locate=True)
    assert np.array_equal(cs, counts[idx_s])
    eng = oracle.Engine(base, 8)
    t = time.time()
    _progress(f"oracle sample of {idx_s.size} patterns")
    oc, oo, _ = eng.search(ss, soo, first_pattern_id=1, threads=THREADS, trie=True)
    t_orc = time.time() - t
    eng.close()
    assert np.array_equal(oc, cs), (idx_s[oc != cs][:8].tolist(), oc[oc != cs][:8].tolist(), cs[oc != cs][:8].tolist())
    assert np.array_equal(oo, os_)
    _report("c5", {"config": "c5", "patterns": int(npat), "planted": int(planted.sum()), "index_s": round(t_index, 1),
                   "count_only_s": round(t_count, 2), "search_groups": st["search_groups"], "occurrences": int(counts.astype(np.uint64).sum()),
                   "located_patterns": int(loc.size), "located_records": int(ol.size), "located_s": round(t_loc, 2),
                   "located_by_length": {str(L): int((lens[loc] == L).sum()) for L in (8, 16, 32, 64)}, "check_records_bad": bad,
                   "deep_overflow": int(dst["deep_overflow"]), "deep_overflow_in_sample": int(ovf_s.size),
                   "tagged_deep": int((tags & edsbwt.PATH_DEEP).astype(bool).sum()), "deep_in_sample": int(deep_s.size),
                   "start_depth": int(st["start_depth"]),
                   "group_ends_in_sample": int(gends.size), "oracle_sample": int(idx_s.size), "oracle_sample_records": int(oo.size),
                   "oracle": "trie-sharing restatement (orc_search_batch_trie, pinned to the literal loop by tests/test_oracle.py)",
                   "oracle_s": round(t_orc, 1),
                   "sample_lengths": {str(L): int((lens[idx_s] == L).sum()) for L in (8, 16, 32, 64)}, "match": True})
