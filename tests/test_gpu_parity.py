"""GPU parity: libedsbwt.so (hand-written gfx950 kernels) vs the oracle, bit-exact.

Counts per pattern and the occurrence records — including their order, which is
the order of <patterns>output_M_LF.csv — must equal the oracle's on the same index."""
import os
import random
import shutil

import numpy as np
import pytest

from conftest import GOLDEN
import edsgen

pytestmark = pytest.mark.gpu


def _pack(pats):
    bs = [p.encode() if isinstance(p, str) else p for p in pats]
    buf = np.frombuffer(b"".join(bs), np.uint8) if bs else np.zeros(0, np.uint8)
    offs = np.concatenate(([0], np.cumsum([len(p) for p in bs]))).astype(np.uint64)
    return buf, offs


def _build(oracle, tmp_path, text, name="idx"):
    (tmp_path / f"{name}.eds").write_text(text)
    base = str(tmp_path / name)
    oracle.transform(str(tmp_path / f"{name}.eds"), base)
    return base


def _compare(oracle, edsbwt, base, pats, table_too=True):
    buf, offs = _pack(pats)
    eng = oracle.Engine(base, 8)
    oc, oo, _ = eng.search(buf, offs)
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc)
        assert np.array_equal(go, oo), (go[:10], oo[:10])
        assert idx.stats()["locate_offsets"] == int(oo["offset"].astype(np.uint64).sum())
        gc2, go2 = idx.search((buf, offs), locate=False)
        assert np.array_equal(gc2, oc) and go2.size == 0
        if table_too:
            gc3, go3 = idx.search((buf, offs), table=True)
            assert np.array_equal(gc3, oc) and np.array_equal(go3, oo)
        st = idx.stats()
        assert st["found"] == int((oc > 0).sum())
        gw, gow = idx.search((buf, offs), walk=True)      # the reference's full walk to '#'
        assert np.array_equal(gw, oc) and np.array_equal(gow, oo)
        assert idx.stats()["locate_lf_steps"] == int(oo["offset"].astype(np.uint64).sum())
        gc4, go4 = idx.search((buf, offs), deep=False)   # level-synchronous path only
        assert np.array_equal(gc4, oc) and np.array_equal(go4, oo)
        # count only on the level path: finishing counts summed inside the step (fused finish),
        # from the table's depth and from depth 0
        for ktab in (True, False):
            gcf, gof = idx.search((buf, offs), locate=False, deep=False, ktab=ktab)
            assert np.array_equal(gcf, oc) and gof.size == 0
        gk, gok = idx.search((buf, offs), ktab=False)     # walk from depth 0, no k-mer start table
        assert np.array_equal(gk, oc) and np.array_equal(gok, oo)
        assert idx.stats()["start_depth"] == 0
        gt, got = idx.search((buf, offs), direct=False)   # trie seeded from the table, never the direct start
        assert np.array_equal(gt, oc) and np.array_equal(got, oo)
        gp, gop = idx.search((buf, offs), pairs=False)   # one character per rank line in k_deep_fast
        assert np.array_equal(gp, oc) and np.array_equal(gop, oo)
        gx, gox = idx.search((buf, offs), text=False)    # single rows stepped, not compared with the text
        assert np.array_equal(gx, oc) and np.array_equal(gox, oo)
        for deep in (True, False):                       # reference-ordered lists at every depth
            gc5, go5 = idx.search((buf, offs), ordered=True, deep=deep)
            assert np.array_equal(gc5, oc) and np.array_equal(go5, oo)
    # the defaults' A/B fallbacks (read when an index opens): the finisher pass instead of the
    # fused count (k_fin_flags / k_fin_emit), no text items, eof_seg link keys without the chain
    # bit (also taken when S >= 2^31), one lane per wide list (k_deep_wide), 64-B segment rows without
    # the dollar step's text-item entries, k_deep's other dispatched build (5 waves per SIMD), the
    # separate count pass instead of the deep kernels' fused counts, the per-pattern scan of the
    # counts instead of per-tile record offsets, the locate kernel's own counts, and k_deep one
    # character per step (no pair entries), k_locate_pp's block-rounds on a 1- and 3-block grid, its
    # 512-record stage, and k_deep_direct's links through the segment table and srow (no seglink lines)
    for var, val in (("EDSBWT_FUSE_FINISH", "0"), ("EDSBWT_TEXT_ITEMS", "0"), ("EDSBWT_LINK_CB", "0"), ("EDSBWT_DEEP_WAVE", "0"),
                     ("EDSBWT_SEGTEXT", "0"), ("EDSBWT_DEEPQ_WAVES", "5"), ("EDSBWT_FUSED_COUNTS", "0"), ("EDSBWT_TILE_SCAN", "0"),
                     ("EDSBWT_LOCATE_COUNTS", "1"), ("EDSBWT_DEEPQ_PAIRS", "0"), ("EDSBWT_LOC_BLOCKS", "1"), ("EDSBWT_LOC_BLOCKS", "3"),
                     ("EDSBWT_LOC_STAGE", "512"), ("EDSBWT_SEGLINK", "0"), ("EDSBWT_DIRECT_BACK", "0")):
        old = os.environ.get(var)
        os.environ[var] = val
        try:
            with edsbwt.Index(base) as idx:
                for kw in ({}, {"locate": False}, {"locate": False, "deep": False}, {"locate": False, "deep": False, "ktab": False}):
                    gv, gov = idx.search((buf, offs), **kw)
                    assert np.array_equal(gv, oc), (var, kw)
                    if kw.get("locate", True):
                        assert np.array_equal(gov, oo), (var, kw)
        finally:
            if old is None:
                os.environ.pop(var)
            else:
                os.environ[var] = old
    return oc, oo


def test_readme_kat_gpu(oracle, edsbwt, tmp_path):
    base = _build(oracle, tmp_path, open(os.path.join(GOLDEN, "test.eds")).read(), "test")
    oc, oo = _compare(oracle, edsbwt, base, ["TATT", "ACT", "TTAT"])
    assert [tuple(int(x) for x in r) for r in oo] == [(1, 3, 2, 0, 0), (1, 4, 3, 0, 1), (1, 7, 4, 0, 1), (1, 1, 1, 1, 0),
                                                      (3, 0, 1, 0, 1), (3, 4, 3, 0, 0), (3, 7, 4, 0, 0)]


def test_move_edsbwt_mirror_csv(oracle, edsbwt, tmp_path):
    base = _build(oracle, tmp_path, open(os.path.join(GOLDEN, "test.eds")).read(), "test")
    shutil.copy(os.path.join(GOLDEN, "kmers.txt"), tmp_path / "kmers.txt")
    m = edsbwt.MoveEDSBWT(base, str(tmp_path / "kmers.txt"))
    assert (m.count_found, m.count_not_found) == (1, 6)
    assert open(tmp_path / "kmers.txtoutput_M_LF.csv", "rb").read() == \
        b"#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n1\t0\t1\t0\t1\n1\t4\t3\t0\t0\n1\t7\t4\t0\t0\n"


def test_example_paper_gpu(oracle, edsbwt, tmp_path):
    base = _build(oracle, tmp_path, open(os.path.join(GOLDEN, "examplePaper.eds")).read(), "ex")
    _compare(oracle, edsbwt, base, ["TAC", "A", "CTA", "GTCT", "ACTAC", "Q", "", "T"])


@pytest.mark.parametrize("seed", range(10))
def test_random_eds_gpu(oracle, edsbwt, tmp_path, seed):
    rng = random.Random(100 + seed)
    segs = edsgen.random_eds(rng, rng.randint(20, 400), alphabet="ACGT" if seed % 3 else "ACGTN",
                             lmax=3 + seed, p_empty=0.0 if seed % 4 == 0 else 0.25)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = []
    for _ in range(400):
        m = rng.randint(1, 24)
        p = edsgen.planted(rng, segs, m) if rng.random() < 0.6 else None
        pats.append(p or "".join(rng.choice("ACGT") for _ in range(m)))
    pats += pats[:40]                     # duplicates share trie nodes
    pats += ["ACGTX", "NNNN", "#A", "A#", "AC\r"]  # bytes outside / the end-marker itself
    _compare(oracle, edsbwt, base, pats)


def test_larger_eds_gpu(oracle, edsbwt, tmp_path):
    rng = random.Random(5)
    segs = edsgen.random_eds(rng, 6000, lmax=7, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.choice([8, 12, 20, 31])) or "ACGT" for _ in range(3000)]
    pats += ["".join(rng.choice("ACGT") for _ in range(20)) for _ in range(3000)]
    _compare(oracle, edsbwt, base, pats)


@pytest.mark.parametrize("alphabet", ["ACGT", "ACGTNRY"])
def test_long_patterns_gpu(oracle, edsbwt, tmp_path, alphabet):
    """Patterns spanning several key chunks (3-bit codes for ACGT, 4-bit once the
    alphabet has 7 symbols + '#'), and blocks of patterns too long to stage in LDS."""
    rng = random.Random(len(alphabet))
    segs = edsgen.random_eds(rng, 3000, alphabet=alphabet, lmax=9, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.choice([15, 16, 17, 21, 22, 33, 48, 64, 70])) or "ACGT" for _ in range(1500)]
    pats += [edsgen.planted(rng, segs, rng.randint(100, 200)) or "A" * 150 for _ in range(300)]
    pats += ["".join(rng.choice(alphabet) for _ in range(rng.randint(1, 90))) for _ in range(1500)]
    # suffixes shared beyond one key chunk (21 / 16 symbols) with different heads: the
    # chunk-0 sort sees ties and the full multi-chunk sort must run
    for _ in range(30):
        tail = edsgen.planted(rng, segs, 26) or "ACGT" * 7
        pats += ["".join(rng.choice(alphabet) for _ in range(rng.randint(1, 12))) + tail for _ in range(5)]
    _compare(oracle, edsbwt, base, pats, table_too=False)
    # one tie group larger than k_fix_ties takes (kTieMax = 256): the full sort runs
    tail = edsgen.planted(rng, segs, 26) or "ACGT" * 7
    big = ["".join(rng.choice(alphabet) for _ in range(rng.randint(3, 10))) + tail for _ in range(400)]
    _compare(oracle, edsbwt, base, pats[:500] + big, table_too=False)


def test_c5_style_gpu(oracle, edsbwt, tmp_path):
    """C5's shape at a size the oracle finishes in seconds: ~20% empty-word segments and
    a mixed 8–64-mer batch (BASELINE.json configs[4] is 1 Gchar; its production index and
    batch are tests/test_production_gpu.py::test_c5_production_parity)."""
    rng = random.Random(55)
    segs = edsgen.random_eds(rng, 20000, kmax=4, lmax=12, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(8, 64)) or "ACGT" for _ in range(3000)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(8, 64))) for _ in range(3000)]
    _compare(oracle, edsbwt, base, pats, table_too=False)


def test_level_table_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """The deep level start table (engine.hip build_ltab; C5 at depth 8), forced on a small
    C5-shaped EDS with a shallow k-mer table (EDSBWT_KTAB_K=3, EDSBWT_LTAB_K=6): batches whose
    patterns are all >= 6 long start at depth 6 from it — patterns of exactly 6 finish at the
    start — located and count-only, on the level path and with the deep cutover, in forced
    trie-subtree groups (the whole C5 batch is grouped because its start passes 2^31 items:
    tests/test_production_gpu.py), with text items stopped at the first cutover-eligible depth
    (the default) or at 32 per node, against the oracle and against the same searches without the table
    (EDSBWT_NO_LTAB); a batch holding a shorter pattern starts from the k-mer table instead."""
    monkeypatch.setenv("EDSBWT_KTAB_K", "3")
    monkeypatch.setenv("EDSBWT_LTAB_K", "6")
    rng = random.Random(8686)
    segs = edsgen.random_eds(rng, 5000, kmax=4, lmax=7, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.choice([6, 6, 7, 9, 12, 16, 24, 40])) or "ACGTAC" for _ in range(2500)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.choice([6, 8, 16, 32]))) for _ in range(1500)]
    pats += [p[:2] + "N" + p[3:] for p in pats[:40]] + pats[:100]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    short = pats[:300] + ["ACGTA"]
    sbuf, soffs = _pack(short)
    soc, soo, _ = oracle.Engine(base, 8).search(sbuf, soffs)
    with edsbwt.Index(base) as idx:
        assert idx.ktab_depth == 3 and idx.ltab_depth == 6 and idx.ltab_groups == 16 and idx.ltab_items > 0
        for kw in ({}, {"locate": False}, {"deep": False}, {"locate": False, "deep": False}, {"direct": False}):
            gc, go = idx.search((buf, offs), **kw)
            assert idx.stats()["start_depth"] == 6, kw
            assert np.array_equal(gc, oc), kw
            if kw.get("locate", True):
                assert np.array_equal(go, oo), kw
        gs, gso = idx.search((sbuf, soffs))
        assert idx.stats()["start_depth"] == 3
        assert np.array_equal(gs, soc) and np.array_equal(gso, soo)
    # ... and the located finishers at the table's start through the emit + sort path, and the records
    # through locate tasks (one wave or one lane per pattern, then k_locate) instead of straight from
    # the lists (k_locate_lists, the default with dense samples)
    for env in ({"EDSBWT_NO_LTAB": "1"}, {"EDSBWT_FORCE_GROUPS": "2"}, {"EDSBWT_FORCE_GROUPS": "1", "EDSBWT_TEXT_STOP": "32"},
                {"EDSBWT_LT_FIN_DIRECT": "0"}, {"EDSBWT_TASKS_WAVE": "2", "EDSBWT_LOCATE_LISTS": "0"},
                {"EDSBWT_TASKS_WAVE": "0", "EDSBWT_LT_FIN_DIRECT": "0", "EDSBWT_LOCATE_LISTS": "0"}, {"EDSBWT_LOCATE_LISTS": "0"}):
        for k_, v_ in env.items():
            monkeypatch.setenv(k_, v_)
        with edsbwt.Index(base) as idx:
            for kw in ({}, {"locate": False}):
                gc, go = idx.search((buf, offs), **kw)
                st = idx.stats()
                assert st["start_depth"] == (3 if "EDSBWT_NO_LTAB" in env else 6), (env, kw)
                if "EDSBWT_FORCE_GROUPS" in env:
                    assert st["search_groups"] > 1, (env, kw)
                assert np.array_equal(gc, oc), (env, kw)
                if kw.get("locate", True):
                    assert np.array_equal(go, oo), (env, kw)
        for k_ in env:
            monkeypatch.delenv(k_)


@pytest.mark.parametrize("k", [1, 2])
def test_grouped_search(oracle, edsbwt, tmp_path, monkeypatch, k):
    """The trie-subtree split a batch falls back to when a depth outgrows 32-bit counts
    (forced here): same counts and records, in the same order."""
    monkeypatch.setenv("EDSBWT_FORCE_GROUPS", str(k))
    rng = random.Random(41 + k)
    segs = edsgen.random_eds(rng, 2000, lmax=6, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 30)) or "ACGT" for _ in range(1500)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 20))) for _ in range(500)] + ["", "N", "#A"]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert idx.stats()["search_groups"] > 1
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)


def test_unaligned_device_bytes(oracle, edsbwt, tmp_path):
    """search_device with a pattern buffer that is not 4-B aligned (the LDS staging
    of the key kernel needs alignment and must fall back)."""
    torch = pytest.importorskip("torch")
    rng = random.Random(3)
    segs = edsgen.random_eds(rng, 800, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(4, 30)) or "ACGT" for _ in range(500)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    with edsbwt.Index(base) as idx:
        raw = torch.zeros(buf.size + 1, dtype=torch.uint8, device="cuda")
        raw[1:] = torch.from_numpy(buf.copy()).cuda()
        d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_counts = torch.zeros(len(pats), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        ptr, n = idx.search_device(raw.data_ptr() + 1, d_offs.data_ptr(), len(pats), d_counts.data_ptr())
        assert np.array_equal(d_counts.cpu().numpy().astype(np.uint32), oc)
        occ = np.zeros(n, dtype=edsbwt.OCC_DTYPE)
        if n:
            assert hip.hipMemcpy(ctypes.c_void_p(occ.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(occ.nbytes), 2) == 0
        assert np.array_equal(occ, oo)


def test_deep_overflow_rerun(oracle, edsbwt, tmp_path):
    """Lists longer than k_deep's registers (many '#' rows / many intervals) fall back
    to the level path: force it with an EDS whose segments repeat one motif."""
    rng = random.Random(9)
    motif = ["AC", "ACA", "CA", "A", ""]
    segs = [[rng.choice(motif) or "A" for _ in range(rng.randint(1, 5))] for _ in range(3000)]
    for s in segs:
        if rng.random() < 0.3 and len(s) > 1:
            s[0] = ""
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = ["".join(rng.choice("AC") for _ in range(rng.randint(6, 30))) for _ in range(2000)]
    pats += [edsgen.planted(rng, segs, 25) or "ACA" for _ in range(2000)]
    oc, oo = _compare(oracle, edsbwt, base, pats, table_too=False)
    with edsbwt.Index(base) as idx:
        buf, offs = _pack(pats)
        idx.search((buf, offs))
        st = idx.stats()
        assert st["deep_from_depth"] > 0 and st["deep_overflow"] > 0, st
        gc, go = idx.search((buf, offs), wide=False)   # overflows straight to the level path
        st2 = idx.stats()
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert st2["deep_level_rerun"] > 0, st2


def _kpos(base):
    """'#'-row rank of every word, from <base>_info.aux (EOF_ID_Copy, Appendix A)."""
    raw = open(base + "_info.aux", "rb").read()
    N, W = np.frombuffer(raw, np.uint32, 2)
    sigma = raw[8]
    eof = np.frombuffer(raw, np.uint32, count=int(W), offset=9 + sigma)
    kp = np.empty(int(W), np.int64)
    kp[eof] = np.arange(int(W))
    return kp


def test_legacy_order_readme(oracle, tmp_path):
    """README.md:144-167 example, produced by the legacy EDSBWTsearch engine: with
    --legacy the CLI's output.csv equals it byte for byte (rows in the legacy order)."""
    import subprocess
    from conftest import ROOT
    base = _build(oracle, tmp_path, open(os.path.join(GOLDEN, "test.eds")).read(), "test")
    shutil.copy(os.path.join(GOLDEN, "readme_kat_patterns.txt"), tmp_path / "p.txt")
    cli = os.path.join(ROOT, "eds-bwt_amd", "_build", "EDSBWTsearch")
    r = subprocess.run([cli, base, str(tmp_path / "p.txt"), "--quiet", "--legacy"], capture_output=True, text=True)
    assert r.returncode == 1, r.stderr
    assert (tmp_path / "p.txtoutput.csv").read_bytes() == open(os.path.join(GOLDEN, "readme_kat_expected.tsv"), "rb").read()


def test_legacy_order_random(oracle, edsbwt, tmp_path):
    """Legacy order = per pattern, by offset, then by the '#'-row rank of the word
    (findMultipleDollarsBackward's rounds, EDSBWTsearch.cpp:300-610)."""
    rng = random.Random(12)
    segs = edsgen.random_eds(rng, 1500, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 12)) or "ACGT" for _ in range(800)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    kp = _kpos(base)
    order = np.lexsort((kp[oo["word"]], oo["offset"], oo["pat"]))
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs), legacy=True)
        assert np.array_equal(gc, oc)
        assert np.array_equal(go, oo[order])


def test_cli_matches_oracle_csv(oracle, tmp_path):
    """EDSBWTsearch (C++ CLI over the C ABI) vs the oracle's MOVE_EDSBWTSearch restatement:
    identical <patterns>output_M_LF.csv bytes, count lines on stderr, exit code 1."""
    import subprocess
    from conftest import ROOT
    rng = random.Random(77)
    segs = edsgen.random_eds(rng, 500, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(4, 18)) or "ACGT" for _ in range(300)] + ["GATTACA", "N"]
    p1 = tmp_path / "p1.txt"
    p1.write_text("\n".join(pats) + "\n")
    p2 = tmp_path / "p2.txt"
    p2.write_text("\n".join(pats) + "\n")
    cli = os.path.join(ROOT, "eds-bwt_amd", "_build", "EDSBWTsearch")
    r = subprocess.run([cli, base, str(p1), "--quiet"], capture_output=True, text=True)
    assert r.returncode == 1, r.stderr   # mainMove_EDSBWT.cpp:61 returns 1 on success
    assert "bs took:" in r.stdout and not r.stdout.endswith("\n")
    ctr, _ = oracle.Engine(base).search_file(str(p2), str(tmp_path / "p2.txtoutput_M_LF.csv"))
    assert f"count_found = {ctr['found']}" in r.stderr and f"count_not_found = {ctr['not_found']}" in r.stderr
    assert (tmp_path / "p1.txtoutput_M_LF.csv").read_bytes() == (tmp_path / "p2.txtoutput_M_LF.csv").read_bytes()
    r = subprocess.run([cli, base], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stderr


def test_short_patterns_4bit_codes_gpu(oracle, edsbwt, tmp_path):
    """7 symbols + '#' (4-bit sort codes) and patterns shorter than one key chunk: the
    chunk's significant bits end at bit 64, the range rocPRIM mis-sorts unless it starts at 0."""
    rng = random.Random(77)
    segs = edsgen.random_eds(rng, 2000, alphabet="ACGTNRY", lmax=6, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(3, 15)) or "ACG" for _ in range(3000)]
    pats += ["".join(rng.choice("ACGTNRY") for _ in range(rng.randint(1, 15))) for _ in range(3000)]
    _compare(oracle, edsbwt, base, pats, table_too=False)


@pytest.mark.parametrize("seed", range(5))
def test_kmer_start_table_gpu(oracle, edsbwt, tmp_path, monkeypatch, seed):
    """Batches whose patterns are all longer than the k-mer start table's depth start
    straight from their D-mers' lists (direct start; forced here, since these small tables
    hold long lists) or from the trie seeded by the table (direct=False); results equal the
    oracle's and the walk from depth 0."""
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
    rng = random.Random(900 + seed)
    alphabet = ("ACGTN", "ACGT", "ACGTN", "ACGT", "ACGTNRY")[seed]  # 3-bit codes; 4-bit codes for 7 symbols
    segs = edsgen.random_eds(rng, 1500 + 500 * seed, alphabet=alphabet, lmax=4 + 2 * (seed % 4), p_empty=0.25 if seed % 2 else 0.1)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D = idx.ktab_depth
        assert D >= 2 and idx.ktab_items > 0
    pats = [edsgen.planted(rng, segs, rng.randint(D + 1, D + 20)) or "ACGT" * 8 for _ in range(800)]
    pats += ["".join(rng.choice(alphabet + "N") for _ in range(rng.randint(D + 1, 40))) for _ in range(400)]
    pats += ["N" * (D + 1), "ACGT" * 10 + "X"]  # a byte outside the alphabet inside / before the last D
    oc, oo = _compare(oracle, edsbwt, base, pats, table_too=seed == 0)
    buf, offs = _pack(pats)
    monkeypatch.setenv("EDSBWT_DIRECT_SORT", "0")  # direct start in input order
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert idx.stats()["trie_nodes"] == 0
    monkeypatch.delenv("EDSBWT_DIRECT_SORT")
    with edsbwt.Index(base) as idx:
        idx.search((buf, offs))
        assert idx.stats()["start_depth"] == D
        assert idx.stats()["trie_nodes"] == 0  # direct start: no trie built
        idx.search((buf, offs), direct=False)
        assert idx.stats()["start_depth"] == D and idx.stats()["trie_nodes"] > 0
        idx.search((buf, offs), ordered=True)  # the ordered path never uses the table
        assert idx.stats()["start_depth"] == 0


def _covid_like(rng, nseg):
    """Solid segments (one long string) alternating with short variant segments, some
    holding the empty word: the shape of BASELINE config C3 at test size."""
    segs = []
    for t in range(nseg):
        if t % 2 == 0:
            segs.append(["".join(rng.choice("ACGT") for _ in range(rng.randint(40, 120)))])
        else:
            segs.append(["" if rng.random() < 0.1 else "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 3)))
                         for _ in range(rng.randint(2, 4))])
    return segs


def test_pair_blocks_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """Two backward steps per rank entry (k_deep_fast, rent2): planted and random 31-mers,
    odd and even remaining lengths, patterns that die between the two steps and ones
    that meet '#' rows after the first — identical counts, records and step counts with
    the pair blocks on and off, and equal to the oracle."""
    monkeypatch.setenv("EDSBWT_TRIPLES", "1")  # three-step entries too (off by default)
    monkeypatch.setenv("EDSBWT_DEEPQ_PAIRS", "0")  # (k_deep's pair steps count a list's two steps at once)
    rng = random.Random(355)
    segs = _covid_like(rng, 800)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.choice([20, 21, 31, 32, 40, 47])) or "ACGT" * 8 for _ in range(3000)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.choice([18, 19, 31]))) for _ in range(1000)]
    buf, offs = _pack(pats)
    eng = oracle.Engine(base, 8)
    oc, oo, _ = eng.search(buf, offs)
    with edsbwt.Index(base) as idx:
        assert idx.pair_blocks
        for direct in (True, False):
            gc, go = idx.search((buf, offs), direct=direct)
            assert np.array_equal(gc, oc) and np.array_equal(go, oo)
            st_on = idx.stats()
            gc2, go2 = idx.search((buf, offs), direct=direct, pairs=False)
            assert np.array_equal(gc2, oc) and np.array_equal(go2, oo)
            st_off = idx.stats()
            assert st_on["intervals_stepped"] == st_off["intervals_stepped"]
    monkeypatch.setenv("EDSBWT_NO_TRIPLES", "1")  # two steps per entry at most
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert idx.stats()["intervals_stepped"] == st_on["intervals_stepped"]
    monkeypatch.setenv("EDSBWT_NO_RANK_ENTRIES", "1")  # the 64-row occ blocks only
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert idx.stats()["intervals_stepped"] == st_on["intervals_stepped"]


def test_packed_direct_start_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """Packed direct start: when every pattern is longer than the k-mer table's depth D0 by at
    most 16 symbols, each pattern's input index and remaining symbols are sorted along with
    its D-mer (k_ktab_direct) and k_deep_fast reads neither lengths nor key chunks.  Patterns
    with a symbol outside the alphabet after D0 take the empty list.  Same results as the
    unpacked direct start and the oracle."""
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")  # small tables hold long lists
    rng = random.Random(4096)
    segs = _covid_like(rng, 600)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    assert D0 >= 2
    pats = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(3000)]
    pats = [p[: D0 + 16] if len(p) > D0 + 16 else p for p in pats]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(D0 + 1, D0 + 16))) for _ in range(500)]
    pats += [p[:-1] + "N" for p in pats[:50]]  # outside the alphabet: in the D-mer (read first) ...
    pats += ["N" + p[1:] for p in pats[50:100]]  # ... and in the remaining symbols
    buf, offs = _pack(pats)
    eng = oracle.Engine(base, 8)
    oc, oo, _ = eng.search(buf, offs)
    got = {}
    for packed in ("1", "0"):
        monkeypatch.setenv("EDSBWT_DIRECT_PACKED", packed)
        with edsbwt.Index(base) as idx:
            gc, go = idx.search((buf, offs))
            assert idx.stats()["start_depth"] == D0 and idx.stats()["trie_nodes"] == 0  # direct start
            assert idx.stats()["text_rows"] > 0  # single rows compared with the text
            assert np.array_equal(gc, oc) and np.array_equal(go, oo)
            got[packed] = (gc, go)
            gp, gop = idx.search((buf, offs), pairs=False)
            assert np.array_equal(gp, oc) and np.array_equal(gop, oo)


def test_wide_kmer_entries_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """The wide k-mer table (k_ktab_wide: 32 B per D-mer, a one-row entry carries the row's
    sample and the 32 text characters before it, so k_deep_fast compares them with no further
    load) against the 8-B entries (EDSBWT_KT1_WIDE=0) and the oracle: patterns finished inside
    the window, ones longer than it (D0 + 33 .. D0 + 60: the compare goes on from the text),
    crossing into earlier segments, mismatching at either end, with bytes outside the alphabet;
    packed and unpacked direct starts, in input order (the default with the wide table) and
    sorted by D-mer, with and without the per-row text-compare entries (EDSBWT_SROW), located and
    count-only, the text compare on and off."""
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
    rng = random.Random(3232)
    segs = _covid_like(rng, 700)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    assert D0 >= 2
    short = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(2500)]
    short = [p[: D0 + 16] if len(p) > D0 + 16 else p for p in short]
    short += [p[:-2] + rng.choice("ACGT") + p[-1:] for p in short[:300]]   # a mismatch near the end
    short += [rng.choice("ACGT") + p[1:] for p in short[300:600]]          # ... at the start
    long_ = [edsgen.planted(rng, segs, rng.randint(D0 + 17, D0 + 60)) or "ACGT" * 20 for _ in range(1200)]
    long_ += [p[:4] + "N" + p[5:] for p in long_[:100]]                       # outside the alphabet
    sizes = {}
    for pats, packed in ((short, "1"), (short + long_, "0")):
        buf, offs = _pack(pats)
        oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
        monkeypatch.setenv("EDSBWT_DIRECT_PACKED", packed)
        monkeypatch.setenv("EDSBWT_DIRECT_SORT_MIN", "0")  # the D-mer sort even for this small batch, when on
        # -1: the default sort (input order when wide); srow: the per-row text-compare entries
        # link "1": 64-B wide entries with the first link's segment ranks (EDSBWT_KT1_LINK=1; "0", the
        # default: 32 B)
        for wide, sort_bits, srow, link in (("1", "-1", "1", "1"), ("1", "16", "1", "1"), ("0", "-1", "1", "1"), ("1", "-1", "0", "1"),
                                            ("0", "-1", "0", "1"), ("1", "-1", "1", "0")):
            monkeypatch.setenv("EDSBWT_KT1_WIDE", wide)
            monkeypatch.setenv("EDSBWT_DIRECT_SORT_BITS", sort_bits)
            monkeypatch.setenv("EDSBWT_SROW", srow)
            monkeypatch.setenv("EDSBWT_KT1_LINK", link)
            with edsbwt.Index(base) as idx:
                sizes[wide + srow + ("" if link == "1" else "n")] = idx.device_bytes
                for kw in ({}, {"locate": False}, {"text": False}):
                    gc, go = idx.search((buf, offs), **kw)
                    st = idx.stats()
                    assert st["start_depth"] == D0, (wide, sort_bits, srow, packed, kw)
                    assert np.array_equal(gc, oc), (wide, sort_bits, srow, packed, kw)
                    if kw.get("locate", True):
                        assert np.array_equal(go, oo), (wide, sort_bits, srow, packed, kw)
                    if not kw:
                        assert st["text_rows"] > 1000, st
    # the packed direct start with its keys computed inside k_deep_direct (the default on the
    # deferred input-order path) against the separate key kernel (EDSBWT_FUSED_KEYS=0), with
    # patterns outside the guessed lengths (the deferred check sends those batches to the redo)
    for pats in (short, short + ["ACGT" * 4, "A" * (D0 + 17)]):
        buf, offs = _pack(pats)
        oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
        # (and k_deep_direct's build without work counters, EDSBWT_DEEP_STATS=0)
        for fused, stats in (("1", "1"), ("0", "1"), ("1", "0")):
            monkeypatch.setenv("EDSBWT_FUSED_KEYS", fused)
            monkeypatch.setenv("EDSBWT_DEEP_STATS", stats)
            for k_ in ("EDSBWT_KT1_WIDE", "EDSBWT_DIRECT_SORT_BITS", "EDSBWT_SROW", "EDSBWT_DIRECT_PACKED", "EDSBWT_KT1_LINK"):
                monkeypatch.delenv(k_, raising=False)
            with edsbwt.Index(base) as idx:
                # (counters=False: the per-call EDSBWT_NO_COUNTERS, bench.py's timed steps)
                for kw in ({}, {"locate": False}, {"counters": False}, {"locate": False, "counters": False}):
                    gc, go = idx.search((buf, offs), **kw)
                    assert np.array_equal(gc, oc), (fused, stats, kw, len(pats))
                    if kw.get("locate", True):
                        assert np.array_equal(go, oo), (fused, stats, kw, len(pats))
    for k_ in ("EDSBWT_FUSED_KEYS", "EDSBWT_DEEP_STATS"):
        monkeypatch.delenv(k_)
    E = (4 ** D0) + 1
    assert sizes["11"] - sizes["01"] == 56 * E  # the wide table was built (64 B instead of 8 per D-mer) ...
    assert sizes["11n"] - sizes["01"] == 24 * E  # ... or 32 B without the link ranks
    assert sizes["11"] > sizes["10"]  # ... and the per-row entries


@pytest.mark.parametrize("pieces", ["2", "3", "5"])
def test_deep_pieces_gpu(oracle, edsbwt, tmp_path, monkeypatch, pieces):
    """The deferred direct start in pieces (engine.hip run_deep_pieces, EDSBWT_DEEP_PIECES): each
    piece's k_deep_direct, then k_deep over that piece's own queue on a second stream beside the
    next piece's k_deep_direct.  Same counts and records as one piece and as the oracle, located
    and count-only, with and without work counters, through search() and the device-resident call,
    and the queue's patterns really walked by k_deep (path tags)."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
    monkeypatch.setenv("EDSBWT_DEEP_PIECE_MIN", "1")
    monkeypatch.setenv("EDSBWT_PATH_TAGS", "1")
    rng = random.Random(4242)
    segs = _covid_like(rng, 900)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    pats = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(7000)]
    pats = [p[: D0 + 16] if len(p) > D0 + 16 else p for p in pats]
    pats += [rng.choice("ACGT") + p[1:] for p in pats[:500]]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=3)
    for np_ in ("1", pieces):
        monkeypatch.setenv("EDSBWT_DEEP_PIECES", np_)
        with edsbwt.Index(base) as idx:
            for kw in ({}, {"locate": False}, {"counters": False}):
                gc, go = idx.search((buf, offs), first_pattern_id=3, **kw)
                assert idx.stats()["start_depth"] == D0 and idx.stats()["redo_searches"] == 0
                assert np.array_equal(gc, oc), (np_, kw)
                if kw.get("locate", True):
                    assert np.array_equal(go, oo), (np_, kw)
            d_bytes = torch.from_numpy(buf.copy()).cuda()
            d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
            d_counts = torch.zeros(len(pats), dtype=torch.int32, device="cuda")
            for counters in (True, False):
                ptr, n = idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), len(pats), d_counts.data_ptr(), first_pattern_id=3,
                                           counters=counters)
                torch.cuda.synchronize()
                assert np.array_equal(d_counts.cpu().numpy().view(np.uint32), oc) and n == oo.size
            tags = idx.path_tags(len(pats))
            assert (tags & edsbwt.PATH_DEEP).sum() > 50  # queued patterns walked by k_deep in every piece
            deep = np.flatnonzero(tags & edsbwt.PATH_DEEP)
            assert deep.min() < len(pats) // int(pieces) and deep.max() >= len(pats) - len(pats) // int(pieces)


@pytest.mark.parametrize("env", [{}, {"EDSBWT_DEEP_K": "2", "EDSBWT_KTAB_K": "7"},
                                 {"EDSBWT_DEEP_K": "2", "EDSBWT_KTAB_K": "7", "EDSBWT_WAVE_TILES": "0"},
                                 {"EDSBWT_DEEP_K": "2", "EDSBWT_KTAB_K": "7", "EDSBWT_DEEP_PIECES": "3"},
                                 {"EDSBWT_DEEP_K": "2", "EDSBWT_KTAB_K": "7", "EDSBWT_STREAM2_EARLY": "0"}],
                         ids=["default", "K=2", "K=2, tiles after k_deep_wave", "K=2, 3 pieces", "K=2, second stream on first use"])
def test_wave_tiles_gpu(oracle, edsbwt, tmp_path, monkeypatch, env):
    """The located deferred direct start sums its record-offset tiles on the second stream beside
    k_deep_wave (engine.hip run_deep: k_mark_wide + k_count_tiles without the patterns k_deep_wave
    walks, then k_tile_fix): counts and every record equal to the oracle's, through search() and the
    device-resident call (with and without work counters, repeated on the same buffers: the bitmap
    must be clear again), with patterns really walked by k_deep_wave (7-mer start lists and K = 2:
    many lists overflow k_deep's registers), and the same with the tiles summed after k_deep_wave."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("EDSBWT_PATH_TAGS", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = random.Random(9091)
    segs = _covid_like(rng, 900)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    pats = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(6000)]
    pats = [p[: D0 + 16] if len(p) > D0 + 16 else p for p in pats]
    pats += [rng.choice("ACGT") + p[1:] for p in pats[:800]]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=2)
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs), first_pattern_id=2)
        assert idx.stats()["start_depth"] == D0 and idx.stats()["redo_searches"] == 0
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        d_bytes = torch.from_numpy(buf.copy()).cuda()
        d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_counts = torch.zeros(len(pats), dtype=torch.int32, device="cuda")
        for counters in (False, False, True):  # (path tags: of the last call, a counted one)
            d_counts.fill_(-1)
            ptr, n = idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), len(pats), d_counts.data_ptr(), first_pattern_id=2,
                                       counters=counters)
            torch.cuda.synchronize()
            assert np.array_equal(d_counts.cpu().numpy().view(np.uint32), oc) and n == oo.size
            assert idx.stats()["redo_searches"] == 0
        tags = idx.path_tags(len(pats))  # (of the last device-resident call)
        if env.get("EDSBWT_DEEP_K") == "2":
            assert (tags & edsbwt.PATH_WIDE).astype(bool).sum() > 20
        gc2, go2 = idx.search((buf, offs), first_pattern_id=2)
        assert np.array_equal(gc2, oc) and np.array_equal(go2, oo)


@pytest.mark.parametrize("direct", [True, False])
def test_single_row_text_compare_gpu(oracle, edsbwt, tmp_path, monkeypatch, direct):
    """Single-row intervals decided by comparing the pattern with the words' text: patterns
    ending inside a word, crossing into earlier segments (the compare stops at the word start
    and the walk goes on from the whole-word row), mismatching before or after the jump, with
    bytes outside the alphabet; count-only and locate; identical to the oracle and to the walk
    with the text compare off, and the compare really ran."""
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
    rng = random.Random(7331)
    segs = _covid_like(rng, 700)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    pats = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(3000)]
    pats += [edsgen.planted(rng, segs, rng.randint(D0 + 17, D0 + 60)) or "ACGT" * 20 for _ in range(1000)]
    pats += [p[:-3] + rng.choice("ACGT") + p[-2:] for p in pats[:500]]       # a mismatch near the end
    pats += [rng.choice("ACGT") + p[1:] for p in pats[500:1000]]            # ... at the start
    pats += [p[:5] + "N" + p[6:] for p in pats[1000:1100]]                  # outside the alphabet
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        for locate in (True, False):
            gc, go = idx.search((buf, offs), direct=direct, locate=locate)
            st = idx.stats()
            assert np.array_equal(gc, oc)
            if locate:
                assert np.array_equal(go, oo)
                assert st["locate_offsets"] == int(oo["offset"].astype(np.uint64).sum())
            assert st["text_rows"] > 1000 and st["text_chars"] > 10000, st
            gc2, go2 = idx.search((buf, offs), direct=direct, locate=locate, text=False)
            assert np.array_equal(gc2, oc) and idx.stats()["text_rows"] == 0
            if locate:
                assert np.array_equal(go2, oo)
    # the same with k_deep_direct's links through the segment table, then the row's srow line, and
    # with its rank steps kept to the end once an interval was wide (no return to the text compare)
    for var in ("EDSBWT_SEGLINK", "EDSBWT_DIRECT_BACK"):
        monkeypatch.setenv(var, "0")
        with edsbwt.Index(base) as idx:
            for locate in (True, False):
                gc3, go3 = idx.search((buf, offs), direct=direct, locate=locate)
                assert np.array_equal(gc3, oc), var
                if locate:
                    assert np.array_equal(go3, oo), var
        monkeypatch.delenv(var)


@pytest.mark.parametrize("env", [{"EDSBWT_LOC_BLOCKS": "1"}, {"EDSBWT_LOC_BLOCKS": "3"}, {"EDSBWT_LOC_BLOCKS": "5", "EDSBWT_LOC_STAGE": "512"},
                                 {"EDSBWT_LOC_BLOCKS": "3", "EDSBWT_LOC_PPT": "1"}, {"EDSBWT_LOC_PPT": "1"}],
                         ids=["1 block", "3 blocks", "5 blocks, stage 512", "3 blocks, 1 pattern per thread", "1 pattern per thread"])
def test_locate_block_rounds_gpu(oracle, edsbwt, tmp_path, monkeypatch, env):
    """k_locate_pp over many block-rounds (a grid of 1-5 blocks for ~6000 patterns: the production
    grid gives C3's 10M patterns 2-3 rounds per block): planted patterns ending in one row (records from the
    result's text position), in a row range and in interval lists, misses; records identical to the
    oracle's, count-only counts too."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = random.Random(4242)
    segs = _covid_like(rng, 700)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    pats = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(3000)]
    pats += [edsgen.planted(rng, segs, rng.randint(4, D0)) or "ACG" for _ in range(2000)]        # short: many occurrences
    pats += [rng.choice("ACGT") + p[1:] for p in pats[:1000]]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=5)
    assert oo.size > 2 * len(pats)
    with edsbwt.Index(base) as idx:
        for kw in ({}, {"direct": False}, {"locate": False}):
            gc, go = idx.search((buf, offs), first_pattern_id=5, **kw)
            assert np.array_equal(gc, oc), kw
            if kw.get("locate", True):
                assert np.array_equal(go, oo), kw
                assert idx.stats()["locate_offsets"] == int(oo["offset"].astype(np.uint64).sum())


def test_split_locate_scans_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """Locate offsets from the two separate scans (the path batches whose totals pass 2^32
    take) give the same records as the packed single scan."""
    rng = random.Random(77)
    segs = edsgen.random_eds(rng, 1500, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(2, 25)) or "ACGT" for _ in range(1500)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    monkeypatch.setenv("EDSBWT_SPLIT_SCANS", "1")
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)


@pytest.mark.parametrize("shift", [0, 2, 3])
def test_locate_sample_rates_gpu(oracle, edsbwt, tmp_path, monkeypatch, shift):
    """Locate from samples of every row (default: one read per occurrence) or of 1 in 2^shift
    word offsets (LF walk to the first sampled row): identical records and Σ offsets."""
    monkeypatch.setenv("EDSBWT_SAMPLE_SHIFT", str(shift))
    rng = random.Random(1200 + shift)
    segs = _covid_like(rng, 300)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(3, 40)) or "ACGT" for _ in range(1500)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        st = idx.stats()
        assert st["locate_offsets"] == int(oo["offset"].astype(np.uint64).sum())
        if shift == 0:
            assert st["locate_lf_steps"] == 0  # no walk: the sample of the row itself


def _lines_search(edsbwt, idx, text: bytes, first_id=1, locate=True, chunk_mb=None, pinned=True):
    """edsbwt_search_lines over `text` (page-locked or pageable): counts and records."""
    import ctypes
    nlines = text.count(b"\n") + (1 if text and not text.endswith(b"\n") else 0)
    if pinned:
        hb = edsbwt.HostBuffer(max(1, len(text)))
        hb.array(np.uint8, len(text))[:] = np.frombuffer(text, np.uint8)
        tptr = hb.ptr
        cb = edsbwt.HostBuffer(4 * max(1, nlines))
        counts = cb.array(np.uint32, nlines)
        cptr = cb.ptr
    else:
        arr = np.frombuffer(text, np.uint8).copy()
        tptr = arr.ctypes.data if arr.size else None
        counts = np.zeros(max(1, nlines), np.uint32)
        cptr = counts.ctypes.data
    npat, ptr, n = idx.search_lines(tptr, len(text), cptr, max(1, nlines), first_pattern_id=first_id, locate=locate, keep=True)
    assert npat == nlines
    occ = idx.occ_view(ptr, n).copy()
    idx.occ_free(ptr)
    return counts[:nlines].copy(), occ


@pytest.mark.parametrize("pinned", [True, False])
def test_search_lines_pipeline_gpu(oracle, edsbwt, tmp_path, monkeypatch, pinned):
    """The pattern file in host memory through edsbwt_search_lines: lines split on the device
    (getline semantics: '\\r' kept, empty lines, a last line without '\\n'), cut into many
    chunks (EDSBWT_CHUNK_MB tiny) so uploads, searches and downloads overlap across slots;
    page-locked and pageable buffers; first_pattern_id != 1 as a shard's would be."""
    rng = random.Random(808)
    segs = _covid_like(rng, 400)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 40)) or "ACGT" for _ in range(5000)]
    pats += ["", "AC\r", "N", "#A"] + ["".join(rng.choice("ACGT") for _ in range(rng.randint(5, 25))) for _ in range(1000)]
    rng.shuffle(pats)
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=77)
    for trailing in (True, False):
        text = ("\n".join(pats) + ("\n" if trailing else "")).encode()
        for mb in ("0.01", "64"):
            monkeypatch.setenv("EDSBWT_CHUNK_MB", mb)
            monkeypatch.setenv("EDSBWT_CHUNK_SINGLE_MB", "0")  # small batches would otherwise be one chunk
            with edsbwt.Index(base) as idx:
                gc, go = _lines_search(edsbwt, idx, text, first_id=77, pinned=pinned)
                st = idx.stats()
                assert np.array_equal(gc, oc) and np.array_equal(go, oo)
                assert st["chunks"] > (5 if mb == "0.01" else 0)
                assert st["patterns"] == len(pats) and st["occurrences"] == oo.size
                gc2, go2 = _lines_search(edsbwt, idx, text, first_id=77, locate=False, pinned=pinned)
                assert np.array_equal(gc2, oc) and go2.size == 0
            # the (bytes, offsets) host path, chunked the same way
            with edsbwt.Index(base) as idx:
                gc3, go3 = idx.search((buf, offs), first_pattern_id=77)
                assert np.array_equal(gc3, oc) and np.array_equal(go3, oo)


@pytest.mark.parametrize("pinned", [True, False])
def test_search_lines_packed_gpu(oracle, edsbwt, tmp_path, monkeypatch, pinned):
    """Fixed-length A/C/G/T lines go over PCIe at 2 bits per base (format.cpp packer,
    k_unpack_lines): the same counts and records as the oracle for several lengths, with a
    stray 'N' line that sends its chunk raw beside packed ones, a last line without '\\n',
    and the packer switched off (EDSBWT_PACK_LINES=0) for comparison."""
    rng = random.Random(909)
    segs = _covid_like(rng, 400)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    for L in (1, 7, 20, 31, 32):
        pats = []
        for _ in range(4000):
            p = edsgen.planted(rng, segs, L)
            pats.append(p if p and len(p) == L and set(p) <= set("ACGT") else "".join(rng.choice("ACGT") for _ in range(L)))
        stray = list(pats)
        stray[len(stray) // 2] = "N" * L
        for lines, trailing in ((pats, True), (pats, False), (stray, True)):
            buf, offs = _pack(lines)
            oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=5)
            text = ("\n".join(lines) + ("\n" if trailing else "")).encode()
            # "": one chunk, packed whole (the default) or its line blocks streamed (EDSBWT_PACK_STREAMED=1)
            for pack, mb, streamed in (("1", "0.02", "0"), ("0", "0.02", "0"), ("1", "", "0"), ("1", "", "1")):
                monkeypatch.setenv("EDSBWT_PACK_LINES", pack)
                monkeypatch.setenv("EDSBWT_PACK_STREAMED", streamed)
                if mb:
                    monkeypatch.setenv("EDSBWT_CHUNK_MB", mb)
                    monkeypatch.setenv("EDSBWT_CHUNK_SINGLE_MB", "0")
                else:
                    monkeypatch.delenv("EDSBWT_CHUNK_MB", raising=False)
                    monkeypatch.delenv("EDSBWT_CHUNK_SINGLE_MB", raising=False)
                with edsbwt.Index(base) as idx:
                    gc, go = _lines_search(edsbwt, idx, text, first_id=5, pinned=pinned)
                    st = idx.stats()
                assert np.array_equal(gc, oc) and np.array_equal(go, oo), (L, trailing, pack, mb, streamed)
                if not mb:
                    assert st["chunks"] == 1
                    continue
                if pack == "1" and lines is pats:
                    assert st["bytes_h2d"] <= len(lines) * ((L + 3) // 4)  # every chunk went packed
                elif pack == "1":
                    assert len(lines) * ((L + 3) // 4) < st["bytes_h2d"] < len(text)  # one chunk raw, the rest packed
                else:
                    assert st["bytes_h2d"] == len(text)


def test_search_lines_hip_streams_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """The host pipeline without explicit SDMA engines (EDSBWT_HSA_COPY=0: HIP-stream copies,
    the fallback when the HSA agents cannot be matched): same counts and records."""
    rng = random.Random(4242)
    segs = _covid_like(rng, 300)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 40)) or "ACGT" for _ in range(3000)] + ["", "AC\r", "N"]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=3)
    monkeypatch.setenv("EDSBWT_HSA_COPY", "0")
    monkeypatch.setenv("EDSBWT_CHUNK_MB", "0.01")
    monkeypatch.setenv("EDSBWT_CHUNK_SINGLE_MB", "0")
    text = ("\n".join(pats) + "\n").encode()
    for pinned in (True, False):
        with edsbwt.Index(base) as idx:
            gc, go = _lines_search(edsbwt, idx, text, first_id=3, pinned=pinned)
            assert idx.stats()["chunks"] > 5
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)


def test_search_lines_empty_and_held_records_gpu(oracle, edsbwt, tmp_path):
    """An empty file; records still held by the caller when the next call runs (the engine
    must not overwrite them) and freed after the index is closed."""
    base = _build(oracle, tmp_path, open(os.path.join(GOLDEN, "test.eds")).read(), "test")
    with edsbwt.Index(base) as idx:
        c, o = _lines_search(edsbwt, idx, b"")
        assert c.size == 0 and o.size == 0
        hb = edsbwt.HostBuffer(64)
        t = b"TATT\nACT\nTTAT\n"
        hb.array(np.uint8, len(t))[:] = np.frombuffer(t, np.uint8)
        cnt = np.zeros(3, np.uint32)
        _, p1, n1 = idx.search_lines(hb.ptr, len(t), cnt.ctypes.data, 3, keep=True)
        first = idx.occ_view(p1, n1).copy()
        _, p2, n2 = idx.search_lines(hb.ptr, len(t), cnt.ctypes.data, 3, keep=True)
        assert p2 != p1 and np.array_equal(idx.occ_view(p1, n1), first)  # the held records survive
        assert np.array_equal(idx.occ_view(p2, n2), first)
        idx.occ_free(p2)
    assert np.array_equal(edsbwt.Index.occ_view(p1, n1), first)  # detached from the closed index
    edsbwt.Index.occ_free(p1)
    assert [tuple(int(x) for x in r) for r in first] == [(1, 3, 2, 0, 0), (1, 4, 3, 0, 1), (1, 7, 4, 0, 1), (1, 1, 1, 1, 0),
                                                         (3, 0, 1, 0, 1), (3, 4, 3, 0, 0), (3, 7, 4, 0, 0)]


def test_search_device_null_stream_ordering(oracle, edsbwt, tmp_path):
    """search_device with stream=NULL after torch filled the inputs on the default stream,
    with no synchronize in between: the engine orders itself after the null stream."""
    torch = pytest.importorskip("torch")
    rng = random.Random(31)
    segs = edsgen.random_eds(rng, 1500, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(4, 30)) or "ACGT" for _ in range(20000)]
    buf, offs = _pack(pats)
    oc, _, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        h_bytes = torch.from_numpy(buf.copy()).pin_memory()
        h_offs = torch.from_numpy(offs.astype(np.int64)).pin_memory()
        torch.cuda.synchronize()
        d_bytes = torch.zeros(buf.size, dtype=torch.uint8, device="cuda")
        d_offs = torch.zeros(offs.size, dtype=torch.int64, device="cuda")
        big = torch.randn(4096, 4096, device="cuda")
        for _ in range(8):
            big = big @ big  # keep the null stream busy before the copies land
        d_bytes.copy_(h_bytes, non_blocking=True)
        d_offs.copy_(h_offs, non_blocking=True)
        d_counts = torch.zeros(len(pats), dtype=torch.int32, device="cuda")
        idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), len(pats), d_counts.data_ptr(), stream=0)
        assert np.array_equal(d_counts.cpu().numpy().astype(np.uint32), oc)


def test_shard_first_pattern_id_gpu(oracle, edsbwt, tmp_path):
    """Two contiguous shards searched with first_pattern_id = lo + 1 (as each multi-GPU rank
    does) concatenate to the single-call oracle output, in MOVE and legacy order."""
    import importlib
    shard = importlib.import_module("eds-bwt_amd.shard")
    rng = random.Random(2024)
    segs = edsgen.random_eds(rng, 1200, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(3, 20)) or "ACGT" for _ in range(3001)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    kp = _kpos(base)
    legacy_ref = oo[np.lexsort((kp[oo["word"]], oo["offset"], oo["pat"]))]
    with edsbwt.Index(base) as idx:
        for legacy, ref in ((False, oo), (True, legacy_ref)):
            cs, os_ = [], []
            for r in range(2):
                b, o, first = shard.shard_patterns(buf, offs, 2, r)
                c, occ = idx.search((b, o), first_pattern_id=first, legacy=legacy)
                cs.append(c)
                os_.append(occ)
            assert np.array_equal(np.concatenate(cs), oc)
            assert np.array_equal(np.concatenate(os_), ref)


def test_deferred_checks_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """The packed direct start defers its checks to one read-back at the end ('#' in a pattern,
    k_deep overflow lists and the wide retry, record / task totals vs pre-sized buffers).  A
    batch that fails one is searched again on the checked path: forced here by a '#' pattern,
    tiny buffer caps, a tiny wide-retry cap and no wide retry.  Identical to the oracle each time,
    and the redo is visible in the stats."""
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
    rng = random.Random(4242)
    # (a) COVID-like: no overflow; the deferred path completes without a redo
    segs = _covid_like(rng, 600)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs), "cov")
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    assert D0 >= 2
    pats = [edsgen.planted(rng, segs, rng.randint(D0 + 1, D0 + 16)) or "ACGT" * 8 for _ in range(3000)]
    pats = [p[: D0 + 16] if len(p) > D0 + 16 else p for p in pats]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(D0 + 1, D0 + 16))) for _ in range(500)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        for locate in (True, False):
            gc, go = idx.search((buf, offs), locate=locate)
            st = idx.stats()
            assert np.array_equal(gc, oc) and (not locate or np.array_equal(go, oo))
            assert st["start_depth"] == D0 and st["trie_nodes"] == 0 and st["redo_searches"] == 0, st
    monkeypatch.setenv("EDSBWT_DEFER_CAP", "64")  # records and tasks pass the pre-sized buffers
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert idx.stats()["redo_searches"] == 1
    monkeypatch.delenv("EDSBWT_DEFER_CAP")
    # a pattern holding '#' (the ordered path), found only at the final check
    pats2 = pats[:500] + ["A" * D0 + "#AC"] + pats[500:1000]
    buf2, offs2 = _pack(pats2)
    oc2, oo2, _ = oracle.Engine(base, 8).search(buf2, offs2)
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf2, offs2))
        assert np.array_equal(gc, oc2) and np.array_equal(go, oo2)
        assert idx.stats()["redo_searches"] == 1
    # (b) one repeated motif: k_deep overflows (some past the wide lists too)
    motif = ["AC", "ACA", "CA", "A", "", "CAC"]
    segs = [[rng.choice(motif) or "A" for _ in range(rng.randint(1, 5))] for _ in range(3000)]
    for s in segs:
        if rng.random() < 0.3 and len(s) > 1:
            s[0] = ""
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs), "motif")
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    pats = ["".join(rng.choice("AC") for _ in range(rng.randint(D0 + 1, D0 + 16))) for _ in range(2000)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        gc, go = idx.search((buf, offs))
        st = idx.stats()
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert st["start_depth"] == D0 and st["deep_overflow"] > 0, st
        gc, go = idx.search((buf, offs), wide=False)  # every overflow fails the check
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        assert idx.stats()["redo_searches"] == 1
    monkeypatch.setenv("EDSBWT_WIDE_CAP", "1")
    with edsbwt.Index(base) as idx:
        for locate in (True, False):
            gc, go = idx.search((buf, offs), locate=locate)
            assert np.array_equal(gc, oc) and (not locate or np.array_equal(go, oo))
            assert idx.stats()["redo_searches"] == 1


def test_short_patterns_3bit_many_gpu(oracle, edsbwt, tmp_path):
    """More than 2000 patterns shorter than one 3-bit key chunk (21 symbols), so the trie-order
    radix sort runs over partial chunks of many keys, on the trie path (direct=False) and the
    ordered path: identical to the oracle (rocPRIM partial bit ranges)."""
    rng = random.Random(2121)
    segs = edsgen.random_eds(rng, 3000, lmax=8, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(2, 20)) or "ACG" for _ in range(2500)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 20))) for _ in range(2500)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    with edsbwt.Index(base) as idx:
        for kw in ({"direct": False}, {"ordered": True}, {"direct": False, "ktab": False}):
            gc, go = idx.search((buf, offs), **kw)
            assert np.array_equal(gc, oc) and np.array_equal(go, oo), kw


def test_search_lines_vt_after_newline_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """Raw chunks are split on the device (k_nl_count, scan, k_nl_compact): a '\\v' byte right
    after a '\\n' (the has-zero-byte trick double-counts that word's newline) must not shift
    the line offsets of later blocks.  getline keeps '\\v' as a pattern byte."""
    rng = random.Random(1313)
    segs = _covid_like(rng, 300)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(3, 30)) or "ACGT" for _ in range(6000)]
    for i in range(0, len(pats), 7):
        pats[i] = "\v" + pats[i]          # '\n' then '\v' in the same 4-byte word
    for i in range(3, len(pats), 11):
        pats[i] = pats[i] + "\v"
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    text = ("\n".join(pats) + "\n").encode()
    monkeypatch.setenv("EDSBWT_PACK_LINES", "0")
    with edsbwt.Index(base) as idx:
        gc, go = _lines_search(edsbwt, idx, text)
    assert np.array_equal(gc, oc) and np.array_equal(go, oo)


def test_search_lines_many_chunks_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """The host pipeline at its default chunk sizes over a batch of more chunks than slots
    (ADVICE r2): ragged and packed chunks, patterns with thousands of records (the record
    arena grows while chunks are in flight) and one chunk that fails a deferred check ('#' in a
    pattern) and is searched again.  Equal to the device-resident search of the whole batch,
    and to the oracle on a strided sample."""
    torch = pytest.importorskip("torch")
    for k in ("EDSBWT_CHUNK_MB", "EDSBWT_CHUNK_SINGLE_MB", "EDSBWT_PACK_LINES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")  # small tables hold long lists: direct start anyway
    rng = random.Random(5150)
    segs = _covid_like(rng, 400)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    with edsbwt.Index(base) as idx:
        D0 = idx.ktab_depth
    assert D0 >= 2
    # lengths D0+1 .. D0+16: the packed direct start with its deferred checks
    uniq = [edsgen.planted(rng, segs, D0 + 8) or ("ACGT" * 8)[:D0 + 8] for _ in range(40000)]
    uniq += ["".join(rng.choice("ACGT") for _ in range(rng.randint(D0 + 1, D0 + 16))) for _ in range(10000)]
    pats = uniq * 150                                   # 7.5M lines, ~150 MB
    for i in range(777, len(pats) // 2, 20011):
        pats[i] = rng.choice(["A", "C", "GT", "TA"])      # thousands of records each (checked-path chunks)
    pats[3 * len(pats) // 4 + 5] = ("ACGT#ACG" * 8)[:D0 + 4]  # '#' in a direct-start chunk: searched again
    text = ("\n".join(pats) + "\n").encode()
    buf, offs = _pack(pats)
    with edsbwt.Index(base) as idx:
        d_bytes = torch.from_numpy(buf.copy()).cuda()
        d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_counts = torch.zeros(len(pats), dtype=torch.int32, device="cuda")
        ptr, n = idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), len(pats), d_counts.data_ptr())
        ref_counts = d_counts.cpu().numpy().view(np.uint32).copy()
        ref_occ = torch.empty(n * 20, dtype=torch.uint8)
        if n:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            assert hip.hipMemcpy(ctypes.c_void_p(ref_occ.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(n * 20), 2) == 0
        ref_occ = ref_occ.numpy().view(edsbwt.OCC_DTYPE)
        del d_bytes, d_offs, d_counts
        gc, go = _lines_search(edsbwt, idx, text)
        st = idx.stats()
    assert st["chunks"] > 5 and st["redo_searches"] >= 1, st
    assert np.array_equal(gc, ref_counts)
    assert go.size == ref_occ.size and np.array_equal(go, ref_occ)
    # the oracle on a strided sample of the batch (records of pattern i carry #Pat = i + 1)
    sample = np.unique(np.concatenate([np.arange(0, len(pats), 997), np.arange(777, len(pats) // 2, 20011)[:20],
                                       [3 * len(pats) // 4 + 5]]))
    sp = [pats[i] for i in sample]
    sbuf, soffs = _pack(sp)
    oc, oo, _ = oracle.Engine(base, 8).search(sbuf, soffs, threads=8)
    assert np.array_equal(gc[sample], oc)
    sel = np.isin(go["pat"], sample + 1)
    got = go[sel].copy()
    got["pat"] = np.searchsorted(sample, got["pat"] - 1) + 1
    assert np.array_equal(got, oo)


def _expected_console(oracle, base, pfile, pats, argv0):
    """The reference's stdout / stderr for `MOVE_EDSBWTSearch base pfile` (mainMove_EDSBWT.cpp:27-59,
    MOVE_EDSBWTSearch.cpp:23-155,664-766), the per-pattern part from the oracle's literal loop
    (orc_search_batch_console: count and early return per pattern); 'bs took:' left as a marker."""
    raw = open(base + "_info.aux", "rb").read()
    N, W = (int(x) for x in np.frombuffer(raw, np.uint32, 2))
    sigma = raw[8]
    alpha = raw[9:9 + sigma].decode("latin1")
    tocc = np.frombuffer(raw, np.uint32, count=sigma * sigma, offset=9 + sigma + 4 * W).reshape(sigma, sigma)
    buf, offs = _pack(pats)
    counts, early = oracle.Engine(base, 8).console(buf, offs)
    out = [f"BCR_eds: {argv0}\n", f"BCR_eds: The input ebwt file is {base}\n", f"BCR_eds: The pattern file is {pfile}\n", "DEBUG: 0\n",
           f"\nFrom {base}_info.aux file:\n", f"\tNumber of sequences: {W}\n", f"\tTotal length (with $): {N}\n",
           f"\tSize alpha: {sigma}\n", "\tAlphabet: " + "".join(c + "\t" for c in alpha) + "\n", f"NUM OF EOF{W}\n",
           f"\nFrom {base}_info.aux file (TableOcc):\n"]
    out += ["".join(f"{v}\t" for v in row) + "\n" for row in tocc]
    out += [f"size= {N}\n", f"BitVector size: {W}\n"]
    err = ["Backward Search\n"]
    for p, c, e in zip(pats, counts, early):
        out.append(f"Pattern: {p} of length {len(p)}\n")
        if not e:
            out.append(f"num occ {c}\n")
        err.append(f"OCCORRENZA DI: {p} {'TROVATA' if c > 0 else 'NON TROVATA'}\n")
    out.append("bs took:")
    found = int((counts > 0).sum())
    err += ["\n", f"count_found = {found}\n", f"count_not_found = {len(pats) - found}\n", "\nThe csv file is ready! \n", "The End!\n"]
    return "".join(out), "".join(err), counts, early


def test_cli_console_transcript(oracle, tmp_path):
    """EDSBWTsearch without --quiet: stdout and stderr byte-identical to the reference's stream
    (banner, index summary, TableOcc, per pattern 'Pattern: ... of length ...', 'num occ' only
    when backwardSearch reaches its locate loop, 'OCCORRENZA DI ...'), from a transcript made by
    the oracle's literal loop; 'bs took:<secs>' compared up to the number."""
    import re
    import subprocess
    from conftest import ROOT
    rng = random.Random(4711)
    segs = edsgen.random_eds(rng, 400, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(2, 14)) or "ACGT" for _ in range(150)]
    pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 12))) for _ in range(150)]  # many die early
    pats += ["A", "N", "NA", "AN", "GATTACA"]
    pfile = tmp_path / "p.txt"
    pfile.write_text("\n".join(pats) + "\n")
    cli = os.path.join(ROOT, "eds-bwt_amd", "_build", "EDSBWTsearch")
    r = subprocess.run([cli, base, str(pfile)], capture_output=True, text=True)
    assert r.returncode == 1, r.stderr
    want_out, want_err, counts, early = _expected_console(oracle, base, str(pfile), pats, cli)
    assert early.any() and (~early).any() and ((counts == 0) & ~early).any()  # all three console shapes occur
    m = re.fullmatch(r"(.*bs took:)[0-9.e+-]+", r.stdout, re.S)
    assert m, r.stdout[-200:]
    assert m.group(1) == want_out
    assert r.stderr == want_err


@pytest.mark.parametrize("alphabet", ["ACGT", "ACG", "AC"])
def test_rank16_level_step_gpu(oracle, edsbwt, tmp_path, monkeypatch, alphabet):
    """The level step's ranks from the all-symbol 16-B rank entries (rk16, sigma <= 5) against the
    64-B occ blocks (EDSBWT_NO_RANK16=1) and the oracle: trie levels at every depth (deep=False),
    the ordered path, and the k-mer start table built with each."""
    rng = random.Random(1616 + len(alphabet))
    segs = edsgen.random_eds(rng, 3000, alphabet=alphabet, lmax=9, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 40)) or alphabet * 3 for _ in range(2500)]
    pats += ["".join(rng.choice(alphabet + "T") for _ in range(rng.randint(1, 30))) for _ in range(1500)]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    for off in ("0", "1"):
        monkeypatch.setenv("EDSBWT_NO_RANK16", off)
        with edsbwt.Index(base) as idx:
            for kw in ({}, {"deep": False}, {"direct": False, "deep": False}, {"ordered": True, "deep": False}, {"ktab": False}):
                gc, go = idx.search((buf, offs), **kw)
                assert np.array_equal(gc, oc) and np.array_equal(go, oo), (off, kw)


def test_counts_mirror_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """edsbwt_set_counts_mirror: the host pipeline also leaves every pattern's u32 count in a
    device array (what bench.py's ranks gather over RCCL), over several chunks; a batch larger
    than the mirror fails with E_ARG; cap 0 turns it off."""
    torch = pytest.importorskip("torch")
    rng = random.Random(6060)
    segs = _covid_like(rng, 300)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 40)) or "ACGT" for _ in range(6000)] + ["", "N"]
    buf, offs = _pack(pats)
    oc, _, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=9)
    text = ("\n".join(pats) + "\n").encode()
    monkeypatch.setenv("EDSBWT_CHUNK_MB", "0.01")
    monkeypatch.setenv("EDSBWT_CHUNK_SINGLE_MB", "0")
    with edsbwt.Index(base) as idx:
        mirror = torch.full((len(pats),), -1, dtype=torch.int32, device="cuda")
        idx.set_counts_mirror(mirror.data_ptr(), len(pats))
        gc, _ = _lines_search(edsbwt, idx, text, first_id=9)
        assert idx.stats()["chunks"] > 5
        assert np.array_equal(gc, oc) and np.array_equal(mirror.cpu().numpy().view(np.uint32), oc)
        small = torch.zeros(10, dtype=torch.int32, device="cuda")
        idx.set_counts_mirror(small.data_ptr(), 10)
        with pytest.raises(edsbwt.EdsBwtError):
            _lines_search(edsbwt, idx, text, first_id=9)
        idx.set_counts_mirror(0, 0)
        gc2, _ = _lines_search(edsbwt, idx, text, first_id=9)
        assert np.array_equal(gc2, oc)
        # the stream pipeline (the fallback when the SDMA path is not taken: here kernel-store
        # downloads, EDSBWT_D2H_KERNEL=1) fills the mirror too
        monkeypatch.setenv("EDSBWT_D2H_KERNEL", "1")
        mirror.fill_(-1)
        idx.set_counts_mirror(mirror.data_ptr(), len(pats))
        gc3, _ = _lines_search(edsbwt, idx, text, first_id=9)
        assert idx.stats()["chunks"] > 5
        assert np.array_equal(gc3, oc) and np.array_equal(mirror.cpu().numpy().view(np.uint32), oc)
        idx.set_counts_mirror(small.data_ptr(), 10)
        with pytest.raises(edsbwt.EdsBwtError):
            _lines_search(edsbwt, idx, text, first_id=9)
        # a packed batch larger than the mirror is refused before any chunk runs: the mirror is untouched
        monkeypatch.delenv("EDSBWT_D2H_KERNEL")
        small.fill_(-7)
        with pytest.raises(edsbwt.EdsBwtError):
            idx.search((buf, offs), first_pattern_id=9)
        assert (small.cpu().numpy() == -7).all()
        idx.set_counts_mirror(0, 0)


# every k_deep build the engine can dispatch (engine.hip run_deep): the register-list lengths
# (EDSBWT_DEEP_K 2 / 3 / 4 / 8), the 4-interval build unbounded (EDSBWT_DEEPQ_WAVES=1) and held to
# 5 / 6 waves per SIMD, and the '#'-row link-row variant (EDSBWT_EOF_ROWS=1) unbounded and at 5 waves
K_DEEP_BUILDS = [{"EDSBWT_DEEPQ_WAVES": "1"}, {"EDSBWT_DEEPQ_WAVES": "5"}, {"EDSBWT_DEEPQ_WAVES": "6"},
                 {"EDSBWT_DEEPQ_WAVES": "6", "EDSBWT_DEEP_STATS": "0"}, {"EDSBWT_DEEPQ_WAVES": "5", "EDSBWT_DEEP_STATS": "0"},
                 # (the builds without work counters)
                 {"EDSBWT_EOF_ROWS": "1", "EDSBWT_DEEPQ_WAVES": "1"}, {"EDSBWT_EOF_ROWS": "1", "EDSBWT_DEEPQ_WAVES": "5"},
                 {"EDSBWT_DEEP_K": "2"}, {"EDSBWT_DEEP_K": "3"}, {"EDSBWT_DEEP_K": "8"},
                 # the packed direct start's queue: the generic build (not the PACKED one) and PACKED at 7 waves
                 {"EDSBWT_DEEPQ_PACKED": "0"}, {"EDSBWT_DEEPQ_WAVES": "7"}, {"EDSBWT_DEEPQ_WAVES": "7", "EDSBWT_DEEP_STATS": "0"},
                 # k_deep_direct at 8 waves per SIMD (the default is 7), and without the return to the text compare
                 {"EDSBWT_DIRECT_WAVES": "8"}, {"EDSBWT_DIRECT_BACK": "0", "EDSBWT_DEEP_STATS": "0"},
                 # k_deep's packed build without the text filter of a list start
                 {"EDSBWT_DEEPQ_FILTER": "0"}]


@pytest.mark.parametrize("build", K_DEEP_BUILDS, ids=lambda b: ",".join(f"{k[7:]}={v}" for k, v in b.items()))
def test_k_deep_builds_gpu(oracle, edsbwt, tmp_path, monkeypatch, build):
    """Each k_deep instantiation exact against the oracle: the README KAT
    (README.md:144-167, the search that once miscounted TATT), random EDSs with empty words and
    'N', and the direct start whose multi-interval D-mer lists k_deep reads from the wide
    entries (inline lists of 2-3 intervals and offset lists), each through the search variants
    that reach k_deep (default, count-only, the walk from depth 0, the trie start, no pair
    entries, no text compare) and repeated, with fresh allocations poisoned where the process
    runs with EDSBWT_POISON (tools/kdeep_stress.py is the many-repetition form of this test)."""
    for k, v in build.items():
        monkeypatch.setenv(k, v)
    kat = _build(oracle, tmp_path, open(os.path.join(GOLDEN, "test.eds")).read(), "test")
    cases = [(kat, ["TATT", "ACT", "TTAT"]), (kat, ["TATT", "ACT", "TTAT", "TTA", "GTT", "T"])]
    for seed in (0, 7):
        rng = random.Random(100 + seed)
        segs = edsgen.random_eds(rng, rng.randint(20, 400), alphabet="ACGTN" if seed % 3 == 0 else "ACGT", lmax=3 + seed,
                                 p_empty=0.25)
        base = _build(oracle, tmp_path, edsgen.eds_text(segs), f"r{seed}")
        pats = [(edsgen.planted(rng, segs, m) if rng.random() < 0.6 else None) or "".join(rng.choice("ACGT") for _ in range(m))
                for m in (rng.randint(1, 24) for _ in range(400))]
        cases.append((base, pats))
    rng = random.Random(3232)
    segs = _covid_like(rng, 700)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    cov = _build(oracle, tmp_path, edsgen.eds_text(segs), "cov")
    cases.append((cov, [edsgen.planted(rng, segs, rng.randint(16, 31)) or "ACGT" * 8 for _ in range(3000)]))
    for base, pats in cases:
        buf, offs = _pack(pats)
        oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
        if base == cov:
            monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")  # the direct start from this small table
        with edsbwt.Index(base) as idx:
            for kw in ({}, {"locate": False}, {"ktab": False}, {"direct": False}, {"pairs": False}, {"text": False}):
                for _ in range(3):
                    gc, go = idx.search((buf, offs), **kw)
                    assert np.array_equal(gc, oc), (build, base, kw)
                    if kw.get("locate", True):
                        assert np.array_equal(go, oo), (build, base, kw)
        monkeypatch.delenv("EDSBWT_DIRECT_ITEMS", raising=False)


@pytest.mark.parametrize("build", [{}, {"EDSBWT_DEEPQ_WAVES": "1"}, {"EDSBWT_DEEP_STATS": "0"}],
                         ids=lambda b: ",".join(f"{k[7:]}={v}" for k, v in b.items()) or "default")
def test_hash_pattern_pair_step_in_k_deep_gpu(oracle, edsbwt, tmp_path, monkeypatch, build):
    """Patterns holding '#' that are still alive when k_deep reaches the '#' (ADVICE r5, high):
    X + '#' + Y with Y a word's head and X a word's tail, so Y's rows survive and the '#' step
    (code 0) is taken inside k_deep with pair entries on (rent2, EDSBWT_DEEPQ_PAIRS default).  A
    pair code for c = '#' would wrap below 1 and index rent2 ~2^32 entries away; the single step is
    the reference's (MOVE_EDSBWTSearch.cpp:376-422 with c = '#').  Such patterns take the ordered
    path (levels()); EDSBWT_DEEP_SHARE=0 cuts over to k_deep at depth 2, so the '#' is met there."""
    for k, v in build.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("EDSBWT_DEEP_SHARE", "0")
    rng = random.Random(2323)
    segs = edsgen.random_eds(rng, 600, lmax=9, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    words = [w for s in segs for w in s if len(w) >= 4]
    assert words
    pats = []
    for _ in range(1500):
        a, b = rng.choice(words), rng.choice(words)
        pats.append(a[-rng.randint(1, 3):] + "#" + b[: rng.randint(2, 4)])      # '#' at depth 2..4
    pats += [rng.choice(words)[-2:] + "#" + "".join(rng.choice("ACGT") for _ in range(3)) for _ in range(300)]
    pats += ["#" + rng.choice(words)[:3] for _ in range(50)] + [rng.choice(words)[-3:] + "#" for _ in range(50)]
    pats += [edsgen.planted(rng, segs, rng.randint(4, 20)) or "ACGT" for _ in range(1000)]  # the same batch, no '#'
    buf, offs = _pack(pats)
    eng = oracle.Engine(base, 8)
    oc, oo, _ = eng.search(buf, offs)
    # every head Y after the '#' occurs (a word's prefix): each such pattern is alive at the '#'
    ybuf, yoffs = _pack([p.split("#", 1)[1] for p in pats[:1500]])
    assert (eng.search(ybuf, yoffs)[0] > 0).all()
    with edsbwt.Index(base) as idx:
        assert idx.pair_blocks
        for kw in ({}, {"locate": False}, {"ktab": False}, {"ordered": True}):
            gc, go = idx.search((buf, offs), **kw)
            assert np.array_equal(gc, oc), (build, kw, np.flatnonzero(gc != oc)[:8].tolist())
            if kw.get("locate", True):
                assert np.array_equal(go, oo), (build, kw)
            if kw.get("ktab") is False:
                assert idx.stats()["deep_from_depth"] == 2  # k_deep walked from depth 2: it met every '#'


@pytest.mark.parametrize("gpus", [2, 3, 5])
def test_cli_gpus_shards(oracle, tmp_path, gpus):
    """EDSBWTsearch --gpus N (the pattern loop MOVE_EDSBWTSearch.cpp:111-136 sharded into N
    contiguous line ranges, one index each — here N handles on the box's one GPU): the CSV is
    byte-identical to --gpus 1's and to the oracle's, count lines equal, in MOVE order, count-only
    and legacy order; the console transcript (no --quiet) equals the single-device one; a file with
    fewer lines than shards works."""
    import re
    import subprocess
    from conftest import ROOT
    rng = random.Random(600 + gpus)
    segs = edsgen.random_eds(rng, 700, p_empty=0.2)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(3, 20)) or "ACGT" for _ in range(1500)]
    pats += ["", "N", "GATTACA", "AC\r"] + ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 16))) for _ in range(500)]
    rng.shuffle(pats)
    cli = os.path.join(ROOT, "eds-bwt_amd", "_build", "EDSBWTsearch")

    def run(name, text, *extra):
        p = tmp_path / name
        p.write_text(text)
        r = subprocess.run([cli, base, str(p)] + list(extra), capture_output=True, text=True)
        assert r.returncode == 1, r.stderr[-500:]
        return p, r

    for trailing in ("\n", ""):
        text = "\n".join(pats) + trailing
        p1, r1 = run(f"one{len(trailing)}.txt", text, "--quiet")
        pn, rn = run(f"many{len(trailing)}.txt", text, "--quiet", "--gpus", str(gpus))
        csv1 = open(str(p1) + "output_M_LF.csv", "rb").read()
        assert open(str(pn) + "output_M_LF.csv", "rb").read() == csv1
        assert rn.stderr.split("count_found")[1] == r1.stderr.split("count_found")[1]
    ctr, _ = oracle.Engine(base).search_file(str(p1), str(tmp_path / "orc.csv"))
    assert open(tmp_path / "orc.csv", "rb").read() == csv1
    for extra in (["--count-only"], ["--legacy"]):
        pa, ra = run("a.txt", "\n".join(pats) + "\n", "--quiet", *extra)
        pb, rb = run("b.txt", "\n".join(pats) + "\n", "--quiet", "--gpus", str(gpus), *extra)
        out = "output.csv" if "--legacy" in extra else "output_M_LF.csv"
        assert open(str(pa) + out, "rb").read() == open(str(pb) + out, "rb").read()
        assert ra.stderr.split("count_found")[1] == rb.stderr.split("count_found")[1]
    # the console stream (reach search sharded too)
    _, c1 = run("c1.txt", "\n".join(pats[:300]) + "\n")
    _, cn = run("c1.txt", "\n".join(pats[:300]) + "\n", "--gpus", str(gpus))
    strip = lambda s: re.sub(r"bs took:[0-9.e+-]+", "bs took:", s)
    assert strip(cn.stdout) == strip(c1.stdout) and cn.stderr == c1.stderr
    # fewer lines than shards
    pf, rf = run("few.txt", "TTAT\nACGT\n", "--quiet", "--gpus", "4")
    _, r2 = run("few1.txt", "TTAT\nACGT\n", "--quiet")
    assert open(str(pf) + "output_M_LF.csv", "rb").read() == open(str(tmp_path / "few1.txt") + "output_M_LF.csv", "rb").read()


def test_prepare_then_search_lines_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """edsbwt_prepare (the CLI's setup before its clock: the pipeline, slots and record arena sized
    by one pass over synthetic lines) changes no result: search_lines after it equals the oracle,
    located and count-only, over many chunks and one; a prepare sized far off the real batch, and
    one for zero lines, are harmless."""
    rng = random.Random(515)
    segs = _covid_like(rng, 400)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, 31) or "ACGT" * 8 for _ in range(6000)] + ["", "N", "AC\r"]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=1)
    text = ("\n".join(pats) + "\n").encode()
    for mb in ("0.02", "64"):
        monkeypatch.setenv("EDSBWT_CHUNK_MB", mb)
        monkeypatch.setenv("EDSBWT_CHUNK_SINGLE_MB", "0")
        with edsbwt.Index(base) as idx:
            idx.prepare(len(text), len(pats))
            gc, go = _lines_search(edsbwt, idx, text)
            assert np.array_equal(gc, oc) and np.array_equal(go, oo), mb
            idx.prepare(len(text), len(pats), locate=False)
            gc2, go2 = _lines_search(edsbwt, idx, text, locate=False)
            assert np.array_equal(gc2, oc) and go2.size == 0
            idx.prepare(10 * len(text), 3)  # far off: 3 lines of a long mean length
            idx.prepare(0, 0)
            gc3, go3 = _lines_search(edsbwt, idx, text)
            assert np.array_equal(gc3, oc) and np.array_equal(go3, oo)


@pytest.mark.parametrize("shape", ["covid", "c5"])
def test_kmer_table_grouped_build_gpu(oracle, edsbwt, tmp_path, monkeypatch, shape):
    """The k-mer start table built group by group (engine.hip build_ktab_grouped: the K-mers
    sharing their last two characters walked together, their lists concatenated into the table's
    layout; C3's production table is built this way so its transient workspace is 1/16 of the
    whole-table walk's) equals the whole-table walk's: same depth, intervals and device bytes, and
    searches through it equal the oracle — direct start and trie start, located and count-only.
    On a C5-shaped EDS with a small interval budget the group walk outgrows its share and the
    build falls back to the whole-table walk at the depth the group reached."""
    rng = random.Random(77 if shape == "covid" else 78)
    if shape == "covid":
        segs = _covid_like(rng, 500)
        if any(w == "" for w in segs[1]):
            segs[1] = ["A"]
    else:
        segs = edsgen.random_eds(rng, 4000, kmax=4, lmax=7, p_empty=0.2)
        monkeypatch.setenv("EDSBWT_KTAB_ITEMS", "20000")
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
    info = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("EDSBWT_KTAB_GROUPED", mode)
        with edsbwt.Index(base) as idx:
            info[mode] = (idx.ktab_depth, idx.ktab_items, idx.device_bytes)
            D = idx.ktab_depth
            assert D >= 2 and idx.open_peak_bytes > 0
            pats = [edsgen.planted(rng, segs, rng.randint(D + 1, D + 16)) or "ACGT" * 8 for _ in range(1500)]
            pats += ["".join(rng.choice("ACGT") for _ in range(rng.randint(D + 1, D + 12))) for _ in range(300)]
            pats += [edsgen.planted(rng, segs, rng.randint(1, D)) or "AC" for _ in range(200)]  # trie start
            buf, offs = _pack(pats)
            oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
            for kw in ({}, {"locate": False}):
                gc, go = idx.search((buf, offs), **kw)
                assert np.array_equal(gc, oc), (mode, kw)
                if kw.get("locate", True):
                    assert np.array_equal(go, oo), (mode, kw)
            long_ = [p for p in pats if len(p) > D]
            lb, lo = _pack(long_)
            lc, loo, _ = oracle.Engine(base, 8).search(lb, lo)
            gc, go = idx.search((lb, lo))
            assert idx.stats()["start_depth"] == D
            assert np.array_equal(gc, lc) and np.array_equal(go, loo)
    if shape == "covid":
        assert info["0"] == info["2"], info


@pytest.mark.parametrize("small", ["1", "2", "0"])
def test_count_only_counts_paths_gpu(oracle, edsbwt, tmp_path, monkeypatch, small):
    """A count-only search_lines call downloads its counts as u32 straight into the caller's array
    (the default), or as bytes widened on the host (EDSBWT_SMALL_COUNTS=2, the located calls' form,
    with counts of 255 and more as exceptions); located calls keep the byte counts unless
    EDSBWT_SMALL_COUNTS=0.  Same counts either way, pinned and pageable, one chunk and many."""
    monkeypatch.setenv("EDSBWT_SMALL_COUNTS", small)
    rng = random.Random(2222)
    segs = _covid_like(rng, 300)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(1, 30)) or "ACGT" for _ in range(4000)] + ["A", "C", "G", "T", "", "N"]
    buf, offs = _pack(pats)
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs)
    assert (oc >= 255).any()  # the byte form's exceptions occur
    text = ("\n".join(pats) + "\n").encode()
    for mb in ("0.01", "64"):
        monkeypatch.setenv("EDSBWT_CHUNK_MB", mb)
        monkeypatch.setenv("EDSBWT_CHUNK_SINGLE_MB", "0")
        with edsbwt.Index(base) as idx:
            for pinned in (True, False):
                gc, _ = _lines_search(edsbwt, idx, text, locate=False, pinned=pinned)
                assert np.array_equal(gc, oc), (mb, pinned)
                gl, gol = _lines_search(edsbwt, idx, text, pinned=pinned)
                assert np.array_equal(gl, oc) and np.array_equal(gol, oo), (mb, pinned)


def _device_search(edsbwt, idx, pats, ids=None, first_id=1, locate=True):
    """search_device (or search_device_ids when ids is given) of pats: counts and records."""
    import ctypes
    torch = pytest.importorskip("torch")
    buf, offs = _pack(pats)
    d_bytes = torch.from_numpy(buf.copy() if buf.size else np.zeros(1, np.uint8)).cuda()
    d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_counts = torch.zeros(max(1, len(pats)), dtype=torch.int32, device="cuda")
    d_ids = torch.from_numpy(np.asarray(ids, np.uint32).view(np.int32)).cuda() if ids is not None else None
    ptr, n = idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), len(pats), d_counts.data_ptr(), first_pattern_id=first_id,
                               locate=locate, ids=d_ids.data_ptr() if d_ids is not None else 0)
    torch.cuda.synchronize()
    occ = np.zeros(n, edsbwt.OCC_DTYPE)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(occ.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(n * 20), 2) == 0
    return d_counts.cpu().numpy().view(np.uint32)[:len(pats)].copy(), occ


@pytest.mark.parametrize("shape", ["level_table", "direct"])
def test_search_device_ids_gpu(oracle, edsbwt, tmp_path, monkeypatch, shape):
    """edsbwt_search_device_ids: a batch cut into suffix-ordered sub-batches (bench.py's C5 located
    chunks) reports each record's #Pat as the pattern's line number from the id map; the counts
    and records of every sub-batch equal the oracle's for those lines, pattern-major in the
    sub-batch's order — on the level-table start with trie-subtree groups (C5's path) and on the
    direct start with its per-pattern locate (k_locate_pp / k_locate_big)."""
    import bench
    rng = random.Random(7070)
    if shape == "level_table":
        monkeypatch.setenv("EDSBWT_KTAB_K", "3")
        monkeypatch.setenv("EDSBWT_LTAB_K", "6")
        monkeypatch.setenv("EDSBWT_FORCE_GROUPS", "2")
        segs = edsgen.random_eds(rng, 5000, kmax=4, lmax=7, p_empty=0.2)
        pats = [edsgen.planted(rng, segs, rng.choice([6, 6, 7, 12, 24])) or "ACGTAC" for _ in range(2000)]
        pats += ["".join(rng.choice("ACGT") for _ in range(rng.choice([6, 8, 16]))) for _ in range(800)]
    else:
        monkeypatch.setenv("EDSBWT_DIRECT_ITEMS", "1e9")
        segs = _covid_like(rng, 300)
        pats = [edsgen.planted(rng, segs, rng.randint(12, 31)) or "ACGTACGTACGTA" for _ in range(2500)]
        pats += ["A", "C", "GT"] * 5 + ["".join(rng.choice("ACGT") for _ in range(20)) for _ in range(500)]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    buf, offs = _pack(pats)
    first_id = 101
    oc, oo, _ = oracle.Engine(base, 8).search(buf, offs, first_pattern_id=first_id)
    ostart = np.zeros(len(pats) + 1, np.int64)
    ostart[1:] = np.cumsum(oc.astype(np.int64))
    order = bench.suffix_order(buf, offs.astype(np.int64), k=6)
    cuts = [0, len(pats) // 3, len(pats) // 3 + 1, len(pats)]
    with edsbwt.Index(base) as idx:
        for a, b in zip(cuts[:-1], cuts[1:]):
            sel = order[a:b]
            gc, go = _device_search(edsbwt, idx, [pats[i] for i in sel], ids=sel + first_id)
            if shape == "level_table":
                assert idx.stats()["start_depth"] == 6 or b - a == 1
            assert np.array_equal(gc, oc[sel]), (a, b)
            want = np.concatenate([oo[ostart[i]:ostart[i + 1]] for i in sel]) if sel.size else oo[:0]
            assert np.array_equal(go, want), (a, b)
        # the whole batch in line order through the id map == first_pattern_id
        ids = np.arange(len(pats)) + first_id
        gc, go = _device_search(edsbwt, idx, pats, ids=ids)
        assert np.array_equal(gc, oc) and np.array_equal(go, oo)
        gc2, go2 = _device_search(edsbwt, idx, pats, first_id=first_id)
        assert np.array_equal(go2, oo)
        # the legacy engine order sorts by #Pat: refused with an id map
        import ctypes
        L = edsbwt.lib()
        occ_p, nocc = ctypes.c_void_p(), ctypes.c_uint64()
        assert L.edsbwt_search_device_ids(idx._h, None, None, 0, None, edsbwt.LOCATE | edsbwt.LEGACY_ORDER, None,
                                          ctypes.byref(occ_p), ctypes.byref(nocc), None) == -5


def test_locate_many_tiles_gpu(oracle, edsbwt, tmp_path, monkeypatch):
    """The per-pattern locate's record offsets over a batch of ~4700 64-pattern tiles (k_count_tiles,
    the scan over tiles, k_locate_pp's wave scans) — blocks of 0 records and of more than the LDS
    stage's records, patterns left to k_locate_big: records and counts identical to the per-pattern
    scan (EDSBWT_TILE_SCAN=0) and the first patterns' records identical to the oracle's, three
    times over.  (Round 5 also ran this against a decoupled look-back inside k_locate_pp: exact,
    but slower — profiles/r05_ab_c3_loc_lookback_v*.txt.)"""
    rng = random.Random(4242)
    segs = _covid_like(rng, 900)
    if any(w == "" for w in segs[1]):
        segs[1] = ["A"]
    base = _build(oracle, tmp_path, edsgen.eds_text(segs), "lb")
    pats = []
    for k in range(300_000):
        m = rng.choice((6, 9, 16, 24, 31))
        if (k // 256) % 7 == 3:  # whole blocks of patterns that occur nowhere (0-record blocks)
            pats.append("N" * m)
        else:
            pats.append(edsgen.planted(rng, segs, m) or "ACGT" * 8)
    buf, offs = _pack(pats)
    n0 = 3000
    b0, o0 = _pack(pats[:n0])
    oc0, oo0, _ = oracle.Engine(base, 8).search(b0, o0)
    got = {}
    for tsc in ("1", "0"):
        monkeypatch.setenv("EDSBWT_TILE_SCAN", tsc)
        with edsbwt.Index(base) as idx:
            for rep in range(3):
                gc, go = idx.search((buf, offs))
                assert np.array_equal(gc[:n0], oc0), (tsc, rep)
                assert np.array_equal(go[:oo0.size], oo0), (tsc, rep)
                assert int(gc.astype(np.int64).sum()) == go.size
                if tsc in got:
                    assert np.array_equal(gc, got[tsc][0]) and np.array_equal(go, got[tsc][1])
                got[tsc] = (gc, go)
    assert np.array_equal(got["1"][0], got["0"][0]) and np.array_equal(got["1"][1], got["0"][1])
    assert got["1"][1].size > 300_000 * 2  # (records well past the blocks' stage sizes)


def test_native_gather_counts_gpu(oracle, edsbwt, tmp_path):
    """The library's own RCCL exchange (edsbwt_comm_init / edsbwt_gather_counts, ABI 7) with one
    rank: counts of alternating device-resident searches gathered into rank 0's output, the
    host pipeline's counts mirror gathered too, in step order (a search writing a buffer waits
    for the gather still reading it), every gather equal to the oracle's counts."""
    torch = pytest.importorskip("torch")
    rng = random.Random(717)
    segs = _covid_like(rng, 300)
    base = _build(oracle, tmp_path, edsgen.eds_text(segs))
    pats = [edsgen.planted(rng, segs, rng.randint(4, 40)) or "ACGT" for _ in range(5000)]
    buf, offs = _pack(pats)
    oc, _, _ = oracle.Engine(base, 8).search(buf, offs)
    n = len(pats)
    sizes = np.array([n], np.uint64)
    with edsbwt.Index(base) as idx:
        idx.comm_init(edsbwt.Index.comm_unique_id(), 1, 0)
        d_bytes = torch.from_numpy(buf.copy()).cuda()
        d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
        bufs = [torch.full((n,), -1, dtype=torch.int32, device="cuda") for _ in range(2)]
        out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        for step in range(6):
            b = bufs[step % 2]
            idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), n, b.data_ptr(), locate=step % 3 != 0)
            idx.gather_counts(b.data_ptr(), n, out.data_ptr(), sizes, 0)
        idx.comm_sync()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), oc)
        # the host pipeline's counts mirror, gathered the same way
        out.fill_(-1)
        text = ("\n".join(pats) + "\n").encode()
        for step in range(3):
            idx.set_counts_mirror(bufs[step % 2].data_ptr(), n)
            gc, _ = _lines_search(edsbwt, idx, text)
            idx.gather_counts(bufs[step % 2].data_ptr(), n, out.data_ptr(), sizes, 0)
        idx.comm_sync()
        idx.set_counts_mirror(0, 0)
        assert np.array_equal(gc, oc) and np.array_equal(out.cpu().numpy().view(np.uint32), oc)
        with pytest.raises(edsbwt.EdsBwtError):
            idx.gather_counts(bufs[0].data_ptr(), n - 1, out.data_ptr(), sizes, 0)  # n differs from sizes[rank]


def test_three_way_list_start_gpu():
    """Round 5's fault, kept reproducible: k_deep with the three-way divergent branch on
    the queue entry's kind (libedsbwt_3way.so, built by `make all` from the same sources with
    -DEDSBWT_KDEEP_THREEWAY), unbounded build (EDSBWT_DEEPQ_WAVES=1), over the README KAT in every
    search variant (tools/threeway_probe.py, its own process).  Before the fix (the interval assigned
    in its own arm) this build returned [0, 0, 0] for [4, 0, 3]; with the interval assigned before the
    branch every variant equals the oracle."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    lib3 = os.path.join(ROOT, "eds-bwt_amd", "_build", "libedsbwt_3way.so")
    if not os.path.exists(lib3):
        pytest.skip("libedsbwt_3way.so not built (make -C eds-bwt_amd all)")
    env = dict(os.environ, EDSBWT_LIB=lib3, EDSBWT_DEEPQ_WAVES="1", EDSBWT_PATH_TAGS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "threeway_probe.py")], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["oracle_counts"] == [4, 0, 3]
    assert all(run.get("match") for run in d["runs"]), d["runs"]
