"""Pin the oracle (CPU restatement of the reference path) before trusting it.

* README.md:144-167 known-answer test (the only expected output the reference holds;
  legacy engine order, so compared as a multiset).
* Survey Appendix C values for sample/test and sample/ExamplePaper (re-derived).
* An independent brute-force EDS matcher over random EDSs with empty words.
* M_LF invariants (move == LF; runs-file build == .ebwt build).
"""
import os
import random
import shutil

import numpy as np
import pytest

from conftest import GOLDEN
import edsgen


def _index(oracle, tmp_path, eds_name_or_text, name="idx", text=False):
    eds = tmp_path / f"{name}.eds"
    if text:
        eds.write_text(eds_name_or_text)
    else:
        shutil.copy(os.path.join(GOLDEN, eds_name_or_text), eds)
    base = str(tmp_path / name)
    oracle.transform(str(eds), base)
    return base


def _rows(occ):
    return [tuple(int(x) for x in r) for r in occ]


def test_readme_kat(oracle, tmp_path):
    base = _index(oracle, tmp_path, "test.eds", "test")
    eng = oracle.Engine(base, 8)
    pats = open(os.path.join(GOLDEN, "readme_kat_patterns.txt"), "rb").read().split(b"\n")[:-1]
    buf = np.frombuffer(b"".join(pats), np.uint8)
    offs = np.concatenate(([0], np.cumsum([len(p) for p in pats]))).astype(np.uint64)
    counts, occ, ctr = eng.search(buf, offs)
    exp = [tuple(int(v) for v in l.split("\t")) for l in open(os.path.join(GOLDEN, "readme_kat_expected.tsv")).read().splitlines()[1:]]
    assert sorted(_rows(occ)) == sorted(exp)
    assert list(counts) == [4, 0, 3]
    # MOVE order (interval order, rows ascending) — survey Appendix C
    assert _rows(occ) == [(1, 3, 2, 0, 0), (1, 4, 3, 0, 1), (1, 7, 4, 0, 1), (1, 1, 1, 1, 0),
                          (3, 0, 1, 0, 1), (3, 4, 3, 0, 0), (3, 7, 4, 0, 0)]


def test_sample_index_files(oracle, tmp_path):
    base = _index(oracle, tmp_path, "test.eds", "test")
    assert open(base + ".ebwt", "rb").read() == b"TACTTAGT#TT####T#TTT####A"
    info = np.fromfile(base + "_info.aux", dtype=np.uint8)
    n, w = np.frombuffer(info[:8].tobytes(), np.uint32)
    assert (n, w) == (25, 10)
    assert info[8] == 5 and bytes(info[9:14]) == b"#ACGT"
    eof = np.frombuffer(info[14:14 + 40].tobytes(), np.uint32)
    assert list(eof) == [8, 5, 9, 2, 6, 3, 1, 0, 4, 7]
    tocc = np.frombuffer(info[54:54 + 100].tobytes(), np.uint32).reshape(5, 5)
    assert tocc.tolist() == [[1, 2, 1, 1, 5], [2, 0, 0, 0, 1], [1, 0, 0, 0, 0], [1, 0, 0, 0, 0], [5, 1, 0, 0, 4]]
    bv = np.fromfile(base + ".bitvector", dtype=np.uint64)
    assert bv[0] == 10 and int(bv[1]) == int("1010011001", 2)  # bits 1001100101 LSB-first
    assert len(open(base + "_runs.aux").read().splitlines()) == 21


def test_sample_kmers(oracle, tmp_path):
    base = _index(oracle, tmp_path, "test.eds", "test")
    eng = oracle.Engine(base, 8)
    shutil.copy(os.path.join(GOLDEN, "kmers.txt"), tmp_path / "kmers.txt")
    ctr, _ = eng.search_file(str(tmp_path / "kmers.txt"), str(tmp_path / "kmers.txtoutput_M_LF.csv"))
    assert (ctr["found"], ctr["not_found"]) == (1, 6)
    csv = open(tmp_path / "kmers.txtoutput_M_LF.csv", "rb").read()
    assert csv == b"#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n1\t0\t1\t0\t1\n1\t4\t3\t0\t0\n1\t7\t4\t0\t0\n"


def test_example_paper(oracle, tmp_path):
    base = _index(oracle, tmp_path, "examplePaper.eds", "ex")
    eng = oracle.Engine(base, 8)
    counts, occ, _ = eng.search(np.frombuffer(b"TAC", np.uint8), np.array([0, 3], np.uint64))
    assert _rows(occ) == [(1, 0, 1, 0, 5), (1, 4, 3, 0, 8), (1, 1, 2, 0, 1), (1, 2, 2, 1, 0), (1, 4, 3, 0, 1)]


@pytest.mark.parametrize("seed", range(12))
def test_oracle_vs_bruteforce(oracle, tmp_path, seed):
    rng = random.Random(seed)
    segs = edsgen.random_eds(rng, rng.randint(5, 60), alphabet="ACGT" if seed % 3 else "ACGTN",
                             p_empty=0.0 if seed % 4 == 0 else 0.25)
    base = _index(oracle, tmp_path, edsgen.eds_text(segs, use_E=(seed % 2 == 1)), text=True)
    eng = oracle.Engine(base, 2 + seed % 7)
    pats = []
    for _ in range(60):
        m = rng.randint(1, 14)
        p = edsgen.planted(rng, segs, m) if rng.random() < 0.7 else None
        pats.append(p or "".join(rng.choice("ACGT") for _ in range(m)))
    buf = np.frombuffer("".join(pats).encode(), np.uint8)
    offs = np.concatenate(([0], np.cumsum([len(p) for p in pats]))).astype(np.uint64)
    counts, occ, _ = eng.search(buf, offs, threads=1 + seed % 3)
    got = {}
    for r in _rows(occ):
        got.setdefault(r[0], []).append(r[1:])
    for i, p in enumerate(pats):
        exp = edsgen.brute_occurrences(segs, p)
        g = got.get(i + 1, [])
        assert len(g) == len(set(g)), (p, g)
        assert set(g) == exp, (seed, p, sorted(g), sorted(exp))
        assert counts[i] == len(exp)


def test_mlf_runs_files_equal_ebwt(oracle, tmp_path):
    rng = random.Random(7)
    segs = edsgen.random_eds(rng, 300, p_empty=0.2)
    base = _index(oracle, tmp_path, edsgen.eds_text(segs), text=True)
    a = oracle.Engine(base, 4, from_runs_files=True)
    b = oracle.Engine(base, 4, from_runs_files=False)
    for x, y in zip(a.mlf_arrays(), b.mlf_arrays()):
        assert np.array_equal(x, y)
    assert not a.last_run_split


@pytest.mark.parametrize("a", [2, 4, 8])
def test_mlf_is_lf(oracle, tmp_path, a):
    """move(x, interval(x)) == LF(x) for every row, and the structure is a-balanced."""
    rng = random.Random(a)
    segs = edsgen.random_eds(rng, 400, kmax=2, lmax=30, p_empty=0.1, alphabet="AC")  # long runs → splits
    base = _index(oracle, tmp_path, edsgen.eds_text(segs), text=True)
    eng = oracle.Engine(base, a)
    p, q, idx, Lp = eng.mlf_arrays()
    L = np.frombuffer(open(base + ".ebwt", "rb").read(), np.uint8)
    n = L.size
    # LF from rank
    C = {}
    acc = 0
    for c in sorted(set(L.tolist())):
        C[c] = acc
        acc += int((L == c).sum())
    seen = {c: 0 for c in C}
    lf = np.zeros(n, np.int64)
    for i, c in enumerate(L.tolist()):
        lf[i] = C[c] + seen[c]
        seen[c] += 1
    r = len(q)
    assert r >= eng.runs
    iv = np.searchsorted(p[:-1], np.arange(n), side="right") - 1
    for x in range(n):
        i = iv[x]
        y = q[i] + (x - p[i])
        assert y == lf[x]
        assert Lp[i] == L[x]
    # balanced: each output interval holds < 2a input starts
    for i in range(r):
        length = int(p[i + 1] - p[i])
        lo, hi = np.searchsorted(p[:-1], [q[i], q[i] + length])
        assert hi - lo < 2 * a


@pytest.mark.parametrize("seed", range(8))
def test_trie_variant_equals_literal(oracle, tmp_path, seed):
    """orc_search_batch_trie (the trie-sharing CPU variant) gives the literal
    pattern loop's counts and records in the same order, including '#' patterns, empty lines,
    duplicates and patterns that are suffixes of others; its interval steps never exceed the
    literal's."""
    rng = random.Random(100 + seed)
    segs = edsgen.random_eds(rng, rng.randint(10, 80), p_empty=0.0 if seed % 4 == 0 else 0.25)
    base = _index(oracle, tmp_path, edsgen.eds_text(segs, use_E=(seed % 2 == 1)), text=True)
    eng = oracle.Engine(base, 2 + seed % 5)
    pats = []
    for _ in range(300):
        m = rng.randint(0, 12)
        p = edsgen.planted(rng, segs, m) if m and rng.random() < 0.6 else None
        p = p or "".join(rng.choice("ACGT#" if rng.random() < 0.05 else "ACGT") for _ in range(m))
        pats.append(p)
        if rng.random() < 0.2:
            pats.append(p[rng.randint(0, len(p)):] if p else p)  # a suffix (or a duplicate)
    buf = np.frombuffer("".join(pats).encode(), np.uint8)
    offs = np.concatenate(([0], np.cumsum([len(p) for p in pats]))).astype(np.uint64)
    lc, lo, lctr = eng.search(buf, offs, first_pattern_id=5)
    for threads in (1, 3):
        tc, to, tctr = eng.search(buf, offs, first_pattern_id=5, threads=threads, trie=True)
        assert np.array_equal(tc, lc) and np.array_equal(to, lo)
        assert tctr["occurrences"] == lctr["occurrences"] and tctr["found"] == lctr["found"]
        assert tctr["interval_steps"] <= lctr["interval_steps"]


def test_console_early_return_rule(oracle, tmp_path):
    """The reference's backwardSearch returns before its locate loop (no 'num occ' line,
    MOVE_EDSBWTSearch.cpp:250-253,295-297,371) exactly when the pattern without its first
    character does not occur (its final list is the pattern's list after all but the first
    character) — the rule the CLI's console stream uses; checked on the literal loop."""
    import random
    import edsgen
    rng = random.Random(99)
    for t in range(3):
        segs = edsgen.random_eds(rng, 300, p_empty=0.25)
        (tmp_path / f"e{t}.eds").write_text(edsgen.eds_text(segs))
        base = str(tmp_path / f"e{t}")
        oracle.transform(str(tmp_path / f"e{t}.eds"), base)
        pats = [edsgen.planted(rng, segs, rng.randint(1, 12)) or "AC" for _ in range(200)]
        pats += ["".join(rng.choice("ACGTN") for _ in range(rng.randint(0, 10))) for _ in range(200)]
        buf = np.frombuffer("".join(pats).encode(), np.uint8)
        offs = np.concatenate(([0], np.cumsum([len(p) for p in pats]))).astype(np.uint64)
        eng = oracle.Engine(base, 8)
        counts, early = eng.console(buf, offs)
        c_ref, _, _ = eng.search(buf, offs)
        assert np.array_equal(counts, c_ref)
        sufs = [p[1:] for p in pats]
        sb = np.frombuffer("".join(sufs).encode(), np.uint8)
        so = np.concatenate(([0], np.cumsum([len(p) for p in sufs]))).astype(np.uint64)
        cs, _, _ = eng.search(sb, so)
        reach = np.array([len(p) == 1 or (len(p) > 1 and c > 0) for p, c in zip(pats, cs)])
        assert np.array_equal(~early, reach)
