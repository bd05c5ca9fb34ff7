"""Product index writer (eds_transform) == oracle transform byte-for-byte; the
synthetic generators are reproducible and planted patterns occur."""
import os
import random
import subprocess

import numpy as np
import pytest

from conftest import ROOT, GOLDEN
import edsgen

BUILD = os.path.join(ROOT, "eds-bwt_amd", "_build")
FILES = [".ebwt", "_info.aux", ".bitvector", "_runs.aux", "_runs.txt"]


def _run(*args):
    return subprocess.run([os.path.join(BUILD, args[0]), *map(str, args[1:])], check=True, capture_output=True)


@pytest.mark.parametrize("seed", range(8))
def test_transform_matches_oracle(oracle, tmp_path, seed):
    rng = random.Random(1000 + seed)
    alpha = ["ACGT", "ACGTN", "AC", "ACGTNRY"][seed % 4]
    segs = edsgen.random_eds(rng, rng.randint(1, 800), alphabet=alpha, lmax=2 + 4 * seed, p_empty=0.3 * (seed % 2))
    eds = tmp_path / "x.eds"
    eds.write_text(edsgen.eds_text(segs, use_E=seed % 3 == 0))
    oracle.transform(str(eds), str(tmp_path / "o"))
    _run("eds_transform", eds, tmp_path / "p", "--threads", 1 + seed % 4)
    for f in FILES:
        assert (tmp_path / ("o" + f)).read_bytes() == (tmp_path / ("p" + f)).read_bytes(), f
    sigma = (tmp_path / "o_info.aux").read_bytes()[8]
    for j in range(sigma):
        assert (tmp_path / f"o_bwt_{j}.aux").read_bytes() == (tmp_path / f"p_bwt_{j}.aux").read_bytes()


def test_transform_repetitive_ties(oracle, tmp_path):
    # long identical words force tie groups beyond one packed chunk
    w = "ACGT" * 30
    segs = [[w, w + "A", "C" + w], ["", w], [w], [w[:-1], w]] * 20
    eds = tmp_path / "r.eds"
    eds.write_text(edsgen.eds_text(segs))
    oracle.transform(str(eds), str(tmp_path / "o"))
    _run("eds_transform", eds, tmp_path / "p")
    for f in FILES:
        assert (tmp_path / ("o" + f)).read_bytes() == (tmp_path / ("p" + f)).read_bytes(), f


def test_transform_rejects_bad_input(tmp_path):
    for bad in ["{A,C}\n", "{A}{}", "{AE}", "A{C}", "{acg}"]:
        p = tmp_path / "b.eds"
        p.write_text(bad)
        r = subprocess.run([os.path.join(BUILD, "eds_transform"), str(p), str(tmp_path / "b")], capture_output=True)
        assert r.returncode != 0, bad


@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_generator_reproducible_and_planted(oracle, tmp_path, cfg):
    eds = tmp_path / "g.eds"
    _run("edsbwt_gen", "eds", "--config", cfg, "--chars", 20000, "--seed", 3, "--out", eds)
    a = eds.read_bytes()
    _run("edsbwt_gen", "eds", "--config", cfg, "--chars", 20000, "--seed", 3, "--out", eds)
    assert eds.read_bytes() == a
    if cfg == "c3":
        assert b",}" in a or b"{," in a or b",," in a  # empty words exist
    pats = tmp_path / "p.txt"
    _run("edsbwt_gen", "patterns", "--eds", eds, "--count", 200, "--len", 12, "--mode", "planted", "--seed", 4, "--out", pats)
    _run("eds_transform", eds, tmp_path / "g")
    buf = np.frombuffer(pats.read_bytes().replace(b"\n", b""), np.uint8)
    offs = np.arange(0, 201 * 12, 12, dtype=np.uint64)
    counts, _, _ = oracle.Engine(str(tmp_path / "g")).search(buf, offs)
    assert (counts > 0).all()  # every planted pattern occurs
