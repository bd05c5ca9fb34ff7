"""The C-ABI library loads and exports every symbol include/edsbwt.h declares
(no compute without a GPU)."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT


def _declared():
    hdr = open(os.path.join(ROOT, "include", "edsbwt.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(edsbwt_[a-z_]+)\s*\(", hdr)))


def test_header_symbols_exported(edsbwt):
    L = edsbwt.lib()
    names = _declared()
    assert "edsbwt_search" in names and "edsbwt_index_open" in names
    for n in names:
        assert hasattr(L, n), n
    assert L.edsbwt_abi_version() == 7
    assert L.edsbwt_device_count() >= 0  # (0 without a GPU: no compute)


def test_build_id_matches_sources(edsbwt):
    """libedsbwt.so carries the hash of the sources it was built from; lib() refuses a stale one."""
    L = edsbwt.lib()
    assert L.edsbwt_build_id().decode() == edsbwt.source_build_id()


def test_open_missing_index_fails_cleanly(edsbwt, tmp_path):
    import pytest
    with pytest.raises(edsbwt.EdsBwtError) as e:
        edsbwt.Index(str(tmp_path / "nope"))
    assert e.value.code in (-1, -4)


def test_format_csv(edsbwt):
    import numpy as np
    occ = np.zeros(3, edsbwt.OCC_DTYPE)
    occ["pat"] = [1, 1, 12]
    occ["word"] = [3, 4000000000, 0]
    occ["seg"] = [2, 3, 1]
    occ["offset"] = [0, 1, 99]
    assert edsbwt.format_csv(occ, threads=2) == b"1\t3\t2\t0\t0\n1\t4000000000\t3\t0\t1\n12\t0\t1\t0\t99\n"


def test_read_pattern_file_getline(edsbwt, tmp_path):
    p = tmp_path / "p.txt"
    p.write_bytes(b"ACG\nT\r\n\nGG")
    buf, offs = edsbwt.read_pattern_file(str(p))
    pats = [bytes(buf[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    assert pats == [b"ACG", b"T\r", b"", b"GG"]
    p.write_bytes(b"A\nC\n")
    buf, offs = edsbwt.read_pattern_file(str(p))
    assert len(offs) == 3


def test_write_csv(edsbwt, tmp_path):
    """edsbwt_write_csv (the CLI's pwrite path) writes the bytes edsbwt_format_csv builds, at
    the given offset, with any thread count."""
    rng = np.random.default_rng(9)
    n = 300_000
    occ = np.zeros(n, edsbwt.OCC_DTYPE)
    for f, hi in (("pat", 10_000_000), ("word", 2**32 - 1), ("seg", 2**31), ("word_in_seg", 50), ("offset", 10**6)):
        occ[f] = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
    want = edsbwt.format_csv(occ, threads=4)
    for threads in (1, 3, 16):
        p = tmp_path / f"o{threads}.csv"
        with open(p, "wb") as f:
            f.write(b"HEADER\n")
            f.flush()
            assert edsbwt.write_csv(occ, f.fileno(), 7, threads) == len(want)
        assert p.read_bytes() == b"HEADER\n" + want
    p = tmp_path / "empty.csv"
    with open(p, "wb") as f:
        assert edsbwt.write_csv(occ[:0], f.fileno(), 0, 4) == 0


def test_header_flags_match_python(edsbwt):
    """Every EDSBWT_* search flag and path tag include/edsbwt.h defines has the same value in the
    Python host (eds-bwt_amd/__init__.py), and no two search flags share a bit."""
    hdr = open(os.path.join(ROOT, "include", "edsbwt.h")).read()
    defs = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"#define EDSBWT_([A-Z_0-9]+)\s+(0x[0-9a-fA-F]+)u?", hdr)}
    flags = {k: v for k, v in defs.items() if not k.startswith(("PATH_", "E_"))}
    assert "NO_COUNTERS" in flags and "NO_TEXT" in flags
    for k, v in flags.items():
        if hasattr(edsbwt, k):
            assert getattr(edsbwt, k) == v, k
    for k in ("COUNT_ONLY", "LOCATE", "NO_TEXT", "NO_COUNTERS", "NO_PAIRS"):
        assert hasattr(edsbwt, k), k
    bits = [v for v in flags.values() if v and (v & (v - 1)) == 0]
    assert len(bits) == len(set(bits))
