"""The host-side 2-bit packer of fixed-length pattern lines (csrc/format.cpp), on CPU.

A chunk of the pattern file whose lines are all L bytes of A/C/G/T (getline lines,
MOVE_EDSBWTSearch.cpp:111) crosses PCIe as 2 bits per base and k_unpack_lines restores the
bytes on the device.  Here: the packed layout against a numpy restatement, the device
unpack restated in numpy (round trip to the exact line bytes), and every form the packer
must refuse so the chunk goes raw (other bytes, ragged or empty lines, '\\r\\n', L > 32).
"""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("EDSBWT_LIB") or os.path.join(ROOT, "eds-bwt_amd", "_build", "libedsbwt.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("libedsbwt.so not built")
    L = ctypes.CDLL(LIB)
    L.edsbwt_lines_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]
    L.edsbwt_lines_fixed.restype = ctypes.c_uint64
    L.edsbwt_pack_lines.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_void_p, ctypes.c_void_p]
    L.edsbwt_pack_lines.restype = ctypes.c_int
    return L


def _pack(lib, text: bytes, parts=1, reverse=False):
    """(P, L, packed bytes) or None when the packer refuses the chunk.  reverse: pack the parts
    last to first (the engine's pool threads finish in any order; a part must not write into
    the bytes of the next part)."""
    src = np.frombuffer(text, np.uint8).copy() if text else np.zeros(1, np.uint8)
    Lo = ctypes.c_uint32(0)
    P = lib.edsbwt_lines_fixed(src.ctypes.data, len(text), ctypes.byref(Lo))
    if not P:
        return None
    L = Lo.value
    S = (L + 3) // 4
    out = np.full(P * S + 16, 0xEE, np.uint8)
    end = src.ctypes.data + len(text)
    order = range(parts - 1, -1, -1) if reverse else range(parts)
    for t in order:  # the engine's pool splits the lines the same way
        p0, p1 = P * t // parts, P * (t + 1) // parts
        if p0 < p1 and not lib.edsbwt_pack_lines(src.ctypes.data, len(text), L, p0, p1, end, out.ctypes.data):
            return None
    return P, L, out[:P * S]


def _expect(lines, L):
    """numpy restatement of the packed layout: code (byte >> 1) & 3, base j at bits 2*(j%4) of byte j/4."""
    S = (L + 3) // 4
    a = np.frombuffer("".join(lines).encode(), np.uint8).reshape(len(lines), L)
    codes = (a >> 1) & 3
    pad = np.zeros((len(lines), S * 4), np.uint8)
    pad[:, :L] = codes
    q = pad.reshape(len(lines), S, 4).astype(np.uint32)
    return (q[:, :, 0] | (q[:, :, 1] << 2) | (q[:, :, 2] << 4) | (q[:, :, 3] << 6)).astype(np.uint8).reshape(-1)


def _unpack(packed, P, L):
    """kernels.hip k_unpack_lines restated: the line bytes (no '\\n') and the offsets."""
    S = (L + 3) // 4
    b = packed.reshape(P, S)
    j = np.arange(L)
    codes = (b[:, j // 4] >> (2 * (j % 4))) & 3
    return np.frombuffer(b"ACTG", np.uint8)[codes].reshape(-1), np.arange(P + 1, dtype=np.uint64) * L


@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 7, 8, 15, 16, 20, 31, 32])
@pytest.mark.parametrize("trailing", [True, False])
def test_pack_round_trip(lib, L, trailing):
    rng = random.Random(L * 2 + trailing)
    lines = ["".join(rng.choice("ACGT") for _ in range(L)) for _ in range(rng.randint(1, 3000))]
    text = ("\n".join(lines) + ("\n" if trailing else "")).encode()
    for parts in (1, 3, 7):
        r = _pack(lib, text, parts)
        assert r is not None
        P, LL, packed = r
        assert P == len(lines) and LL == L
        assert np.array_equal(packed, _expect(lines, L))
        by, offs = _unpack(packed, P, L)
        assert by.tobytes() == "".join(lines).encode() and offs[-1] == P * L


@pytest.mark.parametrize("bad", ["ACGN", "ACG", "ACGTA", "", "acgt", "AC\rT", "AC#T"])
def test_pack_refuses_irregular(lib, bad):
    rng = random.Random(5)
    lines = ["".join(rng.choice("ACGT") for _ in range(4)) for _ in range(500)]
    lines[rng.randrange(1, 500)] = bad
    assert _pack(lib, ("\n".join(lines) + "\n").encode(), 4) is None


def test_pack_refuses_other_forms(lib):
    assert _pack(lib, b"", 1) is None
    assert _pack(lib, b"\nACGT\n", 1) is None                   # an empty first line
    assert _pack(lib, (("A" * 33) + "\n").encode() * 4, 1) is None  # longer than 32 bases
    assert _pack(lib, b"ACGT\r\nACGT\r\n", 1) is None           # '\r' kept by getline
    assert _pack(lib, b"ACGT\nACG", 1) is None                  # a short unterminated last line
    assert _pack(lib, b"ACGT", 1) is None                       # no '\n' at all: sent raw


@pytest.mark.parametrize("L", list(range(1, 13)))
def test_pack_parts_any_order(lib, L):
    """Parts packed last-to-first, and on concurrent threads, over >= 32768 lines (the engine's
    pool uses 2+ threads from there): every line keeps its bases (8-byte stores of a
    part's last lines must not reach into the next part)."""
    import threading
    rng = np.random.default_rng(L)
    P = 40000 + L
    lines = ["".join("ACGT"[c] for c in row) for row in rng.integers(0, 4, (P, L))]
    text = ("\n".join(lines) + "\n").encode()
    want = _expect(lines, L)
    for parts in (2, 7, 12):
        r = _pack(lib, text, parts, reverse=True)
        assert r is not None and np.array_equal(r[2], want), (L, parts)
    src = np.frombuffer(text, np.uint8).copy()
    S = (L + 3) // 4
    out = np.full(P * S + 16, 0xEE, np.uint8)
    end = src.ctypes.data + len(text)
    parts = 12
    ok = []
    th = [threading.Thread(target=lambda t=t: ok.append(lib.edsbwt_pack_lines(
        src.ctypes.data, len(text), L, P * t // parts, P * (t + 1) // parts, end, out.ctypes.data)))
        for t in range(parts - 1, -1, -1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(ok) and np.array_equal(out[:P * S], want)


@pytest.mark.parametrize("L", [3, 20, 31])
def test_pack_refuses_every_other_byte(lib, L):
    """Every byte value other than A/C/G/T at a base, and every value other than '\\n' at a line's
    end, in the middle of a chunk (the packer's bulk path: one table lookup validates a line's
    bases and its '\\n' together), makes the packer refuse the chunk."""
    rng = np.random.default_rng(L)
    P = 3000
    a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, (P, L))]
    base = np.concatenate([a, np.full((P, 1), 10, np.uint8)], 1)
    assert _pack(lib, base.tobytes(), 2) is not None
    for b in range(256):
        for col in (0, L // 2, L - 1, L):
            good = (b == 10) if col == L else (b in b"ACGT")
            if good:
                continue
            t = base.copy()
            t[P // 3 + b, col] = b
            assert _pack(lib, t.tobytes(), 2) is None, (b, col)
