"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes bridge to oracle/_build/liboracle.so, the plain-C restatement of
riccardo-nozza/EDS-BWT's MOVE_EDSBWTSearch path (see edsbwt_oracle.c for the
file:line map).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg import this module; the product (eds-bwt_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# EDSBWT_ORACLE_BUILD: another build directory of this Makefile (the sanitizer build, _build_asan)
_BUILD = os.environ.get("EDSBWT_ORACLE_BUILD") or os.path.join(HERE, "_build")
LIB_PATH = os.path.join(_BUILD, "liboracle.so")
CLI_PATH = os.path.join(_BUILD, "edsbwt_oracle")

OCC_DTYPE = np.dtype([("pat", "<u4"), ("word", "<u4"), ("seg", "<u4"), ("word_in_seg", "<u4"), ("offset", "<u4")])


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("interval_steps", "step_moves", "locate_moves", "pdf_calls",
                                                "eof_reads", "occurrences", "found", "not_found")]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_transform.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_transform.restype = i32
        L.orc_open.argtypes = [ctypes.c_char_p, u32, i32]
        L.orc_open.restype = vp
        L.orc_close.argtypes = [vp]
        for f in ("orc_n", "orc_words", "orc_r_prime", "orc_runs"):
            getattr(L, f).argtypes = [vp]
            getattr(L, f).restype = u32
        L.orc_last_run_split.argtypes = [vp]
        L.orc_last_run_split.restype = i32
        L.orc_mlf_arrays.argtypes = [vp, vp, vp, vp, vp]
        L.orc_search_batch.argtypes = [vp, vp, vp, u64, u32, i32, vp, ctypes.POINTER(vp), ctypes.POINTER(u64),
                                       ctypes.POINTER(Counters)]
        L.orc_search_batch.restype = i32
        L.orc_search_batch_trie.argtypes = L.orc_search_batch.argtypes
        L.orc_search_batch_trie.restype = i32
        L.orc_search_batch_console.argtypes = [vp, vp, vp, u64, u32, i32, vp, vp]
        L.orc_search_batch_console.restype = i32
        L.orc_free.argtypes = [vp]
        L.orc_search_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, u64, i32, ctypes.POINTER(Counters),
                                      ctypes.POINTER(ctypes.c_double)]
        L.orc_search_file.restype = i32
        L.orc_check_records.argtypes = [ctypes.c_char_p, vp, vp, u64, u32, vp, u64, i32, ctypes.POINTER(u64),
                                        ctypes.POINTER(u64)]
        L.orc_check_records.restype = i32
        _L = L
    return _L


def transform(eds_path: str, base: str) -> None:
    """EDS-BWTransform.sh restated (naive suffix sort: small inputs only)."""
    if lib().orc_transform(eds_path.encode(), base.encode()) != 0:
        raise RuntimeError(lib().orc_last_error().decode())


def check_records(eds_path: str, buf: np.ndarray, offs: np.ndarray, occ: np.ndarray, first_pattern_id: int = 1,
                  threads: int = 8) -> tuple[int, int]:
    """BWT-free soundness check of occurrence records against the .eds text (see
    orc_check_records).  Returns (number of bad records, index of the first bad one or -1)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    occ = np.ascontiguousarray(occ, dtype=OCC_DTYPE)
    bad, first = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().orc_check_records(eds_path.encode(), buf.ctypes.data if buf.size else None, offs.ctypes.data, offs.size - 1,
                                 first_pattern_id, occ.ctypes.data if occ.size else None, occ.size, threads,
                                 ctypes.byref(bad), ctypes.byref(first))
    if rc != 0:
        raise RuntimeError(lib().orc_last_error().decode())
    return int(bad.value), (-1 if first.value == 2**64 - 1 else int(first.value))


class Engine:
    def __init__(self, base: str, a: int = 8, from_runs_files: bool = False):
        self._h = lib().orc_open(base.encode(), a, 1 if from_runs_files else 0)
        if not self._h:
            raise RuntimeError(lib().orc_last_error().decode())

    def close(self):
        if self._h:
            lib().orc_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def r_prime(self) -> int:
        return lib().orc_r_prime(self._h)

    @property
    def runs(self) -> int:
        return lib().orc_runs(self._h)

    @property
    def n(self) -> int:
        return lib().orc_n(self._h)

    @property
    def last_run_split(self) -> bool:
        return bool(lib().orc_last_run_split(self._h))

    def mlf_arrays(self):
        r = self.r_prime
        p = np.zeros(r + 1, np.uint32)
        q = np.zeros(r, np.uint32)
        idx = np.zeros(r, np.uint32)
        L = np.zeros(r, np.uint8)
        lib().orc_mlf_arrays(self._h, p.ctypes.data, q.ctypes.data, idx.ctypes.data, L.ctypes.data)
        return p, q, idx, L

    def search(self, buf: np.ndarray, offs: np.ndarray, first_pattern_id: int = 1, threads: int = 1,
               trie: bool = False):
        """The reference's pattern loop over the batch; trie=True shares common pattern suffixes
        (orc_search_batch_trie: same results, deduplicated counters)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        npat = offs.size - 1
        counts = np.zeros(max(npat, 1), np.uint32)
        occ_p = ctypes.c_void_p()
        nocc = ctypes.c_uint64()
        c = Counters()
        fn = lib().orc_search_batch_trie if trie else lib().orc_search_batch
        rc = fn(self._h, buf.ctypes.data if buf.size else None, offs.ctypes.data, npat,
                first_pattern_id, threads, counts.ctypes.data, ctypes.byref(occ_p), ctypes.byref(nocc), ctypes.byref(c))
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        occ = np.zeros(nocc.value, OCC_DTYPE)
        if nocc.value:
            ctypes.memmove(occ.ctypes.data, occ_p.value, nocc.value * OCC_DTYPE.itemsize)
        lib().orc_free(occ_p)
        return counts[:npat], occ, c.as_dict()

    def console(self, buf: np.ndarray, offs: np.ndarray, threads: int = 1):
        """(counts, early): early[i] when the reference's backwardSearch returns before its
        locate loop for pattern i (no "num occ" line, MOVE_EDSBWTSearch.cpp:250-253,295-297,371)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        npat = offs.size - 1
        counts = np.zeros(max(npat, 1), np.uint32)
        early = np.zeros(max(npat, 1), np.uint8)
        rc = lib().orc_search_batch_console(self._h, buf.ctypes.data if buf.size else None, offs.ctypes.data, npat, 1, threads,
                                            counts.ctypes.data, early.ctypes.data)
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return counts[:npat], early[:npat].astype(bool)

    def search_file(self, patterns_path: str, out_csv: str | None, limit: int = 0, threads: int = 1):
        c = Counters()
        secs = ctypes.c_double()
        rc = lib().orc_search_file(self._h, patterns_path.encode(), out_csv.encode() if out_csv else None, limit,
                                   threads, ctypes.byref(c), ctypes.byref(secs))
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return c.as_dict(), secs.value
