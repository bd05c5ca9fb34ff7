"""eds-bwt_amd — MI355X-native EDS-BWT backward search (host side, Python).

Python mirror of the reference's MOVE_EDSBWTSearch path (riccardo-nozza/EDS-BWT):

* :class:`MoveEDSBWT` mirrors ``MOVE_EDSBWT::MOVE_EDSBWT(base, patterns)``
  (MOVE_EDSBWTSearch.cpp:23-176): load the index, search every line of the pattern
  file, write ``<patterns>output_M_LF.csv`` and keep ``count_found`` /
  ``count_not_found``.
* :class:`Index` is the batch API over the C ABI of ``include/edsbwt.h``
  (``libedsbwt.so``, hand-written gfx950 kernels).

Everything computes on the GPU through ``libedsbwt.so``; there is no CPU fallback.
A missing or unloadable library raises :class:`EdsBwtError`.  The package directory
name contains a hyphen, so import it with ``importlib.import_module("eds-bwt_amd")``.
"""
from __future__ import annotations

import ctypes
import os
import time
from typing import Iterable, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(_HERE, "_build")
LIB_PATH = os.environ.get("EDSBWT_LIB") or os.path.join(BUILD_DIR, "libedsbwt.so")

COUNT_ONLY = 0x1
LOCATE = 0x2
LOCATE_TABLE = 0x4
PROFILE = 0x8
NO_DEEP = 0x10
ORDERED = 0x20
PROFILE_LIGHT = 0x40
NO_WIDE = 0x80
LOCATE_WALK = 0x100
LEGACY_ORDER = 0x200
NO_KTAB = 0x400
NO_DIRECT = 0x800
NO_PAIRS = 0x1000
NO_TEXT = 0x2000
NO_COUNTERS = 0x4000

# edsbwt_last_paths bits (EDSBWT_PATH_TAGS=1): the kernels a pattern went through
PATH_DEEP = 0x1
PATH_WIDE = 0x2
PATH_LEVELS = 0x4
PATH_REDO = 0x8

OCC_DTYPE = np.dtype([("pat", "<u4"), ("word", "<u4"), ("seg", "<u4"), ("word_in_seg", "<u4"), ("offset", "<u4")])
CSV_HEADER = b"#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n"  # MOVE_EDSBWTSearch.cpp:59 (note the trailing space)


class EdsBwtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"edsbwt error {code}: {msg}")
        self.code = code


class _Info(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_uint64), ("n_words", ctypes.c_uint64), ("n_segments", ctypes.c_uint64),
                ("sigma", ctypes.c_uint32), ("alphabet", ctypes.c_uint8 * 16), ("device_bytes", ctypes.c_uint64),
                ("ktab_depth", ctypes.c_uint32), ("pair_blocks", ctypes.c_uint32), ("ktab_items", ctypes.c_uint64),
                ("ltab_depth", ctypes.c_uint32), ("ltab_groups", ctypes.c_uint32), ("ltab_items", ctypes.c_uint64),
                ("open_peak_bytes", ctypes.c_uint64), ("open_seconds", ctypes.c_double)]


class _Stats(ctypes.Structure):
    _fields_ = [("patterns", ctypes.c_uint64), ("found", ctypes.c_uint64), ("not_found", ctypes.c_uint64),
                ("occurrences", ctypes.c_uint64), ("depths", ctypes.c_uint64), ("trie_nodes", ctypes.c_uint64),
                ("intervals_stepped", ctypes.c_uint64), ("link_hash_rows", ctypes.c_uint64),
                ("link_ranges", ctypes.c_uint64), ("locate_lf_steps", ctypes.c_uint64),
                ("deep_from_depth", ctypes.c_uint64), ("deep_overflow", ctypes.c_uint64),
                ("deep_level_rerun", ctypes.c_uint64), ("ms_total", ctypes.c_double),
                ("ms_kernel", ctypes.c_double * 16), ("launches_kernel", ctypes.c_uint64 * 16),
                ("bytes_kernel", ctypes.c_uint64 * 16),
                ("lines_kernel", ctypes.c_uint64 * 16),
                ("locate_offsets", ctypes.c_uint64),
                ("search_groups", ctypes.c_uint64), ("start_depth", ctypes.c_uint64),
                ("ms_wall", ctypes.c_double), ("chunks", ctypes.c_uint64), ("bytes_h2d", ctypes.c_uint64),
                ("bytes_d2h", ctypes.c_uint64), ("text_chars", ctypes.c_uint64), ("text_rows", ctypes.c_uint64),
                ("redo_searches", ctypes.c_uint64)]


_LIB = None
# the library's sources, in the order eds-bwt_amd/Makefile hashes them into BUILD_ID
_SOURCES = ("csrc/engine.hip", "csrc/index_io.cpp", "csrc/format.cpp", "csrc/kernels.hip", "csrc/kernels.h", "csrc/index_io.h",
            "../include/edsbwt.h")


def source_build_id() -> str:
    """sha256 (16 hex digits) of the library sources in this tree (Makefile BUILD_ID)."""
    import hashlib
    h = hashlib.sha256()
    for f in _SOURCES:
        with open(os.path.join(_HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def lib() -> ctypes.CDLL:
    """Load libedsbwt.so (built in-tree by __graft_entry__.build()); raise if it is absent or
    was built from other sources than the ones in this tree (EDSBWT_LIB overrides skip the check)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise EdsBwtError(-4, f"{LIB_PATH} not built: run __graft_entry__.build() (make -C eds-bwt_amd)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL, use_errno=True)  # (edsbwt_write_csv reports pwrite's errno)
    L.edsbwt_build_id.argtypes = []
    L.edsbwt_build_id.restype = ctypes.c_char_p
    built = L.edsbwt_build_id().decode()
    if not os.environ.get("EDSBWT_LIB") and built != source_build_id():
        raise EdsBwtError(-4, f"{LIB_PATH} was built from sources {built}, the tree holds {source_build_id()}: "
                              "rebuild it (make -C eds-bwt_amd)")
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    L.edsbwt_index_open.argtypes = [ctypes.c_char_p, i32, u32, ctypes.POINTER(vp)]
    L.edsbwt_index_open.restype = i32
    L.edsbwt_index_close.argtypes = [vp]
    L.edsbwt_index_close.restype = None
    L.edsbwt_index_get_info.argtypes = [vp, ctypes.POINTER(_Info)]
    L.edsbwt_index_get_info.restype = i32
    L.edsbwt_search.argtypes = [vp, vp, vp, u64, u32, u32, vp, ctypes.POINTER(vp), ctypes.POINTER(u64)]
    L.edsbwt_search.restype = i32
    L.edsbwt_search_device.argtypes = [vp, vp, vp, u64, u32, u32, vp, ctypes.POINTER(vp), ctypes.POINTER(u64), vp]
    L.edsbwt_search_device.restype = i32
    if hasattr(L, "edsbwt_search_device_ids"):  # (ABI 6)
        L.edsbwt_search_device_ids.argtypes = [vp, vp, vp, u64, vp, u32, vp, ctypes.POINTER(vp), ctypes.POINTER(u64), vp]
        L.edsbwt_search_device_ids.restype = i32
    L.edsbwt_search_lines.argtypes = [vp, vp, u64, u32, u32, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(vp),
                                      ctypes.POINTER(u64)]
    L.edsbwt_search_lines.restype = i32
    if hasattr(L, "edsbwt_prepare"):  # (ABI 5)
        L.edsbwt_prepare.argtypes = [vp, u64, u64, u64, u32]
        L.edsbwt_prepare.restype = i32
        L.edsbwt_device_count.argtypes = []
        L.edsbwt_device_count.restype = i32
    L.edsbwt_host_alloc.argtypes = [u64, ctypes.POINTER(vp)]
    L.edsbwt_host_alloc.restype = i32
    L.edsbwt_host_free.argtypes = [vp]
    L.edsbwt_host_free.restype = None
    L.edsbwt_occ_free.argtypes = [vp]
    L.edsbwt_occ_free.restype = None
    L.edsbwt_set_counts_mirror.argtypes = [vp, vp, u64]
    L.edsbwt_set_counts_mirror.restype = i32
    if hasattr(L, "edsbwt_comm_init"):  # (ABI 7: the native RCCL exchange)
        L.edsbwt_comm_unique_id.argtypes = [vp, u64]
        L.edsbwt_comm_unique_id.restype = i32
        L.edsbwt_comm_init.argtypes = [vp, vp, u64, i32, i32]
        L.edsbwt_comm_init.restype = i32
        L.edsbwt_gather_counts.argtypes = [vp, vp, u64, vp, vp, i32]
        L.edsbwt_gather_counts.restype = i32
        L.edsbwt_comm_sync.argtypes = [vp]
        L.edsbwt_comm_sync.restype = i32
    L.edsbwt_last_paths.argtypes = [vp, vp, u64]
    L.edsbwt_last_paths.restype = i32
    L.edsbwt_last_stats.argtypes = [vp, ctypes.POINTER(_Stats)]
    L.edsbwt_last_stats.restype = i32
    L.edsbwt_kernel_name.argtypes = [i32]
    L.edsbwt_kernel_name.restype = ctypes.c_char_p
    L.edsbwt_format_csv.argtypes = [vp, u64, vp, u64, i32]
    L.edsbwt_format_csv.restype = u64
    if hasattr(L, "edsbwt_write_csv"):  # (an EDSBWT_LIB override built before ABI 4 lacks it)
        L.edsbwt_write_csv.argtypes = [vp, u64, i32, u64, i32]
        L.edsbwt_write_csv.restype = ctypes.c_int64
    L.edsbwt_last_error.argtypes = []
    L.edsbwt_last_error.restype = ctypes.c_char_p
    L.edsbwt_abi_version.argtypes = []
    L.edsbwt_abi_version.restype = i32
    _LIB = L
    return L


def _check(rc: int) -> None:
    if rc != 0:
        raise EdsBwtError(rc, lib().edsbwt_last_error().decode(errors="replace"))


def pack_patterns(patterns: Iterable[bytes | str]) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate patterns into (bytes u8[], offsets u64[npat+1])."""
    pats = [p.encode() if isinstance(p, str) else bytes(p) for p in patterns]
    offs = np.zeros(len(pats) + 1, dtype=np.uint64)
    if pats:
        offs[1:] = np.cumsum([len(p) for p in pats], dtype=np.uint64)
    buf = np.frombuffer(b"".join(pats), dtype=np.uint8) if pats else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), offs


def read_pattern_file(path: str) -> tuple[np.ndarray, np.ndarray]:
    """std::getline semantics (MOVE_EDSBWTSearch.cpp:111): split at '\\n', keep '\\r',
    a last line without '\\n' counts, a trailing '\\n' does not open a new line."""
    data = np.fromfile(path, dtype=np.uint8)
    nl = np.flatnonzero(data == 10)
    starts = np.concatenate(([0], nl + 1))
    ends = np.concatenate((nl, [data.size]))
    if starts.size and starts[-1] >= data.size:  # file ends with '\n'
        starts, ends = starts[:-1], ends[:-1]
    lens = (ends - starts).astype(np.uint64)
    offs = np.zeros(lens.size + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    keep = np.ones(data.size, dtype=bool)
    keep[nl] = False
    return np.ascontiguousarray(data[keep]), offs


class HostBuffer:
    """Page-locked host memory (edsbwt_host_alloc) viewed as a numpy array: pattern bytes,
    counts and records move over PCIe at full rate from/to it."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _check(lib().edsbwt_host_alloc(int(nbytes), ctypes.byref(p)))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    def array(self, dtype=np.uint8, count: int = -1) -> np.ndarray:
        dt = np.dtype(dtype)
        n = self.nbytes // dt.itemsize if count < 0 else count
        raw = (ctypes.c_char * (n * dt.itemsize)).from_address(self.ptr) if n else bytearray()
        return np.frombuffer(raw, dtype=dt, count=n)

    def free(self) -> None:
        if getattr(self, "ptr", None):
            lib().edsbwt_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def read_pattern_file_pinned(path: str) -> HostBuffer:
    """The pattern file's bytes in page-locked memory (input of Index.search_lines)."""
    n = os.path.getsize(path)
    hb = HostBuffer(max(n, 1))
    if n:
        with open(path, "rb") as f:
            f.readinto(memoryview(hb.array(np.uint8, n)).cast("B"))
    hb.nbytes = n
    return hb


class Index:
    """A loaded EDS-BWT index on one GPU (edsbwt_index_open)."""

    def __init__(self, base: str, device: int = 0, a_balance: int = 8):
        L = lib()
        h = ctypes.c_void_p()
        _check(L.edsbwt_index_open(base.encode(), int(device), int(a_balance), ctypes.byref(h)))
        self._h = h
        self.base = base
        self.device = device
        inf = _Info()
        _check(L.edsbwt_index_get_info(self._h, ctypes.byref(inf)))
        self.n_rows, self.n_words, self.n_segments = inf.n_rows, inf.n_words, inf.n_segments
        self.sigma = inf.sigma
        self.alphabet = bytes(inf.alphabet[: inf.sigma])
        self.device_bytes = inf.device_bytes
        self.ktab_depth, self.ktab_items = inf.ktab_depth, inf.ktab_items
        self.ltab_depth, self.ltab_groups, self.ltab_items = inf.ltab_depth, inf.ltab_groups, inf.ltab_items
        self.pair_blocks = bool(inf.pair_blocks)
        self.open_peak_bytes, self.open_seconds = inf.open_peak_bytes, inf.open_seconds

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().edsbwt_index_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def search(self, patterns: Sequence[bytes | str] | tuple[np.ndarray, np.ndarray], *, first_pattern_id: int = 1,
               locate: bool = True, table: bool = False, profile: bool = False, deep: bool = True,
               ordered: bool = False, wide: bool = True, walk: bool = False, legacy: bool = False,
               ktab: bool = True, direct: bool = True, pairs: bool = True, text: bool = True, counters: bool = True):
        """Search a batch.  Returns (counts u32[npat], occ OCC_DTYPE[nocc]).
        ``table``: (word, offset) per row from the full table; ``walk``: the reference's
        full LF walk to '#'; default: walk to the first sampled row.  ``legacy``: records in
        the legacy EDSBWTsearch engine's order (``<patterns>output.csv``) instead of MOVE's."""
        buf, offs = patterns if isinstance(patterns, tuple) else pack_patterns(patterns)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        npat = offs.size - 1
        counts = np.zeros(max(npat, 0), dtype=np.uint32)
        flags = ((LOCATE if locate else COUNT_ONLY) | (LOCATE_TABLE if table else 0) | (PROFILE if profile else 0)
                 | (0 if deep else NO_DEEP) | (ORDERED if ordered else 0) | (0 if wide else NO_WIDE)
                 | (LOCATE_WALK if walk else 0) | (LEGACY_ORDER if legacy else 0) | (0 if ktab else NO_KTAB)
                 | (0 if direct else NO_DIRECT) | (0 if pairs else NO_PAIRS) | (0 if text else NO_TEXT)
                 | (0 if counters else NO_COUNTERS))
        occ_p = ctypes.c_void_p()
        nocc = ctypes.c_uint64()
        bp = buf.ctypes.data if buf.size else None
        _check(lib().edsbwt_search(self._h, bp, offs.ctypes.data, npat, first_pattern_id, flags,
                                   counts.ctypes.data if npat else None, ctypes.byref(occ_p), ctypes.byref(nocc)))
        n = nocc.value
        occ = np.zeros(n, dtype=OCC_DTYPE)
        if n:
            ctypes.memmove(occ.ctypes.data, occ_p.value, n * OCC_DTYPE.itemsize)
            lib().edsbwt_occ_free(occ_p)
        return counts, occ

    def search_lines(self, text_ptr: int, nbytes: int, counts_ptr: int, counts_cap: int, *, first_pattern_id: int = 1,
                     locate: bool = True, profile: bool = False, keep: bool = False):
        """A pattern file in host memory (ideally page-locked: HostBuffer) through the
        pipelined host path (edsbwt_search_lines).  Returns (patterns, records pointer,
        number of records); the records are page-locked and library-owned: pass keep=True and
        free them with occ_free(ptr), else they are given back at once (timing runs)."""
        pflag = {False: 0, True: PROFILE, "light": PROFILE_LIGHT}[profile]
        flags = (LOCATE if locate else COUNT_ONLY) | pflag
        occ_p = ctypes.c_void_p()
        nocc = ctypes.c_uint64()
        npat = ctypes.c_uint64()
        _check(lib().edsbwt_search_lines(self._h, text_ptr, nbytes, first_pattern_id, flags, counts_ptr, counts_cap,
                                         ctypes.byref(npat), ctypes.byref(occ_p), ctypes.byref(nocc)))
        if not keep and occ_p.value:
            lib().edsbwt_occ_free(occ_p.value)
            return npat.value, 0, nocc.value
        return npat.value, occ_p.value or 0, nocc.value

    def prepare(self, text_bytes: int, npat: int, *, records_hint: int = 0, locate: bool = True) -> None:
        """edsbwt_prepare: set the host pipeline up for a search_lines batch of about this size
        (synthetic lines; nothing of the batch is searched), so its first call runs at steady state."""
        flags = LOCATE if locate else COUNT_ONLY
        _check(lib().edsbwt_prepare(self._h, int(text_bytes), int(npat), int(records_hint), flags))

    @staticmethod
    def occ_view(ptr: int, n: int) -> np.ndarray:
        """numpy view of n records at a library-owned host pointer (valid until occ_free)."""
        if not n:
            return np.zeros(0, OCC_DTYPE)
        raw = (ctypes.c_char * (n * OCC_DTYPE.itemsize)).from_address(ptr)
        return np.frombuffer(raw, dtype=OCC_DTYPE, count=n)

    @staticmethod
    def occ_free(ptr: int) -> None:
        if ptr:
            lib().edsbwt_occ_free(ptr)

    def search_device(self, d_bytes: int, d_offsets: int, npat: int, d_counts: int, *, first_pattern_id: int = 1,
                      locate: bool = True, table: bool = False, profile: bool = False, deep: bool = True,
                      stream: int = 0, walk: bool = False, ktab: bool = True, direct: bool = True,
                      pairs: bool = True, text: bool = True, ids: int = 0, counters: bool = True):
        """Device-resident batch (pointers are device addresses, e.g. torch data_ptr()).
        ids: device array of npat u32 — pattern i is reported as #Pat ids[i] (edsbwt_search_device_ids)
        instead of first_pattern_id + i.  counters=False: EDSBWT_NO_COUNTERS (the deep kernels' work
        statistics read 0; same results).  Returns (device pointer of the records, number of records)."""
        pflag = {False: 0, True: PROFILE, "light": PROFILE_LIGHT}[profile]
        flags = (LOCATE if locate else COUNT_ONLY) | (LOCATE_TABLE if table else 0) | pflag | (0 if deep else NO_DEEP) \
            | (LOCATE_WALK if walk else 0) | (0 if ktab else NO_KTAB) | (0 if direct else NO_DIRECT) \
            | (0 if pairs else NO_PAIRS) | (0 if text else NO_TEXT) | (0 if counters else NO_COUNTERS)
        occ_p = ctypes.c_void_p()
        nocc = ctypes.c_uint64()
        if ids:
            _check(lib().edsbwt_search_device_ids(self._h, d_bytes, d_offsets, npat, ids, flags, d_counts,
                                                  ctypes.byref(occ_p), ctypes.byref(nocc), stream or None))
        else:
            _check(lib().edsbwt_search_device(self._h, d_bytes, d_offsets, npat, first_pattern_id, flags, d_counts,
                                              ctypes.byref(occ_p), ctypes.byref(nocc), stream or None))
        return occ_p.value or 0, nocc.value

    def set_counts_mirror(self, d_counts: int, cap: int) -> None:
        """Host-pipeline calls also leave the u32 counts in device array d_counts[cap] (the
        multi-GPU exchange gathers them over RCCL); 0 turns it off."""
        _check(lib().edsbwt_set_counts_mirror(self._h, d_counts or None, int(cap) if d_counts else 0))

    # ---- the native RCCL exchange (ABI 7, include/edsbwt.h): one process per GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        """rank 0: a new RCCL unique id (128 bytes) to hand to every rank's comm_init."""
        buf = ctypes.create_string_buffer(128)
        _check(lib().edsbwt_comm_unique_id(buf, 128))
        return buf.raw

    def comm_init(self, uid: bytes, nranks: int, rank: int) -> None:
        """An RCCL communicator on this index's device (edsbwt_comm_init)."""
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        _check(lib().edsbwt_comm_init(self._h, buf, len(uid), int(nranks), int(rank)))

    def gather_counts(self, d_counts: int, n: int, d_out: int, sizes: np.ndarray, dst: int = 0) -> None:
        """Queue the gather of every rank's counts to rank dst (device pointers; sizes: uint64 per
        rank, kept alive by the caller); returns at once (edsbwt_gather_counts)."""
        sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
        _check(lib().edsbwt_gather_counts(self._h, d_counts or None, int(n), d_out or None, sizes.ctypes.data, int(dst)))

    def comm_sync(self) -> None:
        """Wait until every queued gather is done (edsbwt_comm_sync)."""
        _check(lib().edsbwt_comm_sync(self._h))

    def path_tags(self, n: int) -> np.ndarray:
        """PATH_* bits per pattern of the last search_device call (the process must run with
        EDSBWT_PATH_TAGS=1 before the index is opened): which patterns took k_deep, the wide
        lists, the level re-run, or a searched-again batch."""
        out = np.zeros(max(n, 1), np.uint8)
        _check(lib().edsbwt_last_paths(self._h, out.ctypes.data, n))
        return out[:n]

    def stats(self) -> dict:
        s = _Stats()
        _check(lib().edsbwt_last_stats(self._h, ctypes.byref(s)))
        out = {k: getattr(s, k) for k, _ in _Stats._fields_ if k not in ("ms_kernel", "launches_kernel", "bytes_kernel", "lines_kernel")}
        out["kernels"] = {n: {"ms": s.ms_kernel[i], "launches": s.launches_kernel[i], "bytes": s.bytes_kernel[i],
                              "lines": s.lines_kernel[i]}
                          for i, n in enumerate(kernel_names()) if n}
        return out

    # ---- cheap per-call statistics for timed loops (bench.py): one preallocated struct, no dict
    def stats_struct(self) -> "_Stats":
        """The last call's edsbwt_stats, refreshed into one struct owned by this Index."""
        if getattr(self, "_st", None) is None:
            self._st = _Stats()
            st = self._st
            self._st_views = [np.ctypeslib.as_array(st.ms_kernel), np.ctypeslib.as_array(st.launches_kernel),
                              np.ctypeslib.as_array(st.bytes_kernel), np.ctypeslib.as_array(st.lines_kernel)]
        _check(lib().edsbwt_last_stats(self._h, ctypes.byref(self._st)))
        return self._st

    @staticmethod
    def kernel_acc() -> np.ndarray:
        """Accumulator for add_kernel_stats: rows ms, launches, bytes, lines per kernel class."""
        return np.zeros((4, 16), np.float64)

    def add_kernel_stats(self, acc: np.ndarray) -> "_Stats":
        """acc += the last call's per-class kernel times / launches / bytes / lines."""
        st = self.stats_struct()
        for r, v in enumerate(self._st_views):
            acc[r] += v
        return st

    @staticmethod
    def kernel_acc_dict(acc: np.ndarray) -> dict:
        return {n: {"ms": float(acc[0, i]), "launches": int(acc[1, i]), "bytes": int(acc[2, i]), "lines": int(acc[3, i])}
                for i, n in enumerate(kernel_names()) if n}


_KNAMES = None


def kernel_names() -> list:
    """engine.hip kernel class names (edsbwt_kernel_name), cached."""
    global _KNAMES
    if _KNAMES is None:
        _KNAMES = [lib().edsbwt_kernel_name(i).decode() for i in range(16)]
    return _KNAMES


def write_csv(occ: np.ndarray, fd: int, at: int = 0, threads: int = 8) -> int:
    """CSV body rows written to file descriptor fd at byte offset `at` (edsbwt_write_csv)."""
    occ = np.ascontiguousarray(occ, dtype=OCC_DTYPE)
    n = int(lib().edsbwt_write_csv(occ.ctypes.data if occ.size else None, occ.size, fd, at, threads))
    if n < 0:
        raise OSError(ctypes.get_errno(), "edsbwt_write_csv failed")
    return n


def format_csv(occ: np.ndarray, threads: int = 8) -> bytes:
    """CSV body rows "%u\\t%u\\t%u\\t%u\\t%u\\n" (MOVE_EDSBWTSearch.cpp:365)."""
    occ = np.ascontiguousarray(occ, dtype=OCC_DTYPE)
    n = occ.size
    if n == 0:
        return b""
    L = lib()
    size = L.edsbwt_format_csv(occ.ctypes.data, n, None, 0, threads)
    out = ctypes.create_string_buffer(int(size))
    L.edsbwt_format_csv(occ.ctypes.data, n, out, size, threads)
    return out.raw[:size]


class MoveEDSBWT:
    """Mirror of ``MOVE_EDSBWT(inputFileName, filepatterns)`` (MOVE_EDSBWTSearch.cpp:23-176):
    the constructor does all the work.  Attributes ``count_found``, ``count_not_found``,
    ``counts`` (per pattern) and ``seconds`` (the ``bs took:`` region, :109,:145)."""

    def __init__(self, input_file_name: str, file_patterns: str, device: int = 0, *, table: bool = False):
        with Index(input_file_name, device) as idx:
            buf, offs = read_pattern_file(file_patterns)
            t0 = time.perf_counter()
            counts, occ = idx.search((buf, offs), first_pattern_id=1, locate=True, table=table)
            out_path = file_patterns + "output_M_LF.csv"
            try:
                with open(out_path, "wb") as f:
                    f.write(CSV_HEADER)
                    f.write(format_csv(occ))
            except OSError as e:  # :61-64
                raise EdsBwtError(-1, f"ERROR opening file {out_path} to write output") from e
            self.seconds = time.perf_counter() - t0
            self.counts = counts
            self.occ = occ
            self.count_found = int((counts > 0).sum())
            self.count_not_found = int(counts.size - self.count_found)
            self.stats = idx.stats()
