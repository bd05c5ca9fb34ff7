"""Synthetic workloads of SURVEY.md §8(d) (BASELINE.json `configs`), shared by bench.py
and the production-scale parity tests.

    C1  sample/test/test.eds + kmers.txt (tests/golden; plumbing, tests only)
    C2  10 Mchar EDS (seed 1, ~3 strings/segment), 1M random 20-mers per GPU (seed 2), count-only
    C3  ~100 Mchar COVID-like EDS (seed 3), 10M planted 31-mers per GPU (seed 4), full locate
    C4  the C3 index, 100M planted 31-mers in total (seed 5) sharded over the ranks, full locate
    C5  1 Gchar EDS with 20% empty-word segments (seed 6), mixed 8-64-mers (seed 7); BASELINE
        names no count-only mode for it and the reference always locates: bench.py's timed C5
        leg is count-only (the COUNT_ONLY flag, labelled in the line) and its `located` leg
        locates every pattern in pattern-range chunks whose records fit in HBM

Pattern i of a stream is drawn from its own seeded generator (edsbwt_gen --first), so a
rank generates exactly its contiguous shard of the stream: per-GPU configs (C2, C3, C5:
weak scaling) give rank r the stream ids [r*P, (r+1)*P); C4 (strong: a fixed 100M batch)
gives rank r its shard_range of the 100M.  #Pat of stream id i is i + 1
(MOVE_EDSBWTSearch.cpp:101,121: 1-based line number of the pattern file).
"""
from __future__ import annotations

import os
import subprocess
import time
from dataclasses import dataclass

ROOT = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(ROOT, "eds-bwt_amd", "_build")


@dataclass(frozen=True)
class Workload:
    name: str
    gen: str            # edsbwt_gen eds --config
    chars: int          # EDS size
    eds_seed: int
    patterns: int       # per GPU (per_gpu) or in total
    per_gpu: bool       # weak scaling (fixed patterns per GPU) vs a fixed total batch
    lens: str
    mode: str           # random | planted | mixed
    pat_seed: int
    locate: bool
    index_tag: str      # workloads sharing an index share its files
    text: str


CONFIGS = {
    "c2": Workload("c2", "c2", 10_000_000, 1, 1_000_000, True, "20", "random", 2, False, "c2",
                   "C2: 10 Mchar synthetic EDS (sigma=4, ~3 strings/segment), 1M random 20-mers per GPU, count-only"),
    "c3": Workload("c3", "c3", 100_000_000, 3, 10_000_000, True, "31", "planted", 4, True, "c3",
                   "C3: ~100 Mchar COVID-like synthetic EDS, 10M planted 31-mers per GPU, full position recovery"),
    "c4": Workload("c4", "c3", 100_000_000, 3, 100_000_000, False, "31", "planted", 5, True, "c3",
                   "C4: the C3 index replicated, 100M planted 31-mers in total sharded over the GPUs, full position recovery"),
    "c5": Workload("c5", "c5", 1_000_000_000, 6, 200_000, True, "8,16,32,64", "mixed", 7, False, "c5",
                   "C5: 1 Gchar synthetic EDS with 20% empty-string segments, mixed 8-64-mers per GPU; timed leg: the "
                   "located search (every occurrence's record, in record-budget chunks); the e2e leg is count-only"),
}


def shard_range(npat: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of a contiguous shard (same cut as eds-bwt_amd/shard.py)."""
    return npat * rank // world, npat * (rank + 1) // world


def run(args, **kw):
    subprocess.run([str(a) for a in args], check=True, **kw)


def ensure_built():
    need = [os.path.join(BUILD, f) for f in ("libedsbwt.so", "eds_transform", "edsbwt_gen", "EDSBWTsearch")]
    if not all(os.path.exists(p) for p in need):
        run(["make", "-s", "-j", "16", "-C", os.path.join(ROOT, "eds-bwt_amd"), "all"])


def default_workdir() -> str:
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), "edsbwt_bench")


def build_index(w: Workload, workdir: str, chars: int = 0, log=None) -> tuple[str, str]:
    """Generate the workload's EDS and write its index (eds_transform); cached in workdir.
    Returns (eds path, index base)."""
    chars = chars or w.chars
    tag = w.index_tag if chars == w.chars else f"{w.index_tag}_{chars}"
    os.makedirs(workdir, exist_ok=True)
    eds = os.path.join(workdir, f"{tag}.eds")
    base = os.path.join(workdir, tag)
    if not os.path.exists(base + "_info.aux"):
        t = time.time()
        run([os.path.join(BUILD, "edsbwt_gen"), "eds", "--config", w.gen, "--chars", chars, "--seed", w.eds_seed, "--out", eds])
        # big indexes: the suffix sort on the GPU (eds_transform --gpu; C5's 1.26G suffixes:
        # 0.4 s against 17 s on 16 host threads, same files)
        gpu = chars >= 200_000_000 and os.path.exists("/dev/kfd") and os.environ.get("EDSBWT_WRITER_GPU", "1") != "0"
        run([os.path.join(BUILD, "eds_transform"), eds, base, "--no-runs"] + (["--gpu", "0"] if gpu else []))
        if log:
            log(f"[workloads] index {base} built in {time.time() - t:.1f}s")
    return eds, base


def shard(w: Workload, rank: int, world: int, patterns: int = 0) -> tuple[int, int]:
    """Stream ids [lo, hi) of rank's patterns (patterns overrides the count: per GPU for
    per-GPU workloads, in total otherwise)."""
    n = patterns or w.patterns
    if w.per_gpu:
        return rank * n, (rank + 1) * n
    return shard_range(n, world, rank)


def pattern_file(w: Workload, eds: str, workdir: str, lo: int, hi: int, tag: str = "") -> str:
    """The pattern file of stream ids [lo, hi) (generated once, cached), with its planted mask
    (planted_mask(): one byte per pattern, 1 = spelled along a path of the EDS)."""
    path = os.path.join(workdir, f"{w.name}{tag}_pats_{w.pat_seed}_{lo}_{hi}.txt")
    if not os.path.exists(path) or not os.path.exists(path + ".planted"):
        tmp = path + f".tmp{os.getpid()}"
        run([os.path.join(BUILD, "edsbwt_gen"), "patterns", "--eds", eds, "--count", hi - lo, "--first", lo, "--lens", w.lens,
             "--mode", w.mode, "--seed", w.pat_seed, "--out", tmp, "--planted-mask", tmp + ".planted"])
        os.replace(tmp + ".planted", path + ".planted")
        os.replace(tmp, path)
    return path


def planted_mask(pattern_path: str):
    """bool per pattern of a pattern_file(): True when it was planted (it must occur)."""
    import numpy as np
    return np.fromfile(pattern_path + ".planted", dtype=np.uint8).astype(bool)
