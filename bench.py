#!/usr/bin/env python3
"""Benchmark: EDS-BWT backward search on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5]

A *step* is one pass of the hot path — MOVE_EDSBWTSearch's pattern loop with position
recovery (MOVE_EDSBWTSearch.cpp:97-155, 228-374) — over one batch of synthetic patterns:
the pattern file's bytes in (page-locked) host memory go through edsbwt_search_lines,
the library's pipelined host path (H2D of chunk k+1 overlaps the search of chunk k and the
D2H of chunk k-1), until every count and occurrence record is back in host memory: SURVEY.md
§8(d)'s PCIe-inclusive clock, reported as `e2e` (value, ms_per_step, per-call walls).  The same
batch with its bytes and offsets already in HBM and the counts and records left there
(edsbwt_search_device) is timed next: that leg is `value` / `ms_per_step` (the task's
contract: inputs resident in HBM when the timed region starts; the PCIe-inclusive rate is
never `value`) and `device_resident`, and the kernel roofline comes from it.

Default workload = C3 (BASELINE.json configs[2]): ~100 Mchar COVID-like synthetic EDS,
10M planted 31-mers per GPU, full locate.  C4 = the C3 index with 100M patterns in total,
sharded over the ranks.  N>1: one process per GPU (torchrun; `--gpus N` without torchrun
starts it), each rank searches its contiguous shard against a replicated index; the
exchange step — sizes all-gathered, per-pattern counts gathered to rank 0 over RCCL — is
inside both timed legs' steps.  rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import workloads  # noqa: E402

MI355X_HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak
MI355X_MALL_BYTES = 256 << 20  # Infinity Cache: index tables smaller than this are cache-resident
# bench.py kernel class (engine.hip KClass) -> the kernels it times
KERNELS_OF_CLASS = {"deep": "k_deep_direct (packed start, wide k-mer entries; else k_deep_fast)", "deep_list": "k_deep",
                    "deep_wide": "k_deep_wave",
                    "step": "k_lvl_items + k_lvl_dollar + k_lvl_chunks", "locate": "k_locate_pp + k_locate_big (+ k_locate)"}
# Practical ceilings of the deep kernels' access shape on MI355X (tools/calib_gather.hip,
# profiles/r02_calib_gather.json): one random 16-B rank entry per lane per step from a
# table of the C3 rank entries' size, issued as the kernel issues them.
CALIB = os.path.join(ROOT, "profiles", "r02_calib_chain.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def traffic_from_profile(cfg: str, kernel: str):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 PMC summary of
    this command (profiles/traffic_<cfg>.json, tools/profile_summary.py: separate --pmc
    FETCH_SIZE / WRITE_SIZE passes); None when there is none."""
    path = os.path.join(ROOT, "profiles", f"traffic_{cfg}.json")
    try:
        t = json.load(open(path))
        if t.get("classes_version") != "r3b":  # the current classes: deep = k_deep_direct / k_deep_fast
            return None, None
        c = t["classes"][kernel]
        # calibrated DRAM bytes (TCC_EA0_RDREQ_DRAM_32B x 32 + WRITE_SIZE; profiles/r03_calib_counters.json)
        # when the TCC pass was taken, else FETCH_SIZE + WRITE_SIZE
        f = t.get("traffic_field", "pmc_hbm_bytes_per_launch")
        return int(c[f]), f"profiles/traffic_{cfg}.json: {f} ({t.get('source', '')})"
    except (OSError, KeyError, ValueError):
        return None, None


def gather_ceiling():
    """Line-rate ceiling of the deep walk's own access shape: chain2 = each lane walks
    dependent steps of two random 16-B rank-entry loads (one per interval end), several
    patterns per lane in flight, from a 1 GB table (the C3 rent2 entries' size)."""
    try:
        rows = [json.loads(x) for x in open(CALIB) if x.strip()]
        best = max((r for r in rows if r["shape"].startswith("chain2") and r["table_MB"] >= 1024),
                   key=lambda r: r["lines_per_s"])
        return float(best["lines_per_s"]), f"{best['shape']} over {best['table_MB']} MB ({os.path.basename(CALIB)})"
    except (OSError, KeyError, ValueError):
        return None, None


def pin_to_gpu_numa(torch, dev: int):
    """Run this rank's host threads (and so place its page-locked buffers) on the NUMA node of its
    GPU's PCIe root, within the CPUs the process may use: the host pipeline's DMA then stays off
    the inter-socket link.  Returns the node, or None when the platform does not say."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read().strip())
        if node < 0:
            return None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        allowed = os.sched_getaffinity(0) & cpus
        if not allowed:
            return None
        os.sched_setaffinity(0, allowed)
        return node
    except (OSError, ValueError, AttributeError):
        return None


def cpu_baseline(base: str, buf, offs, first_id: int, sample: int, threads: int, trie: bool = False) -> dict:
    """The oracle (faithful C restatement of MOVE_EDSBWTSearch: a-balanced M_LF, literal
    per-pattern link/step/locate, MOVE_EDSBWTSearch.cpp:228-374) on the first `sample`
    patterns of this rank's batch, on `threads` host threads over contiguous shards; index
    load excluded, as the reference's `bs took:` region excludes it (:109,145).  trie=True: the
    trie-sharing variant (orc_search_batch_trie: common pattern suffixes searched once)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # checker / CPU baseline only

    import threading

    o = offs[: sample + 1]
    b = buf[: int(o[-1])]
    done = threading.Event()
    t_start = time.time()

    def beat():  # a long oracle run (C5's index) still shows progress
        while not done.wait(30):
            log(f"[bench] cpu baseline ({sample} patterns, {'trie' if trie else 'literal'}) running {time.time() - t_start:.0f}s")

    threading.Thread(target=beat, daemon=True).start()
    try:
        t = time.time()
        eng = orc.Engine(base, 8)
        t_open = time.time() - t
        t = time.time()
        counts, occ, ctr = eng.search(b, o, first_pattern_id=first_id, threads=threads, trie=trie)
        dt = time.time() - t
        eng.close()
    finally:
        done.set()
    return {"value": sample / dt, "seconds": dt, "open_s": t_open, "counts": counts, "occ": occ, "ctr": ctr}


# HIP-event times of the timed steps' kernel classes: the light set (deep, step, locate, link sort)
# by default; EDSBWT_BENCH_PROFILE=full times every class (diagnostics: more events in the step)
PROFILE_TIMED = True if os.environ.get("EDSBWT_BENCH_PROFILE") == "full" else "light"


def record_chunks(counts, budget: float) -> list:
    """Cut points [0, ..., n] of contiguous pattern ranges holding at most `budget` records each
    (greedy; a single pattern above the budget is a chunk of its own)."""
    c = np.asarray(counts, np.int64)
    cuts = [0]
    csum = np.concatenate(([0], np.cumsum(c)))
    n = c.size
    while cuts[-1] < n:
        a = cuts[-1]
        # the furthest b with csum[b] - csum[a] <= budget, at least a + 1
        b = int(np.searchsorted(csum, csum[a] + budget, side="right")) - 1
        cuts.append(min(n, max(a + 1, b)))
    return cuts


def suffix_order(buf, offs, k: int = 8) -> np.ndarray:
    """Pattern indices ordered by their last k characters read backwards (the first k levels of the
    reversed-pattern trie the search walks: MOVE_EDSBWTSearch.cpp:240-258 starts each pattern at its
    last character), stable: patterns sharing a trie node at depth <= k are contiguous in the order,
    so record-budget batches cut in it (located_chunks) share almost no trie nodes.  A pattern shorter
    than k sorts before its longer extensions (missing characters count as 0)."""
    b = np.asarray(buf, np.uint8)
    o = np.asarray(offs, np.int64)
    lens = np.diff(o)
    key = np.zeros(lens.size, np.uint64)
    for j in range(k):
        pos = o[1:] - 1 - j
        c = np.where(lens > j, b[np.clip(pos, 0, max(0, b.size - 1))] if b.size else 0, 0).astype(np.uint64)
        key |= c << np.uint64(8 * (k - 1 - j))
    return np.argsort(key, kind="stable")


# HBM per located record when sizing C5's batches (k_locate_lists needs no task arrays): 30 B — 6 batches,
# 1.189 s, against 8 at 40 B (1.229 s) and 12 at round 5's first 64 B (1.305 s); EDSBWT_LOCATED_BPR overrides
LOCATED_BYTES_PER_RECORD = float(os.environ.get("EDSBWT_LOCATED_BPR", "30"))


def located_chunks(buf, offs, counts, dev, budget: float, torch, first_id: int, order: str = "suffix") -> tuple:
    """C5's located search: the reference always recovers positions (MOVE_EDSBWTSearch.cpp:328-369),
    and C5's 8.7e9 occurrences (20-B records: ~174 GB) do not fit in HBM beside the index, so the
    batch is searched WITH locate in batches (chunks) whose records fit `budget` (at most what the
    free HBM holds at ~30 B of locate workspace per record: the 20-B record, its interval in the archive and
    the walk's share); each chunk's counts + records are left
    in HBM and the next chunk reuses the buffers.  The chunks are cut in suffix_order(), not in line
    order: contiguous line ranges share the shallow trie nodes (C5: ~62K depth-8 nodes whose lists
    hold ~1.5e5 intervals each), which every range would walk again (round 5: 12 line-range chunks
    walked 1.19 s of level steps against 0.61 s for the whole batch count-only).  Each chunk reports
    its patterns' file line numbers through an id map (edsbwt_search_device_ids).  Returns the chunks
    (pattern indices, device bytes, offsets, ids, counts), the budget and the host seconds the
    ordering and gathering took (setup, before the timed steps, like the uploads)."""
    t = time.perf_counter()
    c64 = counts.astype(np.int64)
    free_b, _ = torch.cuda.mem_get_info(dev)
    budget = min(budget, 0.6 * free_b / LOCATED_BYTES_PER_RECORD)
    order = suffix_order(buf, offs) if order == "suffix" else np.arange(c64.size)
    cuts = record_chunks(c64[order], budget)
    lens = np.diff(offs.astype(np.int64))
    chunks = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        sel = order[a:b]
        so = np.concatenate(([0], np.cumsum(lens[sel]))).astype(np.int64)
        # the chunk's pattern bytes in its order: one gather of every selected byte
        starts = offs[sel].astype(np.int64)
        src = (np.repeat(starts - so[:-1], lens[sel]) + np.arange(int(so[-1]), dtype=np.int64)) if so[-1] else np.zeros(0, np.int64)
        cb = np.asarray(buf)[src] if src.size else np.zeros(1, np.uint8)
        ids = (sel.astype(np.int64) + first_id).astype(np.uint32)
        chunks.append((sel, torch.from_numpy(np.ascontiguousarray(cb)).to(dev), torch.from_numpy(so).to(dev),
                       torch.from_numpy(ids.view(np.int32)).to(dev), torch.zeros(max(1, b - a), dtype=torch.int32, device=dev)))
    torch.cuda.synchronize()
    return chunks, budget, time.perf_counter() - t


def pat_column(p_occ: int, n: int, dev, torch):
    """The #Pat column of n device records (20-B edsbwt_occ at device address p_occ) as a device
    int32 tensor: one strided device-to-device copy (hipMemcpy2D), no host round trip."""
    import ctypes
    out = torch.empty(n, dtype=torch.int32, device=dev)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy2D.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                    ctypes.c_size_t, ctypes.c_int]
        rc = hip.hipMemcpy2D(out.data_ptr(), 4, p_occ, 20, 4, n, 3)  # 3: hipMemcpyDeviceToDevice
        if rc != 0:
            raise RuntimeError(f"hipMemcpy2D of the records' #Pat column failed ({rc})")
    return out


def survey_B_whole_step(dstat: dict, npat: int, pattern_bytes: int, locate: bool, d_ms: float) -> dict:
    """SURVEY §8(d)'s algorithmic bytes of one whole device-resident step, every term, from the
    device's own counters of the (untimed, counted) step:
        B = 64·(2·S_steps + 2·K_pdf + W_lf + 3·O) + 4·D_eof + Σ(|P|+1) + 4·N_pat + 20·O
    S_steps = intervals_stepped; K_pdf = D_eof = link_hash_rows (each '#' row an interval holds is one
    preceding_dollars_finder call, MOVE_EDSBWTSearch.cpp:570-625, and one EOF_ID entry read); W_lf =
    locate_lf_steps (0 with dense samples); O = occurrences when the step locates (count-only: 0 — no
    locate lines, no records written).  The device's counters are its own work, not the survey's
    deduplicated trie counts, and a text-compared pattern's characters are not interval steps (the
    single-row compare replaces them: text_rows / text_chars)."""
    S = int(dstat["intervals_stepped"])
    K = int(dstat["link_hash_rows"])
    W = int(dstat["locate_lf_steps"])
    O = int(dstat["occurrences"]) if locate else 0
    terms = {"lines_2S": 64 * 2 * S, "lines_2K_pdf": 64 * 2 * K, "lines_W_lf": 64 * W, "lines_3O": 64 * 3 * O,
             "eof_4D": 4 * K, "patterns_sum_len_plus_1": pattern_bytes + npat, "counts_4N": 4 * npat, "records_20O": 20 * O}
    B = sum(terms.values())
    return {"bytes_per_step": B, "terms": terms,
            "counters": {"S_steps": S, "K_pdf": K, "D_eof": K, "W_lf": W, "O": O, "N_pat": npat,
                         "text_rows": int(dstat.get("text_rows", 0)), "text_chars": int(dstat.get("text_chars", 0))},
            "device_ms_per_step": round(d_ms, 4),
            "achieved_gbs": round(B / (d_ms * 1e-3) / 1e9, 1) if d_ms > 0 else None,
            "frac": round(B / (d_ms * 1e-3) / 1e9 / MI355X_HBM_PEAK_GBS, 4) if d_ms > 0 else None,
            "what": "SURVEY §8(d) B over the whole device-resident step (every term), from the device counters of the "
                    "counted step; `roofline.frac` is the dominant kernel's line model, this is the whole step's"}


def d2h_records(p_occ: int, n: int, pkg) -> np.ndarray:
    """The first n 20-B records at device address p_occ, copied to host memory (hipMemcpy)."""
    import ctypes
    out = np.zeros(max(1, n), pkg.OCC_DTYPE)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        rc = hip.hipMemcpy(out.ctypes.data, p_occ, n * pkg.OCC_DTYPE.itemsize, 2)  # 2: hipMemcpyDeviceToHost
        if rc != 0:
            raise RuntimeError(f"hipMemcpy of the timed step's records failed ({rc})")
    return out[:n]


def located_pass(idx, chunks, counts, stream, torch, kacc=None, check=False) -> dict:
    """Every chunk searched with locate (device-resident: its bytes, offsets and ids in HBM, counts
    and records left there); kacc: the HIP-event kernel times summed in; check: each chunk's records
    == Σ its counts from the count-only search, its counts equal them and its records name its
    patterns' line numbers (pattern-major in the chunk's order; synchronises per chunk)."""
    per, recs, ok = [], 0, True
    for sel, db, do, di, dc in chunks:
        t = time.perf_counter()
        p_occ, n = idx.search_device(db.data_ptr(), do.data_ptr(), sel.size, dc.data_ptr(), ids=di.data_ptr(), locate=True,
                                     stream=stream, profile=PROFILE_TIMED if kacc is not None else False)
        if kacc is not None:
            idx.add_kernel_stats(kacc)
        recs += n
        if check:
            torch.cuda.synchronize()
            want_c = counts[sel]
            want = int(want_c.astype(np.int64).sum())
            cm = bool(np.array_equal(dc.cpu().numpy().view(np.uint32)[:sel.size], want_c))
            pm = True
            if n:
                # the records' #Pat column: pattern-major in the chunk's order, ids[i] count(i) times
                got = pat_column(p_occ, n, db.device, torch)
                want_p = torch.repeat_interleave(di, torch.from_numpy(want_c.astype(np.int64)).to(db.device))
                pm = bool(torch.equal(got, want_p))
                del got, want_p
            ok = ok and cm and pm and n == want
            per.append({"patterns": int(sel.size), "records": int(n), "records_expected": want, "counts_match": cm,
                        "pat_column_match": pm, "s": round(time.perf_counter() - t, 3)})
    return {"records": recs, "ok": ok, "per_chunk": per}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(workloads.CONFIGS))
    ap.add_argument("--patterns", type=int, default=0, help="patterns per GPU (C4: in total; default: the config's)")
    ap.add_argument("--chars", type=int, default=0, help="EDS size override (scaled-down diagnostic runs)")
    ap.add_argument("--locate", default="sampled", choices=("sampled", "walk", "table"),
                    help="position recovery: per-row samples (default), the reference's full walk to '#', or the per-row table")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-sample", type=int, default=0)
    ap.add_argument("--no-device", action="store_true", help="skip the device-resident leg")
    ap.add_argument("--timed-counters", action="store_true",
                    help="run the timed steps with the deep kernels' work counters (rounds 1-5); default: the timed "
                         "steps pass EDSBWT_NO_COUNTERS and one untimed counted step gives the line model")
    ap.add_argument("--no-e2e", action="store_true",
                    help="profiling runs: only the device-resident leg (its kernel averages then match a rocprofv3 "
                         "trace of the whole run); the line's value is then the device-resident rate")
    ap.add_argument("--no-located", action="store_true", help="C5: skip the located leg")
    ap.add_argument("--dist-self", action="store_true",
                    help="run the N>1 exchange path (process group, RCCL gather of the device counts) with one rank too "
                         "(launch with torchrun --nproc-per-node 1): exercises RCCL on a one-GPU box")
    ap.add_argument("--located-budget", type=float, default=2.0e9,
                    help="C5 located leg: most records per pattern-range chunk (20 B each, left in HBM)")
    ap.add_argument("--located-order", default="suffix", choices=("suffix", "lines"),
                    help="C5 located leg: batches cut in the patterns' suffix order (default) or in line order")
    ap.add_argument("--workdir", default=workloads.default_workdir())
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on GPU nodes; gloo to rehearse ranks on one GPU")
    ap.add_argument("--gather", default="auto", choices=("auto", "none", "counts"),
                    help="N>1 exchange: 'counts' (the default when N>1) gathers the per-pattern counts to rank 0 over "
                         "RCCL inside the timed step (every rank's (patterns, records) offsets follow from them); 'none': "
                         "no exchange, every rank keeps its counts and records")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    # --dist-self: the exchange path (process group, all-gather of sizes, counts gathered over RCCL
    # from the device mirror) even with one rank — it exercises RCCL on a one-GPU box
    multi = world > 1 or args.dist_self
    if args.gather == "auto":
        args.gather = "counts" if multi else "none"
    # the CPUs this process may use, before the NUMA pinning below; the CPU baseline uses them,
    # capped by the job's CPU share when the launcher states one (OMP_NUM_THREADS: 16 per GPU
    # on the GPU box, whose os.cpu_count() shows the whole machine)
    cpus_usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cpu_share = int(os.environ.get("OMP_NUM_THREADS") or cpus_usable)
    cpu_threads = max(1, min(cpus_usable, cpu_share))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start torchrun as a child (nothing has touched the GPU yet)
        port = free_port()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    # the JSON line is the only thing on stdout: libraries that print there (RCCL's version banner
    # at communicator init) write to stderr instead
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev  # rehearsal: several ranks may share one GPU (gloo)
    gdev = torch.device("cpu")
    if multi:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        for k_, v_ in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(free_port())), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k_, v_)  # --dist-self run bare: a one-rank group
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            gdev = torch.device("cuda", local)
        else:
            dist.init_process_group(args.dist_backend)
        barrier = lambda: dist.barrier()  # noqa: E731
    else:
        torch.cuda.set_device(0)
        barrier = lambda: None  # noqa: E731
    numa = pin_to_gpu_numa(torch, local) if torch.cuda.is_available() else None
    if rank == 0:
        workloads.ensure_built()
    barrier()
    pkg = importlib.import_module("eds-bwt_amd")
    shard = importlib.import_module("eds-bwt_amd.shard")
    w = workloads.CONFIGS[args.config]
    locate = w.locate

    # ---- inputs (outside the timed region): index, this rank's shard of the pattern stream
    t = time.time()
    if rank == 0:
        eds, base = workloads.build_index(w, args.workdir, args.chars, log)
    barrier()
    eds, base = workloads.build_index(w, args.workdir, args.chars)
    lo, hi = workloads.shard(w, rank, world, args.patterns)
    pats_path = workloads.pattern_file(w, eds, args.workdir, lo, hi, tag=f"_{args.chars}" if args.chars else "")
    barrier()
    t_prep = time.time() - t
    npat = hi - lo
    first_id = lo + 1
    t = time.time()
    if world > 1 and ndev < world:
        # ranks sharing a GPU (gloo rehearsal) open the index one at a time, each sizing its optional
        # tables (k-mer table budget, wide entries, per-row text entries, level table) for its share
        # of the device (EDSBWT_HBM_SHARE; the production config otherwise: no depth overrides)
        share = 0.9 * ndev / world
        os.environ.setdefault("EDSBWT_HBM_SHARE", f"{share:.4f}")
        idx = None
        for r in range(world):
            if r == rank:
                idx = pkg.Index(base, device=local)
            barrier()
    else:
        idx = pkg.Index(base, device=local)
    t_open = time.time() - t
    if args.locate == "table" and locate:
        idx.search([b"A"], table=True)  # builds the table outside the timed region
    text = pkg.read_pattern_file_pinned(pats_path)
    counts_hb = pkg.HostBuffer(4 * (npat + 1))
    counts = counts_hb.array(np.uint32, npat + 1)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    flags_kw = dict(table=args.locate == "table", walk=args.locate == "walk")
    rccl = multi and args.dist_backend == "nccl"

    # ---- the exchange step (N > 1), set up once per batch shape: the per-pattern counts gathered to
    # rank 0.  Every rank's shard size follows from the static split and its records are the sum of
    # its counts, so rank 0 has every rank's (patterns, records) offsets from the gather itself: one
    # collective per step, no size read back to the host, nothing allocated per step.  On GPUs the
    # gather is the library's own (edsbwt_gather_counts, ABI 7: an RCCL communicator per index, the
    # gather queued on the library's exchange stream with no Python or host wait on the search's
    # path); the searches alternate two count buffers and the library orders a search that writes a
    # buffer after the gather still reading it, so the gather of step i overlaps step i + 1.  gloo
    # (rehearsal): counts staged through host memory (shard.CountsGather), synchronous
    shard_sizes = [b_ - a_ for a_, b_ in (workloads.shard(w, r, world, args.patterns) for r in range(world))]
    assert shard_sizes[rank] == npat
    # (EDSBWT_BENCH_TORCH_EXCHANGE=1: torch.distributed's gather instead — the fallback, tested)
    native = rccl and args.gather == "counts" and os.environ.get("EDSBWT_BENCH_TORCH_EXCHANGE") != "1"
    native_err = None if native or not rccl else "EDSBWT_BENCH_TORCH_EXCHANGE=1"
    sizes_np = np.array(shard_sizes, np.uint64)
    d_gather_out = None
    if native:
        # every rank tries; if any rank's communicator fails (no librccl, an init error) all fall back to
        # torch.distributed's gather (shard.CountsGather over the same RCCL process group) together
        try:
            uid = [idx.comm_unique_id() if rank == 0 else None]
        except Exception as e:  # noqa: BLE001
            uid, native_err = [None], repr(e)
        dist.broadcast_object_list(uid, src=0)
        ok = torch.tensor([0 if (uid[0] is None or native_err) else 1], dtype=torch.int32, device=gdev)
        if ok.item():
            try:
                idx.comm_init(uid[0], world, rank)
            except Exception as e:  # noqa: BLE001
                native_err = repr(e)
                ok.fill_(0)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not ok.item():
            log(f"[bench] rank {rank}: the library's RCCL exchange is unavailable ({native_err}); torch.distributed gather instead")
            native = False
        else:
            d_gather_out = torch.zeros(max(1, sum(shard_sizes)), dtype=torch.int32, device=dev) if rank == 0 else None
    cg = shard.CountsGather(shard_sizes, gdev) if multi and args.gather == "counts" and not native else None
    # e2e leg: the engine leaves each call's u32 counts in a device mirror too (a device-to-device copy
    # per chunk): the gather reads them from HBM, no second upload; two mirrors, alternated per call
    d_counts_x = [torch.zeros(max(1, npat), dtype=torch.int32, device=dev) for _ in range(2 if native else 0)]
    n_e2e = [0]
    # the last exchanged step's record count per leg (checked against rank 0's view after the timing)
    last_nocc = {}

    def e2e_step(keep=False):
        if d_counts_x:
            idx.set_counts_mirror(d_counts_x[n_e2e[0] % 2].data_ptr(), npat)
        n, ptr, nocc = idx.search_lines(text.ptr, text.nbytes, counts_hb.ptr, npat + 1, first_pattern_id=first_id,
                                        locate=locate, keep=keep)
        assert n == npat, (n, npat)
        return ptr, nocc

    def exchange(nocc, d_src=None, leg="e2e"):
        # the path's exchange step: the per-pattern counts to rank 0, where they also
        # give every rank's (patterns, records) — its offsets in the output.  d_src: the device leg's
        # counts (else the e2e leg's mirror / host counts)
        if not multi or args.gather != "counts":
            return
        last_nocc[leg] = nocc
        if native:
            if d_src is None:
                d_src = d_counts_x[n_e2e[0] % 2]
                n_e2e[0] += 1
            idx.gather_counts(d_src.data_ptr(), npat, d_gather_out.data_ptr() if d_gather_out is not None else 0, sizes_np, 0)
        elif rccl:  # (fallback) torch.distributed's gather over RCCL, from device tensors, synchronous
            cg.start(d_src if d_src is not None else torch.from_numpy(counts[:npat].view(np.int32)).to(dev))
            cg.wait()
        else:
            cg.start(d_src.cpu() if d_src is not None else torch.from_numpy(counts[:npat].view(np.int32)))

    def exchange_drain():
        if native:
            idx.comm_sync()
        elif cg is not None:
            cg.wait()

    def exchange_check(leg):
        """Outside the timed region: rank 0's per-rank records from the gathered counts == every
        rank's own record count of its last exchanged step."""
        if not multi or args.gather != "counts" or leg not in last_nocc:
            return None
        mine = torch.tensor([last_nocc[leg]], dtype=torch.int64, device=gdev)
        allr = torch.empty(world, dtype=torch.int64, device=gdev)
        dist.all_gather_into_tensor(allr, mine)
        got = d_gather_out if native else cg.result()
        if rank != 0:
            return None
        sums = [int(t_.cpu().numpy().view(np.uint32).astype(np.int64).sum()) for t_ in torch.split(got[:sum(shard_sizes)], shard_sizes)]
        return {"records_per_rank_from_counts": sums, "records_per_rank_reported": [int(x) for x in allr.tolist()],
                "match": sums == [int(x) for x in allr.tolist()]}

    # ---- timed: end-to-end (host memory -> host memory)
    for _ in range(0 if args.no_e2e else args.warmup):
        _, nocc = e2e_step()
        exchange(nocc)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c0 = time.process_time()
    search_ms = exch_ms = 0.0
    held = (0, 0)
    total_occ = 0
    walls = []
    redo_calls = 0
    for i in range(0 if args.no_e2e else args.steps):
        ta = time.perf_counter()
        last = i == args.steps - 1
        ptr, nocc = e2e_step(keep=last)
        if last:
            held = (ptr, nocc)
        tb = time.perf_counter()
        exchange(nocc)
        search_ms += 1e3 * (tb - ta)
        exch_ms += 1e3 * (time.perf_counter() - tb)
        st_call = idx.stats_struct()  # one preallocated struct: no per-step dict building in the timed loop
        walls.append(st_call.ms_wall)
        redo_calls += st_call.redo_searches
        total_occ += nocc
    exchange_drain()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    xchk = {"e2e": exchange_check("e2e")}
    if d_counts_x:
        idx.set_counts_mirror(0, 0)
    host_cores = (time.process_time() - c0) / max(1e-9, elapsed)  # host CPU the pipeline kept busy
    e2e_stats = idx.stats()
    if args.no_e2e:
        e2e_stats = dict(e2e_stats, ms_wall=0.0, found=0)
        walls = [0.0]
    per_rank = [search_ms / args.steps, exch_ms / args.steps]
    if multi:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        pr = torch.tensor(per_rank, dtype=torch.float64, device=gdev)
        allpr = [torch.zeros_like(pr) for _ in range(world)]
        dist.all_gather(allpr, pr)
        per_rank_all = [[round(float(x), 3) for x in t_.tolist()] for t_ in allpr]
        agg = torch.tensor([total_occ], dtype=torch.float64, device=gdev)
        dist.all_reduce(agg)
        total_occ = float(agg.item())
    else:
        per_rank_all = [[round(x, 3) for x in per_rank]]

    # records of the last step (kept) for the parity sample
    occ_last = idx.occ_view(*held).copy() if held[1] else np.zeros(0, pkg.OCC_DTYPE)
    counts_last = counts[:npat].copy()
    idx.occ_free(held[0])

    # ---- timed: device-resident (bytes + offsets in HBM, results left in HBM); C5: the located search
    dres = None
    located_timed = w.name == "c5" and not args.no_located
    if not args.no_device:
        buf, offs = pkg.read_pattern_file(pats_path)
        d_bytes = torch.from_numpy(buf).to(dev)
        d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
        # two count buffers when the counts are gathered natively: step i's gather reads one while
        # step i + 1 searches into the other; else one
        d_counts_b = [torch.zeros(max(1, npat), dtype=torch.int32, device=dev) for _ in range(2 if native else 1)]
        d_counts = d_counts_b[0]
        n_dev = [0]

        # the timed steps run the deep kernels' builds without their work counters (EDSBWT_NO_COUNTERS:
        # same results, fewer registers); the line model (bytes / lines per launch, intervals stepped)
        # comes from one counted step, untimed, before the warm-up
        counted = args.timed_counters or located_timed

        def dev_step(profile=False, counters=counted):
            # returns (records pointer, records, the counts buffer this step wrote)
            dc = d_counts_b[n_dev[0] % len(d_counts_b)]
            n_dev[0] += 1
            p_, n_ = idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), npat, dc.data_ptr(), first_pattern_id=first_id,
                                       locate=locate, profile=profile, stream=stream, counters=counters, **flags_kw)
            return p_, n_, dc

        kacc_c = stats_c = None
        if not counted:
            kacc_c = idx.kernel_acc()
            _, dn, dc = dev_step(profile=PROFILE_TIMED, counters=True)
            exchange(dn, dc, "device")
            idx.add_kernel_stats(kacc_c)
            stats_c = idx.stats()
        for _ in range(max(1, args.warmup)):
            _, dn, dc = dev_step()
            exchange(dn, dc, "device")
        exchange_drain()
        d_counts = dc
        located = None
        count_only = None
        if located_timed:
            # the count-only device-resident step (C5's timed step through round 4), timed on its own so
            # the C5 series stays comparable across rounds: same batch, counts left in HBM
            torch.cuda.synchronize()
            tc = time.perf_counter()
            for _ in range(args.steps):
                dev_step(counters=False)
            torch.cuda.synchronize()
            dt_c = (time.perf_counter() - tc) / args.steps
            count_only = {"value": round(npat / dt_c, 1), "ms_per_step": round(1e3 * dt_c, 3), "steps": args.steps,
                          "what": "the count-only device-resident search of the same batch (C5's timed step through "
                                  "round 4), timed separately; `value` is the located step since round 5"}
        if located_timed:
            # C5: the timed step is the located search (the reference always locates), in record-budget
            # chunks; the count-only warm-up above gave the counts the chunks are cut by
            counts_c = d_counts.cpu().numpy().view(np.uint32)[:npat].copy()
            exchange_drain()
            for b_ in d_counts_b:  # (each located step gathers the batch's counts, in line order)
                if b_.data_ptr() != d_counts.data_ptr():
                    b_.copy_(d_counts)
            chunks, budget, setup_s = located_chunks(buf, offs, counts_c, dev, args.located_budget, torch, first_id,
                                                      order=args.located_order)
            chk = located_pass(idx, chunks, counts_c, stream, torch, check=True)  # warm-up pass, checked
            lens = np.diff(offs.astype(np.int64))
            c64 = counts_c.astype(np.int64)
            located = {"chunks": len(chunks), "records_budget_per_chunk": int(budget), "records_per_step": int(chk["records"]),
                       "records_equal_counts": chk["ok"], "per_chunk_check": chk["per_chunk"],
                       "lengths": {str(L): {"patterns": int((lens == L).sum()), "records": int(c64[lens == L].sum())}
                                   for L in np.unique(lens)},
                       "order": args.located_order, "setup_s": round(setup_s, 3),
                       "what": "the timed step: every pattern searched WITH locate (counts + 20-B records left in HBM, "
                               "device-resident) in batches whose records fit the budget, cut in the patterns' suffix order "
                               "(--located-order suffix; 'lines': contiguous line ranges) with each record's #Pat the pattern's "
                               "line number (id map); checked once (records == the count-only counts, and the #Pat column, "
                               "per chunk) before the timed steps; setup_s: the host ordering + gathers + uploads, untimed"}
        barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        kacc = idx.kernel_acc()
        p_last = n_last = 0
        for _ in range(args.steps):
            if located_timed:
                lp = located_pass(idx, chunks, counts_c, stream, torch, kacc=kacc)
                exchange(lp["records"], d_counts_b[n_dev[0] % len(d_counts_b)], "device")  # (the batch's counts, line order)
                n_dev[0] += 1
            else:
                p_last, n_last, d_counts = dev_step(profile=PROFILE_TIMED)
                exchange(n_last, d_counts, "device")
                idx.add_kernel_stats(kacc)  # HIP-event times of this call's kernel classes, summed in place
        exchange_drain()
        torch.cuda.synchronize()
        barrier()
        d_elapsed = time.perf_counter() - t1
        xchk["device_resident"] = exchange_check("device")
        # the last TIMED step's results (its build: counter-free unless --timed-counters), kept for the
        # oracle sample below (the records the headline times are the ones compared)
        timed_counts = d_counts.cpu().numpy().view(np.uint32)[:npat].copy()
        timed_head = None
        if locate and not located_timed and n_last:
            k_head = int(timed_counts[: min(npat, 4096)].astype(np.int64).sum())
            timed_head = d2h_records(p_last, min(k_head, n_last), pkg)
        if located is not None:
            located["seconds_per_step"] = round(d_elapsed / args.steps, 4)
            located["records_per_sec"] = round(located["records_per_step"] * args.steps / d_elapsed, 1)
        if multi:
            tt = torch.tensor([d_elapsed], dtype=torch.float64, device=gdev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            d_elapsed = float(tt.item())
        dstats = idx.stats()
        if kacc_c is not None:
            # the timed steps' HIP-event times and launches; bytes and lines per step from the counted
            # step (a step's work is the same every step); its statistics for the interval steps
            kacc[2:4] = kacc_c[2:4] * args.steps
            dstats = stats_c
        kstats = idx.kernel_acc_dict(kacc)
        dres = {"elapsed": d_elapsed, "kstats": kstats, "stats": dstats, "timed_counts": timed_counts, "timed_head": timed_head,
                "pattern_bytes": int(offs[-1]),
                "counters": "timed" if counted else "one untimed counted step (timed steps: EDSBWT_NO_COUNTERS)"}
        if not located_timed and not args.no_e2e and not np.array_equal(timed_counts, counts_last[:npat]):
            raise SystemExit("bench.py: device-resident counts differ from the end-to-end counts")
        if located is not None:
            if not located["records_equal_counts"]:
                raise SystemExit("bench.py: located chunks' records differ from the count-only counts")
            dres["located"] = located
            dres["count_only"] = count_only

    # ---- N > 1: every rank's first patterns against the oracle, outside the timed region: the e2e
    # leg's results and the last timed device-resident step's (the counter-free build the line times)
    rank_parity = None
    if multi and not args.no_cpu:
        n_par = min(16 if w.name == "c5" else 256, npat)
        pbuf, poffs = pkg.read_pattern_file(pats_path)
        ok = ok_t = 0
        try:
            pr_ = cpu_baseline(base, pbuf, poffs, first_id, n_par, cpu_threads)
            kk = int(pr_["counts"].astype(np.int64).sum())
            ok = int(np.array_equal(pr_["counts"], counts_last[:n_par]) and (not locate or np.array_equal(pr_["occ"], occ_last[:kk])))
            ok_t = ok
            if dres is not None and not located_timed:
                th = dres["timed_head"]
                ok_t = int(np.array_equal(pr_["counts"], dres["timed_counts"][:n_par])
                           and (not locate or (th is not None and np.array_equal(pr_["occ"], th[:kk]))))
        except Exception as e:  # noqa: BLE001 - reported as a mismatch
            log(f"[bench] rank {rank} parity sample failed: {e!r}")
        tt = torch.tensor([min(ok, ok_t), n_par], dtype=torch.float64, device=gdev)
        mn = tt.clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        sm = tt.clone()
        dist.all_reduce(sm)
        rank_parity = {"n_per_rank": n_par, "ranks": world, "n": int(sm[1].item()), "match": bool(mn[0].item() == 1),
                       "compared": "counts and records" if locate else "counts (count-only workload)",
                       "legs": ["e2e", "device_resident timed step"] if dres is not None and not located_timed else ["e2e"],
                       "what": "each rank's first n_per_rank patterns (its first_pattern_id offset) against the oracle "
                               "(literal MOVE_EDSBWTSearch restatement), all-reduced (min), for the e2e leg's results and "
                               "the last timed device-resident step's"}

    if rank == 0:
        total_pats = npat * world if w.per_gpu else (args.patterns or w.patterns)  # every rank's shard
        e2e_value = None if args.no_e2e else total_pats * args.steps / elapsed
        e2e_ms = None if args.no_e2e else 1000.0 * elapsed / args.steps
        # value: the device-resident leg (inputs in HBM); --no-device runs (host-pipeline studies)
        # fall back to the end-to-end rate, labelled in timed_region
        v_elapsed = dres["elapsed"] if dres else elapsed
        value = total_pats * args.steps / v_elapsed
        ms_step = 1000.0 * v_elapsed / args.steps
        rows = idx.n_rows
        # tables the deep kernels gather from: occ blocks (1 B/row), rent1 (sigma/2 B/row), rent2 (10 B/row)
        rank_bytes = rows * (1 + idx.sigma / 2 + (10 if idx.pair_blocks else 0))
        out = {
            "metric": "patterns/sec + LF-steps/sec, 100 Mchar EDS, 10M 31-mers, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "patterns/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "value_kind": ("device_resident: pattern bytes + offsets in HBM -> counts + records left in HBM (since round 3; "
                           "rounds 1-2 reported the PCIe-inclusive rate, now e2e.value)"
                           + ("; C5: the located search in record-budget chunks (round 5)" if located_timed else "") if dres else
                           "end_to_end (--no-device): host memory -> host memory"),
            "higher_is_better": True,
            "scaling": "weak" if w.per_gpu else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (edsbwt_gen, seeded; SURVEY.md §8(d) generators)",
            "config": {"workload": w.text, "config": w.name, "patterns_per_gpu": npat,
                       "patterns_total": total_pats,
                       "index_rows": rows, "words": idx.n_words, "segments": idx.n_segments,
                       "locate": ({"sampled": "per-row samples (word, offset, segment, word-in-segment), one read per occurrence",
                                   "walk": "lf-walk to '#' (reference)", "table": "per-row table"}[args.locate]
                                  if locate else ("per-row samples, the located search in record-budget chunks is the timed "
                                                  "step (`located`); the e2e leg is count-only" if located_timed else "count-only")),
                       "parallelism": f"pattern-shard x{world}",
                       "timed_region": ("edsbwt_search_device: pattern bytes + offsets resident in HBM -> counts + records "
                                        "in HBM, plus the exchange step when N>1; the PCIe-inclusive rate is `e2e`"
                                        if dres else
                                        "(--no-device) edsbwt_search_lines: page-locked pattern-file bytes H2D -> search -> "
                                        "counts + records D2H (SURVEY §8(d)), plus the exchange step when N>1"),
                       "exchange": ("none (one GPU)" if not multi else
                                    "none (--gather none: every rank keeps its counts + records)" if args.gather != "counts" else
                                    ("per-pattern counts gathered to rank 0 over RCCL by torch.distributed (the library's "
                                     f"exchange was unavailable: {native_err})" if rccl and not native else
                                     "per-pattern counts gathered to rank 0 over RCCL (xGMI) by the library itself "
                                     "(edsbwt_gather_counts: its own communicator and exchange stream), two alternating "
                                     "count buffers (the gather of step i beside the search of step i + 1); every rank's "
                                     "(patterns, records) offsets follow from the gathered counts"
                                     if args.dist_backend == "nccl" else
                                     f"per-pattern counts gathered to rank 0 over {args.dist_backend} (rehearsal: counts "
                                     "staged through host memory, synchronous)")),
                       "dist_backend": args.dist_backend if multi else None,
                       "ktab_depth": idx.ktab_depth, "ltab_depth": idx.ltab_depth, "ltab_items": idx.ltab_items,
                       "index_device_bytes": idx.device_bytes,
                       "index_open_peak_bytes": getattr(idx, "open_peak_bytes", None),
                       "host_numa_node": numa,
                       # every table the search reads (rank tables, k-mer table, samples) within the 256 MB MALL
                       "cache_resident": bool(idx.device_bytes <= MI355X_MALL_BYTES), "rank_tables_bytes": int(rank_bytes)},
            "occurrences_per_step": int(total_occ / args.steps),
            "found_per_step": int((dres["stats"] if dres else e2e_stats)["found"]) if world == 1 else None,
            "e2e": {"value": round(e2e_value, 1) if e2e_value else None, "ms_per_step": round(e2e_ms, 3) if e2e_ms else None,
                    "what": "SURVEY §8(d)'s clock: page-locked pattern-file bytes H2D -> search -> every count and 20-B "
                            "record D2H (edsbwt_search_lines), plus the exchange step when N>1",
                    "ms_wall_per_call": round(float(np.mean(walls)), 3), "ms_wall_median": round(float(np.median(walls)), 3),
                    "ms_wall_min": round(float(np.min(walls)), 3), "ms_wall_p90": round(float(np.percentile(walls, 90)), 3),
                    "ms_wall_max": round(float(np.max(walls)), 3), "ms_walls": [round(float(x), 3) for x in walls],
                    "redo_searches": redo_calls, "host_cores": round(host_cores, 2), "chunks": e2e_stats["chunks"],
                    "bytes_h2d": e2e_stats["bytes_h2d"], "bytes_d2h": e2e_stats["bytes_d2h"],
                    "pcie_gbs": round((e2e_stats["bytes_h2d"] + e2e_stats["bytes_d2h"]) / max(1e-9, np.mean(walls) * 1e-3) / 1e9, 2),
                    "device_ms_per_call": round(e2e_stats["ms_total"], 3),
                    "per_rank_search_exchange_ms": per_rank_all},
            "bs_took": round(elapsed / args.steps, 6) if not args.no_e2e else None,
            "index_open_s": round(t_open, 2),
            "inputs_prepare_s": round(t_prep, 1),
        }
        if dres:
            kstats = dres["kstats"]
            dstat = dres["stats"]
            d_ms = 1000.0 * dres["elapsed"] / args.steps
            ceil, ceil_shape = gather_ceiling()

            def kclass(name):
                d = kstats.get(name)
                if not d or not d["launches"] or d["ms"] <= 0:
                    return None
                avg_ms = d["ms"] / d["launches"]
                bpl = d["bytes"] / d["launches"]
                lpl = d["lines"] / d["launches"]
                ach = bpl / (avg_ms * 1e-3) / 1e9
                rate = lpl / (avg_ms * 1e-3)
                traffic, tsrc = traffic_from_profile(w.name, name)
                return {"kernels": KERNELS_OF_CLASS.get(name, name), "ms_per_step": round(d["ms"] / args.steps, 4),
                        "traffic_frac": round(traffic / (avg_ms * 1e-3) / 1e9 / MI355X_HBM_PEAK_GBS, 4) if traffic else None,
                        "launches_per_step": round(d["launches"] / args.steps, 2), "avg_launch_ms": round(avg_ms, 4),
                        "bytes_per_launch": int(bpl), "lines_per_launch": int(lpl),
                        "achieved": round(ach, 1), "frac": round(ach / MI355X_HBM_PEAK_GBS, 4) if bpl else None,
                        # (the random-line ceiling bounds the gathering classes; locate's lines are mostly its
                        # streamed records, bounded by HBM bandwidth: `frac`)
                        "lines_per_s": round(rate, 1),
                        "frac_of_gather_ceiling": round(rate / ceil, 4) if (ceil and lpl and name != "locate") else None,
                        "traffic": traffic, "traffic_source": tsrc}

            per_class = {k: v for k in ("deep", "deep_list", "deep_wide", "step", "locate") if (v := kclass(k))}
            # the dominant timed class (under a PMC pass the event times may be missing: then the
            # first class that has them)
            timed_k = [k for k in kstats if k != "scan" and kclass(k)]
            dom = max(timed_k, key=lambda k: kstats[k]["ms"]) if timed_k else None
            dk = (per_class.get(dom) or kclass(dom)) if dom else None
            if dk is None:
                dk = {"kernels": None, "achieved": None, "frac": None, "traffic": None, "traffic_source": None, "traffic_frac": None,
                      "avg_launch_ms": None, "bytes_per_launch": None, "lines_per_launch": None, "lines_per_s": None,
                      "frac_of_gather_ceiling": None}
                dom = dom or "none"
                kstats.setdefault(dom, {"ms": 0.0, "launches": 0, "bytes": 0, "lines": 0})
            # SURVEY §8(d)'s per-step model: two 64-B lines per interval step, whichever kernel
            # takes it (level step, dollar step, deep walk), over the whole device-resident step
            survey_b = 2 * 64 * dstat["intervals_stepped"]
            out["roofline"] = {
                "bound": "hbm", "kernel": dom, "kernels": dk["kernels"], "achieved": dk["achieved"], "peak": MI355X_HBM_PEAK_GBS,
                "unit": "GB/s", "frac": dk["frac"], "traffic": dk["traffic"], "traffic_source": dk["traffic_source"],
                "traffic_frac": dk["traffic_frac"],
                "traffic_note": ("DRAM bytes per launch from the PMC (calibrated: a random 16-B load moves one 128-B line, "
                                 "profiles/r03_calib_counters.json), over this line's event-timed launch; the line model counts "
                                 "64 B per line, so traffic ~ 2x bytes_per_launch is the DRAM line size, not re-reads"),
                "avg_launch_ms": dk["avg_launch_ms"], "launches": kstats[dom]["launches"],
                "bytes_model": "line model: the 64-B lines the kernel gathers as it counts them (a narrow interval's two ends in "
                               "one line count once; one 16-B two-step rank entry per end; the single-row text compare's sample, "
                               "text-position and text lines) + 24 B of per-pattern streams (DESIGN.md §6)",
                "bytes_per_launch": dk["bytes_per_launch"], "lines_per_launch": dk["lines_per_launch"], "lines_per_s": dk["lines_per_s"],
                "gather_ceiling_lines_per_s": ceil, "gather_ceiling_shape": ceil_shape,
                "frac_of_gather_ceiling": dk["frac_of_gather_ceiling"],
                "per_kernel": per_class,
                "survey_model_whole_step": {"interval_steps_per_step": int(dstat["intervals_stepped"]),
                                            "bytes_per_step": int(survey_b), "device_ms_per_step": round(d_ms, 4),
                                            "frac": round(survey_b / (d_ms * 1e-3) / 1e9 / MI355X_HBM_PEAK_GBS, 4) if d_ms > 0 else None,
                                            "what": "SURVEY §8(d): 2 x 64 B per interval step (every kernel that steps "
                                                    "intervals) over the whole device-resident step; omits the text "
                                                    "compares, table entries, link sorts and stores"},
                "survey_B_whole_step": survey_B_whole_step(dstat, npat, dres["pattern_bytes"], locate, d_ms),
                "from": "device_resident leg (HIP events on the library stream, EDSBWT_PROFILE_LIGHT)",
                "counters": dres["counters"],
            }
            out["device_resident"] = {
                "value": round(total_pats * args.steps / dres["elapsed"], 1), "ms_per_step": round(d_ms, 3),
                "what": "pattern bytes + u64 offsets resident in HBM before the timed region; counts + records left in HBM"
                        + ("; the exchange step (counts gathered to rank 0) in every step" if multi else ""),
                "kernel_ms_per_step": {k: round(v["ms"] / args.steps, 3) for k, v in sorted(kstats.items()) if v["ms"]},
                "kernel_lines_per_s": {k: round((v["lines"] / (v["ms"] * 1e-3)) if v["ms"] > 0 else 0.0, 1)
                                       for k, v in sorted(kstats.items()) if v["lines"]},
                "engine": {k: dstat[k] for k in ("depths", "deep_from_depth", "deep_overflow", "deep_level_rerun", "search_groups",
                                                 "trie_nodes", "intervals_stepped", "link_hash_rows", "start_depth",
                                                 "locate_lf_steps", "redo_searches", "text_rows", "text_chars")},
                # LF steps the device executed: 2 per interval step (one per end) + locate walk moves
                "device_lf_steps_per_sec": round((2 * dstat["intervals_stepped"] + dstat["locate_lf_steps"]) * args.steps
                                                 / dres["elapsed"], 1),
                "reference_locate_lf_steps_per_sec": round(dstat["locate_offsets"] * args.steps / dres["elapsed"], 1),
            }
            if "located" in dres:
                out["located"] = dres["located"]
                out["device_resident_count_only"] = dres.get("count_only")
            # the LF steps the device executed (measured: 2 rank queries per interval step + locate moves)
            out["lf_steps_per_sec"] = out["device_resident"]["device_lf_steps_per_sec"]
            out["lf_steps_note"] = ("lf_steps_per_sec: LF steps the device executed (2 per interval step + locate walk moves), "
                                    "measured over the device-resident leg; reference_equivalent_lf_steps.modelled_per_sec: "
                                    "oracle-counted reference M_LF moves per pattern x value (SURVEY §8(d)), a model, not executed")
        if rank_parity is not None:
            out["parity_sample"] = rank_parity
        if multi and cg is not None:
            out["exchange_check"] = dict(xchk, what="rank 0: every rank's records of its last exchanged step from the "
                                                    "gathered counts (sum per rank) == the record count each rank reported")
        if world == 1 and not args.no_cpu:
            buf, offs = pkg.read_pattern_file(pats_path)
            threads = cpu_threads
            try:
                # a fixed prefix of the batch on every usable CPU, and the reference's
                # single thread; C5's literal loop runs ~1.9 patterns/s on 16 threads, so its
                # samples are scaled to ~30 s
                samp_n = min(args.cpu_sample or (48 if w.name == "c5" else 4096), npat)
                samp1 = min(4 if w.name == "c5" else 128, npat)
                cb = cpu_baseline(base, buf, offs, first_id, samp_n, threads)
                c1 = cpu_baseline(base, buf, offs, first_id, samp1, 1)
                # parity of the sample: the oracle's counts and records vs the GPU's (end-to-end run)
                k = int(cb["counts"].astype(np.int64).sum())
                # count-only workloads (C2, C5) return no records: their counts are compared
                match_e2e = None if args.no_e2e else bool(np.array_equal(cb["counts"], counts_last[:samp_n])
                                                         and (not locate or np.array_equal(cb["occ"], occ_last[:k])))
                match_timed = None
                if dres is not None and not located_timed:
                    th = dres["timed_head"]
                    match_timed = bool(np.array_equal(cb["counts"], dres["timed_counts"][:samp_n])
                                       and (not locate or (th is not None and th.size >= k and np.array_equal(cb["occ"], th[:k]))))
                match = all(m_ is not False for m_ in (match_e2e, match_timed)) and (match_e2e, match_timed) != (None, None)
                ctr = cb["ctr"]
                lf_ref = (ctr["step_moves"] + ctr["locate_moves"]) / samp_n  # reference-literal M_LF moves per pattern
                out["parity_sample"] = {"n": samp_n, "ranks": 1, "records": k if locate else None, "occurrences": k,
                                        "compared": "counts and records" if locate else "counts (count-only workload)",
                                        "match": match, "match_e2e": match_e2e, "match_timed_device_step": match_timed,
                                        "timed_build": dres["counters"] if dres else None,
                                        "what": "oracle (literal MOVE_EDSBWTSearch restatement) vs the GPU's results "
                                                "(`compared`), in order, for the first n patterns: the e2e leg's last call "
                                                "and the last TIMED device-resident step (the build `value` is measured on)"}
                out["cpu_baseline"] = {
                    "value": round(cb["value"], 3), "unit": "patterns/sec", "cores": threads, "kind": "port",
                    "sample": f"first {samp_n} patterns of the batch; oracle/edsbwt_oracle.c (literal MOVE_EDSBWTSearch "
                              f"restatement, a=8 M_LF) on {threads} host threads over contiguous shards; index load "
                              f"{cb['open_s']:.1f}s excluded",
                    "seconds": round(cb["seconds"], 3),
                    "single_thread": {"value": round(c1["value"], 3), "cores": 1, "sample": f"first {samp1} patterns",
                                      "seconds": round(c1["seconds"], 3)},
                    "cpus_usable": cpus_usable, "cpu_share": cpu_share, "host_cpus_visible": os.cpu_count(),
                    "cores_note": ("threads = the CPUs this process may use (sched_getaffinity, before NUMA pinning), capped by "
                                   "the job's CPU share OMP_NUM_THREADS when set (16 per GPU on the GPU box, whose "
                                   "os.cpu_count() shows the whole machine)"),
                    "lf_steps_per_pattern": round(lf_ref, 1), "interval_steps_per_pattern": round(ctr["interval_steps"] / samp_n, 1),
                }
                # SURVEY §8(d) LF-steps, reference-equivalent: the reference-literal M_LF moves
                # (oracle-counted on the sample) per pattern, times the measured patterns/s — a
                # MODELLED rate (the device does not execute those moves)
                out["reference_equivalent_lf_steps"] = {
                    "modelled_per_sec": round(lf_ref * value, 1), "measured": False,
                    "what": "MODELLED, not executed by the device: the reference-literal M_LF moves per pattern (oracle-"
                            "counted on the CPU sample) x the measured patterns/s; the LF steps the device executed are "
                            "lf_steps_per_sec"}
                out["cpu_baseline"]["lf_steps_per_sec"] = round(lf_ref * cb["value"], 1)
                # the trie-sharing CPU variant on the same sample
                ct = cpu_baseline(base, buf, offs, first_id, samp_n, threads, trie=True)
                tc = ct["ctr"]
                out["cpu_baseline"]["trie_sharing"] = {
                    "value": round(ct["value"], 3), "cores": threads, "seconds": round(ct["seconds"], 3),
                    "sample": f"first {samp_n} patterns, sorted by reversed pattern, each thread a contiguous range of "
                              "that order (orc_search_batch_trie)",
                    "match_literal": bool(np.array_equal(ct["counts"], cb["counts"]) and np.array_equal(ct["occ"], cb["occ"])),
                    "interval_steps_per_pattern": round(tc["interval_steps"] / samp_n, 1),
                }
                if match_e2e is False:
                    diff = np.nonzero(cb["counts"] != counts_last[:samp_n])[0]
                    log("[bench] PARITY SAMPLE MISMATCH", "counts differ at", diff[:8].tolist(),
                        cb["counts"][diff[:8]].tolist(), counts_last[:samp_n][diff[:8]].tolist())
            except Exception as e:  # the GPU line is still valid
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), file=json_out, flush=True)
    text.free()
    counts_hb.free()
    idx.close()
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
