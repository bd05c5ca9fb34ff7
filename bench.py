#!/usr/bin/env python3
"""Benchmark: EDS-BWT backward search on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5]

A *step* is one pass of the hot path (MOVE_EDSBWTSearch's pattern loop + locate,
MOVE_EDSBWTSearch.cpp:97-155) over one batch of synthetic patterns whose bytes and
offsets are already resident in HBM: the whole trie-level search plus position
recovery through libedsbwt.so, results (counts + occurrence records) left in HBM.
Default workload = config C3 of SURVEY.md §8(d) (BASELINE.json configs[2]): a
~100 Mchar COVID-like synthetic EDS, 10M planted 31-mers, full locate.  N>1 ranks
(one per GPU, torchrun) each search their own contiguous shard of 10M patterns
against a replicated index (weak scaling) and the per-pattern counts are gathered
over RCCL.  rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(ROOT, "eds-bwt_amd", "_build")
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (generator config, EDS chars, EDS seed, patterns per GPU, lengths, mode, pattern seed, locate)
    "c2": ("c2", 10_000_000, 1, 1_000_000, "20", "random", 2, False),
    "c3": ("c3", 100_000_000, 3, 10_000_000, "31", "planted", 4, True),
    "c5": ("c5", 1_000_000_000, 6, 200_000, "8,16,32,64", "mixed", 7, False),
}
WORKLOAD = {
    "c2": "C2: 10 Mchar synthetic EDS (sigma=4, ~3 strings/segment), 1M random 20-mers per GPU, count-only",
    "c3": "C3: ~100 Mchar COVID-like synthetic EDS, 10M planted 31-mers per GPU, full position recovery",
    "c5": "C5: 1 Gchar synthetic EDS with 20% empty-string segments, mixed 8-64-mers per GPU, counts (a random 8-mer has ~1e4-1e5 occurrences)",
}
MI355X_HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak
# Practical ceiling of the rank queries' access shape — one random 64-B line per lane
# from a table of the C3 index's size (100 MB, Infinity-Cache resident): measured on
# MI355X by tools/calib_gather.hip (profiles/r01_calib_gather.json), 3.4-3.5 TB/s.
GATHER64_CEILING_LINES_PER_S = 5.48e10


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def run(args, **kw):
    subprocess.run([str(a) for a in args], check=True, **kw)


def ensure_built():
    need = [os.path.join(BUILD, f) for f in ("libedsbwt.so", "eds_transform", "edsbwt_gen")]
    if not all(os.path.exists(p) for p in need):
        run(["make", "-s", "-j", "16", "-C", os.path.join(ROOT, "eds-bwt_amd"), "all"])


def prepare(cfg: str, workdir: str, rank: int, world: int, npat: int, barrier, chars_override: int = 0):
    gcfg, chars, eseed, _, lens, mode, pseed, _ = CONFIGS[cfg]
    tag = cfg
    if chars_override:
        chars, tag = chars_override, f"{cfg}_{chars_override}"
    os.makedirs(workdir, exist_ok=True)
    eds = os.path.join(workdir, f"{tag}.eds")
    base = os.path.join(workdir, tag)
    if rank == 0 and not os.path.exists(base + "_info.aux"):
        t = time.time()
        run([os.path.join(BUILD, "edsbwt_gen"), "eds", "--config", gcfg, "--chars", chars, "--seed", eseed, "--out", eds])
        run([os.path.join(BUILD, "eds_transform"), eds, base, "--no-runs"])
        log(f"[bench] index {base} built in {time.time() - t:.1f}s")
    barrier()
    pats = os.path.join(workdir, f"{tag}_pats_{npat}_r{rank}of{world}.txt")
    if not os.path.exists(pats):
        run([os.path.join(BUILD, "edsbwt_gen"), "patterns", "--eds", eds, "--count", npat, "--lens", lens, "--mode", mode,
             "--seed", pseed * 1000003 + rank, "--out", pats])
    barrier()
    return base, pats


def traffic_from_profile(cfg: str, kernel: str, locate: bool):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 PMC summary of
    this same command (profiles/traffic_<cfg>.json, written by tools/profile_summary.py
    from separate --pmc FETCH_SIZE / WRITE_SIZE passes); None when there is none."""
    path = os.path.join(ROOT, "profiles", f"traffic_{cfg}.json")
    try:
        t = json.load(open(path))
        c = t["classes"][kernel]
        return int(c["pmc_hbm_bytes_per_launch"]), f"profiles/traffic_{cfg}.json ({t.get('source', '')})"
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(base: str, pats_path: str, sample: int, threads: int) -> dict:
    """The oracle (faithful C restatement of MOVE_EDSBWTSearch: a-balanced M_LF,
    literal per-pattern link/step/locate) on the first `sample` patterns."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # checker / CPU baseline only

    pkg = importlib.import_module("eds-bwt_amd")
    buf, offs = pkg.read_pattern_file(pats_path)
    offs = offs[: sample + 1]
    buf = buf[: int(offs[-1])]
    t = time.time()
    eng = orc.Engine(base, 8)
    t_open = time.time() - t
    t = time.time()
    counts, occ, ctr = eng.search(buf, offs, threads=threads)
    dt = time.time() - t
    eng.close()
    return {"value": round(sample / dt, 3), "unit": "patterns/sec", "cores": threads, "kind": "port",
            "sample": f"first {sample} patterns of rank 0's batch, oracle/edsbwt_oracle.c (literal MOVE_EDSBWTSearch "
                      f"restatement, a=8 M_LF) on {threads} host threads; index load {t_open:.1f}s excluded",
            "seconds": round(dt, 3), "lf_steps": int(ctr["step_moves"] + ctr["locate_moves"]),
            "interval_steps": int(ctr["interval_steps"]), "occurrences": int(ctr["occurrences"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--patterns", type=int, default=0, help="patterns per GPU (default: the config's)")
    ap.add_argument("--chars", type=int, default=0, help="EDS size override (scaled-down parity/diagnostic runs)")
    ap.add_argument("--locate", default="sampled", choices=("sampled", "walk", "table"),
                    help="position recovery: LF walk to the first sampled row (default), the reference's full "
                         "walk to '#', or the per-row (word, offset) table")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-sample", type=int, default=0)
    ap.add_argument("--workdir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "edsbwt_bench"))
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on GPU nodes; gloo to rehearse ranks on one GPU")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev  # rehearsal: several ranks may share one GPU (gloo)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
        barrier = lambda: dist.barrier()  # noqa: E731
    else:
        torch.cuda.set_device(0)
        barrier = lambda: None  # noqa: E731
    if rank == 0:
        ensure_built()
    barrier()
    pkg = importlib.import_module("eds-bwt_amd")
    cfg = args.config
    npat = args.patterns or CONFIGS[cfg][3]
    locate = CONFIGS[cfg][7]
    base, pats_path = prepare(cfg, args.workdir, rank, world, npat, barrier, args.chars)

    t = time.time()
    if world > 1 and ndev < world:
        # ranks sharing a GPU (gloo rehearsal) open the index one at a time: the k-mer table
        # build's transient workspace is sized for a whole GPU
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
    buf, offs = pkg.read_pattern_file(pats_path)
    dev = torch.device("cuda", local)
    d_bytes = torch.from_numpy(buf).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_counts = torch.zeros(npat, dtype=torch.int32, device=dev)
    first_id = rank * npat + 1
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(profile=False):
        return idx.search_device(d_bytes.data_ptr(), d_offs.data_ptr(), npat, d_counts.data_ptr(),
                                 first_pattern_id=first_id, locate=locate, table=args.locate == "table", profile=profile,
                                 stream=stream, walk=args.locate == "walk")

    gdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    gathered = torch.zeros(npat * world, dtype=torch.int32, device=gdev) if world > 1 else None

    def exchange():
        # the path's one exchange: every rank's per-pattern counts, gathered over RCCL/xGMI
        if world > 1:
            src = d_counts if args.dist_backend == "nccl" else d_counts.cpu()
            dist.all_gather_into_tensor(gathered, src)

    for _ in range(args.warmup):
        step()
        exchange()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kstats = {}
    total_occ = 0
    lf_steps = 0
    ref_loc_steps = 0
    for i in range(args.steps):
        _, nocc = step(profile="light")
        exchange()
        st = idx.stats()
        total_occ += nocc
        lf_steps += 2 * st["intervals_stepped"] + st["locate_lf_steps"]
        ref_loc_steps += st["locate_offsets"]
        for k, v in st["kernels"].items():
            a = kstats.setdefault(k, {"ms": 0.0, "launches": 0, "bytes": 0, "lines": 0})
            a["ms"] += v["ms"]
            a["launches"] += v["launches"]
            a["bytes"] += v["bytes"]
            a["lines"] += v["lines"]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        agg = torch.tensor([lf_steps, total_occ, ref_loc_steps], dtype=torch.float64, device=gdev)
        dist.all_reduce(agg)
        lf_steps, total_occ, ref_loc_steps = float(agg[0].item()), float(agg[1].item()), float(agg[2].item())
    last = idx.stats()

    if rank == 0:
        ms_step = 1000.0 * elapsed / args.steps
        value = npat * world * args.steps / elapsed
        # dominant kernel class by device time over the timed region
        dom = max((k for k in kstats if k != "scan"), key=lambda k: kstats[k]["ms"])
        d = kstats[dom]
        avg_ms = d["ms"] / max(1, d["launches"])
        achieved = (d["bytes"] / d["launches"]) / (avg_ms * 1e-3) / 1e9 if d["launches"] and avg_ms > 0 else 0.0
        line_rate = (d["lines"] / d["launches"]) / (avg_ms * 1e-3) if d["launches"] and avg_ms > 0 else 0.0
        traffic, traffic_src = traffic_from_profile(cfg, dom, locate)
        out = {
            "metric": "patterns/sec + LF-steps/sec, 100 Mchar EDS, 10M 31-mers, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "patterns/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (edsbwt_gen, seeded)",
            "config": {"workload": WORKLOAD[cfg], "config": cfg, "patterns_per_gpu": npat,
                       "index_rows": idx.n_rows, "words": idx.n_words, "segments": idx.n_segments,
                       "locate": {"sampled": "per-row samples (word, offset, segment, word-in-segment), one read per occurrence",
                                  "walk": "lf-walk to '#' (reference)", "table": "per-row table"}[args.locate]
                       if locate else "count-only",
                       "parallelism": f"pattern-shard x{world}"},
            # LF steps the device executed (2 per interval step + locate walk moves)
            "lf_steps_per_sec": round(lf_steps / elapsed, 1),
            # the reference's locate walk moves for the same records (sum of offsets, :348-353)
            "reference_locate_lf_steps_per_sec": round(ref_loc_steps / elapsed, 1),
            "occurrences_per_step": int(total_occ / args.steps / max(1, world)) if world == 1 else int(total_occ / args.steps),
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": MI355X_HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / MI355X_HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "avg_launch_ms": round(avg_ms, 4), "launches": d["launches"],
                         "bytes_per_launch": int(d["bytes"] / max(1, d["launches"])),
                         # random 64-B lines: the rate the access shape is actually bound by
                         "lines_per_launch": int(d["lines"] / max(1, d["launches"])),
                         "lines_per_s": round(line_rate, 1),
                         "gather_ceiling_lines_per_s": GATHER64_CEILING_LINES_PER_S,
                         "frac_of_gather_ceiling": round(line_rate / GATHER64_CEILING_LINES_PER_S, 4)},
            "kernel_lines_per_s": {k: round((v["lines"] / (v["ms"] * 1e-3)) if v["ms"] > 0 else 0.0, 1)
                                   for k, v in sorted(kstats.items()) if v["lines"]},
            "kernel_ms_per_step": {k: round(v["ms"] / args.steps, 3) for k, v in sorted(kstats.items())},
            "index_open_s": round(t_open, 2),
            "engine": {k: last[k] for k in ("depths", "deep_from_depth", "deep_overflow", "deep_level_rerun", "search_groups", "trie_nodes", "intervals_stepped",
                                              "link_hash_rows", "link_ranges", "locate_lf_steps")},
            "found_per_step": int(last["found"]),
        }
        if world == 1 and not args.no_cpu:
            threads = min(16, os.cpu_count() or 1)
            sample = args.cpu_sample or (64 * threads if cfg != "c2" else 512 * threads)
            sample = min(sample, npat)
            try:
                out["cpu_baseline"] = cpu_baseline(base, pats_path, sample, threads)
            except Exception as e:  # the GPU line is still valid
                out["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(out), flush=True)
    idx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
