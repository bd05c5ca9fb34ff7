#!/usr/bin/env python3
"""Summarise rocprofv3 output of a bench.py run.

    python tools/profile_summary.py <trace_dir> <pmc_fetch_dir> <pmc_write_dir> <bench.json> <out_summary.json> \
        [--traffic profiles/traffic_<cfg>.json --source "<what was run>"]

* kernel trace (--kernel-trace --stats): per kernel calls / total / average duration,
  and per bench.py kernel class (the `roofline.kernel` the bench line names);
* PMC (separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes, as MI355X_MICROARCH.md
  §HBM prescribes): per kernel bytes fetched / written.  FETCH_SIZE is in KB and its
  byte factor depends on the access shape; tools/calib_gather.hip measured it on
  MI355X (profiles/r01_calib_fetch.csv): 1.00 for one random 64-B line per lane — the
  shape of every rank query, which dominates the step / deep / locate classes — and
  2.0 for 16-B-per-lane streaming reads (the guide's gfx950 correction).  The classes
  below use the gather factor; WRITE_SIZE × 1024 as is.
* --tcc <dir>: a third PMC pass of TCC_EA0_RDREQ_sum, TCC_BUBBLE_sum, TCC_EA0_RDREQ_32B_sum and
  TCC_EA0_RDREQ_DRAM_32B_sum.  Round 3 calibration on MI355X (tools/calib_gather.hip, 4 GB table,
  profiles/r03_calib_counters.json): TCC_EA0_RDREQ_DRAM_32B x 32 equals the bytes of a 16-B-per-lane
  streaming read exactly (FETCH_SIZE shows half of them, as the guide says), and a random 16-, 64-
  or 128-B access is ONE 128-B request (RDREQ = accesses, DRAM_32B = 4 per access) while
  FETCH_SIZE tallies it at 64 B.  So DRAM read bytes = TCC_EA0_RDREQ_DRAM_32B x 32 for every
  shape, and = 2 x FETCH_SIZE for the random gathers; with --tcc the classes' HBM traffic uses it.
* --traffic writes the per-class HBM bytes per launch that bench.py reports as
  `roofline.traffic`.
"""
import argparse
import collections
import csv
import json
import os

# bench.py kernel class -> kernels (engine.hip KClass)
# (round 3: the deep stage's three kernels are classes of their own, KC_DEEP / KC_DEEPQ /
# KC_DEEPW, so each has its own rocprof average and PMC bytes per launch; "r3b": deep is
# k_deep_direct on the packed start with the wide k-mer table, deep_wide k_deep_wave)
CLASSES = {
    "step": ("k_lvl_items", "k_lvl_dollar", "k_lvl_chunks"),
    "deep": ("k_deep_direct", "k_deep_fast"),
    "deep_list": ("k_deep",),
    "deep_wide": ("k_deep_wave", "k_deep_wide"),
    "locate": ("k_locate", "k_locate_pp", "k_locate_big", "k_locate_lists"),
    # the link key sort (KC_LINKSORT, hipcub SortKeys on u64 keys: the only keys-only radix sort
    # the engine runs); one "launch" = one sort = one global-offsets kernel + its onesweep passes
    "link_sort": ("rocprim_sortkeys_offsets", "rocprim_sortkeys"),
}
# the kernel whose dispatches count a class's launches, where one launch is several kernels
CLASS_UNIT = {"link_sort": "rocprim_sortkeys_offsets"}
FETCH_FACTOR_GATHER64 = 1.0


def short(name: str) -> str:
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("edsbwt::", "")
    if not n.startswith("rocprim"):
        return n.split("<")[0]
    if "radix_sort" in name and "empty_type" in name:
        return "rocprim_sortkeys_offsets" if "global_offsets" in name else "rocprim_sortkeys"
    return "rocprim"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("bench_json")
    ap.add_argument("out")
    ap.add_argument("--traffic")
    ap.add_argument("--tcc")
    ap.add_argument("--source", default="")
    a = ap.parse_args()

    def first_csv(d, suffix):
        for f in sorted(os.listdir(d)):
            if f.endswith(suffix):
                return os.path.join(d, f)
        raise FileNotFoundError(f"{d}/*{suffix}")

    stats = list(csv.DictReader(open(first_csv(a.trace_dir, "kernel_stats.csv"))))
    per = collections.defaultdict(lambda: {"calls": 0, "total_ms": 0.0})
    for r in stats:
        k = short(r["Name"])
        per[k]["calls"] += int(r["Calls"])
        per[k]["total_ms"] += float(r["TotalDurationNs"]) / 1e6
    for v in per.values():
        v["avg_us"] = 1e3 * v["total_ms"] / max(1, v["calls"])
    pmc = collections.defaultdict(lambda: {"fetch_bytes": 0.0, "write_bytes": 0.0, "dispatches": 0})
    # (tools/prof_reduce.py may have summed the rows per (kernel, counter): "Dispatches" then
    # holds the number of dispatches each sum covers)
    for d, key in ((a.fetch_dir, "fetch_bytes"), (a.write_dir, "write_bytes")):
        for r in csv.DictReader(open(first_csv(d, "counter_collection.csv"))):
            k = short(r["Kernel_Name"])
            v = float(r["Counter_Value"]) * 1024.0
            pmc[k][key] += FETCH_FACTOR_GATHER64 * v if key == "fetch_bytes" else v
            if key == "fetch_bytes":
                pmc[k]["dispatches"] += int(r.get("Dispatches") or 1)
    tcc = collections.defaultdict(lambda: collections.defaultdict(float))
    if a.tcc:
        for r in csv.DictReader(open(first_csv(a.tcc, "counter_collection.csv"))):
            tcc[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "TCC_EA0_RDREQ_sum":
                tcc[short(r["Kernel_Name"])]["dispatches"] += int(r.get("Dispatches") or 1)
    # registers, LDS and the occupancy they allow, per kernel (kernel trace columns).  gfx950:
    # 512 VGPRs per lane per SIMD shared by the arch and accumulation registers (granule 8),
    # at most 8 waves per SIMD, 160 KB of LDS per CU (4 SIMDs)
    res = {}
    for r in csv.DictReader(open(first_csv(a.trace_dir, "kernel_trace.csv"))):
        k = short(r["Kernel_Name"])
        if k in res:
            continue
        v, acc = int(r["VGPR_Count"]), int(r.get("Accum_VGPR_Count") or 0)
        lds, wg = int(r["LDS_Block_Size"]), max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
        regs = max(8, -(-(v + acc) // 8) * 8)
        w_reg = min(8, 512 // regs)
        waves_per_wg = -(-wg // 64)
        w_lds = 8 if lds == 0 else min(8, (160 * 1024 // lds) * waves_per_wg // 4)
        res[k] = {"vgpr": v, "agpr": acc, "sgpr": int(r["SGPR_Count"]), "lds_bytes": lds, "scratch_bytes": int(r["Scratch_Size"]),
                  "workgroup": wg, "waves_per_simd": min(w_reg, w_lds), "occupancy_limit": "vgpr" if w_reg <= w_lds else "lds"}
    bench = json.load(open(a.bench_json))
    classes = {}
    for c, ks in CLASSES.items():
        unit = (CLASS_UNIT[c],) if c in CLASS_UNIT else ks
        calls = sum(per[k]["calls"] for k in unit if k in per)
        tot = sum(per[k]["total_ms"] for k in ks if k in per)
        disp = sum(pmc[k]["dispatches"] for k in unit if k in pmc)
        fb = sum(pmc[k]["fetch_bytes"] for k in ks if k in pmc)
        wb = sum(pmc[k]["write_bytes"] for k in ks if k in pmc)
        classes[c] = {"rocprof_calls": calls, "rocprof_avg_launch_ms": tot / max(1, calls),
                      "pmc_hbm_bytes_per_launch": (fb + wb) / max(1, disp),
                      "pmc_fetch_bytes_per_launch": fb / max(1, disp), "pmc_write_bytes_per_launch": wb / max(1, disp)}
        if a.tcc:
            td = sum(tcc[k]["dispatches"] for k in unit if k in tcc)
            dram = 32.0 * sum(tcc[k]["TCC_EA0_RDREQ_DRAM_32B_sum"] for k in ks if k in tcc)
            req = sum(tcc[k]["TCC_EA0_RDREQ_sum"] for k in ks if k in tcc)
            classes[c].update({"pmc_dram_read_bytes_per_launch": dram / max(1, td), "pmc_read_requests_per_launch": req / max(1, td),
                               "pmc_dram_bytes_per_launch": dram / max(1, td) + wb / max(1, disp)})
    out_d = {"bench": {k: bench.get(k) for k in ("value", "ms_per_step", "roofline", "kernel_ms_per_step")},
             "fetch_factor": FETCH_FACTOR_GATHER64,
             "classes": classes,
             "kernels": {k: {**per[k], **pmc.get(k, {}), **res.get(k, {})} for k in sorted(per, key=lambda k: -per[k]["total_ms"])}}
    json.dump(out_d, open(a.out, "w"), indent=1)
    if a.traffic:
        json.dump({"source": a.source, "classes_version": "r3b", "fetch_factor": FETCH_FACTOR_GATHER64,
                   "traffic_field": "pmc_dram_bytes_per_launch" if a.tcc else "pmc_hbm_bytes_per_launch",
                   "classes": classes}, open(a.traffic, "w"), indent=1)
    print(json.dumps(classes, indent=1))


if __name__ == "__main__":
    main()
