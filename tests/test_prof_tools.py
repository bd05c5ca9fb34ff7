"""tools/prof_reduce.py and tools/profile_summary.py on synthetic rocprofv3 CSVs (CPU only): the
on-box reduction keeps one kernel-trace row per kernel and sums the PMC rows per (kernel, counter)
with their dispatch count, and the summary's per-class launches and bytes are the same before and
after the reduction (the link-key sort class counts one launch per sort)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SORT_OFF = ("void rocprim::detail::trampoline_kernel<radix_sort_onesweep_global_offsets<unsigned long const*, "
            "rocprim::empty_type*>(unsigned long const*)")
SORT_IT = "void rocprim::detail::trampoline_kernel<radix_sort_onesweep_iteration<unsigned long, rocprim::empty_type*>(unsigned long*)"
DEEP = "void edsbwt::k_deep_direct<8, true>(unsigned long, unsigned int)"


def _write(path, rows, fields):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        w.writerows(rows)


def _make(d):
    os.makedirs(os.path.join(d, "trace"))
    for sub in ("fetch", "write", "tcc"):
        os.makedirs(os.path.join(d, sub))
    names = [DEEP] * 3 + [SORT_OFF] * 2 + [SORT_IT] * 8
    _write(os.path.join(d, "trace", "t_kernel_trace.csv"),
           [{"Kernel_Name": n, "VGPR_Count": 64, "Accum_VGPR_Count": 0, "SGPR_Count": 80, "LDS_Block_Size": 512, "Scratch_Size": 36,
             "Workgroup_Size_X": 256, "Workgroup_Size_Y": 1, "Workgroup_Size_Z": 1} for n in names],
           ["Kernel_Name", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Scratch_Size", "Workgroup_Size_X",
            "Workgroup_Size_Y", "Workgroup_Size_Z"])
    _write(os.path.join(d, "trace", "t_kernel_stats.csv"),
           [{"Name": DEEP, "Calls": 3, "TotalDurationNs": 3_000_000}, {"Name": SORT_OFF, "Calls": 2, "TotalDurationNs": 40_000},
            {"Name": SORT_IT, "Calls": 8, "TotalDurationNs": 800_000}], ["Name", "Calls", "TotalDurationNs"])
    for sub, counters in (("fetch", [("FETCH_SIZE", 1000.0)]), ("write", [("WRITE_SIZE", 500.0)]),
                          ("tcc", [("TCC_EA0_RDREQ_sum", 10.0), ("TCC_EA0_RDREQ_DRAM_32B_sum", 40.0)])):
        rows = [{"Kernel_Name": n, "Counter_Name": c, "Counter_Value": v, "Dispatch_Id": k} for k, n in enumerate(names) for c, v in counters]
        _write(os.path.join(d, sub, "p_counter_collection.csv"), rows, ["Kernel_Name", "Counter_Name", "Counter_Value", "Dispatch_Id"])
    json.dump({"value": 1.0, "ms_per_step": 1.0}, open(os.path.join(d, "bench.json"), "w"))


def _summary(d, out):
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "profile_summary.py"), os.path.join(d, "trace"), os.path.join(d, "fetch"),
                    os.path.join(d, "write"), os.path.join(d, "bench.json"), out, "--tcc", os.path.join(d, "tcc")],
                   check=True, capture_output=True)
    return json.load(open(out))["classes"]


def test_reduce_keeps_class_numbers(tmp_path):
    d = str(tmp_path)
    _make(d)
    before = _summary(d, os.path.join(d, "s0.json"))
    # (as tools/gpu.sh calls it: on the rocprofv3 output directories)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_reduce.py")] + [os.path.join(d, x) for x in ("trace", "fetch", "write", "tcc")],
                   check=True)
    with open(os.path.join(d, "trace", "t_kernel_trace.csv")) as f:
        assert len(list(csv.DictReader(f))) == 3  # one row per kernel
    with open(os.path.join(d, "fetch", "p_counter_collection.csv")) as f:
        rows = list(csv.DictReader(f))
    assert {r["Kernel_Name"]: int(r["Dispatches"]) for r in rows} == {DEEP: 3, SORT_OFF: 2, SORT_IT: 8}
    after = _summary(d, os.path.join(d, "s1.json"))
    assert before == after
    # k_deep_direct: 3 launches of 1 ms, 1000 KB fetched + 500 KB written each; DRAM bytes 40 x 32 + write
    deep = after["deep"]
    assert deep["rocprof_calls"] == 3 and abs(deep["rocprof_avg_launch_ms"] - 1.0) < 1e-9
    assert deep["pmc_hbm_bytes_per_launch"] == 1500 * 1024 and deep["pmc_dram_bytes_per_launch"] == 40 * 32 + 500 * 1024
    # the link-key sort: one launch per global-offsets kernel (2 sorts), all ten kernels' time and bytes
    ls = after["link_sort"]
    assert ls["rocprof_calls"] == 2 and abs(ls["rocprof_avg_launch_ms"] - 0.42) < 1e-9
    assert ls["pmc_fetch_bytes_per_launch"] == 10 * 1000 * 1024 / 2
