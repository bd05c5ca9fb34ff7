#!/usr/bin/env python3
"""Host-contention rehearsal for the 8-GPU run, on a 1-GPU box.

    python tools/host_contention.py [--procs 0,1,3] [--threads 2] [--steps 30] > out.json

On an 8-GPU node every rank runs the host pipeline of edsbwt_search_lines beside the others:
its packer streams the pattern file (C3: 320 MB read, 80 MB written per call) and the copy
engines read the packed bytes and land 242 MB of counts and records in host memory — about
130 GB/s of host-memory traffic per rank.  This tool runs ONE real bench.py rank
(C3, end-to-end leg only) while K background processes, pinned to the same NUMA node, repeat
the CPU side of other ranks' pipelines: the same 2-bit packer (libedsbwt.so's
edsbwt_pack_lines, no GPU call) over a 40 MB chunk of fixed-length lines, plus a 30 MB memcpy
into page-locked memory (the widening of landed records).  It reports the rank's per-call
walls for each K and the background processes' achieved host bandwidth.

The box gives one job 16 CPUs (cgroup cpu.max 1600000/100000), so K is small here: this
measures the sensitivity of a rank's end-to-end time to neighbours on its socket, not the
8-rank node itself.
"""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "eds-bwt_amd", "_build", "libedsbwt.so")


def gpu_numa_cpus():
    """CPUs of GPU 0's NUMA node (read in a child process: only it touches the GPU)."""
    code = ("import torch,os;p=torch.cuda.get_device_properties(0);"
            "b=f'{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0';"
            "n=int(open(f'/sys/bus/pci/devices/{b}/numa_node').read());"
            "print(n, open(f'/sys/devices/system/node/node{n}/cpulist').read().strip() if n>=0 else '')")
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300).stdout.split()
        node, spec = int(out[0]), out[1] if len(out) > 1 else ""
    except Exception:  # noqa: BLE001
        return None, None
    cpus = set()
    for part in spec.split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    return node, cpus


def neighbour(cpus, threads, mb, stop, out_q):
    """One emulated neighbour rank: pack + memcpy loops on `threads` threads until `stop`."""
    if cpus:
        os.sched_setaffinity(0, cpus & os.sched_getaffinity(0) or os.sched_getaffinity(0))
    L = ctypes.CDLL(LIB)
    L.edsbwt_lines_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]
    L.edsbwt_lines_fixed.restype = ctypes.c_uint64
    L.edsbwt_pack_lines.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_void_p, ctypes.c_void_p]
    L.edsbwt_pack_lines.restype = ctypes.c_int
    n = int(mb * 2**20) // 32
    rng = np.random.default_rng(os.getpid())
    a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=(n, 32))]
    a[:, 31] = ord("\n")
    text = np.ascontiguousarray(a).reshape(-1)
    Lo = ctypes.c_uint32(0)
    P = L.edsbwt_lines_fixed(text.ctypes.data, text.size, ctypes.byref(Lo))
    packed = np.zeros(P * 8 + 16, np.uint8)
    src = np.ones(30 << 20, np.uint8)
    dst = np.zeros(30 << 20, np.uint8)
    moved = [0] * threads

    def work(t):
        lo, hi = P * t // threads, P * (t + 1) // threads
        s0, s1 = src.size * t // threads, src.size * (t + 1) // threads
        while not stop.is_set():
            L.edsbwt_pack_lines(text.ctypes.data, text.size, Lo.value, lo, hi, text.ctypes.data + text.size, packed.ctypes.data)
            ctypes.memmove(dst.ctypes.data + s0, src.ctypes.data + s0, s1 - s0)
            moved[t] += (hi - lo) * (32 + 8) + 2 * (s1 - s0)
    t0 = time.time()
    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    out_q.put(sum(moved) / (time.time() - t0) / 1e9)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="0,1,3")
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--mb", type=float, default=40)
    a = ap.parse_args()
    node, cpus = gpu_numa_cpus()
    res = {"what": __doc__.split("\n\n")[1].strip(), "gpu_numa_node": node, "runs": []}
    ctx = mp.get_context("spawn")
    for K in [int(x) for x in a.procs.split(",")]:
        stop = ctx.Event()
        q = ctx.Queue()
        ps = [ctx.Process(target=neighbour, args=(cpus, a.threads, a.mb, stop, q)) for _ in range(K)]
        for p in ps:
            p.start()
        time.sleep(2.0 if K else 0.0)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-device", "--steps", str(a.steps),
                            "--warmup", "3"], capture_output=True, text=True, timeout=600)
        stop.set()
        gbs = [q.get(timeout=60) for _ in ps]
        for p in ps:
            p.join(timeout=60)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        e = line["e2e"]
        res["runs"].append({"neighbours": K, "threads_each": a.threads, "neighbour_host_GBps": [round(x, 1) for x in gbs],
                            "value": line["value"], "ms_per_step": line["ms_per_step"], "ms_wall_median": e["ms_wall_median"],
                            "ms_wall_p90": e["ms_wall_p90"], "ms_wall_max": e["ms_wall_max"], "host_cores": e["host_cores"]})
        print(json.dumps(res["runs"][-1]), file=sys.stderr, flush=True)
    base = res["runs"][0]["ms_wall_median"] if res["runs"] else None
    for r_ in res["runs"]:
        r_["median_vs_alone"] = round(r_["ms_wall_median"] / base, 3) if base else None
    print(json.dumps(res))


if __name__ == "__main__":
    main()
