#!/bin/bash
# Round-3 final measurement pass (C3, then the C5 and C2 lines): smoke, a kernel trace
# and separate PMC passes of the device-resident leg (FETCH_SIZE; WRITE_SIZE; TCC requests and
# DRAM 32-B requests; SQ stalls), the per-class traffic summary written into profiles/ of this
# tree (so the bench line that follows carries it), then the default bench line.
export TMPDIR=/tmp
TAG=${1:-r3m2}
mkdir -p gpurun_out
B="python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o pmc --output-format csv -- $B > gpurun_out/${TAG}_fetch.json 2> gpurun_out/${TAG}_fetch.log &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o pmc --output-format csv -- $B > gpurun_out/${TAG}_write.json 2> gpurun_out/${TAG}_write.log &&
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_tcc -o pmc --output-format csv -- $B > gpurun_out/${TAG}_tcc.json 2> gpurun_out/${TAG}_tcc.log &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/${TAG}_sq -o pmc --output-format csv -- $B > gpurun_out/${TAG}_sq.json 2> gpurun_out/${TAG}_sq.log &&
python tools/profile_summary.py gpurun_out/${TAG}_trace gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_trace_bench.json gpurun_out/${TAG}_c3_summary.json --tcc gpurun_out/${TAG}_tcc --traffic profiles/traffic_c3.json --source "tools/gpu_r3meas.sh: rocprofv3 --pmc passes of bench.py --no-cpu --no-e2e --steps 3 --warmup 1 (C3)" > gpurun_out/${TAG}_classes.json &&
cp profiles/traffic_c3.json gpurun_out/traffic_c3.json &&
python - "$TAG" <<'PY' &&
import csv, collections, glob, json, os, sys
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"gpurun_out/{tag}_sq/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("edsbwt::", "").split("<")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
json.dump({k: dict(v) for k, v in agg.items() if k.startswith("k_")}, open(f"gpurun_out/{tag}_sq_summary.json", "w"), indent=1)
for d in ("trace", "fetch", "write", "tcc", "sq"):
    for f in glob.glob(f"gpurun_out/{tag}_{d}/*.csv"):
        if not f.endswith("kernel_stats.csv"):
            os.remove(f)
PY
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log
rc=$?
[ $rc -eq 0 ] && timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.log
[ $? -eq 0 ] && timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.log
echo EXIT $rc $?
# C5: a depth-4 k-mer start table (EDSBWT_KTAB_ITEMS=2e9: 1.8G intervals) against the default budget (depth 3)
[ $rc -eq 0 ] && bash tools/gpu_ab3.sh ${TAG} c5 3 X=1 EDSBWT_KTAB_ITEMS=2000000000
du -sh gpurun_out
