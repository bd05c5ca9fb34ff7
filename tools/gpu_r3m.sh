#!/bin/bash
# As gpu_r3l.sh without the tests; bulky per-dispatch CSVs are summarised on the box and removed.
export TMPDIR=/tmp
TAG=${1:-r3m}
mkdir -p gpurun_out
w() { python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])"; }
for spec in "X=1" "EDSBWT_DEEP_WAVE=0"; do
  echo "== c2 $spec" >> gpurun_out/${TAG}_ab.txt
  env $spec timeout -k 10 200 python bench.py --config c2 --no-cpu --no-e2e --steps 10 --warmup 2 2>/dev/null | w >> gpurun_out/${TAG}_ab.txt || exit 1
  echo "== c3 $spec" >> gpurun_out/${TAG}_ab.txt
  env $spec timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 10 --warmup 2 2>/dev/null | w >> gpurun_out/${TAG}_ab.txt || exit 1
done
EDSBWT_TRACE=1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 1 --warmup 1 > gpurun_out/${TAG}_c3_trace.json 2> gpurun_out/${TAG}_c3_trace.full.log
grep -v "^\[edsbwt\] t " gpurun_out/${TAG}_c3_trace.full.log | tail -200 > gpurun_out/${TAG}_c3_trace.log; rm -f gpurun_out/${TAG}_c3_trace.full.log
B="python3 bench.py --config c5 --no-cpu --no-e2e --steps 1 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_tcc -o pmc --output-format csv -- $B > gpurun_out/${TAG}_tcc.json 2> gpurun_out/${TAG}_tcc.log
echo EXIT $?
python - "$TAG" <<'PY'
import csv, collections, json, sys, glob, os
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"gpurun_out/{tag}_tcc/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("edsbwt::", "").split("<")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "TCC_EA0_RDREQ_sum": agg[k]["dispatches"] += 1
json.dump({k: dict(v) for k, v in agg.items()}, open(f"gpurun_out/{tag}_tcc_summary.json", "w"), indent=1)
for f in glob.glob(f"gpurun_out/{tag}_tcc/*") + glob.glob(f"gpurun_out/{tag}_trace/*kernel_trace.csv"):
    os.remove(f)
PY
du -sh gpurun_out
