#!/bin/bash
# C5 profiles: kernel trace + separate FETCH_SIZE / WRITE_SIZE passes (tools/profile_summary.py).
export TMPDIR=/tmp
TAG=${1:-c5p}
mkdir -p gpurun_out
B="python3 bench.py --config c5 --no-cpu --no-e2e --steps 1 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o pmc --output-format csv -- $B > gpurun_out/${TAG}_fetch.json 2> gpurun_out/${TAG}_fetch.log &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o pmc --output-format csv -- $B > gpurun_out/${TAG}_write.json 2> gpurun_out/${TAG}_write.log
echo EXIT $?
