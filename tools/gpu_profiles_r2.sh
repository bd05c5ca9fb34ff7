#!/bin/bash
# Round-2 profiles: kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of a short C3 bench
# (tools/profile_summary.py reads them), the C2 bench line, smoke().   bash tools/gpu_profiles_r2.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
B="python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o pmc --output-format csv -- $B > gpurun_out/${TAG}_fetch.json 2> gpurun_out/${TAG}_fetch.log &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o pmc --output-format csv -- $B > gpurun_out/${TAG}_write.json 2> gpurun_out/${TAG}_write.log &&
timeout -k 10 300 python bench.py --no-cpu --config c2 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo EXIT $?
