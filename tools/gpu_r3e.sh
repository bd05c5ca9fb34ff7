#!/bin/bash
# Host pipeline timelines (EDSBWT_TRACE=1 marks per chunk: upload / uploaded / search / searched /
# download / downloaded / counted) for the C2 and C3 end-to-end calls, and the C2 line.
export TMPDIR=/tmp
TAG=${1:-r3e}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.log &&
EDSBWT_TRACE=1 timeout -k 10 300 python bench.py --config c2 --no-cpu --no-device --steps 8 --warmup 2 > gpurun_out/${TAG}_trace_c2.json 2> gpurun_out/${TAG}_trace_c2.log &&
EDSBWT_TRACE=1 timeout -k 10 300 python bench.py --no-cpu --no-device --steps 12 --warmup 2 > gpurun_out/${TAG}_trace_c3.json 2> gpurun_out/${TAG}_trace_c3.log
echo EXIT $?
