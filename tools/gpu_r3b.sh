#!/bin/bash
# Round 3 measurement pass (C3): smoke, the default bench line, a kernel trace and separate PMC
# passes of the device-resident leg (FETCH_SIZE; WRITE_SIZE; TCC request counters; SQ stall +
# L2 hit counters), and the counter calibration of tools/calib_gather (gather16 / stream16).
#   bash tools/gpu_r3b.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3b}
mkdir -p gpurun_out
B="python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1"
set -o pipefail
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o pmc --output-format csv -- $B > gpurun_out/${TAG}_fetch.json 2> gpurun_out/${TAG}_fetch.log &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o pmc --output-format csv -- $B > gpurun_out/${TAG}_write.json 2> gpurun_out/${TAG}_write.log &&
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d gpurun_out/${TAG}_tccreq -o pmc --output-format csv -- $B > gpurun_out/${TAG}_tccreq.json 2> gpurun_out/${TAG}_tccreq.log &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_sq -o pmc --output-format csv -- $B > gpurun_out/${TAG}_sq.json 2> gpurun_out/${TAG}_sq.log &&
timeout -k 10 120 tools/_build/calib_gather 4096 > gpurun_out/${TAG}_calib.json 2> gpurun_out/${TAG}_calib.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_calib_fetch -o pmc --output-format csv -- tools/_build/calib_gather 4096 > /dev/null 2> gpurun_out/${TAG}_calib_fetch.log &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d gpurun_out/${TAG}_calib_tcc -o pmc --output-format csv -- tools/_build/calib_gather 4096 > /dev/null 2> gpurun_out/${TAG}_calib_tcc.log
echo EXIT $?
