#!/bin/bash
# C5 level-step counters: kernel trace + one TCC pass (requests, DRAM bytes, L2 hit/miss) of one
# device-resident C5 step, to see how many of the step's modelled lines reach the L2 / DRAM.
export TMPDIR=/tmp
TAG=${1:-r3k}
mkdir -p gpurun_out
B="python3 bench.py --config c5 --no-cpu --no-e2e --steps 1 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_tcc -o pmc --output-format csv -- $B > gpurun_out/${TAG}_tcc.json 2> gpurun_out/${TAG}_tcc.log
echo EXIT $?
EDSBWT_TRACE=1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 1 --warmup 1 > gpurun_out/${TAG}_c3_trace.json 2> gpurun_out/${TAG}_c3_trace.log
echo EXIT2 $?
