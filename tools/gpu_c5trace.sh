#!/bin/bash
# Kernel trace of one C5 step (device-resident leg).   bash tools/gpu_c5trace.sh <tag>
export TMPDIR=/tmp
TAG=${1:-c5t}
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- python3 bench.py --config c5 --no-cpu --no-e2e --steps 1 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || { echo FAIL; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
cat gpurun_out/${TAG}_bench.json
