#!/bin/bash
# Kernel trace of a short bench run.   bash tools/gpu_trace.sh <tag> [bench args]
export TMPDIR=/tmp
TAG=${1:-tr}; shift
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/${TAG}_trace.json 2> gpurun_out/${TAG}_trace.log
echo EXIT $?
