#!/bin/bash
# Kernel + memory-copy trace of a short end-to-end bench run (no PMC).   bash tools/gpu_copytrace.sh <tag> [bench args]
export TMPDIR=/tmp
TAG=${1:-ct}; shift
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/${TAG}_ct -o ct --output-format csv -- python3 bench.py --no-cpu --no-device --steps 2 --warmup 1 "$@" > gpurun_out/${TAG}_ct.json 2> gpurun_out/${TAG}_ct.log
echo EXIT $?
