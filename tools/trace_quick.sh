#!/bin/bash
# rocprofv3 kernel trace of a short bench run: bash tools/trace_quick.sh <tag> [bench args...]
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG} -o trace --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.log
