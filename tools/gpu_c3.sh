#!/bin/bash
# GPU parity tests, then the C3 bench line and a kernel trace of a short C3 run.
#   bash tools/gpu_c3.sh <tag> [extra bench args]
export TMPDIR=/tmp
TAG=${1:-c3}; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/${TAG}_trace.json 2> gpurun_out/${TAG}_trace.log
