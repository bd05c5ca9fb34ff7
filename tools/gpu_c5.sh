#!/bin/bash
# GPU parity suite, then the C5 bench line.   bash tools/gpu_c5.sh <tag> [extra bench args]
export TMPDIR=/tmp
TAG=${1:-c5}
shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 600 python bench.py --config c5 --no-cpu "$@" > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.log || { echo BENCH_FAIL; tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
cat gpurun_out/${TAG}_bench_c5.json
