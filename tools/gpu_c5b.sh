#!/bin/bash
# GPU parity suite, then a kernel trace of one C5 step.   bash tools/gpu_c5b.sh <tag>
export TMPDIR=/tmp
TAG=${1:-c5b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
bash tools/gpu_c5trace.sh $TAG
