#!/bin/bash
# Full parity suite, then the round-2 profiles (device-resident leg only) and the C2 line.
export TMPDIR=/tmp
TAG=${1:-r2f}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
bash tools/gpu_profiles_r2.sh $TAG
