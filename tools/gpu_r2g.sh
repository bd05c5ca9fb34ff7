#!/bin/bash
# Parity suite, the default bench line (C3, with the CPU baseline and parity sample), then the
# round-2 profiles.   bash tools/gpu_r2g.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r2g}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log || { echo BENCH_FAIL; tail -30 gpurun_out/${TAG}_bench_c3.log; exit 1; }
cat gpurun_out/${TAG}_bench_c3.json
bash tools/gpu_profiles_r2.sh $TAG
