#!/bin/bash
# Round-2 GPU pass: parity tests (incl. production-scale C2/C3), the default bench line,
# the dependent-chain gather calibration.   bash tools/gpu_r2.sh <tag> [pytest -k expr]
export TMPDIR=/tmp
TAG=${1:-r2}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread "${KARG[@]}" > gpurun_out/${TAG}_pytest_gpu.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log &&
timeout -k 10 120 tools/_build/calib_gather --chain 100 1024 > gpurun_out/${TAG}_calib_chain.json 2>&1
echo EXIT $?
