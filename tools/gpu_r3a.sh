#!/bin/bash
# Round 3: the whole GPU parity suite (incl. the C4 / C5 production tests), then a default bench line.
export TMPDIR=/tmp
TAG=${1:-r3a}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest_gpu.log
