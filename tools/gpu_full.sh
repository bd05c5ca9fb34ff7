#!/bin/bash
# The whole GPU test suite, one process, each test under its own time limit.
export TMPDIR=/tmp
TAG=${1:-full}
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
exit $rc
