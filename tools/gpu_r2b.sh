#!/bin/bash
# GPU pass: full parity suite, then the default bench line (no CPU leg) and a traced e2e run.
#   bash tools/gpu_r2b.sh <tag> [pytest -k expr]
export TMPDIR=/tmp
TAG=${1:-r2b}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread "${KARG[@]}" > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || { echo BENCH_FAIL; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
EDSBWT_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu --no-device --steps 2 --warmup 2 > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.log
echo EXIT $?
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('e2e',d['value'],d['ms_per_step'],'dev',d['device_resident']['value'],d['device_resident']['ms_per_step'],d['device_resident']['kernel_ms_per_step'])"
