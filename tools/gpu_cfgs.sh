#!/bin/bash
# Parity suite, then the C3, C2 and C5 bench lines (no CPU leg).   bash tools/gpu_cfgs.sh <tag> [skip-tests]
export TMPDIR=/tmp
TAG=${1:-cfg}
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
fi
for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.log || { echo BENCH_FAIL $c; tail -20 gpurun_out/${TAG}_bench_$c.log; exit 1; }
done
timeout -k 10 600 python -u bench.py --config c5 --no-cpu --steps 1 --warmup 1 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.log || { echo BENCH_FAIL c5; tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
for c in c3 c2 c5; do
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));r=d.get('device_resident',{});print('$c', 'e2e', d['value'], d['ms_per_step'], 'dev', r.get('value'), r.get('ms_per_step'), r.get('kernel_ms_per_step'), 'ktab', d['config']['ktab_depth'], 'open', d['index_open_s'], 'bytes', d['config']['index_device_bytes'], r.get('engine'))"
done
echo EXIT 0
