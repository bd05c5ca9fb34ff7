#!/bin/bash
# Parity tests, then A/B bench lines (no CPU leg) under env settings.
#   bash tools/gpu_ab.sh <tag> "ENV=1 ENV2=x" "ENV=0" ...     (first arg after tag may be "-" for no tests)
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
if [ "$1" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
else shift; fi
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_ab$i.json 2> gpurun_out/${TAG}_ab$i.log || { echo BENCH_FAIL $i; tail -20 gpurun_out/${TAG}_ab$i.log; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_ab$i.json'));r=d.get('device_resident',{});print('$e', 'e2e', d['value'], d['ms_per_step'], 'dev', r.get('value'), r.get('ms_per_step'), r.get('kernel_ms_per_step'))"
done
echo EXIT 0
