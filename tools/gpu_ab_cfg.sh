#!/bin/bash
# A/B bench lines of one config under env settings (no CPU leg, no tests).
#   bash tools/gpu_ab_cfg.sh <tag> <config> "ENV=1 ENV2=x" "ENV=0" ...
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --config $CFG --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_ab$i.json 2> gpurun_out/${TAG}_ab$i.log || { echo BENCH_FAIL $i; tail -20 gpurun_out/${TAG}_ab$i.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_ab$i.json'));r=d.get('device_resident',{});print('$e', 'e2e', d['value'], d['ms_per_step'], 'dev', r.get('value'), r.get('ms_per_step'), r.get('kernel_ms_per_step'), 'ktab', d['config']['ktab_depth'], 'open', d['index_open_s'], r.get('engine',{}).get('start_depth'), r.get('engine',{}).get('depths'))"
done
echo EXIT 0
