#!/bin/bash
# Device-resident A/B of engine switches: bash tools/gpu_ab3.sh TAG CONFIG STEPS "A=1,B=2" "C=0" ...
# (each argument after STEPS is one variant: comma-separated environment assignments)
export TMPDIR=/tmp
TAG=$1; CFG=$2; STEPS=$3; shift 3
mkdir -p gpurun_out
for spec in "$@"; do
  echo "== $CFG $spec" >> gpurun_out/${TAG}_ab.txt
  env ${spec//,/ } timeout -k 10 300 python bench.py --config $CFG --no-cpu --no-e2e --steps $STEPS --warmup 3 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(round(d['value']), d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" \
    >> gpurun_out/${TAG}_ab.txt || exit 1
done
cat gpurun_out/${TAG}_ab.txt
