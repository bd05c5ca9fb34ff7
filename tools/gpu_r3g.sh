#!/bin/bash
# C3 end-to-end A/B of the host pipeline's chunk ramp (EDSBWT_RAMP_STEPS) and chunk size.
export TMPDIR=/tmp
TAG=${1:-r3g}
mkdir -p gpurun_out
w() { python -c "import json,sys; d=json.loads(sys.stdin.readline()); e=d['e2e']; print(d['value'], d['ms_per_step'], e['ms_wall_median'], e['ms_wall_p90'], e['ms_wall_max'], e['chunks'])"; }
for spec in "X=1" "EDSBWT_RAMP_STEPS=4" "EDSBWT_RAMP_STEPS=5" "EDSBWT_RAMP_STEPS=6" "EDSBWT_RAMP_STEPS=5 EDSBWT_CHUNK_MB=32" "EDSBWT_RAMP_STEPS=5 EDSBWT_CHUNK_MB=56" "X=2"; do
  echo "== c3 $spec" >> gpurun_out/${TAG}_walls.txt
  env $spec timeout -k 10 200 python bench.py --no-cpu --no-device --steps 30 --warmup 3 2>/dev/null | w >> gpurun_out/${TAG}_walls.txt || exit 1
done
echo EXIT $?
