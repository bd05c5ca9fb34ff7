#!/bin/bash
# e2e tail study (C3): cgroup CPU limits on the box, then per-call walls over 30 calls with the
# default host pipeline, with fewer pack threads, and with the C2 upload variants.
export TMPDIR=/tmp
TAG=${1:-r3f}
mkdir -p gpurun_out
{ cat /sys/fs/cgroup/cpu.max 2>&1; cat /proc/self/status | grep -i cpus_allowed_list; nproc; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/${TAG}_host.txt 2>&1
w() { python -c "import json,sys; d=json.loads(sys.stdin.readline()); e=d['e2e']; print(d['value'], d['ms_per_step'], e['ms_wall_median'], e['ms_wall_p90'], e['ms_wall_max'], e['ms_walls'])"; }
for spec in "X=1" "EDSBWT_HOST_THREADS=8" "EDSBWT_HOST_THREADS=16" "X=2"; do
  echo "== c3 $spec" >> gpurun_out/${TAG}_walls.txt
  env $spec timeout -k 10 200 python bench.py --no-cpu --no-device --steps 30 --warmup 3 2>/dev/null | w >> gpurun_out/${TAG}_walls.txt || exit 1
done
for spec in "X=1" "EDSBWT_PACK_LINES=0" "EDSBWT_PACK_LINES=0 EDSBWT_CHUNK_SINGLE_MB=0 EDSBWT_CHUNK_MB=8" "EDSBWT_CHUNK_SINGLE_MB=0 EDSBWT_CHUNK_MB=8" "EDSBWT_PACK_LINES=0 EDSBWT_CHUNK_SINGLE_MB=0 EDSBWT_CHUNK_MB=16"; do
  echo "== c2 $spec" >> gpurun_out/${TAG}_walls.txt
  env $spec timeout -k 10 200 python bench.py --config c2 --no-cpu --no-device --steps 30 --warmup 3 2>/dev/null | w >> gpurun_out/${TAG}_walls.txt || exit 1
done
echo EXIT $?
