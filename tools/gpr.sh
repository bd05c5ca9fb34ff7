#!/bin/bash
# gpurun with retries while no box/slot is free (nothing ran, nothing charged); any other outcome returns
for i in $(seq 1 ${R:-10}); do
  out=$(timeout 2400 /usr/local/graft/bin/gpurun --timeout ${T:-1200} -- "$1" 2>&1)
  if echo "$out" | grep -q "status=transient"; then echo "[gpr] attempt $i: no box ($(date +%T))"; sleep 120; continue; fi
  echo "$out" | tail -${N:-25}; exit 0
done
echo "[gpr] gave up"
