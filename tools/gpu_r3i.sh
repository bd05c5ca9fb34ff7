#!/bin/bash
# Multi-rank rehearsal on one GPU (2 ranks over gloo: per-rank parity sample + counts gather
# in the timed step) and the host-contention rehearsal (tools/host_contention.py).
export TMPDIR=/tmp
TAG=${1:-r3i}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/${TAG}_gloo2_c3.json 2> gpurun_out/${TAG}_gloo2_c3.log &&
timeout -k 10 700 python tools/host_contention.py --procs 0,1,2,3 --threads 2 --steps 30 > gpurun_out/${TAG}_contention.json 2> gpurun_out/${TAG}_contention.log
echo EXIT $?
