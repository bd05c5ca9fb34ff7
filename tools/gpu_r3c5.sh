#!/bin/bash
# C5: a depth-4 k-mer start table (EDSBWT_KTAB_ITEMS=2e9: 1.8G intervals) against the default
# budget (depth 3), then the C5 bench line with its located >= 32-mers.
export TMPDIR=/tmp
TAG=${1:-r3c5}
mkdir -p gpurun_out
bash tools/gpu_ab3.sh ${TAG} c5 3 X=1 EDSBWT_KTAB_ITEMS=2000000000 || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 ${C5ENV:-} > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.log
echo EXIT $?
