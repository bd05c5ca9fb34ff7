#!/bin/bash
# C5 with a depth-4 k-mer start table (EDSBWT_KTAB_ITEMS=2e9): why the A/B line was missing.
export TMPDIR=/tmp
TAG=${1:-r3kt4}
mkdir -p gpurun_out
EDSBWT_KTAB_ITEMS=2000000000 timeout -k 10 500 python bench.py --config c5 --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.log
rc=$?
tail -30 gpurun_out/${TAG}_bench_c5.log
echo EXIT $rc
