#!/bin/bash
# C5 breakdown: the 200K mixed batch and each length class, per kernel class, with per-depth
# trace lines (EDSBWT_TRACE=1: items, single-row items, link keys, step lines per depth and group).
export TMPDIR=/tmp
TAG=${1:-r3c}
mkdir -p gpurun_out
EDSBWT_TRACE=1 timeout -k 10 900 python tools/c5_breakdown.py --steps 2 > gpurun_out/${TAG}_c5_breakdown.json 2> gpurun_out/${TAG}_c5_breakdown.log
echo EXIT $?
