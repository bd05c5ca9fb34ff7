# round-5 GPU pass r: PMC profile of C5's located step (its headline since round 5)
export TMPDIR=/tmp
bash tools/gpu.sh r5r prof:c5:loc || exit 1
