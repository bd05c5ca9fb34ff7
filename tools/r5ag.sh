# round-5 GPU pass ag: the C4 line on one GPU (the fixed 100M batch) and the EDSBWTsearch CLI on C3
# (bs took / search phase, CSV head and tail against the oracle) on the final tree
export TMPDIR=/tmp
bash tools/gpu.sh r5ag quick:c4:3 cli:c3 || exit 1
