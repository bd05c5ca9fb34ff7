# round-5 GPU pass x: k_deep_direct built without its per-lane work counters (EDSBWT_DEEP_STATS=0):
# parity, then C3 A/B on one box
export TMPDIR=/tmp
bash tools/gpu.sh r5x "test:wide_kmer or packed_direct" || exit 1
bash tools/gpu.sh r5x ab:c3:EDSBWT_DEEP_STATS=0:EDSBWT_DEEP_STATS=1:EDSBWT_DEEP_STATS=0 || exit 2
bash tools/gpu.sh r5x2 ab:c3:EDSBWT_DEEP_STATS=1:EDSBWT_DEEP_STATS=0:EDSBWT_DEEP_STATS=1 || exit 3
