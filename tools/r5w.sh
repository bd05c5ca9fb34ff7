# round-5 GPU pass w: k_deep_direct without the split-walk / segtab3 code (back to round 5's lean
# kernel): direct-start parity, then C3 A/B against the build that carried them (libedsbwt_ab0.so)
export TMPDIR=/tmp
bash tools/gpu.sh r5w "test:wide_kmer or packed_direct or c3_production or deferred or readme or random_eds" || exit 1
bash tools/gpu.sh r5w ab:c3:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0 || exit 2
bash tools/gpu.sh r5w2 ab:c3:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so || exit 3
