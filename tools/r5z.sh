# round-5 GPU pass z: k_deep on 32-bit queue indices and a 32-bit term counter in k_deep_direct —
# parity, C3 A/B against the previous build (libedsbwt_ab0.so), and k_deep at 6 waves per SIMD
export TMPDIR=/tmp
bash tools/gpu.sh r5z "test:wide_kmer or packed_direct or c3_production or deferred or readme or random_eds or k_deep_builds" || exit 1
bash tools/gpu.sh r5z ab:c3:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0 || exit 2
bash tools/gpu.sh r5z2 ab:c3:EDSBWT_DEEPQ_WAVES=6:EDSBWT_TRACE=0:EDSBWT_DEEPQ_WAVES=6 || exit 3
