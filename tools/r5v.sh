# round-5 GPU pass v: k_deep_direct with the next pattern's offsets loaded one iteration ahead —
# direct-start parity, then C3 A/B against the previous build (libedsbwt_ab0.so)
export TMPDIR=/tmp
bash tools/gpu.sh r5v "test:wide_kmer or packed_direct or c3_production or deferred or readme" || exit 1
bash tools/gpu.sh r5v ab:c3:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0 || exit 2
bash tools/gpu.sh r5v2 ab:c3:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so || exit 3
