# round-5 GPU pass y: k_deep_direct on 32-bit pattern indices — direct-start parity, then C3 A/B
# against the previous build (libedsbwt_ab0.so) on one box
export TMPDIR=/tmp
bash tools/gpu.sh r5y "test:wide_kmer or packed_direct or c3_production or deferred" || exit 1
bash tools/gpu.sh r5y ab:c3:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0 || exit 2
bash tools/gpu.sh r5y2 ab:c3:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so:EDSBWT_TRACE=0:EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so || exit 3
