# round-5 GPU pass t: the segment link + two characters table (k_deep_direct's links past a matched
# word in one read): parity on the direct-start tests and the C3 production test, then the C3 A/B
export TMPDIR=/tmp
bash tools/gpu.sh r5t "test:wide_kmer or packed_direct or single_row_text or c3_production or random_eds or readme or deferred" || exit 1
bash tools/gpu.sh r5t ab:c3:EDSBWT_SEGTAB3=1:EDSBWT_SEGTAB3=0:EDSBWT_SEGTAB3=1 || exit 2
