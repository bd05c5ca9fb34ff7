# round-5 GPU pass af: the device-invariant build (libedsbwt_dbg.so: queue slots, packed lengths, wide
# entries, list intervals checked on the device; a violation fails the search) with every fresh
# allocation poisoned, over the parity tests that reach k_deep / k_deep_direct / the level walk
export TMPDIR=/tmp
EDSBWT_LIB=$PWD/eds-bwt_amd/_build/libedsbwt_dbg.so EDSBWT_POISON=1 bash tools/gpu.sh r5af "test:k_deep_builds or random_eds or wide_kmer or packed_direct or level_table or device_ids or c5_style or readme or deferred or grouped" || exit 1
