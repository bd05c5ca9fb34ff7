# round-5 GPU pass h: fused record-offset tiles (parity + C3 A/B)
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "random_eds or wide_kmer or packed_direct or single_row or deferred or locate or search_lines_packed or k_deep_builds or readme or larger_eds" > gpurun_out/r5h_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5h_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu.sh r5h ab:c3:EDSBWT_TILE_FUSE=1:EDSBWT_TILE_FUSE=0:EDSBWT_TILE_FUSE=1 || exit 2
