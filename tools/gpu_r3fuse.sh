#!/bin/bash
# Count-only finishing fused into the level step, the segment-chain bitmap in k_run_flags and
# two-character steps in k_deep: parity (random EDSs through _compare, grouped / C5-style
# searches, the pair / deferred / overflow cases, production C2 / C5), then C5 with the fusion
# on and off, then the C3 device-resident line.
export TMPDIR=/tmp
TAG=${1:-r3fuse}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "${TESTS:-readme_kat or example_paper or random_eds or larger_eds or long_patterns or c5_style or grouped or short_patterns or kmer_start or rank16 or pair_blocks or deferred or deep_overflow or packed_direct or wide_kmer or single_row or c5_production or c2_production or c3_production}" \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_ab3.sh ${TAG} c5 3 X=1 EDSBWT_FUSE_FINISH=0 || exit 1
bash tools/gpu_ab3.sh ${TAG}c3 c3 20 X=1 X=2
