#!/bin/bash
# Occupancy round: parity over the direct start and the level path, then C3 (k_deep_direct 7 / 8
# waves) and C5 (level step 7 / 8 waves) device legs.
export TMPDIR=/tmp
TAG=${1:-r3w}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTS:-wide_kmer or packed_direct or pair or single_row or deferred or random_eds or deep_overflow or kmer_start or c5_style or grouped or c3_production or smoke}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_ab3.sh ${TAG} c3 20 X=1 EDSBWT_DIRECT_WAVES=8 X=2 || exit 1
bash tools/gpu_ab3.sh ${TAG}c5 c5 2 X=1 EDSBWT_LVL_WAVES=8
