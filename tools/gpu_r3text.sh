#!/bin/bash
# Text items in the count-only level walk, the per-row entries built after the k-mer table:
# parity (random EDSs through _compare incl. count-only level walks, grouped / C5-style,
# production C2 / C3 / C5), then C5 with text items on and off, then the C3 line.
export TMPDIR=/tmp
TAG=${1:-r3text}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "${TESTS:-readme_kat or example_paper or random_eds or larger_eds or long_patterns or c5_style or grouped or short_patterns or kmer_start or rank16 or deep_overflow or c5_production or c2_production or c3_production}" \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_ab3.sh ${TAG} c5 3 X=1 EDSBWT_TEXT_ITEMS=0 || exit 1
bash tools/gpu_ab3.sh ${TAG}c3 c3 20 X=1
