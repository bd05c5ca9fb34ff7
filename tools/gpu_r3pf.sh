#!/bin/bash
# k_lvl_items and k_lvl_dollar loading each lane's next item one iteration ahead (EDSBWT_LVL_PREFETCH): parity over the level
# walks (random EDSs, grouped / C5-style, production C2 / C5), then C5 with the prefetch on and off.
export TMPDIR=/tmp
TAG=${1:-r3pf}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "${TESTS:-readme_kat or example_paper or random_eds or larger_eds or long_patterns or c5_style or grouped or short_patterns or kmer_start or rank16 or legacy or c5_production or c2_production}" \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_ab3.sh ${TAG} c5 3 X=1 EDSBWT_LVL_PREFETCH=0 X=2
