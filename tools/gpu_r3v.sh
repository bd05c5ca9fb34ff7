#!/bin/bash
# k_deep_direct: parity tests of the direct start, then occupancy A/B on C3 and C2.
export TMPDIR=/tmp
TAG=${1:-r3v}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTS:-wide_kmer or packed_direct or pair or single_row or deferred or c3_production or c2_production or smoke}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_ab3.sh ${TAG} c3 20 X=1 EDSBWT_DIRECT_WAVES=7 EDSBWT_DIRECT_WAVES=8 EDSBWT_DEEP_DIRECT=0 X=2 || exit 1
bash tools/gpu_ab3.sh ${TAG}c2 c2 20 X=1 EDSBWT_DIRECT_WAVES=7 EDSBWT_DEEP_DIRECT=0
