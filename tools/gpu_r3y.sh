#!/bin/bash
# Per-row text-compare entries (srow): parity over the direct start, the deep kernels and the
# level path, then C3 / C2 device legs with the entries on and off.
export TMPDIR=/tmp
TAG=${1:-r3y}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTS:-wide_kmer or packed_direct or pair or single_row or deferred or random_eds or deep_overflow or kmer_start or larger_eds or c3_production or c2_production or smoke}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_ab3.sh ${TAG} c3 20 X=1 EDSBWT_SROW=0 X=2 || exit 1
bash tools/gpu_ab3.sh ${TAG}c2 c2 20 X=1 EDSBWT_SROW=0
